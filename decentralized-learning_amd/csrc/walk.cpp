// walk.cpp — the host path's one-pass walk over every parameter of every model, in native code.
//
// FedAvg.aggregate (accdfl/core/gradient_aggregation/fedavg.py:23-25) touches every parameter of every
// model: `for m, w in zip(models, weights): for c1, p1 in zip(center.parameters(), m.parameters())`.
// The MI355X path needs, once per round, each parameter's host or device pointer, checked against
// models[0]'s shapes, one dtype, one device and dense storage (accdfl_amd fedavg._host_layout /
// _device_layout).  In Python every parameter costs ~0.8 us of attribute lookups (128 google_speech
// ResNet-34 models: 14 080 parameters, ~10 ms — more than the whole device-resident reduce); here it
// is a few tens of nanoseconds.
//
// layout(models, device, plain) walks each model exactly as nn.Module.parameters() does — pre-order
// over modules through `_modules`, each module's `_parameters` in order, a module or parameter seen
// before skipped — for module classes in `plain` (classes that keep nn.Module's own walk; the caller
// decides and caches that).  It returns None when a model's tree holds another class or the round
// does not qualify (then the caller's general path handles it), else
//     (dtype name, [numel of each of models[0]'s parameters], pointer table bytearray, device index)
// with the table tensor-major ([n_tensors][n_models] uint64) or peer-major ([n_models][n_tensors]).
// `device`: -1 for CPU parameters, a HIP device index every parameter must be on, or -2 for the HIP
// device of models[0]'s first parameter (the returned device index; -1 for CPU).  `ref`, when given, is a
// model outside the list whose parameters set the layout (shapes, dtype, device) every listed model must
// match — a round laid out group by group checks each group against its first model this way — and is
// not part of the table.
//
// This is host plumbing of the Python binding, not part of the C ABI (include/dlagg.h): it takes
// Python objects and is built against torch's headers.
#include <torch/extension.h>
#include <torch/csrc/autograd/python_variable.h>
#include <pybind11/numpy.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#ifndef DLA_WALK_BUILD_ID
#define DLA_WALK_BUILD_ID "unversioned"
#endif

namespace {

// Embedded as plain bytes too, so the build's id can be read from the file without loading it.
__attribute__((used)) const char kWalkIdTag[] = "dlagg-walk-build-id:" DLA_WALK_BUILD_ID;

// The objects one walk has met (modules, parameters): open addressing with linear probing over a
// power-of-two table of (address, stamp) slots, emptied in O(1) by moving to the next stamp.  A
// node-based std::unordered_set allocates on every insert, which was most of the walk's cost per parameter.
class PtrSet {
 public:
  PtrSet() : slots_(256) {}
  void clear() {
    size_ = 0;
    if (++stamp_ == 0) {  // stamps wrapped: forget every slot for real
      std::fill(slots_.begin(), slots_.end(), Slot{});
      stamp_ = 1;
    }
  }
  // true if `p` was not in the set (and is now)
  bool insert(PyObject* p) {
    if (2 * (size_ + 1) > slots_.size()) grow();
    Slot& s = find(p);
    if (s.stamp == stamp_) return false;
    s = Slot{p, stamp_};
    ++size_;
    return true;
  }

 private:
  struct Slot {
    PyObject* p = nullptr;
    uint32_t stamp = 0;
  };
  Slot& find(PyObject* p) {
    const size_t mask = slots_.size() - 1;
    size_t i = (reinterpret_cast<uintptr_t>(p) >> 4) * 0x9E3779B97F4A7C15ull >> 20 & mask;
    while (slots_[i].stamp == stamp_ && slots_[i].p != p) i = (i + 1) & mask;
    return slots_[i];
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(old.size() * 2, Slot{});
    for (const Slot& s : old)
      if (s.stamp == stamp_) find(s.p) = s;
  }
  std::vector<Slot> slots_;
  size_t size_ = 0;
  uint32_t stamp_ = 1;
};

// Interned attribute names (their hashes cached): a module's dicts are looked up without making a str
// per lookup (PyDict_GetItemString does), ~0.1 us a module of a model's walk.
PyObject* interned(const char* s) {
  PyObject* o = PyUnicode_InternFromString(s);
  if (!o) throw py::error_already_set();
  return o;  // immortal for the module's lifetime
}
PyObject* const kParameters = interned("_parameters");
PyObject* const kBuffers = interned("_buffers");
PyObject* const kModules = interned("_modules");

// One model's parameters in nn.Module.parameters() order (`which` = "_parameters"; "_buffers": its
// buffers in nn.Module.buffers() order); false if a class is not plain.
bool walk(PyObject* mod, PyObject* plain, PtrSet& seen_m, PtrSet& seen_p, std::vector<PyObject*>& out,
          PyObject* which = kParameters) {
  if (!seen_m.insert(mod)) return true;
  const int ok = PySet_Contains(plain, reinterpret_cast<PyObject*>(Py_TYPE(mod)));
  if (ok != 1) {
    if (ok < 0) PyErr_Clear();
    return false;
  }
  PyObject** dp = _PyObject_GetDictPtr(mod);  // the instance __dict__ (borrowed)
  PyObject* d = dp ? *dp : nullptr;
  if (!d || !PyDict_Check(d)) return false;
  PyObject* params = PyDict_GetItemWithError(d, which);  // borrowed
  PyObject* mods = params ? PyDict_GetItemWithError(d, kModules) : nullptr;
  if (!mods && PyErr_Occurred()) PyErr_Clear();
  bool good = params && mods && PyDict_Check(params) && PyDict_Check(mods);
  if (good) {
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(params, &pos, &k, &v)) {
      if (v == Py_None || !seen_p.insert(v)) continue;
      out.push_back(v);
    }
    pos = 0;
    while (good && PyDict_Next(mods, &pos, &k, &v)) {
      if (v == Py_None) continue;
      good = walk(v, plain, seen_m, seen_p, out, which);
    }
  }
  return good;
}

const char* dtype_name(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return "float32";
    case at::kBFloat16: return "bfloat16";
    case at::kHalf: return "float16";
    case at::kDouble: return "float64";
    default: return nullptr;
  }
}

py::object layout(py::list models, int device, py::object plain, bool tensor_major, py::object ref) {
  const Py_ssize_t n = static_cast<Py_ssize_t>(py::len(models));
  if (n < 1 || !PySet_Check(plain.ptr())) return py::none();
  std::vector<PyObject*> ps;
  std::vector<at::Tensor> p0;  // the reference layout: `ref`'s parameters, else models[0]'s
  std::vector<uint64_t> ptrs;
  at::ScalarType dt = at::kFloat;
  PtrSet seen_m, seen_p;  // per model, cleared (table kept) between models
  // m = -1: `ref` (a model of the round outside this list — the first model of a round laid out group
  // by group), walked for the layout only
  for (Py_ssize_t m = ref.is_none() ? 0 : -1; m < n; ++m) {
    ps.clear();
    seen_m.clear();
    seen_p.clear();
    if (!walk(m < 0 ? ref.ptr() : PyList_GET_ITEM(models.ptr(), m), plain.ptr(), seen_m, seen_p, ps)) return py::none();
    if (p0.empty()) {
      if (ps.empty()) return py::none();
      ptrs.resize(static_cast<size_t>(n) * ps.size());
    } else if (ps.size() != p0.size()) {
      return py::none();
    }
    const size_t nt = ps.size();
    const bool first = p0.empty();
    for (size_t t = 0; t < nt; ++t) {
      if (!THPVariable_Check(ps[t])) return py::none();
      const at::Tensor& x = THPVariable_Unpack(ps[t]);
      if (first) {
        if (t == 0) {
          dt = x.scalar_type();
          if (!dtype_name(dt)) return py::none();
          if (device == -2) {
            if (!x.is_cuda()) return py::none();
            device = x.get_device();
          }
        }
        p0.push_back(x);
      } else if (x.sizes() != p0[t].sizes()) {
        return py::none();
      }
      if (x.scalar_type() != dt || !x.is_contiguous() || !x.has_storage()) return py::none();
      if (device < 0 ? !x.is_cpu() : !(x.is_cuda() && x.get_device() == device)) return py::none();
      if (m >= 0) ptrs[tensor_major ? t * n + m : m * nt + t] = reinterpret_cast<uint64_t>(x.data_ptr());
    }
  }
  py::list numels;
  for (const at::Tensor& x : p0) numels.append(x.numel());
  // writable, so the caller's ctypes / numpy views of it need no copy
  py::bytearray table(reinterpret_cast<const char*>(ptrs.data()), ptrs.size() * sizeof(uint64_t));
  return py::make_tuple(py::str(dtype_name(dt)), numels, table, device);
}

// (parameters, buffers) of one model as lists, in parameters() / buffers() order, or None when its tree
// holds a class outside `plain`: the result module's fresh tensors are made from these without another
// Python walk of models[0] (fedavg._device_round).
py::object tensors(py::object model, py::object plain) {
  if (!PySet_Check(plain.ptr())) return py::none();
  PtrSet seen_m, seen_p;
  std::vector<PyObject*> ps, bs;
  if (!walk(model.ptr(), plain.ptr(), seen_m, seen_p, ps)) return py::none();
  seen_m.clear();
  seen_p.clear();
  if (!walk(model.ptr(), plain.ptr(), seen_m, seen_p, bs, kBuffers)) return py::none();
  py::list pl, bl;
  for (PyObject* o : ps) pl.append(py::reinterpret_borrow<py::object>(o));
  for (PyObject* o : bs) bl.append(py::reinterpret_borrow<py::object>(o));
  return py::make_tuple(pl, bl);
}

// A model's parameters' identities as bytes — (object address, data pointer, in-place version counter) of
// each, parameters() order — or None when its tree holds a class outside `plain`.  DeviceModelManager
// compares these at aggregation time with the ones taken when the model was staged into HBM on arrival
// (a registered model written in place since no longer matches, accdfl/core/model_manager.py:42-47): a few
// microseconds per ResNet-34 model here against ~60 us of Python (128 models: ~8 ms per round).
py::object fingerprint(py::object model, py::object plain) {
  if (!PySet_Check(plain.ptr())) return py::none();
  PtrSet seen_m, seen_p;
  std::vector<PyObject*> ps;
  if (!walk(model.ptr(), plain.ptr(), seen_m, seen_p, ps)) return py::none();
  std::vector<uint64_t> v;
  v.reserve(3 * ps.size());
  for (PyObject* o : ps) {
    if (!THPVariable_Check(o)) return py::none();
    const at::Tensor& x = THPVariable_Unpack(o);
    v.push_back(reinterpret_cast<uint64_t>(o));
    v.push_back(x.has_storage() ? reinterpret_cast<uint64_t>(x.data_ptr()) : 0);
    v.push_back(static_cast<uint64_t>(x._version()));
  }
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(uint64_t));
}

// (addresses, byte lengths) of a list of byte blocks as two int64 arrays — the block list an EVA transfer
// receives (accdfl/util/eva/transfer/incoming.py:35 joins it; accdfl_amd.core.wire reads it in place):
// ~1 700 blocks per 100 MB model, a few nanoseconds each here against ~0.2 us of Python per block.
// bytes objects are read directly; any other block through the buffer protocol (C-contiguous, e.g. the
// memoryview halves wire.split_blocks cuts), whose address stays valid while the block lives.
py::tuple block_table(py::list blocks) {
  const py::ssize_t n = PyList_GET_SIZE(blocks.ptr());
  py::array_t<int64_t> addrs(n), lens(n);
  int64_t* a = addrs.mutable_data();
  int64_t* l = lens.mutable_data();
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(blocks.ptr(), i);
    if (PyBytes_CheckExact(o)) {
      a[i] = reinterpret_cast<int64_t>(PyBytes_AS_STRING(o));
      l[i] = PyBytes_GET_SIZE(o);
      continue;
    }
    Py_buffer view;
    if (PyObject_GetBuffer(o, &view, PyBUF_C_CONTIGUOUS) != 0) throw py::error_already_set();
    a[i] = reinterpret_cast<int64_t>(view.buf);
    l[i] = view.len;
    PyBuffer_Release(&view);
  }
  return py::make_tuple(addrs, lens);
}

// A tensor over part of `flat`'s allocation with the given sizes, strides and element offset, holding a
// storage of its OWN (its bytes only) whose data pointer keeps `flat`'s storage alive: what deepcopy
// gives each tensor (a storage per tensor, so pickle.dumps(state_dict()) — the reference's
// serialize_model — writes each tensor's bytes once, not the whole allocation per tensor), while the
// reduce and the buffer gather still write ONE allocation.  Same dtype, device and dispatch keys as
// `flat`, no view or autograd history, metadata changeable; resizable through `flat`'s allocator, or the
// device's default one (a resize reallocates and lets go of `flat`).  One TensorImpl, no dispatched op.
at::Tensor alias_of(const at::Tensor& flat, at::IntArrayRef sizes, at::IntArrayRef strides, int64_t offset) {
  const int64_t es = static_cast<int64_t>(flat.element_size());
  int64_t extent = 1;  // elements the tensor spans
  for (size_t d = 0; d < sizes.size(); ++d) {
    if (sizes[d] == 0) {
      extent = 0;
      break;
    }
    extent += (sizes[d] - 1) * strides[d];
  }
  char* base = static_cast<char*>(flat.data_ptr()) + offset * es;
  if (offset < 0 || (offset + extent) * es > static_cast<int64_t>(flat.nbytes()))
    throw std::invalid_argument("alias_of: outside the allocation");
  auto* keep = new c10::Storage(flat.storage());  // released by the DataPtr's deleter
  c10::DataPtr dp(base, keep, [](void* ctx) { delete static_cast<c10::Storage*>(ctx); }, flat.device());
  at::Allocator* alloc = flat.storage().allocator();  // none for memory torch did not allocate (a pool's)
  if (!alloc) alloc = c10::GetAllocator(flat.device().type());
  c10::Storage st(c10::Storage::use_byte_size_t(), static_cast<size_t>(extent * es), std::move(dp), alloc,
                  /*resizable=*/alloc != nullptr);
  auto impl = c10::make_intrusive<c10::TensorImpl>(std::move(st), flat.key_set(), flat.dtype());
  impl->set_sizes_and_strides(sizes, strides, 0);
  impl->set_allow_tensor_metadata_change(true);
  return at::Tensor(std::move(impl));
}

// Fresh tensors like a given one (sizes, strides, dtype, device; no data) straight from the allocator torch's
// own tensors of that device come from — one allocate() and one TensorImpl each, no dispatched op (~0.6 us
// a tensor less than at::empty_strided).  The DataPtr is the allocator's own (its deleter and context), so
// the caching allocator knows the block: record_stream and CUDA IPC work as on any torch tensor.  Dense
// device tensors only; anything else through at::empty_strided.
class FreshAlloc {
 public:
  at::Tensor like(const at::Tensor& p) {
    if (!(p.is_cuda() && p.is_contiguous() && p.layout() == at::kStrided))
      return at::empty_strided(p.sizes(), p.strides(), at::TensorOptions().dtype(p.scalar_type()).device(p.device()));
    if (!guard_ || guard_->current_device() != p.device()) {
      guard_.emplace(p.device());
      // on ROCm the allocator behind the wrapper that labels its memory "cuda" (c10::GetAllocator(kCUDA)
      // is the unwrapped HIP one, whose tensors would say "hip"), and a plain device tensor's dispatch keys
      const at::Tensor probe = at::empty({0}, at::TensorOptions().dtype(p.scalar_type()).device(p.device()));
      alloc_ = probe.storage().allocator();
      keys_ = probe.key_set();
      if (!alloc_) throw std::runtime_error("walk: no device allocator");
    }
    const size_t nbytes = static_cast<size_t>(p.numel()) * p.element_size();
    c10::Storage st(c10::Storage::use_byte_size_t(), nbytes, alloc_->allocate(nbytes), alloc_, /*resizable=*/true);
    auto impl = c10::make_intrusive<c10::TensorImpl>(std::move(st), keys_, p.dtype());
    impl->set_sizes_and_strides(p.sizes(), p.strides(), 0);
    return at::Tensor(std::move(impl));
  }

 private:
  c10::optional<c10::DeviceGuard> guard_;
  at::Allocator* alloc_ = nullptr;
  c10::DispatchKeySet keys_;
};

// The result module's fresh parameters of a device round (fedavg._device_round: deepcopy(models[0]) of
// fedavg.py:20 with every parameter over part of ONE allocation the reduce writes): for each of
// models[0]'s parameters p and its element offset in `flat`, an nn.Parameter over alias_of(flat, p's
// sizes, p's strides, offset) with p's requires_grad — what torch.Tensor._make_subclass(nn.Parameter,
// data, rg) builds (a detached tensor whose metadata may change, wrapped as the Parameter class), without its ~8 us
// of Python per parameter (110 parameters of a google_speech ResNet-34: ~0.4 ms per round) — stored
// straight into the deepcopy memo as memo[id(p)].
void param_views(const at::Tensor& flat, py::list params, const std::vector<int64_t>& offsets, py::dict memo) {
  const py::ssize_t n = PyList_GET_SIZE(params.ptr());
  if (static_cast<size_t>(n) != offsets.size()) throw std::invalid_argument("param_views: one offset per parameter");
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(params.ptr(), i);
    if (!THPVariable_Check(o)) throw std::invalid_argument("param_views: not a tensor");
    const at::Tensor& p = THPVariable_Unpack(o);
    at::Tensor v = alias_of(flat, p.sizes(), p.strides(), offsets[i]);
    v.set_requires_grad(p.requires_grad());
    py::object w = py::reinterpret_steal<py::object>(THPVariable_Wrap(v, reinterpret_cast<PyTypeObject*>(ParameterClass)));
    if (!w) throw py::error_already_set();
    py::object id = py::reinterpret_steal<py::object>(PyLong_FromVoidPtr(o));
    if (!id || PyDict_SetItem(memo.ptr(), id.ptr(), w.ptr()) < 0) throw py::error_already_set();
  }
}

// The result module's fresh parameters of a device round (fedavg._device_round: deepcopy(models[0]) of
// fedavg.py:20, the reduce writing into them): for each of models[0]'s parameters p, an nn.Parameter over
// a NEW tensor from the device's caching allocator with p's sizes, strides and dtype and p's
// requires_grad — a storage of its own from the allocator, as deepcopy gives, so Tensor.record_stream,
// CUDA IPC and pickling behave exactly as for a deepcopy (round 6; rounds 4-5 made
// them aliases of one allocation, which the allocator did not know) — stored into the deepcopy memo as
// memo[id(p)].  Returns their data pointers (the reduce's outputs), one uint64 each.  One TensorImpl and
// one allocator call per parameter, no Python frame.
py::array_t<uint64_t> param_fresh(py::list params, py::dict memo) {
  const py::ssize_t n = PyList_GET_SIZE(params.ptr());
  py::array_t<uint64_t> ptrs(n);
  uint64_t* out = ptrs.mutable_data();
  FreshAlloc fresh;
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(params.ptr(), i);
    if (!THPVariable_Check(o)) throw std::invalid_argument("param_fresh: not a tensor");
    const at::Tensor& p = THPVariable_Unpack(o);
    at::Tensor v = fresh.like(p);
    v.set_requires_grad(p.requires_grad());
    out[i] = reinterpret_cast<uint64_t>(v.data_ptr());
    py::object w = py::reinterpret_steal<py::object>(THPVariable_Wrap(v, reinterpret_cast<PyTypeObject*>(ParameterClass)));
    if (!w) throw py::error_already_set();
    py::object id = py::reinterpret_steal<py::object>(PyLong_FromVoidPtr(o));
    if (!id || PyDict_SetItem(memo.ptr(), id.ptr(), w.ptr()) < 0) throw py::error_already_set();
  }
  return ptrs;
}

// param_fresh in two halves around the launch (fedavg._device_round): param_blocks takes the blocks from
// the allocator (the reduce needs only their addresses), param_wrap turns them into the nn.Parameters of
// the deepcopy memo while the reduce runs — the Python objects, autograd metadata and memo entries (~0.3 us
// a parameter) leave the time before the launch.  Blocks a FreshParams still holds when it is dropped go
// back to the allocator, ordered after the work queued on the stream they came from.
struct FreshParams {
  std::vector<at::Tensor> t;
};

py::tuple param_blocks(py::list params) {
  const py::ssize_t n = PyList_GET_SIZE(params.ptr());
  py::array_t<uint64_t> ptrs(n);
  uint64_t* out = ptrs.mutable_data();
  auto h = std::make_unique<FreshParams>();
  h->t.reserve(n);
  FreshAlloc fresh;
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(params.ptr(), i);
    if (!THPVariable_Check(o)) throw std::invalid_argument("param_blocks: not a tensor");
    h->t.push_back(fresh.like(THPVariable_Unpack(o)));
    out[i] = reinterpret_cast<uint64_t>(h->t.back().data_ptr());
  }
  return py::make_tuple(py::cast(std::move(h)), ptrs);
}

void param_wrap(FreshParams& h, py::list params, py::dict memo) {
  const py::ssize_t n = PyList_GET_SIZE(params.ptr());
  if (static_cast<size_t>(n) != h.t.size()) throw std::invalid_argument("param_wrap: one block per parameter");
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(params.ptr(), i);
    if (!THPVariable_Check(o)) throw std::invalid_argument("param_wrap: not a tensor");
    at::Tensor& v = h.t[i];
    v.set_requires_grad(THPVariable_Unpack(o).requires_grad());
    py::object w = py::reinterpret_steal<py::object>(THPVariable_Wrap(v, reinterpret_cast<PyTypeObject*>(ParameterClass)));
    if (!w) throw py::error_already_set();
    py::object id = py::reinterpret_steal<py::object>(PyLong_FromVoidPtr(o));
    if (!id || PyDict_SetItem(memo.ptr(), id.ptr(), w.ptr()) < 0) throw py::error_already_set();
  }
  h.t.clear();
}

// deepcopy of models[0]'s device buffers (fedavg.py:20 copies them, it does not average them) in one
// fused copy per (device, dtype), stored into the deepcopy memo: for each entry of `buffers` not already in
// `memo`, memo[id(buffer)] = a fresh tensor from the device's allocator (a storage of its own, as deepcopy
// gives: record_stream and IPC work on it; rounds 4-5 made the copies views of one allocation per group),
// all of a group filled by ONE fused multi-tensor copy.  Entries that are not plain dense CPU or CUDA
// tensors without grad, alone in their group, or sharing a storage with another buffer get no entry (the
// caller's deepcopy copies them, keeping the sharing).  Replaces a Python pass over every buffer (108 BN
// buffers of a google_speech ResNet-34: ~0.15 ms per round).
void buffer_copies(py::list buffers, py::dict memo) {
  const py::ssize_t n = PyList_GET_SIZE(buffers.ptr());
  std::vector<std::pair<int, int>> keys;  // (device index, scalar type) of each group
  std::vector<std::vector<py::ssize_t>> members;
  std::vector<py::object> ids(n);
  std::unordered_set<PyObject*> seen;
  std::vector<char> take(n, 0);
  // tensors sharing a storage keep the stock deepcopy, which keeps them sharing one
  std::unordered_map<const void*, int> storage_uses;
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(buffers.ptr(), i);
    if (Py_TYPE(o) != reinterpret_cast<PyTypeObject*>(THPVariableClass) || !seen.insert(o).second) continue;
    ids[i] = py::reinterpret_steal<py::object>(PyLong_FromVoidPtr(o));
    if (!ids[i]) throw py::error_already_set();
    const int in_memo = PyDict_Contains(memo.ptr(), ids[i].ptr());
    if (in_memo < 0) throw py::error_already_set();
    if (in_memo) continue;
    take[i] = 1;
    const at::Tensor& t = THPVariable_Unpack(o);
    if (t.has_storage()) ++storage_uses[t.storage().unsafeGetStorageImpl()];
  }
  for (py::ssize_t i = 0; i < n; ++i) {
    if (!take[i]) continue;
    const at::Tensor& t = THPVariable_Unpack(PyList_GET_ITEM(buffers.ptr(), i));
    if (t.requires_grad() || !t.is_contiguous() || !t.has_storage() || !(t.is_cuda() || t.is_cpu())) continue;
    if (storage_uses[t.storage().unsafeGetStorageImpl()] > 1) continue;
    const std::pair<int, int> key{t.get_device(), static_cast<int>(t.scalar_type())};
    size_t g = 0;
    while (g < keys.size() && keys[g] != key) ++g;
    if (g == keys.size()) {
      keys.push_back(key);
      members.emplace_back();
    }
    members[g].push_back(i);
  }
  for (const auto& mem : members) {
    if (mem.size() < 2) continue;
    // a fresh allocator tensor per buffer, then ONE fused multi-tensor copy
    std::vector<at::Tensor> srcs, dsts;
    srcs.reserve(mem.size());
    dsts.reserve(mem.size());
    FreshAlloc fresh;
    for (py::ssize_t i : mem) {
      srcs.push_back(THPVariable_Unpack(PyList_GET_ITEM(buffers.ptr(), i)));
      dsts.push_back(fresh.like(srcs.back()));
    }
    at::_foreach_copy_(dsts, srcs);
    for (size_t j = 0; j < mem.size(); ++j) {
      py::object w = py::reinterpret_steal<py::object>(THPVariable_Wrap(dsts[j]));
      if (!w || PyDict_SetItem(memo.ptr(), ids[mem[j]].ptr(), w.ptr()) < 0) throw py::error_already_set();
    }
  }
}

// The module-tree clone (fedavg._clone_value, deepcopy's protocol restated) in native code.  Ctx: the
// deepcopy memo (id -> copy), the set of types copied as themselves, the set of module classes cloned
// here (fedavg._plain_module: torch's __getstate__, no other copy hook), `fallback(obj, memo)` (the
// Python _clone_value, for every other object), collections.OrderedDict, "_compiled_call_impl" (the
// __dict__ entry a module clone leaves out), and — when fedavg found that torch's nn.Module.__setstate__
// only updates __dict__ for a state holding every attribute a fresh module has — that function and those
// attribute names (else both null).
struct CloneCtx {
  PyObject* memo;
  PyObject* atomic;
  PyObject* modules;
  PyObject* fallback;
  PyObject* odict;
  PyObject* skip;
  PyObject* setstate_fn;
  PyObject* full_state;  // tuple of str
  bool scalar_atomic;    // str, int, bool, float and None are in `atomic`
  bool containers_not_atomic;  // dict and OrderedDict are not
};

// x is a str, int, bool, float or None: copied as itself, and never in the memo (deepcopy memoizes only
// objects whose copy is a new object), so no memo lookup is needed for it.
inline bool scalar(PyObject* x) {
  return PyUnicode_CheckExact(x) || PyLong_CheckExact(x) || PyBool_Check(x) || PyFloat_CheckExact(x) || x == Py_None;
}

// `key`: id(x) as the caller already made it for its memo lookup (else made here)
PyObject* clone_mapping(PyObject* v, const CloneCtx& c, bool module_state = false, PyObject* key = nullptr);
PyObject* clone_sequence(PyObject* x, const CloneCtx& c, PyObject* key = nullptr);

bool memo_put(PyObject* memo, PyObject* x, PyObject* y, PyObject* key = nullptr) {
  PyObject* id = key ? Py_NewRef(key) : PyLong_FromVoidPtr(x);
  const int rc = id ? PyDict_SetItem(memo, id, y) : -1;
  Py_XDECREF(id);
  return rc == 0;
}

// (_PyType_Lookup and _PyObject_GetDictPtr below are CPython's own, exported by the 3.10 this extension
// is built against; the build id ties the .so to that interpreter's headers.)
// y.__setstate__(state) is y.__dict__.update(state) on a fresh y: its class keeps torch's
// nn.Module.__setstate__, and the state holds every attribute whose absence that function repairs.
// 1 yes, 0 no, -1 error.
int setstate_is_update(PyTypeObject* tp, PyObject* state, const CloneCtx& c) {
  static PyObject* const setstate = PyUnicode_InternFromString("__setstate__");
  if (!c.setstate_fn || _PyType_Lookup(tp, setstate) != c.setstate_fn) return 0;
  const Py_ssize_t n = PyTuple_GET_SIZE(c.full_state);
  if (PyDict_GET_SIZE(state) < n) return 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const int has = PyDict_Contains(state, PyTuple_GET_ITEM(c.full_state, i));
    if (has <= 0) return has;
  }
  return 1;
}

// A module of a class in ctx.modules, as copy._reconstruct does it: y = cls.__new__(cls), registered in
// the memo, state = a clone of x.__dict__ without _compiled_call_impl, y.__setstate__(state) — or, when
// that call would only copy the state into y's empty __dict__ (setstate_is_update), the state made y's
// __dict__ directly: the same entries in the same order, without a Python frame per module.  (The memo
// then maps x.__dict__ to y's own __dict__ rather than to a detached copy of it: only an object that held
// a module's __dict__ itself could tell.)
PyObject* clone_module(PyObject* x, const CloneCtx& c, PyObject* key = nullptr) {
  PyTypeObject* tp = Py_TYPE(x);
  static PyObject* const no_args = PyTuple_New(0);
  static PyObject* const setstate = PyUnicode_InternFromString("__setstate__");
  PyObject* y = tp->tp_new(tp, no_args, nullptr);
  if (!y) return nullptr;
  if (!memo_put(c.memo, x, y, key)) {
    Py_DECREF(y);
    return nullptr;
  }
  PyObject* d = PyObject_GenericGetDict(x, nullptr);
  PyObject* state = d ? clone_mapping(d, c, /*module_state=*/true) : nullptr;
  Py_XDECREF(d);
  if (!state) {
    Py_DECREF(y);
    return nullptr;
  }
  const int update = setstate_is_update(tp, state, c);
  PyObject** yd = update > 0 ? _PyObject_GetDictPtr(y) : nullptr;
  if (yd && (!*yd || PyDict_GET_SIZE(*yd) == 0)) {
    const int rc = PyObject_GenericSetDict(y, state, nullptr);
    Py_DECREF(state);
    if (rc < 0) {
      Py_DECREF(y);
      return nullptr;
    }
    return y;
  }
  PyObject* r = update >= 0 ? PyObject_CallMethodOneArg(y, setstate, state) : nullptr;
  Py_DECREF(state);
  if (!r) {
    Py_DECREF(y);
    return nullptr;
  }
  Py_DECREF(r);
  return y;
}

// One value, in fedavg._clone_value's order: the memo's copy if it holds one (seeded parameters and
// buffers, objects met before), the value itself if its type is atomic, a clone of a dict /
// OrderedDict / tuple / list / empty set / plain module made here, else fallback(value, memo).  New
// reference, or nullptr with the Python error set.
PyObject* clone_one(PyObject* x, const CloneCtx& c) {
  if (c.scalar_atomic && scalar(x)) return Py_NewRef(x);
  PyObject* key = PyLong_FromVoidPtr(x);
  if (!key) return nullptr;
  const py::object keep = py::reinterpret_steal<py::object>(key);  // released on every return
  PyObject* hit = PyDict_GetItemWithError(c.memo, key);  // borrowed
  if (hit) return Py_NewRef(hit);
  if (PyErr_Occurred()) return nullptr;
  // the containers a module's __dict__ holds are never atomic (clone_value checks): no set lookup for them
  const bool mapping = PyDict_CheckExact(x) || Py_TYPE(x) == reinterpret_cast<PyTypeObject*>(c.odict);
  if (!(mapping && c.containers_not_atomic)) {
    const int at = PySet_Contains(c.atomic, reinterpret_cast<PyObject*>(Py_TYPE(x)));
    if (at < 0) return nullptr;
    if (at) return Py_NewRef(x);
  }
  if (mapping) return clone_mapping(x, c, false, key);
  if (PyTuple_CheckExact(x) || PyList_CheckExact(x)) return clone_sequence(x, c, key);
  if (PySet_CheckExact(x) && PySet_GET_SIZE(x) == 0) {  // _non_persistent_buffers_set: a new empty set
    PyObject* y = PySet_New(nullptr);
    if (!y || !memo_put(c.memo, x, y, key)) {
      Py_XDECREF(y);
      return nullptr;
    }
    return y;
  }
  const int mod = PySet_Contains(c.modules, reinterpret_cast<PyObject*>(Py_TYPE(x)));
  if (mod < 0) return nullptr;
  if (mod) return clone_module(x, c, key);
  return PyObject_CallFunctionObjArgs(c.fallback, x, c.memo, nullptr);
}

// A tuple or list (a conv's kernel_size / stride / padding, _reversed_padding_repeated_twice), as
// copy.deepcopy copies them: a list is a new list registered in the memo before its items; a tuple is
// itself when every item clones to itself (tuples of numbers), else a new tuple registered in the memo.
PyObject* clone_sequence(PyObject* x, const CloneCtx& c, PyObject* key) {
  if (PyList_CheckExact(x)) {
    PyObject* y = PyList_New(0);
    if (!y || !memo_put(c.memo, x, y, key)) {
      Py_XDECREF(y);
      return nullptr;
    }
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(x); ++i) {
      PyObject* item = Py_NewRef(PyList_GET_ITEM(x, i));
      PyObject* ci = clone_one(item, c);
      Py_DECREF(item);
      if (!ci || PyList_Append(y, ci) < 0) {
        Py_XDECREF(ci);
        Py_DECREF(y);
        return nullptr;
      }
      Py_DECREF(ci);
    }
    return y;
  }
  const Py_ssize_t n = PyTuple_GET_SIZE(x);
  PyObject* y = PyTuple_New(n);
  if (!y) return nullptr;
  bool same = true;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* ci = clone_one(PyTuple_GET_ITEM(x, i), c);
    if (!ci) {
      Py_DECREF(y);
      return nullptr;
    }
    same = same && ci == PyTuple_GET_ITEM(x, i);
    PyTuple_SET_ITEM(y, i, ci);
  }
  if (same) {
    Py_DECREF(y);
    return Py_NewRef(x);
  }
  // an item's copy may have copied this tuple already (a cycle through a mutable item): use that one
  PyObject* id = key ? Py_NewRef(key) : PyLong_FromVoidPtr(x);
  PyObject* prev = id ? PyDict_GetItemWithError(c.memo, id) : nullptr;
  Py_XDECREF(id);
  if (prev || PyErr_Occurred()) {
    Py_DECREF(y);
    return prev ? Py_NewRef(prev) : nullptr;
  }
  if (!memo_put(c.memo, x, y, key)) {
    Py_DECREF(y);
    return nullptr;
  }
  return y;
}

// A dict or OrderedDict of the module tree (a module's _parameters, _buffers, _modules, hook dicts), or
// a module's __dict__ as the state its clone is set from (module_state: "_compiled_call_impl" left out):
// a new mapping of the same type registered in the memo first (deepcopy's order, so a cycle finds it),
// then every entry in iteration order with its value cloned by clone_one and a non-atomic key through
// the fallback.
PyObject* clone_mapping(PyObject* v, const CloneCtx& c, bool module_state, PyObject* key) {
  // an empty OrderedDict (a module's hook dicts) iterates like a dict: no items() view needed
  const bool exact = PyDict_CheckExact(v);
  const bool plain_iter = exact || PyDict_GET_SIZE(v) == 0;
  // an exact OrderedDict (the hook dicts, _parameters, _buffers, _modules) without a type call
  const bool odict = !exact && PyODict_CheckExact(v);
  PyObject* y = exact ? PyDict_New() : odict ? PyODict_New() : PyObject_CallNoArgs(reinterpret_cast<PyObject*>(Py_TYPE(v)));
  if (!y || !memo_put(c.memo, v, y, key)) {
    Py_XDECREF(y);
    return nullptr;
  }
  auto put = [&](PyObject* k, PyObject* x) -> bool {
    if (module_state && PyUnicode_Check(k) &&
        (k == c.skip || (PyUnicode_GET_LENGTH(k) == PyUnicode_GET_LENGTH(c.skip) && PyUnicode_Compare(k, c.skip) == 0)))
      return true;
    const int at = c.scalar_atomic && PyUnicode_CheckExact(k) ? 1 : PySet_Contains(c.atomic, reinterpret_cast<PyObject*>(Py_TYPE(k)));
    if (at < 0) return false;
    PyObject* kc = at ? Py_NewRef(k) : PyObject_CallFunctionObjArgs(c.fallback, k, c.memo, nullptr);
    if (!kc) return false;
    PyObject* ci = clone_one(x, c);
    const int rc = ci ? (exact ? PyDict_SetItem(y, kc, ci) : odict ? PyODict_SetItem(y, kc, ci) : PyObject_SetItem(y, kc, ci)) : -1;
    Py_DECREF(kc);
    Py_XDECREF(ci);
    return rc == 0;
  };
  bool ok = true;
  if (plain_iter) {
    // entries are cloned into another dict, so `v` is not resized by the loop; a fallback that
    // mutated it would be caught by the size check
    const Py_ssize_t size = PyDict_GET_SIZE(v);
    Py_ssize_t pos = 0;
    PyObject *k, *x;
    while (ok && PyDict_Next(v, &pos, &k, &x)) {
      Py_INCREF(k);
      Py_INCREF(x);
      ok = put(k, x);
      Py_DECREF(k);
      Py_DECREF(x);
      if (ok && PyDict_GET_SIZE(v) != size) {
        PyErr_SetString(PyExc_RuntimeError, "dictionary changed size during iteration");
        ok = false;
      }
    }
  } else {
    static PyObject* const items_name = PyUnicode_InternFromString("items");
    PyObject* items = PyObject_CallMethodNoArgs(v, items_name);
    PyObject* it = items ? PyObject_GetIter(items) : nullptr;
    Py_XDECREF(items);
    ok = it != nullptr;
    while (ok) {
      PyObject* kv = PyIter_Next(it);
      if (!kv) {
        ok = !PyErr_Occurred();
        break;
      }
      ok = PyTuple_Check(kv) && PyTuple_GET_SIZE(kv) == 2 && put(PyTuple_GET_ITEM(kv, 0), PyTuple_GET_ITEM(kv, 1));
      Py_DECREF(kv);
    }
    Py_XDECREF(it);
  }
  if (!ok) {
    Py_DECREF(y);
    return nullptr;
  }
  return y;
}

// fedavg._clone_value in native code, for a value of the result module's tree: the memo's entries are
// looked up without a Python call each (a google_speech ResNet-34's _parameters and _buffers hold 218
// seeded entries), and the tree's dicts, containers and plain modules are cloned here.  `atomic`: the set
// of types copied as themselves; `modules`: the set of module classes cloned here; `fallback(obj, memo)`:
// _clone_value, for every other object and for non-atomic keys (hashable: _clone_value copies them as
// deepcopy does); `odict`: collections.OrderedDict.
py::object clone_value(py::object v, py::dict memo, py::object atomic, py::object modules, py::object fallback,
                       py::object odict, py::object setstate_fn, py::object full_state) {
  if (!PyAnySet_Check(atomic.ptr()) || !PyAnySet_Check(modules.ptr()))
    throw std::invalid_argument("clone_value: sets of atomic types and module classes");
  const bool fast = !setstate_fn.is_none();
  if (fast) {
    if (!PyTuple_Check(full_state.ptr())) throw std::invalid_argument("clone_value: full_state is a tuple of str");
    for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(full_state.ptr()); ++i) {
      PyObject* k = PyTuple_GET_ITEM(full_state.ptr(), i);
      if (!PyUnicode_CheckExact(k)) throw std::invalid_argument("clone_value: full_state is a tuple of str");
    }
  }
  static PyObject* const skip = PyUnicode_InternFromString("_compiled_call_impl");
  bool scalar_atomic = true;
  for (PyTypeObject* t : {&PyUnicode_Type, &PyLong_Type, &PyBool_Type, &PyFloat_Type, Py_TYPE(Py_None)}) {
    const int has = PySet_Contains(atomic.ptr(), reinterpret_cast<PyObject*>(t));
    if (has < 0) throw py::error_already_set();
    scalar_atomic = scalar_atomic && has;
  }
  bool containers_not_atomic = true;
  for (PyObject* t : {reinterpret_cast<PyObject*>(&PyDict_Type), odict.ptr()}) {
    const int has = PySet_Contains(atomic.ptr(), t);
    if (has < 0) throw py::error_already_set();
    containers_not_atomic = containers_not_atomic && !has;
  }
  const CloneCtx c{memo.ptr(), atomic.ptr(), modules.ptr(), fallback.ptr(), odict.ptr(), skip,
                   fast ? setstate_fn.ptr() : nullptr, fast ? full_state.ptr() : nullptr, scalar_atomic,
                   containers_not_atomic};
  PyObject* y = clone_one(v.ptr(), c);
  if (!y) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(y);
}

// ------------------------------------------------------------------------------------------------
// Wire ingress: the state-dict pickle scanned natively.
//
// accdfl ships a model as serialize_model(model) = pickle.dumps(model.state_dict())
// (accdfl/core/models/__init__.py:9-10) and decodes it with pickle.loads + load_state_dict (:13-16) after
// EVA joined the blocks (accdfl/util/eva/transfer/incoming.py:35).  accdfl_amd.core.wire decodes the same
// bytes with a restricted pickle VM in Python; for a google_speech ResNet-34 (218 entries) that VM and
// the per-storage blob parse cost ~10 ms per peer on the MI355X hosts, 13x the peer's PCIe time.
//
// scan_state_dict runs the same restricted opcode subset here, over the block list in place: the only
// callables it knows are collections.OrderedDict (called, with no arguments), torch._utils.
// _rebuild_tensor_v2 and torch.storage._load_from_bytes (neither called: they become descriptions), and
// every other global makes it give up.  It builds no tensor and copies no element byte: it returns
//     (top, storages)
// where `top` is the pickled OrderedDict with every tensor replaced by a description tuple
// (scan_tensor_tag, storage index, storage offset, sizes, strides, requires_grad) — one object per pickled
// tensor, so entries the pickle ties stay tied — and `storages` lists (dtype name, numel, byte position of
// the element data in the payload, nbytes) for each legacy storage blob (torch.save of one storage:
// magic, protocol, sys info, the storage's persistent id, its key list, its element count, its bytes).
// None: something outside this subset (the caller's Python VM then decodes or refuses the payload, with
// its own errors).  span_pieces turns storages' payload ranges into the (dst, src, len) copies of one
// batched gather; build_state_dict makes the tensors over a buffer holding the gathered storages.

namespace wirescan {

struct Tags {
  PyObject* bytes;     // (tag, position, length): a BINBYTES argument left in the payload
  PyObject* global;    // (tag, which): an allowed global
  PyObject* storage;   // (tag, storage index)
  PyObject* tensor;    // (tag, storage index, storage offset, sizes, strides, requires_grad)
  PyObject* sclass;    // (tag, dtype index): torch.<X>Storage inside a storage blob
  PyObject* pstorage;  // (tag, dtype index, key, numel): a storage blob's persistent id
};

const Tags& tags() {
  static const Tags t = [] {
    auto mk = [] {
      PyObject* o = PyObject_CallNoArgs(reinterpret_cast<PyObject*>(&PyBaseObject_Type));
      if (!o) throw py::error_already_set();
      return o;  // immortal for the module's lifetime
    };
    return Tags{mk(), mk(), mk(), mk(), mk(), mk()};
  }();
  return t;
}

// torch.<X>Storage of a legacy blob -> (torch dtype name, element size, scalar type)
struct StorageType {
  const char* cls;
  const char* dtype;
  int esize;
  at::ScalarType st;
};
const StorageType kStorageTypes[] = {
    {"FloatStorage", "float32", 4, at::kFloat},     {"DoubleStorage", "float64", 8, at::kDouble},
    {"HalfStorage", "float16", 2, at::kHalf},       {"BFloat16Storage", "bfloat16", 2, at::kBFloat16},
    {"LongStorage", "int64", 8, at::kLong},         {"IntStorage", "int32", 4, at::kInt},
    {"ShortStorage", "int16", 2, at::kShort},       {"CharStorage", "int8", 1, at::kChar},
    {"ByteStorage", "uint8", 1, at::kByte},         {"BoolStorage", "bool", 1, at::kBool},
};
constexpr int kNumStorageTypes = static_cast<int>(sizeof(kStorageTypes) / sizeof(kStorageTypes[0]));

enum Global { G_ODICT = 0, G_REBUILD = 1, G_LOAD_BYTES = 2 };

struct StorageRec {
  int type;
  int64_t numel;
  int64_t data_pos;
  int64_t nbytes;
};

// The payload: a list of blocks read as one stream (EVA's data_list, or one bytes object).
struct Blocks {
  const int64_t* addr;
  const int64_t* len;
  int64_t n;
  std::vector<int64_t> start;
  int64_t total = 0;
  int64_t pos = 0;
  int64_t bi = 0;  // the block holding `pos`

  Blocks(const int64_t* a, const int64_t* l, int64_t nb) : addr(a), len(l), n(nb), start(static_cast<size_t>(nb)) {
    for (int64_t i = 0; i < n; ++i) {
      start[i] = total;
      total += len[i];
    }
    settle();
  }
  void settle() {
    while (bi < n && pos >= start[bi] + len[bi]) ++bi;
  }
  bool read(char* dst, int64_t k) {
    if (k < 0 || k > total - pos) return false;
    while (k > 0) {
      const int64_t off = pos - start[bi];
      const int64_t take = std::min(k, len[bi] - off);
      std::memcpy(dst, reinterpret_cast<const char*>(addr[bi]) + off, static_cast<size_t>(take));
      dst += take;
      k -= take;
      pos += take;
      settle();
    }
    return true;
  }
  bool skip(int64_t k) {
    if (k < 0 || k > total - pos) return false;
    pos += k;
    settle();
    return true;
  }
  // random access (the blob headers): k bytes from stream position p
  bool read_at(int64_t p, char* dst, int64_t k) const {
    if (p < 0 || k < 0 || p + k > total) return false;
    int64_t i = static_cast<int64_t>(std::upper_bound(start.begin(), start.end(), p) - start.begin()) - 1;
    while (k > 0) {
      while (i < n && p >= start[i] + len[i]) ++i;
      const int64_t off = p - start[i];
      const int64_t take = std::min(k, len[i] - off);
      std::memcpy(dst, reinterpret_cast<const char*>(addr[i]) + off, static_cast<size_t>(take));
      dst += take;
      k -= take;
      p += take;
    }
    return true;
  }
};

// A storage blob's header, copied out of the payload.
struct Mem {
  const char* p;
  int64_t n;
  int64_t pos = 0;
  bool read(char* dst, int64_t k) {
    if (k < 0 || k > n - pos) return false;
    std::memcpy(dst, p + pos, static_cast<size_t>(k));
    pos += k;
    return true;
  }
  bool skip(int64_t k) {
    if (k < 0 || k > n - pos) return false;
    pos += k;
    return true;
  }
};

// Owned references, released on scope exit.
struct Refs {
  std::vector<PyObject*> v;
  ~Refs() {
    for (PyObject* o : v) Py_XDECREF(o);
  }
};

struct Scanner {
  Blocks& blocks;
  PyObject* odict_cls;
  std::vector<StorageRec> storages;
  std::string prefix;  // the first checked blob's magic / protocol / sys-info pickles, byte for byte

  bool is_tagged(PyObject* o, PyObject* tag, Py_ssize_t n) const {
    return PyTuple_CheckExact(o) && PyTuple_GET_SIZE(o) == n && PyTuple_GET_ITEM(o, 0) == tag;
  }

  // One pickle (up to STOP) from `src`: new reference, or nullptr (outside the subset; any Python error
  // is cleared by the caller).  blob: the pickles of a legacy storage blob (persistent ids, torch.<X>Storage
  // globals) instead of the state dict's (the three allowed globals, BINBYTES left in the payload).
  template <class Src>
  PyObject* run(Src& src, bool blob) {
    const Tags& T = tags();
    Refs stack, memo;  // memo slots may be null
    std::vector<size_t> marks;
    auto& st = stack.v;
    auto u = [&](int k, uint64_t* out) -> bool {
      unsigned char b[8] = {0};
      if (!src.read(reinterpret_cast<char*>(b), k)) return false;
      uint64_t x = 0;
      for (int i = k - 1; i >= 0; --i) x = (x << 8) | b[i];
      *out = x;
      return true;
    };
    auto push = [&](PyObject* o) -> bool {
      if (!o) return false;
      st.push_back(o);
      return true;
    };
    auto pop = [&]() -> PyObject* {  // new reference (the caller owns it)
      PyObject* o = st.back();
      st.pop_back();
      return o;
    };
    auto pop_mark = [&](size_t* at) -> bool {
      if (marks.empty() || marks.back() > st.size()) return false;
      *at = marks.back();
      marks.pop_back();
      return true;
    };
    auto put_memo = [&](uint64_t i) -> bool {
      // a state dict's pickle memoizes a few objects per entry, in order: an index far past that is refused
      // (a 5-byte opcode must not grow the memo by hundreds of MB)
      if (st.empty() || i > (uint64_t{1} << 22) || i > memo.v.size() + 4096) return false;
      if (memo.v.size() <= i) memo.v.resize(static_cast<size_t>(i) + 1, nullptr);
      Py_XDECREF(memo.v[i]);
      memo.v[i] = Py_NewRef(st.back());
      return true;
    };
    auto get_memo = [&](uint64_t i) -> bool {
      if (i >= memo.v.size() || !memo.v[i]) return false;
      return push(Py_NewRef(memo.v[i]));
    };
    auto text = [&](uint64_t n) -> PyObject* {
      if (n > (uint64_t{1} << 20)) return nullptr;
      std::string s(static_cast<size_t>(n), '\0');
      if (!src.read(s.data(), static_cast<int64_t>(n))) return nullptr;
      return PyUnicode_DecodeUTF8(s.data(), static_cast<Py_ssize_t>(n), "strict");
    };
    auto global = [&](PyObject* module, PyObject* name) -> PyObject* {
      if (!PyUnicode_Check(module) || !PyUnicode_Check(name)) return nullptr;
      const char* m = PyUnicode_AsUTF8(module);
      const char* nm = PyUnicode_AsUTF8(name);
      if (!m || !nm) return nullptr;
      if (blob) {
        if (std::strcmp(m, "torch") != 0) return nullptr;
        for (int i = 0; i < kNumStorageTypes; ++i)
          if (std::strcmp(nm, kStorageTypes[i].cls) == 0) return Py_BuildValue("(Oi)", T.sclass, i);
        return nullptr;
      }
      int g = -1;
      if (!std::strcmp(m, "collections") && !std::strcmp(nm, "OrderedDict")) g = G_ODICT;
      else if (!std::strcmp(m, "torch._utils") && !std::strcmp(nm, "_rebuild_tensor_v2")) g = G_REBUILD;
      else if (!std::strcmp(m, "torch.storage") && !std::strcmp(nm, "_load_from_bytes")) g = G_LOAD_BYTES;
      return g < 0 ? nullptr : Py_BuildValue("(Oi)", T.global, g);
    };
    auto tuple_of = [&](size_t from) -> PyObject* {
      const Py_ssize_t n = static_cast<Py_ssize_t>(st.size() - from);
      PyObject* t = PyTuple_New(n);
      if (!t) return nullptr;
      for (Py_ssize_t i = 0; i < n; ++i) PyTuple_SET_ITEM(t, i, st[from + static_cast<size_t>(i)]);
      st.resize(from);  // references moved into the tuple
      return t;
    };
    for (;;) {
      unsigned char op;
      if (!src.read(reinterpret_cast<char*>(&op), 1)) return nullptr;
      uint64_t x = 0;
      switch (op) {
        case 0x80:  // PROTO
          if (!u(1, &x) || x > 5) return nullptr;
          break;
        case 0x95:  // FRAME: frames are inline
          if (!src.skip(8)) return nullptr;
          break;
        case 0x2E:  // STOP
          if (st.size() != 1 || !marks.empty()) return nullptr;
          return pop();
        case 0x28:  // MARK
          marks.push_back(st.size());
          break;
        case 0x8C:  // SHORT_BINUNICODE
          if (!u(1, &x) || !push(text(x))) return nullptr;
          break;
        case 0x58:  // BINUNICODE
          if (!u(4, &x) || !push(text(x))) return nullptr;
          break;
        case 0x8D:  // BINUNICODE8
          if (!u(8, &x) || !push(text(x))) return nullptr;
          break;
        case 0x94:  // MEMOIZE
          if (!put_memo(memo.v.size())) return nullptr;
          break;
        case 0x71:  // BINPUT
          if (!u(1, &x) || !put_memo(x)) return nullptr;
          break;
        case 0x72:  // LONG_BINPUT
          if (!u(4, &x) || !put_memo(x)) return nullptr;
          break;
        case 0x68:  // BINGET
          if (!u(1, &x) || !get_memo(x)) return nullptr;
          break;
        case 0x6A:  // LONG_BINGET
          if (!u(4, &x) || !get_memo(x)) return nullptr;
          break;
        case 0x93: {  // STACK_GLOBAL
          if (st.size() < 2) return nullptr;
          PyObject* name = pop();
          PyObject* module = pop();
          PyObject* g = global(module, name);
          Py_DECREF(name);
          Py_DECREF(module);
          if (!push(g)) return nullptr;
          break;
        }
        case 0x63: {  // GLOBAL: "module\nname\n"
          std::string line[2];
          for (auto& s : line) {
            char ch;
            while (true) {
              if (!src.read(&ch, 1) || s.size() > 256) return nullptr;
              if (ch == '\n') break;
              s.push_back(ch);
            }
          }
          PyObject* module = PyUnicode_DecodeUTF8(line[0].data(), static_cast<Py_ssize_t>(line[0].size()), "strict");
          PyObject* name = PyUnicode_DecodeUTF8(line[1].data(), static_cast<Py_ssize_t>(line[1].size()), "strict");
          PyObject* g = module && name ? global(module, name) : nullptr;
          Py_XDECREF(module);
          Py_XDECREF(name);
          if (!push(g)) return nullptr;
          break;
        }
        case 0x29:  // EMPTY_TUPLE
          if (!push(PyTuple_New(0))) return nullptr;
          break;
        case 0x85:  // TUPLE1
        case 0x86:  // TUPLE2
        case 0x87: {  // TUPLE3
          const size_t k = op - 0x84;
          if (st.size() < k || (!marks.empty() && marks.back() > st.size() - k)) return nullptr;
          if (!push(tuple_of(st.size() - k))) return nullptr;
          break;
        }
        case 0x74: {  // TUPLE
          size_t at;
          if (!pop_mark(&at) || !push(tuple_of(at))) return nullptr;
          break;
        }
        case 0x52: {  // REDUCE
          if (st.size() < 2) return nullptr;
          PyObject* args = pop();
          PyObject* fn = pop();
          PyObject* r = is_tagged(fn, T.global, 2) && PyTuple_CheckExact(args) ? reduce(fn, args) : nullptr;
          Py_DECREF(args);
          Py_DECREF(fn);
          if (!push(r)) return nullptr;
          break;
        }
        case 0x51: {  // BINPERSID (storage blobs only)
          if (!blob || st.empty()) return nullptr;
          PyObject* pid = pop();
          PyObject* r = nullptr;
          if (PyTuple_CheckExact(pid) && PyTuple_GET_SIZE(pid) == 6 && PyUnicode_Check(PyTuple_GET_ITEM(pid, 0)) &&
              PyUnicode_CompareWithASCIIString(PyTuple_GET_ITEM(pid, 0), "storage") == 0 &&
              is_tagged(PyTuple_GET_ITEM(pid, 1), T.sclass, 2) && PyTuple_GET_ITEM(pid, 5) == Py_None &&
              PyLong_CheckExact(PyTuple_GET_ITEM(pid, 4))) {
            PyObject* key = PyObject_Str(PyTuple_GET_ITEM(pid, 2));
            if (key) {
              r = Py_BuildValue("(OOOO)", T.pstorage, PyTuple_GET_ITEM(PyTuple_GET_ITEM(pid, 1), 1), key,
                                PyTuple_GET_ITEM(pid, 4));
              Py_DECREF(key);
            }
          }
          Py_DECREF(pid);
          if (!push(r)) return nullptr;
          break;
        }
        case 0x4A: {  // BININT
          if (!u(4, &x)) return nullptr;
          if (!push(PyLong_FromLong(static_cast<int32_t>(static_cast<uint32_t>(x))))) return nullptr;
          break;
        }
        case 0x4B:  // BININT1
          if (!u(1, &x) || !push(PyLong_FromUnsignedLongLong(x))) return nullptr;
          break;
        case 0x4D:  // BININT2
          if (!u(2, &x) || !push(PyLong_FromUnsignedLongLong(x))) return nullptr;
          break;
        case 0x8A: {  // LONG1
          if (!u(1, &x)) return nullptr;
          unsigned char b[256];
          if (!src.read(reinterpret_cast<char*>(b), static_cast<int64_t>(x))) return nullptr;
          if (!push(x ? _PyLong_FromByteArray(b, static_cast<size_t>(x), 1, 1) : PyLong_FromLong(0))) return nullptr;
          break;
        }
        case 0x4E:  // NONE
          if (!push(Py_NewRef(Py_None))) return nullptr;
          break;
        case 0x88:  // NEWTRUE
          if (!push(Py_NewRef(Py_True))) return nullptr;
          break;
        case 0x89:  // NEWFALSE
          if (!push(Py_NewRef(Py_False))) return nullptr;
          break;
        case 0x7D:  // EMPTY_DICT
          if (!push(PyDict_New())) return nullptr;
          break;
        case 0x5D:  // EMPTY_LIST
          if (!push(PyList_New(0))) return nullptr;
          break;
        case 0x61: {  // APPEND
          if (st.size() < 2 || !PyList_CheckExact(st[st.size() - 2])) return nullptr;
          PyObject* v = pop();
          const int rc = PyList_Append(st.back(), v);
          Py_DECREF(v);
          if (rc < 0) return nullptr;
          break;
        }
        case 0x65: {  // APPENDS
          size_t at;
          if (!pop_mark(&at) || at < 1 || !PyList_CheckExact(st[at - 1])) return nullptr;
          for (size_t i = at; i < st.size(); ++i)
            if (PyList_Append(st[at - 1], st[i]) < 0) return nullptr;
          for (size_t i = at; i < st.size(); ++i) Py_DECREF(st[i]);
          st.resize(at);
          break;
        }
        case 0x73: {  // SETITEM
          if (st.size() < 3 || !PyDict_Check(st[st.size() - 3])) return nullptr;
          PyObject* v = pop();
          PyObject* k = pop();
          const int rc = PyObject_SetItem(st.back(), k, v);
          Py_DECREF(k);
          Py_DECREF(v);
          if (rc < 0) return nullptr;
          break;
        }
        case 0x75: {  // SETITEMS
          size_t at;
          if (!pop_mark(&at) || at < 1 || !PyDict_Check(st[at - 1]) || (st.size() - at) % 2) return nullptr;
          for (size_t i = at; i + 1 < st.size(); i += 2)
            if (PyObject_SetItem(st[at - 1], st[i], st[i + 1]) < 0) return nullptr;
          for (size_t i = at; i < st.size(); ++i) Py_DECREF(st[i]);
          st.resize(at);
          break;
        }
        case 0x62: {  // BUILD: only an OrderedDict's _metadata (state_dict's instance attribute)
          if (blob || st.size() < 2) return nullptr;
          PyObject* state = pop();
          PyObject* inst = st.back();
          bool ok = Py_TYPE(inst) == reinterpret_cast<PyTypeObject*>(odict_cls) && PyDict_CheckExact(state);
          Py_ssize_t pos = 0;
          PyObject *k, *v;
          while (ok && PyDict_Next(state, &pos, &k, &v))
            ok = PyUnicode_Check(k) && PyUnicode_CompareWithASCIIString(k, "_metadata") == 0 &&
                 PyObject_SetAttr(inst, k, v) == 0;
          Py_DECREF(state);
          if (!ok) return nullptr;
          break;
        }
        case 0x42:    // BINBYTES
        case 0x43:    // SHORT_BINBYTES
        case 0x8E: {  // BINBYTES8: left in the payload (position, length)
          if (blob || !u(op == 0x43 ? 1 : op == 0x42 ? 4 : 8, &x)) return nullptr;
          const int64_t at = blocks.pos;
          if (x > static_cast<uint64_t>(blocks.total) || !src.skip(static_cast<int64_t>(x))) return nullptr;
          if (!push(Py_BuildValue("(OLL)", T.bytes, static_cast<long long>(at), static_cast<long long>(x)))) return nullptr;
          break;
        }
        case 0x47: {  // BINFLOAT (big-endian double)
          unsigned char b[8];
          if (!src.read(reinterpret_cast<char*>(b), 8)) return nullptr;
          uint64_t bits = 0;
          for (int i = 0; i < 8; ++i) bits = (bits << 8) | b[i];
          double d;
          std::memcpy(&d, &bits, 8);
          if (!push(PyFloat_FromDouble(d))) return nullptr;
          break;
        }
        default:
          return nullptr;
      }
    }
  }

  // REDUCE of an allowed global: OrderedDict() is called; the storage blob and the tensor rebuild become
  // descriptions.  nullptr: arguments outside what a state_dict pickle holds.
  PyObject* reduce(PyObject* fn, PyObject* args) {
    const Tags& T = tags();
    const long g = PyLong_AsLong(PyTuple_GET_ITEM(fn, 1));
    const Py_ssize_t na = PyTuple_GET_SIZE(args);
    if (g == G_ODICT) return na == 0 ? PyObject_CallNoArgs(odict_cls) : nullptr;
    if (g == G_LOAD_BYTES) {
      if (na != 1 || !is_tagged(PyTuple_GET_ITEM(args, 0), T.bytes, 3)) return nullptr;
      const long long at = PyLong_AsLongLong(PyTuple_GET_ITEM(PyTuple_GET_ITEM(args, 0), 1));
      const long long n = PyLong_AsLongLong(PyTuple_GET_ITEM(PyTuple_GET_ITEM(args, 0), 2));
      const int64_t idx = storage_blob(at, n);
      return idx < 0 ? nullptr : Py_BuildValue("(OL)", T.storage, static_cast<long long>(idx));
    }
    if (g != G_REBUILD || (na != 6 && na != 7)) return nullptr;
    // _rebuild_tensor_v2(storage, storage_offset, size, stride, requires_grad, backward_hooks[, metadata])
    PyObject* s = PyTuple_GET_ITEM(args, 0);
    PyObject* off = PyTuple_GET_ITEM(args, 1);
    PyObject* size = PyTuple_GET_ITEM(args, 2);
    PyObject* stride = PyTuple_GET_ITEM(args, 3);
    PyObject* rg = PyTuple_GET_ITEM(args, 4);
    PyObject* hooks = PyTuple_GET_ITEM(args, 5);
    if (!is_tagged(s, T.storage, 2) || !PyLong_CheckExact(off) || !PyTuple_CheckExact(size) ||
        !PyTuple_CheckExact(stride) || PyTuple_GET_SIZE(size) != PyTuple_GET_SIZE(stride) || !PyBool_Check(rg) ||
        !PyDict_Check(hooks) || PyDict_GET_SIZE(hooks) != 0 || (na == 7 && PyTuple_GET_ITEM(args, 6) != Py_None))
      return nullptr;
    const long long sidx = PyLong_AsLongLong(PyTuple_GET_ITEM(s, 1));
    const long long o = PyLong_AsLongLong(off);
    if (sidx < 0 || sidx >= static_cast<long long>(storages.size()) || o < 0) return nullptr;
    const StorageRec& rec = storages[static_cast<size_t>(sidx)];
    if (rg == Py_True && !at::isFloatingType(kStorageTypes[rec.type].st)) return nullptr;
    __int128 extent = 1;  // the elements the tensor spans must lie inside its storage
    bool empty = false;
    for (Py_ssize_t d = 0; d < PyTuple_GET_SIZE(size); ++d) {
      PyObject* a = PyTuple_GET_ITEM(size, d);
      PyObject* b = PyTuple_GET_ITEM(stride, d);
      if (!PyLong_CheckExact(a) || !PyLong_CheckExact(b)) return nullptr;
      const long long sz = PyLong_AsLongLong(a), sd = PyLong_AsLongLong(b);
      if (sz < 0 || sd < 0 || sz > (1LL << 40) || sd > (1LL << 40)) return nullptr;
      if (sz == 0) empty = true;
      extent += static_cast<__int128>(sz - 1) * sd;
    }
    if (!empty && o + extent > rec.numel) return nullptr;
    return PyTuple_Pack(6, T.tensor, PyTuple_GET_ITEM(s, 1), off, size, stride, rg);
  }

  // A legacy storage blob (torch.save of one storage, what TypedStorage.__reduce__ embeds) at payload
  // position `at`, `n` bytes: its index in `storages`, or -1.
  int64_t storage_blob(int64_t at, int64_t n) {
    // the header pickles are a few hundred bytes: parse from the first 1 KiB, and from 64 KiB (the Python
    // decoder's bound) only when they run past it
    const int64_t r = storage_blob_head(at, n, 1024);
    return r == -2 ? storage_blob_head(at, n, 65536) : r;
  }

  // -1: not a storage blob; -2: its header runs past `cap` bytes
  int64_t storage_blob_head(int64_t at, int64_t n, int64_t cap) {
    const Tags& T = tags();
    char small[1024];
    std::string big;
    const int64_t hn = std::min<int64_t>(n, cap);
    char* hp = small;
    if (hn > static_cast<int64_t>(sizeof(small))) {
      big.resize(static_cast<size_t>(hn));
      hp = big.data();
    }
    if (!blocks.read_at(at, hp, hn)) return -1;
    Mem m{hp, hn};
    static PyObject* const magic = PyLong_FromString("1950A86A20F9469CFC6C", nullptr, 16);
    PyObject* objs[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    int64_t idx = -1;
    bool ok = magic != nullptr;
    // The first three pickles (magic number, protocol, sys info) are the same bytes in every blob one
    // torch wrote: once a blob's have been checked, a blob that starts with the same bytes skips them (the
    // sys-info dict is most of a header's objects: ~2 us -> ~1 us per tensor)
    const bool same_prefix = !prefix.empty() && static_cast<size_t>(hn) >= prefix.size() &&
                             std::memcmp(hp, prefix.data(), prefix.size()) == 0;
    int64_t prefix_end = 0;
    if (same_prefix) {
      m.pos = static_cast<int64_t>(prefix.size());
      for (int i = 3; ok && i < 5; ++i) ok = (objs[i] = run(m, true)) != nullptr;
    } else {
      for (int i = 0; ok && i < 5; ++i) {
        ok = (objs[i] = run(m, true)) != nullptr;
        if (i == 2) prefix_end = m.pos;
      }
    }
    if (ok) {
      PyObject* ps = objs[3];
      if (!same_prefix) {
        PyObject* le = PyDict_CheckExact(objs[2]) ? PyDict_GetItemString(objs[2], "little_endian") : nullptr;
        ok = PyObject_RichCompareBool(objs[0], magic, Py_EQ) == 1 && PyLong_CheckExact(objs[1]) &&
             PyLong_AsLong(objs[1]) == 1001 && le == Py_True;
      }
      ok = ok && is_tagged(ps, T.pstorage, 4) && PyList_CheckExact(objs[4]) && PyList_GET_SIZE(objs[4]) == 1 &&
           PyObject_RichCompareBool(PyList_GET_ITEM(objs[4], 0), PyTuple_GET_ITEM(ps, 2), Py_EQ) == 1;
      if (ok && !same_prefix && prefix.empty()) prefix.assign(hp, static_cast<size_t>(prefix_end));
      unsigned char b[8];
      if (ok && m.read(reinterpret_cast<char*>(b), 8)) {
        uint64_t saved = 0;
        for (int i = 7; i >= 0; --i) saved = (saved << 8) | b[i];
        const int type = static_cast<int>(PyLong_AsLong(PyTuple_GET_ITEM(ps, 1)));
        const long long numel = PyLong_AsLongLong(PyTuple_GET_ITEM(ps, 3));
        if (type >= 0 && type < kNumStorageTypes && numel >= 0 && static_cast<uint64_t>(numel) == saved &&
            numel <= (int64_t{1} << 40) && m.pos + numel * kStorageTypes[type].esize == n) {
          idx = static_cast<int64_t>(storages.size());
          storages.push_back({type, numel, at + m.pos, numel * kStorageTypes[type].esize});
        }
      }
    }
    for (PyObject* o : objs) Py_XDECREF(o);
    if (idx < 0) PyErr_Clear();
    // failed on a cut header: try again with the whole 64 KiB the Python decoder reads
    return idx < 0 && hn < n && cap < 65536 ? -2 : idx;
  }
};

}  // namespace wirescan

// See the block comment above: (top, [(dtype name, numel, data position, nbytes)]) or None.
py::object scan_state_dict(py::array_t<int64_t, py::array::c_style> addrs, py::array_t<int64_t, py::array::c_style> lens,
                           py::object odict_cls) {
  if (addrs.size() != lens.size()) throw std::invalid_argument("scan_state_dict: one length per block");
  wirescan::Blocks blocks(addrs.data(), lens.data(), static_cast<int64_t>(lens.size()));
  wirescan::Scanner sc{blocks, odict_cls.ptr(), {}, {}};
  PyObject* top = sc.run(blocks, false);
  if (!top) {
    PyErr_Clear();
    return py::none();
  }
  py::object t = py::reinterpret_steal<py::object>(top);
  if (blocks.pos != blocks.total || !PyDict_Check(top)) return py::none();  // trailing bytes: not a lone pickle
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(top, &pos, &k, &v))
    if (!PyUnicode_Check(k) || !sc.is_tagged(v, wirescan::tags().tensor, 6)) return py::none();
  py::list st;
  for (const auto& r : sc.storages)
    st.append(py::make_tuple(wirescan::kStorageTypes[r.type].dtype, r.numel, r.data_pos, r.nbytes));
  return py::make_tuple(t, st);
}

// StateDictScan.row_layout in native code: where a PeerSlab row's parameters come from in one piece.  When
// the entries `names` (template.named_parameters() order) are dense tensors of dtype `dtype` and the sizes
// `shapes`, each the whole of a storage of its own (storage offset 0, row-major strides, numel = the
// storage's), returns (byte offset of every storage — those parameters back to back from byte 0, every
// other storage after them 256-byte aligned —, total bytes, row bytes); else None.
py::object row_layout(py::dict top, py::list storages, py::list names, std::string dtype, py::list shapes) {
  const py::ssize_t ns = PyList_GET_SIZE(storages.ptr());
  const py::ssize_t nn = PyList_GET_SIZE(names.ptr());
  if (PyList_GET_SIZE(shapes.ptr()) != nn) throw std::invalid_argument("row_layout: one shape per name");
  py::array_t<int64_t> offsets(ns);
  int64_t* off = offsets.mutable_data();
  for (py::ssize_t i = 0; i < ns; ++i) off[i] = -1;
  PyObject* tensor_tag = wirescan::tags().tensor;
  auto none = []() -> py::object {  // not a row (a conversion that failed on the way leaves no error behind)
    PyErr_Clear();
    return py::none();
  };
  int64_t o = 0;
  for (py::ssize_t i = 0; i < nn; ++i) {
    PyObject* d = PyDict_GetItemWithError(top.ptr(), PyList_GET_ITEM(names.ptr(), i));  // borrowed
    if (!d) {
      if (PyErr_Occurred()) throw py::error_already_set();
      return none();
    }
    if (!PyTuple_CheckExact(d) || PyTuple_GET_SIZE(d) != 6 || PyTuple_GET_ITEM(d, 0) != tensor_tag)
      return none();
    const long long sidx = PyLong_AsLongLong(PyTuple_GET_ITEM(d, 1));
    if (sidx < 0 || sidx >= ns || off[sidx] >= 0 || PyLong_AsLongLong(PyTuple_GET_ITEM(d, 2)) != 0) return none();
    PyObject* size = PyTuple_GET_ITEM(d, 3);
    PyObject* stride = PyTuple_GET_ITEM(d, 4);
    PyObject* want = PyList_GET_ITEM(shapes.ptr(), i);
    if (!PyTuple_Check(want) || PyTuple_GET_SIZE(want) != PyTuple_GET_SIZE(size)) return none();
    const Py_ssize_t nd = PyTuple_GET_SIZE(size);
    int64_t numel = 1, expect = 1;
    for (Py_ssize_t k = nd - 1; k >= 0; --k) {  // sizes equal the shape's, strides row-major
      const long long sz = PyLong_AsLongLong(PyTuple_GET_ITEM(size, k));
      if (sz != PyLong_AsLongLong(PyTuple_GET_ITEM(want, k)) || PyLong_AsLongLong(PyTuple_GET_ITEM(stride, k)) != expect)
        return none();
      expect *= sz;
      numel *= sz;
    }
    if (PyErr_Occurred()) throw py::error_already_set();
    py::tuple rec = py::reinterpret_borrow<py::tuple>(PyList_GET_ITEM(storages.ptr(), sidx));
    if (rec[0].cast<std::string>() != dtype || rec[1].cast<int64_t>() != numel) return none();
    off[sidx] = o;
    o += rec[3].cast<int64_t>();
  }
  const int64_t row = o;
  o = (o + 255) / 256 * 256;
  for (py::ssize_t i = 0; i < ns; ++i) {
    if (off[i] >= 0) continue;
    off[i] = o;
    o += (py::reinterpret_borrow<py::tuple>(PyList_GET_ITEM(storages.ptr(), i))[3].cast<int64_t>() + 255) / 256 * 256;
  }
  return py::make_tuple(offsets, o > 0 ? o : 1, row);
}

// The copies that gather storages out of the payload: storage i's `nbytes[i]` bytes from stream position
// `src_pos[i]` to host address `dst[i]`, split at block boundaries — (dst, src, len) int64 arrays for one
// batched memcpy (libdlagg dla_host_copy_batch).
py::tuple span_pieces(py::array_t<int64_t, py::array::c_style> addrs, py::array_t<int64_t, py::array::c_style> lens,
                      py::array_t<int64_t, py::array::c_style> src_pos, py::array_t<int64_t, py::array::c_style> nbytes,
                      py::array_t<int64_t, py::array::c_style> dst) {
  const int64_t nb = static_cast<int64_t>(lens.size());
  const int64_t ns = static_cast<int64_t>(src_pos.size());
  if (addrs.size() != lens.size() || nbytes.size() != src_pos.size() || dst.size() != src_pos.size())
    throw std::invalid_argument("span_pieces: mismatched arrays");
  const int64_t* A = addrs.data();
  const int64_t* L = lens.data();
  std::vector<int64_t> start(static_cast<size_t>(nb) + 1, 0);
  for (int64_t i = 0; i < nb; ++i) start[i + 1] = start[i] + L[i];
  std::vector<int64_t> d, s, l;
  for (int64_t j = 0; j < ns; ++j) {
    int64_t p = src_pos.data()[j], k = nbytes.data()[j], to = dst.data()[j];
    if (p < 0 || k < 0 || p + k > start[nb]) throw std::invalid_argument("span_pieces: range outside the payload");
    int64_t i = static_cast<int64_t>(std::upper_bound(start.begin(), start.end(), p) - start.begin()) - 1;
    while (k > 0) {
      while (p >= start[i + 1]) ++i;
      const int64_t off = p - start[i];
      const int64_t take = std::min(k, L[i] - off);
      d.push_back(to);
      s.push_back(A[i] + off);
      l.push_back(take);
      to += take;
      p += take;
      k -= take;
    }
  }
  auto arr = [](const std::vector<int64_t>& v) {
    py::array_t<int64_t> a(static_cast<py::ssize_t>(v.size()));
    if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(int64_t));
    return a;
  };
  return py::make_tuple(arr(d), arr(s), arr(l));
}

// The decoded state dict over `buf` (a CPU uint8 tensor holding every storage of a scan, storage i at
// byte offset offsets[i]): an OrderedDict of `top`'s keys with, per description, a tensor over a storage
// of its OWN (storage i's bytes; its data pointer keeps `buf` alive) at the description's storage offset,
// sizes and strides — what pickle.loads + _rebuild_tensor_v2 give (one storage per pickled storage,
// tied entries one tensor), without a Python frame per tensor.  `top`'s _metadata is carried over.
py::object build_state_dict(const at::Tensor& buf, py::array_t<int64_t, py::array::c_style> offsets, py::object top,
                            py::list storages, py::object odict_cls) {
  if (!buf.is_cpu() || buf.scalar_type() != at::kByte || !buf.is_contiguous())
    throw std::invalid_argument("build_state_dict: buf must be a contiguous CPU uint8 tensor");
  const py::ssize_t ns = PyList_GET_SIZE(storages.ptr());
  if (offsets.size() != ns) throw std::invalid_argument("build_state_dict: one offset per storage");
  std::vector<c10::Storage> made(static_cast<size_t>(ns));
  std::vector<at::ScalarType> types(static_cast<size_t>(ns));
  char* base = static_cast<char*>(buf.data_ptr());
  at::Allocator* alloc = buf.storage().allocator();
  if (!alloc) alloc = c10::GetAllocator(c10::DeviceType::CPU);
  for (py::ssize_t i = 0; i < ns; ++i) {
    py::tuple rec = py::reinterpret_borrow<py::tuple>(PyList_GET_ITEM(storages.ptr(), i));
    const std::string dt = rec[0].cast<std::string>();
    const int64_t nbytes = rec[3].cast<int64_t>();
    const int64_t at = offsets.data()[i];
    if (at < 0 || at + nbytes > static_cast<int64_t>(buf.nbytes()))
      throw std::invalid_argument("build_state_dict: storage outside the buffer");
    int ty = -1;
    for (int j = 0; j < wirescan::kNumStorageTypes; ++j)
      if (dt == wirescan::kStorageTypes[j].dtype) ty = j;
    if (ty < 0) throw std::invalid_argument("build_state_dict: unknown dtype " + dt);
    types[i] = wirescan::kStorageTypes[ty].st;
    auto* keep = new c10::Storage(buf.storage());
    c10::DataPtr dp(base + at, keep, [](void* ctx) { delete static_cast<c10::Storage*>(ctx); }, buf.device());
    made[i] = c10::Storage(c10::Storage::use_byte_size_t(), static_cast<size_t>(nbytes), std::move(dp), alloc,
                           /*resizable=*/true);
  }
  py::object out = odict_cls();
  std::unordered_map<PyObject*, py::object> done;  // description -> its tensor (tied entries)
  PyObject* tensor_tag = wirescan::tags().tensor;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(top.ptr(), &pos, &k, &v)) {
    auto it = done.find(v);
    if (it == done.end()) {
      if (!PyTuple_CheckExact(v) || PyTuple_GET_SIZE(v) != 6 || PyTuple_GET_ITEM(v, 0) != tensor_tag)
        throw std::invalid_argument("build_state_dict: not a scanned tensor");
      const int64_t sidx = PyLong_AsLongLong(PyTuple_GET_ITEM(v, 1));
      if (sidx < 0 || sidx >= ns) throw std::invalid_argument("build_state_dict: bad storage index");
      const int64_t off = PyLong_AsLongLong(PyTuple_GET_ITEM(v, 2));
      PyObject* szt = PyTuple_GET_ITEM(v, 3);
      PyObject* stt = PyTuple_GET_ITEM(v, 4);
      if (!PyTuple_Check(szt) || !PyTuple_Check(stt) || PyTuple_GET_SIZE(szt) != PyTuple_GET_SIZE(stt) || off < 0)
        throw std::invalid_argument("build_state_dict: bad tensor description");
      std::vector<int64_t> sizes, strides;
      __int128 extent = 1;  // the elements the view spans lie inside its storage (whoever made `top`)
      bool empty = false;
      for (Py_ssize_t d = 0; d < PyTuple_GET_SIZE(szt); ++d) {
        sizes.push_back(PyLong_AsLongLong(PyTuple_GET_ITEM(szt, d)));
        strides.push_back(PyLong_AsLongLong(PyTuple_GET_ITEM(stt, d)));
        if (sizes.back() < 0 || strides.back() < 0) throw std::invalid_argument("build_state_dict: negative size");
        if (sizes.back() == 0) empty = true;
        extent += static_cast<__int128>(sizes.back() - 1) * strides.back();
      }
      if (PyErr_Occurred()) throw py::error_already_set();
      const int64_t esz = static_cast<int64_t>(c10::elementSize(types[sidx]));
      if (!empty && (off + extent) * esz > static_cast<__int128>(made[sidx].nbytes()))
        throw std::invalid_argument("build_state_dict: a tensor outside its storage");
      auto impl = c10::make_intrusive<c10::TensorImpl>(c10::Storage(made[sidx]), buf.key_set(),
                                                       c10::scalarTypeToTypeMeta(types[sidx]));
      impl->set_sizes_and_strides(sizes, strides, off);
      at::Tensor t(std::move(impl));
      if (PyTuple_GET_ITEM(v, 5) == Py_True) t.set_requires_grad(true);
      py::object w = py::reinterpret_steal<py::object>(THPVariable_Wrap(t));
      if (!w) throw py::error_already_set();
      it = done.emplace(v, w).first;
    }
    if (PyObject_SetItem(out.ptr(), k, it->second.ptr()) < 0) throw py::error_already_set();
  }
  py::object meta = py::getattr(top, "_metadata", py::none());
  if (!meta.is_none()) out.attr("_metadata") = meta;
  return out;
}

}  // namespace

PYBIND11_MODULE(_dla_walk, m) {
  m.doc() = "accdfl_amd host plumbing: the per-round walk over every parameter of every model";
  m.def("layout", &layout, py::arg("models"), py::arg("device"), py::arg("plain"), py::arg("tensor_major"),
        py::arg("ref") = py::none());
  m.def("tensors", &tensors, py::arg("model"), py::arg("plain"));
  m.def("block_table", &block_table, py::arg("blocks"));
  m.def("fingerprint", &fingerprint, py::arg("model"), py::arg("plain"));
  m.def("param_views", &param_views, py::arg("flat"), py::arg("params"), py::arg("offsets"), py::arg("memo"));
  m.def("param_fresh", &param_fresh, py::arg("params"), py::arg("memo"));
  py::class_<FreshParams>(m, "FreshParams").def("__len__", [](const FreshParams& h) { return h.t.size(); });
  m.def("param_blocks", &param_blocks, py::arg("params"));
  m.def("param_wrap", &param_wrap, py::arg("blocks"), py::arg("params"), py::arg("memo"));
  m.def("buffer_copies", &buffer_copies, py::arg("buffers"), py::arg("memo"));
  m.def("clone_value", &clone_value, py::arg("v"), py::arg("memo"), py::arg("atomic"), py::arg("modules"),
        py::arg("fallback"), py::arg("odict"), py::arg("setstate_fn") = py::none(), py::arg("full_state") = py::none());
  m.def("scan_state_dict", &scan_state_dict, py::arg("addrs"), py::arg("lens"), py::arg("odict_cls"));
  m.def("row_layout", &row_layout, py::arg("top"), py::arg("storages"), py::arg("names"), py::arg("dtype"),
        py::arg("shapes"));
  m.def("span_pieces", &span_pieces, py::arg("addrs"), py::arg("lens"), py::arg("src_pos"), py::arg("nbytes"),
        py::arg("dst"));
  m.def("build_state_dict", &build_state_dict, py::arg("buf"), py::arg("offsets"), py::arg("top"),
        py::arg("storages"), py::arg("odict_cls"));
  m.attr("scan_tensor_tag") = py::reinterpret_borrow<py::object>(wirescan::tags().tensor);
  m.attr("build_id") = py::str(kWalkIdTag + sizeof("dlagg-walk-build-id:") - 1);
}
