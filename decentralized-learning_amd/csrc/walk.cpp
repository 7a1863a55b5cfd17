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

// One model's parameters in nn.Module.parameters() order (`which` = "_parameters"; "_buffers": its
// buffers in nn.Module.buffers() order); false if a class is not plain.
bool walk(PyObject* mod, PyObject* plain, PtrSet& seen_m, PtrSet& seen_p, std::vector<PyObject*>& out,
          const char* which = "_parameters") {
  if (!seen_m.insert(mod)) return true;
  const int ok = PySet_Contains(plain, reinterpret_cast<PyObject*>(Py_TYPE(mod)));
  if (ok != 1) {
    if (ok < 0) PyErr_Clear();
    return false;
  }
  PyObject* d = PyObject_GenericGetDict(mod, nullptr);  // the instance __dict__ (new reference)
  if (!d) {
    PyErr_Clear();
    return false;
  }
  PyObject* params = PyDict_GetItemString(d, which);  // borrowed
  PyObject* mods = PyDict_GetItemString(d, "_modules");
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
  Py_DECREF(d);
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
  if (!walk(model.ptr(), plain.ptr(), seen_m, seen_p, bs, "_buffers")) return py::none();
  py::list pl, bl;
  for (PyObject* o : ps) pl.append(py::reinterpret_borrow<py::object>(o));
  for (PyObject* o : bs) bl.append(py::reinterpret_borrow<py::object>(o));
  return py::make_tuple(pl, bl);
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

// deepcopy of models[0]'s device buffers (fedavg.py:20 copies them, it does not average them) in one
// gather per (device, dtype), stored into the deepcopy memo: for each entry of `buffers` not already in
// `memo`, memo[id(buffer)] = a copy that is a view of one fresh allocation per group (views made first,
// then one fused multi-tensor copy into them).  Entries that are not plain dense CPU or CUDA tensors
// without grad, alone in their group, or sharing a storage with another buffer get no entry (the caller's
// deepcopy copies them, keeping the sharing).  Replaces a Python pass over every buffer (108 BN buffers
// of a google_speech ResNet-34: ~0.15 ms per round).
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
    // one allocation, a contiguous view of it per buffer, then ONE fused multi-tensor copy
    std::vector<at::Tensor> srcs, dsts;
    srcs.reserve(mem.size());
    dsts.reserve(mem.size());
    int64_t total = 0;
    for (py::ssize_t i : mem) {
      srcs.push_back(THPVariable_Unpack(PyList_GET_ITEM(buffers.ptr(), i)));
      total += srcs.back().numel();
    }
    const at::Tensor flat = at::empty({total}, srcs[0].options());
    int64_t off = 0;
    for (const at::Tensor& t : srcs) {
      dsts.push_back(alias_of(flat, t.sizes(), t.strides(), off));  // contiguous source: contiguous strides
      off += t.numel();
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
// Python _clone_value, for every other object), collections.OrderedDict, and "_compiled_call_impl" (the
// __dict__ entry a module clone leaves out).
struct CloneCtx {
  PyObject* memo;
  PyObject* atomic;
  PyObject* modules;
  PyObject* fallback;
  PyObject* odict;
  PyObject* skip;
};

PyObject* clone_mapping(PyObject* v, const CloneCtx& c, bool module_state = false);
PyObject* clone_sequence(PyObject* x, const CloneCtx& c);

bool memo_put(PyObject* memo, PyObject* x, PyObject* y) {
  PyObject* id = PyLong_FromVoidPtr(x);
  const int rc = id ? PyDict_SetItem(memo, id, y) : -1;
  Py_XDECREF(id);
  return rc == 0;
}

// A module of a class in ctx.modules, as copy._reconstruct does it: y = cls.__new__(cls), registered in
// the memo, state = a clone of x.__dict__ without _compiled_call_impl, y.__setstate__(state).
PyObject* clone_module(PyObject* x, const CloneCtx& c) {
  PyTypeObject* tp = Py_TYPE(x);
  static PyObject* const no_args = PyTuple_New(0);
  static PyObject* const setstate = PyUnicode_InternFromString("__setstate__");
  PyObject* y = tp->tp_new(tp, no_args, nullptr);
  if (!y) return nullptr;
  if (!memo_put(c.memo, x, y)) {
    Py_DECREF(y);
    return nullptr;
  }
  PyObject* d = PyObject_GenericGetDict(x, nullptr);
  PyObject* state = d ? clone_mapping(d, c, /*module_state=*/true) : nullptr;
  Py_XDECREF(d);
  PyObject* r = state ? PyObject_CallMethodOneArg(y, setstate, state) : nullptr;
  Py_XDECREF(state);
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
  PyObject* key = PyLong_FromVoidPtr(x);
  if (!key) return nullptr;
  PyObject* hit = PyDict_GetItemWithError(c.memo, key);  // borrowed
  Py_DECREF(key);
  if (hit) return Py_NewRef(hit);
  if (PyErr_Occurred()) return nullptr;
  const int at = PySet_Contains(c.atomic, reinterpret_cast<PyObject*>(Py_TYPE(x)));
  if (at < 0) return nullptr;
  if (at) return Py_NewRef(x);
  if (PyDict_CheckExact(x) || Py_TYPE(x) == reinterpret_cast<PyTypeObject*>(c.odict)) return clone_mapping(x, c);
  if (PyTuple_CheckExact(x) || PyList_CheckExact(x)) return clone_sequence(x, c);
  if (PySet_CheckExact(x) && PySet_GET_SIZE(x) == 0) {  // _non_persistent_buffers_set: a new empty set
    PyObject* y = PySet_New(nullptr);
    if (!y || !memo_put(c.memo, x, y)) {
      Py_XDECREF(y);
      return nullptr;
    }
    return y;
  }
  const int mod = PySet_Contains(c.modules, reinterpret_cast<PyObject*>(Py_TYPE(x)));
  if (mod < 0) return nullptr;
  if (mod) return clone_module(x, c);
  return PyObject_CallFunctionObjArgs(c.fallback, x, c.memo, nullptr);
}

// A tuple or list (a conv's kernel_size / stride / padding, _reversed_padding_repeated_twice), as
// copy.deepcopy copies them: a list is a new list registered in the memo before its items; a tuple is
// itself when every item clones to itself (tuples of numbers), else a new tuple registered in the memo.
PyObject* clone_sequence(PyObject* x, const CloneCtx& c) {
  if (PyList_CheckExact(x)) {
    PyObject* y = PyList_New(0);
    if (!y || !memo_put(c.memo, x, y)) {
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
  PyObject* id = PyLong_FromVoidPtr(x);
  PyObject* prev = id ? PyDict_GetItemWithError(c.memo, id) : nullptr;
  Py_XDECREF(id);
  if (prev || PyErr_Occurred()) {
    Py_DECREF(y);
    return prev ? Py_NewRef(prev) : nullptr;
  }
  if (!memo_put(c.memo, x, y)) {
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
PyObject* clone_mapping(PyObject* v, const CloneCtx& c, bool module_state) {
  // an empty OrderedDict (a module's hook dicts) iterates like a dict: no items() view needed
  const bool exact = PyDict_CheckExact(v);
  const bool plain_iter = exact || PyDict_GET_SIZE(v) == 0;
  PyObject* y = exact ? PyDict_New() : PyObject_CallNoArgs(reinterpret_cast<PyObject*>(Py_TYPE(v)));
  if (!y || !memo_put(c.memo, v, y)) {
    Py_XDECREF(y);
    return nullptr;
  }
  auto put = [&](PyObject* k, PyObject* x) -> bool {
    if (module_state && PyUnicode_Check(k) && PyUnicode_Compare(k, c.skip) == 0) return true;
    const int at = PySet_Contains(c.atomic, reinterpret_cast<PyObject*>(Py_TYPE(k)));
    if (at < 0) return false;
    PyObject* kc = at ? Py_NewRef(k) : PyObject_CallFunctionObjArgs(c.fallback, k, c.memo, nullptr);
    if (!kc) return false;
    PyObject* ci = clone_one(x, c);
    const int rc = ci ? (exact ? PyDict_SetItem(y, kc, ci) : PyObject_SetItem(y, kc, ci)) : -1;
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
                       py::object odict) {
  if (!PyAnySet_Check(atomic.ptr()) || !PyAnySet_Check(modules.ptr()))
    throw std::invalid_argument("clone_value: sets of atomic types and module classes");
  static PyObject* const skip = PyUnicode_InternFromString("_compiled_call_impl");
  const CloneCtx c{memo.ptr(), atomic.ptr(), modules.ptr(), fallback.ptr(), odict.ptr(), skip};
  PyObject* y = clone_one(v.ptr(), c);
  if (!y) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(y);
}

}  // namespace

PYBIND11_MODULE(_dla_walk, m) {
  m.doc() = "accdfl_amd host plumbing: the per-round walk over every parameter of every model";
  m.def("layout", &layout, py::arg("models"), py::arg("device"), py::arg("plain"), py::arg("tensor_major"),
        py::arg("ref") = py::none());
  m.def("tensors", &tensors, py::arg("model"), py::arg("plain"));
  m.def("block_table", &block_table, py::arg("blocks"));
  m.def("param_views", &param_views, py::arg("flat"), py::arg("params"), py::arg("offsets"), py::arg("memo"));
  m.def("buffer_copies", &buffer_copies, py::arg("buffers"), py::arg("memo"));
  m.def("clone_value", &clone_value, py::arg("v"), py::arg("memo"), py::arg("atomic"), py::arg("modules"),
        py::arg("fallback"), py::arg("odict"));
  m.attr("build_id") = py::str(kWalkIdTag + sizeof("dlagg-walk-build-id:") - 1);
}
