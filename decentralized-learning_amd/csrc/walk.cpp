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
//     (dtype name, [numel of each of models[0]'s parameters], pointer table bytes, device index)
// with the table tensor-major ([n_tensors][n_models] uint64) or peer-major ([n_models][n_tensors]).
// `device`: -1 for CPU parameters, a HIP device index every parameter must be on, or -2 for the HIP
// device of models[0]'s first parameter (the returned device index; -1 for CPU).
//
// This is host plumbing of the Python binding, not part of the C ABI (include/dlagg.h): it takes
// Python objects and is built against torch's headers.
#include <torch/extension.h>
#include <torch/csrc/autograd/python_variable.h>
#include <pybind11/numpy.h>

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

// One model's parameters in nn.Module.parameters() order (`which` = "_parameters"; "_buffers": its
// buffers in nn.Module.buffers() order); false if a class is not plain.
bool walk(PyObject* mod, PyObject* plain, std::unordered_set<PyObject*>& seen_m,
          std::unordered_set<PyObject*>& seen_p, std::vector<PyObject*>& out, const char* which = "_parameters") {
  if (seen_m.count(mod)) return true;
  const int ok = PySet_Contains(plain, reinterpret_cast<PyObject*>(Py_TYPE(mod)));
  if (ok != 1) {
    if (ok < 0) PyErr_Clear();
    return false;
  }
  seen_m.insert(mod);
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
      if (v == Py_None || seen_p.count(v)) continue;
      seen_p.insert(v);
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

py::object layout(py::list models, int device, py::object plain, bool tensor_major) {
  const Py_ssize_t n = static_cast<Py_ssize_t>(py::len(models));
  if (n < 1 || !PySet_Check(plain.ptr())) return py::none();
  std::vector<PyObject*> ps;
  std::vector<at::Tensor> p0;  // models[0]'s parameters (the reference layout)
  std::vector<uint64_t> ptrs;
  at::ScalarType dt = at::kFloat;
  std::unordered_set<PyObject*> seen_m, seen_p;  // per model, cleared (buckets kept) between models
  seen_m.reserve(512);
  seen_p.reserve(512);
  for (Py_ssize_t m = 0; m < n; ++m) {
    ps.clear();
    seen_m.clear();
    seen_p.clear();
    if (!walk(PyList_GET_ITEM(models.ptr(), m), plain.ptr(), seen_m, seen_p, ps)) return py::none();
    if (m == 0) {
      if (ps.empty()) return py::none();
      ptrs.resize(static_cast<size_t>(n) * ps.size());
    } else if (ps.size() != p0.size()) {
      return py::none();
    }
    const size_t nt = ps.size();
    for (size_t t = 0; t < nt; ++t) {
      if (!THPVariable_Check(ps[t])) return py::none();
      const at::Tensor& x = THPVariable_Unpack(ps[t]);
      if (m == 0) {
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
      ptrs[tensor_major ? t * n + m : m * nt + t] = reinterpret_cast<uint64_t>(x.data_ptr());
    }
  }
  py::list numels;
  for (const at::Tensor& x : p0) numels.append(x.numel());
  py::bytes table(reinterpret_cast<const char*>(ptrs.data()), ptrs.size() * sizeof(uint64_t));
  return py::make_tuple(py::str(dtype_name(dt)), numels, table, device);
}

// (parameters, buffers) of one model as lists, in parameters() / buffers() order, or None when its tree
// holds a class outside `plain`: the result module's fresh tensors are made from these without another
// Python walk of models[0] (fedavg._device_round).
py::object tensors(py::object model, py::object plain) {
  if (!PySet_Check(plain.ptr())) return py::none();
  std::unordered_set<PyObject*> seen_m, seen_p;
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

// The result module's fresh parameters of a device round (fedavg._device_round: deepcopy(models[0]) of
// fedavg.py:20 with every parameter a view of ONE allocation the reduce writes): for each of models[0]'s
// parameters p and its element offset in `flat`, an nn.Parameter over flat.as_strided(p's sizes, p's
// strides, offset) with p's requires_grad — what torch.Tensor._make_subclass(nn.Parameter, view, rg)
// builds (a detached alias whose metadata may change, wrapped as the Parameter class), without its ~8 us
// of Python per parameter (110 parameters of a google_speech ResNet-34: ~0.4 ms per round).
py::list param_views(const at::Tensor& flat, py::list params, const std::vector<int64_t>& offsets) {
  const py::ssize_t n = PyList_GET_SIZE(params.ptr());
  if (static_cast<size_t>(n) != offsets.size()) throw std::invalid_argument("param_views: one offset per parameter");
  py::list out(n);
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(params.ptr(), i);
    if (!THPVariable_Check(o)) throw std::invalid_argument("param_views: not a tensor");
    const at::Tensor& p = THPVariable_Unpack(o);
    at::Tensor v = flat.as_strided(p.sizes(), p.strides(), offsets[i]).detach();
    v.unsafeGetTensorImpl()->set_allow_tensor_metadata_change(true);
    v.set_requires_grad(p.requires_grad());
    PyObject* w = THPVariable_Wrap(v, reinterpret_cast<PyTypeObject*>(ParameterClass));
    if (!w) throw py::error_already_set();
    PyList_SET_ITEM(out.ptr(), i, w);  // steals the reference
  }
  return out;
}

// deepcopy of models[0]'s device buffers (fedavg.py:20 copies them, it does not average them) in one
// gather per (device, dtype): for each entry of `buffers`, a copy that is a view of one fresh allocation
// per group (views made first, then one fused multi-tensor copy into them), or None for an entry that is not a plain dense CPU or
// CUDA tensor without grad (the caller deep-copies those) or is alone in its group.  An object listed twice
// gets one copy (deepcopy's memo); buffers that share a storage are left to deepcopy.  Replaces a Python pass over every buffer (108 BN buffers of a
// google_speech ResNet-34: ~0.15 ms per round).
py::list buffer_copies(py::list buffers) {
  const py::ssize_t n = PyList_GET_SIZE(buffers.ptr());
  std::vector<int> group(n, -1);
  std::vector<std::pair<int, int>> keys;  // (device index, scalar type) of each group
  std::vector<std::vector<py::ssize_t>> members;
  std::unordered_map<PyObject*, py::ssize_t> first_of;
  std::vector<py::ssize_t> alias(n, -1);
  // tensors sharing a storage keep the stock deepcopy, which keeps them sharing one
  std::unordered_map<const void*, int> storage_uses;
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(buffers.ptr(), i);
    if (Py_TYPE(o) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) continue;
    const at::Tensor& t = THPVariable_Unpack(o);
    if (t.has_storage() && first_of.emplace(o, i).second) ++storage_uses[t.storage().unsafeGetStorageImpl()];
  }
  first_of.clear();
  for (py::ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(buffers.ptr(), i);
    if (Py_TYPE(o) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) continue;
    auto it = first_of.find(o);
    if (it != first_of.end()) {
      alias[i] = it->second;
      continue;
    }
    first_of.emplace(o, i);
    const at::Tensor& t = THPVariable_Unpack(o);
    if (t.requires_grad() || !t.is_contiguous() || !t.has_storage() || !(t.is_cuda() || t.is_cpu())) continue;
    if (storage_uses[t.storage().unsafeGetStorageImpl()] > 1) continue;
    const std::pair<int, int> key{t.get_device(), static_cast<int>(t.scalar_type())};
    size_t g = 0;
    while (g < keys.size() && keys[g] != key) ++g;
    if (g == keys.size()) {
      keys.push_back(key);
      members.emplace_back();
    }
    group[i] = static_cast<int>(g);
    members[g].push_back(i);
  }
  py::list out(n);
  for (py::ssize_t i = 0; i < n; ++i) PyList_SET_ITEM(out.ptr(), i, py::none().release().ptr());
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
      dsts.push_back(flat.as_strided(t.sizes(), t.strides(), off));  // contiguous source: contiguous strides
      off += t.numel();
    }
    at::_foreach_copy_(dsts, srcs);
    for (size_t j = 0; j < mem.size(); ++j) {
      const py::ssize_t i = mem[j];
      PyObject* w = THPVariable_Wrap(dsts[j]);
      if (!w) throw py::error_already_set();
      PyObject* old = PyList_GET_ITEM(out.ptr(), i);
      PyList_SET_ITEM(out.ptr(), i, w);
      Py_DECREF(old);
    }
  }
  for (py::ssize_t i = 0; i < n; ++i)
    if (alias[i] >= 0) {
      PyObject* c = PyList_GET_ITEM(out.ptr(), alias[i]);
      Py_INCREF(c);
      PyObject* old = PyList_GET_ITEM(out.ptr(), i);
      PyList_SET_ITEM(out.ptr(), i, c);
      Py_DECREF(old);
    }
  return out;
}

}  // namespace

PYBIND11_MODULE(_dla_walk, m) {
  m.doc() = "accdfl_amd host plumbing: the per-round walk over every parameter of every model";
  m.def("layout", &layout, py::arg("models"), py::arg("device"), py::arg("plain"), py::arg("tensor_major"));
  m.def("tensors", &tensors, py::arg("model"), py::arg("plain"));
  m.def("block_table", &block_table, py::arg("blocks"));
  m.def("param_views", &param_views, py::arg("flat"), py::arg("params"), py::arg("offsets"));
  m.def("buffer_copies", &buffer_copies, py::arg("buffers"));
  m.attr("build_id") = py::str(kWalkIdTag + sizeof("dlagg-walk-build-id:") - 1);
}
