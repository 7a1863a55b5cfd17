"""ctypes access to the C restatement of the reference reduce (oracle/fedavg_ref.c, test
infrastructure only: the checker the GPU tests compare the HIP path against)."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_so = None


def lib():
    global _so
    if _so is None:
        so = os.path.join(ROOT, "oracle", "_build", "liboracle_fedavg.so")
        if not os.path.exists(so):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        _so = ctypes.CDLL(so)
    return _so


def c_wsum(flat_peers, weights, dtype):
    """fedavg.py:20-25 over flat peer arrays (f32/f64 values, bf16/f16 raw uint16 bits)."""
    so = lib()
    n = len(flat_peers)
    fn = {"f32": so.oracle_wsum_f32, "f64": so.oracle_wsum_f64, "bf16": so.oracle_wsum_bf16,
          "f16": so.oracle_wsum_f16}[dtype]
    arrs = [np.ascontiguousarray(p) for p in flat_peers]
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    w = (ctypes.c_double * n)(*[float(x) for x in weights])
    out = np.empty_like(arrs[0])
    fn(ptrs, w, ctypes.c_int(n), ctypes.c_int64(out.size), ctypes.c_void_p(out.ctypes.data))
    return out


_CODE = {"f32": 0, "bf16": 1, "f16": 2, "f64": 3}
_NP = {"f32": np.float32, "bf16": np.uint16, "f16": np.uint16, "f64": np.float64}


def c_wsum_mixed(flat_peers, dtypes, weights):
    """fedavg.py:20-25 for peers of several dtypes (oracle_wsum_mixed; f32/f64 values, bf16/f16 raw
    uint16 bits); the result has dtypes[0]."""
    so = lib()
    n = len(flat_peers)
    arrs = [np.ascontiguousarray(p) for p in flat_peers]
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    w = (ctypes.c_double * n)(*[float(x) for x in weights])
    codes = (ctypes.c_int * n)(*[_CODE[d] for d in dtypes])
    out = np.empty(arrs[0].size, dtype=_NP[dtypes[0]])
    so.oracle_wsum_mixed(ctypes.c_int(_CODE[dtypes[0]]), codes, ptrs, w, ctypes.c_int(n), ctypes.c_int64(out.size),
                         ctypes.c_void_p(out.ctypes.data))
    return out
