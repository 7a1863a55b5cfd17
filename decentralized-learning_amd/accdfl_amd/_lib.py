"""ctypes binding of libdlagg.so (C ABI declared in include/dlagg.h).

This is the only way the package reaches the GPU reduce.  There is no CPU or
PyTorch fallback: if the library is missing, fails to load, or no HIP device is
visible, every entry point raises.  (The reference's CPU path is the thing being
replaced; a silent fallback would report reference numbers as ours.)
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
import threading
from typing import Optional, Sequence

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # decentralized-learning_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc", "dlagg.hip")
INCLUDE = os.path.join(REPO_ROOT, "include")
HEADER = os.path.join(INCLUDE, "dlagg.h")
# ACCDFL_AMD_TUNING=1 loads the tuning build (lib/libdlagg_tuning.so, -DDLA_TUNING=1: the same library
# plus the A/B environment knobs the profiles/ scripts sweep); the product build reads no environment.
TUNING = os.environ.get("ACCDFL_AMD_TUNING", "") == "1"


def tuning_env(name: str, default: str) -> str:
    """An A/B knob of the host side (the profiles/ scripts sweep them): read from the environment only
    under ACCDFL_AMD_TUNING=1, as the C library reads its knobs only in the tuning build; the product
    runs the measured policy and reads only the documented variables (ACCDFL_AMD_DEVICES,
    ACCDFL_AMD_RESULT_MEMORY)."""
    return os.environ.get(name, default) if TUNING else default

LIB_PATH = os.environ.get("DLAGG_LIB", os.path.join(PKG_ROOT, "lib",
                                                    "libdlagg_tuning.so" if TUNING else "libdlagg.so"))

# dtype codes (include/dlagg.h)
DLA_F32, DLA_BF16, DLA_F16, DLA_F64 = 0, 1, 2, 3
ABI_VERSION = 13

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",  # bit parity: no FMA contraction of w*p + acc
    "-fno-fast-math",
    "-fPIC",
    "-shared",
]

EXPORTED = (
    "dla_version",
    "dla_build_id",
    "dla_last_error",
    "dla_max_peers_per_pass",
    "dla_select_kernel",
    "dla_wsum",
    "dla_wsum_ex",
    "dla_wsum_slab",
    "dla_wsum_multi",
    "dla_plan_create",
    "dla_plan_set_weights",
    "dla_plan_launch",
    "dla_plan_destroy",
    "dla_mean",
    "dla_host_copy_batch",
    "dla_host_copy_batch_ex",
    "dla_wsum_sharded",
    "dla_shard_range",
    "dla_shutdown",
    "dla_wsum_slab_tiled",
    "dla_slab_tile_elems",
    "dla_host_round_start",
    "dla_host_round_finish",
    "dla_host_reduce",
    "dla_host_reduce_deferred",
    "dla_host_reduce_launch",
    "dla_host_reduce_join",
    "dla_wsum_multi_table_bytes",
    "dla_wsum_multi_table",
    "dla_slab_stage",
    "dla_host_in_place_rounds",
    "dla_wsum_multi_table_acc",
    "dla_wsum_mixed",
)


class DlaggError(RuntimeError):
    """A libdlagg call returned a non-zero status."""


def source_build_id(tuning: bool = False) -> str:
    """Hash of the sources and flags libdlagg.so is built from (csrc/dlagg.hip,
    include/dlagg.h, HIPCC_FLAGS; the tuning build's flag too).  build() compiles it into the
    library, and lib() refuses a library whose dla_build_id() differs from the tree's."""
    h = hashlib.sha256()
    for path in (CSRC, HEADER):
        with open(path, "rb") as f:
            h.update(f.read())
    h.update(" ".join(HIPCC_FLAGS + (_TUNING_FLAGS if tuning else [])).encode())
    return h.hexdigest()[:20]


_TUNING_FLAGS = ["-DDLA_TUNING=1"]


_ID_PREFIX = b"dlagg-build-id:"


def file_build_id(path: str, prefix: bytes = _ID_PREFIX) -> Optional[str]:
    """The build id embedded in a built library file (read from its bytes, not loaded)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(prefix)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(prefix):j].decode(errors="replace")


def build(force: bool = False, verbose: bool = False, tuning: bool = False) -> str:
    """Compile csrc/dlagg.hip for gfx950 into lib/libdlagg.so (in-tree; tuning=True: the A/B build,
    lib/libdlagg_tuning.so), unless the library there already carries this tree's build id."""
    out = os.path.join(PKG_ROOT, "lib", "libdlagg_tuning.so" if tuning else "libdlagg.so")
    bid = source_build_id(tuning)
    if not force and file_build_id(out) == bid:
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = out + ".tmp"
    cmd = [hipcc, *HIPCC_FLAGS, *(_TUNING_FLAGS if tuning else []), '-DDLA_BUILD_ID="%s"' % bid, "-I", INCLUDE,
           "-o", tmp, CSRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


_PROBE_ID_PREFIX = b"dlagg-probe-build-id:"


def probe_build_id() -> str:
    """Hash of csrc/probe.hip and HIPCC_FLAGS (the probe library's build id)."""
    h = hashlib.sha256()
    with open(os.path.join(PKG_ROOT, "csrc", "probe.hip"), "rb") as f:
        h.update(f.read())
    h.update(" ".join(HIPCC_FLAGS).encode())
    return h.hexdigest()[:20]


def build_probe(force: bool = False) -> str:
    """Compile the HBM ceiling probes (csrc/probe.hip -> lib/libdlagg_probe.so; diagnostics only),
    unless the library there already carries this tree's probe build id (as build() does)."""
    src = os.path.join(PKG_ROOT, "csrc", "probe.hip")
    out = os.path.join(PKG_ROOT, "lib", "libdlagg_probe.so")
    bid = probe_build_id()
    if not force and file_build_id(out, _PROBE_ID_PREFIX) == bid:
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, *HIPCC_FLAGS, '-DDLP_BUILD_ID="%s"' % bid, "-o", out + ".tmp", src], check=True)
    os.replace(out + ".tmp", out)
    return out


# ------------------------------------------------------------------ host walk extension
# csrc/walk.cpp: the per-round walk over every parameter of every model (host plumbing, built
# against torch's headers; not part of the C ABI).  Optional: without it the Python walk runs.
WALK_SRC = os.path.join(PKG_ROOT, "csrc", "walk.cpp")
_WALK_ID_PREFIX = b"dlagg-walk-build-id:"


def _walk_path() -> str:
    import sysconfig

    return os.path.join(PKG_ROOT, "lib", "_dla_walk" + sysconfig.get_config_var("EXT_SUFFIX"))


def walk_build_id() -> str:
    """Hash of csrc/walk.cpp, the torch version it is built against and its flags."""
    import torch

    h = hashlib.sha256()
    with open(WALK_SRC, "rb") as f:
        h.update(f.read())
    h.update(torch.__version__.encode())
    h.update(" ".join(_walk_flags()).encode())
    return h.hexdigest()[:20]


def _walk_flags():
    import sysconfig

    import torch
    from torch.utils import cpp_extension

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = cpp_extension.include_paths() + [sysconfig.get_paths()["include"]]
    libdir = cpp_extension.library_paths()[0]
    return (["-O2", "-shared", "-fPIC", "-std=c++17", "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi,
             "-DTORCH_EXTENSION_NAME=_dla_walk", "-DTORCH_API_INCLUDE_EXTENSION_H"] + ["-I" + d for d in inc] +
            ["-L" + libdir, "-ltorch_python", "-ltorch", "-ltorch_cpu", "-lc10", "-Wl,-rpath," + libdir])


def build_walk(force: bool = False) -> str:
    """Compile csrc/walk.cpp (g++) into lib/_dla_walk*.so unless it already carries this tree's id."""
    out = _walk_path()
    bid = walk_build_id()
    if not force and file_build_id(out, _WALK_ID_PREFIX) == bid:
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    subprocess.run([cxx, WALK_SRC, "-o", out + ".tmp", '-DDLA_WALK_BUILD_ID="%s"' % bid] + _walk_flags(), check=True)
    os.replace(out + ".tmp", out)
    return out


_walk_mod = None
_walk_tried = False


def walk_module():
    """The loaded host walk extension, or None when it is absent or not built from this tree (the
    callers then walk in Python: same result, ~10x slower per parameter)."""
    global _walk_mod, _walk_tried
    if not _walk_tried:
        _walk_tried = True
        path = _walk_path()
        try:
            if os.path.exists(path) and file_build_id(path, _WALK_ID_PREFIX) == walk_build_id():
                import importlib.machinery
                import importlib.util

                loader = importlib.machinery.ExtensionFileLoader("_dla_walk", path)
                spec = importlib.util.spec_from_file_location("_dla_walk", path, loader=loader)
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
                _walk_mod = mod
        except (ImportError, OSError):
            _walk_mod = None
    return _walk_mod


class _Lib:
    def __init__(self, path: str):
        if not os.path.exists(path):
            raise RuntimeError(
                "libdlagg.so not found at %s — build it first "
                "(python -c 'import __graft_entry__ as g; g.build()')" % path)
        self.path = path
        self.so = ctypes.CDLL(path)
        so = self.so
        vp = ctypes.c_void_p
        so.dla_version.restype = ctypes.c_int
        so.dla_build_id.restype = ctypes.c_char_p
        so.dla_last_error.restype = ctypes.c_char_p
        so.dla_max_peers_per_pass.restype = ctypes.c_int
        so.dla_select_kernel.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64]
        so.dla_select_kernel.restype = ctypes.c_char_p
        so.dla_wsum.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                ctypes.c_int64, vp, vp]
        so.dla_wsum.restype = ctypes.c_int
        so.dla_wsum_ex.argtypes = so.dla_wsum.argtypes + [ctypes.POINTER(LaunchCfg)]
        so.dla_wsum_ex.restype = ctypes.c_int
        so.dla_wsum_slab.argtypes = [ctypes.c_int, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                     ctypes.c_int64, vp, vp]
        so.dla_wsum_slab.restype = ctypes.c_int
        so.dla_wsum_multi.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                      vp]
        so.dla_wsum_multi.restype = ctypes.c_int
        so.dla_plan_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(vp),
                                       ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64, vp,
                                       ctypes.POINTER(LaunchCfg)]
        so.dla_plan_create.restype = ctypes.c_int
        so.dla_plan_set_weights.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        so.dla_plan_set_weights.restype = ctypes.c_int
        so.dla_plan_launch.argtypes = [vp, vp]
        so.dla_plan_launch.restype = ctypes.c_int
        so.dla_mean.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int64, vp, vp]
        so.dla_mean.restype = ctypes.c_int
        so.dla_host_copy_batch.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                           ctypes.c_int]
        so.dla_host_copy_batch.restype = ctypes.c_int
        so.dla_host_copy_batch_ex.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                              ctypes.c_int, ctypes.c_int]
        so.dla_host_copy_batch_ex.restype = ctypes.c_int
        so.dla_wsum_sharded.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                         ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64,
                                         ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(vp)]
        so.dla_wsum_sharded.restype = ctypes.c_int
        so.dla_shard_range.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        so.dla_shard_range.restype = ctypes.c_int
        so.dla_shutdown.restype = ctypes.c_int
        so.dla_wsum_slab_tiled.argtypes = [ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64, vp, vp,
                                           ctypes.POINTER(LaunchCfg)]
        so.dla_wsum_slab_tiled.restype = ctypes.c_int
        so.dla_slab_tile_elems.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64]
        so.dla_slab_tile_elems.restype = ctypes.c_int64
        so.dla_host_round_start.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp),
                                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double), vp,
                                            ctypes.c_int64, vp, vp]
        so.dla_host_round_start.restype = ctypes.c_int
        so.dla_host_round_finish.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64), vp,
                                             ctypes.POINTER(vp), vp]
        so.dla_host_round_finish.restype = ctypes.c_int
        so.dla_host_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(vp), ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, vp, vp,
                                       vp, vp, vp, vp]
        so.dla_host_reduce.restype = ctypes.c_int
        so.dla_host_reduce_deferred.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int), ctypes.c_int64,
                                                ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, vp]
        so.dla_host_reduce_deferred.restype = ctypes.c_int
        so.dla_host_reduce_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(vp),
                                              ctypes.POINTER(ctypes.c_int), ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, vp, vp, vp, vp, vp, vp, ctypes.POINTER(vp)]
        so.dla_host_reduce_launch.restype = ctypes.c_int
        so.dla_host_reduce_join.argtypes = [vp]
        so.dla_host_reduce_join.restype = ctypes.c_int
        so.dla_wsum_multi_table_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
        so.dla_wsum_multi_table_bytes.restype = ctypes.c_int64
        so.dla_wsum_multi_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                            ctypes.c_int, vp, vp, vp]
        so.dla_wsum_multi_table.restype = ctypes.c_int
        so.dla_wsum_multi_table_acc.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                                ctypes.c_int, ctypes.c_int, vp, vp, vp]
        so.dla_wsum_multi_table_acc.restype = ctypes.c_int
        so.dla_slab_stage.argtypes = [ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_int64, vp, ctypes.c_int64, vp]
        so.dla_slab_stage.restype = ctypes.c_int
        so.dla_host_in_place_rounds.argtypes = []
        so.dla_host_in_place_rounds.restype = ctypes.c_int64
        so.dla_wsum_mixed.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                      ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int64, vp, vp]
        so.dla_wsum_mixed.restype = ctypes.c_int
        so.dla_plan_destroy.argtypes = [vp]
        so.dla_plan_destroy.restype = None
        v = so.dla_version()
        if v != ABI_VERSION:
            raise RuntimeError("libdlagg ABI version %d, expected %d" % (v, ABI_VERSION))
        self.build_id = so.dla_build_id().decode()
        if os.path.exists(CSRC) and os.path.exists(HEADER):
            want = source_build_id(tuning=os.path.basename(path) == "libdlagg_tuning.so")
            if self.build_id != want:
                raise RuntimeError(
                    "stale libdlagg.so at %s: built from sources %s, the tree's are %s — rebuild it "
                    "(python -c 'import __graft_entry__ as g; g.build()')" % (path, self.build_id, want))
        self.max_peers_per_pass = so.dla_max_peers_per_pass()

    def check(self, rc: int, what: str):
        if rc != 0:
            msg = self.so.dla_last_error().decode(errors="replace")
            raise DlaggError("%s failed (status %d): %s" % (what, rc, msg))


class LaunchCfg(ctypes.Structure):
    """dla_launch_cfg_t (include/dlagg.h)."""
    _fields_ = [("variant", ctypes.c_int), ("chunks", ctypes.c_int), ("grid_blocks", ctypes.c_int),
                ("block", ctypes.c_int)]


_lib: Optional[_Lib] = None
_lock = threading.Lock()


def lib() -> _Lib:
    """The loaded library (loads on first use; raises if it cannot)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                _lib = _Lib(LIB_PATH)
    return _lib


def loaded_path() -> Optional[str]:
    return _lib.path if _lib is not None else None


# ------------------------------------------------------------------ typed calls
def _ptr_array(ptrs: Sequence[int]):
    arr = (ctypes.c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def _dbl_array(vals: Sequence[float]):
    arr = (ctypes.c_double * len(vals))()
    for i, v in enumerate(vals):
        arr[i] = float(v)
    return arr


def wsum_ptrs(dtype_code: int, peer_ptrs: Sequence[int], weights: Sequence[float], n_elems: int, out_ptr: int,
              stream_ptr: int, cfg: Optional[LaunchCfg] = None) -> None:
    """dla_wsum / dla_wsum_ex on raw device pointers."""
    L = lib()
    n = len(peer_ptrs)
    _check_tables("wsum", n, 1, weights=weights)
    if cfg is None:
        rc = L.so.dla_wsum(dtype_code, _ptr_array(peer_ptrs), _dbl_array(weights), n, n_elems, out_ptr, stream_ptr)
    else:
        rc = L.so.dla_wsum_ex(dtype_code, _ptr_array(peer_ptrs), _dbl_array(weights), n, n_elems, out_ptr,
                              stream_ptr, ctypes.byref(cfg))
    L.check(rc, "dla_wsum")


def wsum_mixed_ptrs(out_code: int, peer_codes: Sequence[int], peer_ptrs: Sequence[int], weights: Sequence[float],
                    n_elems: int, out_ptr: int, stream_ptr: int) -> None:
    """dla_wsum_mixed: one parameter whose peers have several dtypes (peer_codes[0] == out_code)."""
    L = lib()
    n = len(peer_ptrs)
    _check_tables("wsum_mixed", n, 1, weights=weights)
    if len(peer_codes) != n:
        raise ValueError("wsum_mixed: %d dtypes for %d peers" % (len(peer_codes), n))
    rc = L.so.dla_wsum_mixed(out_code, (ctypes.c_int * n)(*peer_codes), _ptr_array(peer_ptrs), _dbl_array(weights), n,
                             n_elems, out_ptr, stream_ptr)
    L.check(rc, "dla_wsum_mixed")


def select_kernel(dtype_code: int, n_peers: int, n_elems: int) -> str:
    """dla_select_kernel: the kernel family a default dla_wsum launch uses for this shape."""
    return lib().so.dla_select_kernel(dtype_code, n_peers, n_elems).decode()


def mean_ptrs(dtype_code: int, peer_ptrs: Sequence[int], n_elems: int, out_ptr: int, stream_ptr: int) -> None:
    """dla_mean: sequential sum / N (teacher-logit aggregation)."""
    L = lib()
    rc = L.so.dla_mean(dtype_code, _ptr_array(peer_ptrs), len(peer_ptrs), n_elems, out_ptr, stream_ptr)
    L.check(rc, "dla_mean")


def wsum_slab_ptr(dtype_code: int, base_ptr: int, pitch_elems: int, weights: Sequence[float], n_peers: int,
                  n_elems: int, out_ptr: int, stream_ptr: int) -> None:
    L = lib()
    _check_tables("wsum_slab", n_peers, 1, weights=weights)
    rc = L.so.dla_wsum_slab(dtype_code, base_ptr, pitch_elems, _dbl_array(weights), n_peers, n_elems, out_ptr,
                            stream_ptr)
    L.check(rc, "dla_wsum_slab")


def wsum_multi_ptrs(dtype_code: int, peer_ptrs: Sequence[int], out_ptrs: Sequence[int], numels: Sequence[int],
                    weights: Sequence[float], stream_ptr: int) -> None:
    """peer_ptrs is [n_tensors * n_peers] (tensor-major); sequences or ctypes arrays."""
    L = lib()
    t = len(out_ptrs)
    n = len(weights)
    if len(peer_ptrs) != t * n:
        raise ValueError("peer_ptrs must hold n_tensors * n_peers pointers")
    if len(numels) != t:
        raise ValueError("wsum_multi: %d numels for %d tensors" % (len(numels), t))
    num = numels if isinstance(numels, ctypes.Array) else (ctypes.c_int64 * t)(*[int(x) for x in numels])
    pa = peer_ptrs if isinstance(peer_ptrs, ctypes.Array) else _ptr_array(peer_ptrs)
    oa = out_ptrs if isinstance(out_ptrs, ctypes.Array) else _ptr_array(out_ptrs)
    rc = L.so.dla_wsum_multi(dtype_code, t, pa, oa, num, _dbl_array(weights), n, stream_ptr)
    L.check(rc, "dla_wsum_multi")


def wsum_multi_table_bytes(n_tensors: int, n_peers: int) -> int:
    """dla_wsum_multi_table_bytes: size of the device table of a dla_wsum_multi_table call."""
    return int(lib().so.dla_wsum_multi_table_bytes(n_tensors, n_peers))


def wsum_multi_table_ptrs(dtype_code: int, peer_ptrs, out_ptrs, numels, weights: Sequence[float], table_host: int,
                          table_dev: int, stream_ptr: int, acc_in: bool = False) -> None:
    """dla_wsum_multi_table (acc_in: dla_wsum_multi_table_acc, folding into the running sum the outputs
    hold): peer_ptrs is [n_tensors * n_peers] (tensor-major); sequences or ctypes arrays."""
    L = lib()
    n = len(weights)
    if not isinstance(out_ptrs, ctypes.Array):
        out_ptrs = _ptr_array(out_ptrs)
    t = len(out_ptrs)
    if not isinstance(peer_ptrs, ctypes.Array):
        peer_ptrs = (ctypes.c_void_p * len(peer_ptrs))(*peer_ptrs)
    if len(peer_ptrs) != t * n:
        raise ValueError("peer_ptrs must hold n_tensors * n_peers pointers")
    if len(numels) != t:
        raise ValueError("wsum_multi_table: %d numels for %d tensors" % (len(numels), t))
    if not isinstance(numels, ctypes.Array):
        numels = (ctypes.c_int64 * t)(*[int(x) for x in numels])
    if acc_in:
        rc = L.so.dla_wsum_multi_table_acc(dtype_code, t, peer_ptrs, out_ptrs, numels, _dbl_array(weights), n, 1,
                                           table_host, table_dev, stream_ptr)
    else:
        rc = L.so.dla_wsum_multi_table(dtype_code, t, peer_ptrs, out_ptrs, numels, _dbl_array(weights), n,
                                       table_host, table_dev, stream_ptr)
    if rc != 0:
        L.check(rc, "dla_wsum_multi_table")


DLA_COPY_STREAMING = 1


def host_copy_batch(dst_ptrs: Sequence[int], src_ptrs: Sequence[int], nbytes: Sequence[int],
                    streaming: bool = False) -> None:
    """dla_host_copy_batch(_ex): dst_ptrs[i] <- src_ptrs[i] (host memory), nbytes[i] bytes each;
    ``streaming``: non-temporal stores (destinations only the GPU reads next)."""
    L = lib()
    m = len(nbytes)
    if isinstance(nbytes, np.ndarray):  # int64 arrays (wire's EVA block gathers): no per-element conversion
        arrs = [np.ascontiguousarray(a, dtype=np.int64) for a in (dst_ptrs, src_ptrs, nbytes)]
        vpp = ctypes.POINTER(ctypes.c_void_p)
        rc = L.so.dla_host_copy_batch_ex(arrs[0].ctypes.data_as(vpp), arrs[1].ctypes.data_as(vpp),
                                         arrs[2].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), m,
                                         DLA_COPY_STREAMING if streaming else 0)
    else:
        rc = L.so.dla_host_copy_batch_ex((ctypes.c_void_p * m)(*dst_ptrs), (ctypes.c_void_p * m)(*src_ptrs),
                                         (ctypes.c_int64 * m)(*nbytes), m, DLA_COPY_STREAMING if streaming else 0)
    if rc != 0:
        L.check(rc, "dla_host_copy_batch")


def _check_tables(what: str, n_peers: int, n_tensors: int, tensor_ptrs=None, out_ptrs=None, weights=None):
    """The host-round entry points read n_peers x n_tensors peer pointers, n_tensors outputs and
    n_peers weights from the tables they are given: refuse shorter (or longer) tables here instead of
    letting the library read past their end."""
    if tensor_ptrs is not None and len(tensor_ptrs) != n_peers * n_tensors:
        raise ValueError("%s: %d peer pointers for %d tensors of %d peers" % (what, len(tensor_ptrs), n_tensors, n_peers))
    if out_ptrs is not None and len(out_ptrs) != n_tensors:
        raise ValueError("%s: %d output pointers for %d tensors" % (what, len(out_ptrs), n_tensors))
    if weights is not None and len(weights) != n_peers:
        raise ValueError("%s: %d weights for %d peers" % (what, len(weights), n_peers))


def host_round_start(dtype_code: int, n_peers: int, tensor_ptrs: Sequence[int], numels, weights: Sequence[float],
                     rows_ptr: int, pitch_elems: int, result_ptr: int, stream_ptr: int) -> None:
    """dla_host_round_start: pack the peers' host tensors (peer-major) into the page-locked rows
    and enqueue the reduce into the page-locked result.  ``numels``: a sequence or a ctypes
    int64 array (reused across rounds of one layout)."""
    L = lib()
    _check_tables("host_round_start", n_peers, len(numels), tensor_ptrs, weights=weights)
    if not isinstance(numels, ctypes.Array):
        numels = (ctypes.c_int64 * len(numels))(*numels)
    if not isinstance(tensor_ptrs, ctypes.Array):
        tensor_ptrs = (ctypes.c_void_p * len(tensor_ptrs))(*tensor_ptrs)
    rc = L.so.dla_host_round_start(dtype_code, n_peers, len(numels), tensor_ptrs, numels, _dbl_array(weights),
                                   rows_ptr, pitch_elems, result_ptr, stream_ptr)
    if rc != 0:
        L.check(rc, "dla_host_round_start")


def host_reduce(dtype_code: int, n_peers: int, tensor_ptrs, numels, weights: Sequence[float], out_ptrs,
                begin: int, end: int, chunk_elems: int, h_stage: int, d_stage: int, h_out: int, d_out: int,
                stream_ptr: int, copy_stream_ptr: int, outs_ready: "ctypes.c_int | None" = None) -> None:
    """dla_host_reduce: flat elements [begin, end) of a round of host tensors through the GPU in packed
    chunks (synchronous).  ``tensor_ptrs``: peer-major, n_peers * len(numels) host pointers;
    ``out_ptrs``: one per tensor.  Sequences or ctypes arrays (reused across the buckets of a round).
    ``outs_ready`` (a ctypes.c_int): dla_host_reduce_deferred — ``out_ptrs`` must then be a ctypes
    array the caller fills in place, then sets ``outs_ready.value`` to 1 (or -1 to give up)."""
    L = lib()
    _check_tables("host_reduce", n_peers, len(numels), tensor_ptrs, out_ptrs, weights)
    if not isinstance(numels, ctypes.Array):
        numels = (ctypes.c_int64 * len(numels))(*numels)
    if not isinstance(tensor_ptrs, ctypes.Array):
        tensor_ptrs = (ctypes.c_void_p * len(tensor_ptrs))(*tensor_ptrs)
    if not isinstance(out_ptrs, ctypes.Array):
        out_ptrs = (ctypes.c_void_p * len(out_ptrs))(*out_ptrs)
    if outs_ready is None:
        rc = L.so.dla_host_reduce(dtype_code, n_peers, len(numels), tensor_ptrs, numels, _dbl_array(weights),
                                  out_ptrs, begin, end, chunk_elems, h_stage, d_stage, h_out, d_out, stream_ptr,
                                  copy_stream_ptr)
    else:
        rc = L.so.dla_host_reduce_deferred(dtype_code, n_peers, len(numels), tensor_ptrs, numels,
                                           _dbl_array(weights), out_ptrs, ctypes.byref(outs_ready), begin, end,
                                           chunk_elems, h_stage, d_stage, h_out, d_out, stream_ptr, copy_stream_ptr)
    if rc != 0:
        L.check(rc, "dla_host_reduce")


class HostReduceJob:
    """A dla_host_reduce_launch job: holds every array the library reads until join()."""

    def __init__(self, handle: int, keep: tuple):
        self._handle = handle
        self._keep = keep

    def join(self) -> None:
        """dla_host_reduce_join (the wait releases the interpreter lock); raises DlaggError on failure.
        A job is joined once; later calls do nothing."""
        h, self._handle = self._handle, None
        if h is None:
            return
        L = lib()
        rc = L.so.dla_host_reduce_join(h)
        self._keep = None
        L.check(rc, "dla_host_reduce")

    def __del__(self):  # a job never joined would leak its thread: join it (errors dropped)
        if getattr(self, "_handle", None) is not None:
            try:
                lib().so.dla_host_reduce_join(self._handle)
            except Exception:  # noqa: BLE001  (interpreter shutdown)
                pass


def host_reduce_launch(device: int, dtype_code: int, n_peers: int, tensor_ptrs, numels, weights: Sequence[float],
                       out_ptrs, outs_ready, begin: int, end: int, chunk_elems: int, h_stage: int, d_stage: int,
                       h_out: int, d_out: int, stream_ptr: int, copy_stream_ptr: int) -> HostReduceJob:
    """dla_host_reduce_launch: dla_host_reduce_deferred on a library thread; returns at once.
    ``out_ptrs`` (a ctypes array) is filled by the caller, then ``outs_ready.value`` set to 1 (or -1)."""
    L = lib()
    _check_tables("host_reduce_launch", n_peers, len(numels), tensor_ptrs, out_ptrs, weights)
    if not isinstance(numels, ctypes.Array):
        numels = (ctypes.c_int64 * len(numels))(*numels)
    if not isinstance(tensor_ptrs, ctypes.Array):
        tensor_ptrs = (ctypes.c_void_p * len(tensor_ptrs))(*tensor_ptrs)
    h = ctypes.c_void_p()
    rc = L.so.dla_host_reduce_launch(device, dtype_code, n_peers, len(numels), tensor_ptrs, numels,
                                     _dbl_array(weights), out_ptrs, ctypes.byref(outs_ready), begin, end, chunk_elems,
                                     h_stage, d_stage, h_out, d_out, stream_ptr, copy_stream_ptr, ctypes.byref(h))
    L.check(rc, "dla_host_reduce_launch")
    return HostReduceJob(h.value, (tensor_ptrs, numels, out_ptrs, outs_ready))


def host_round_finish(dtype_code: int, numels, result_ptr: int, out_ptrs: Sequence[int], stream_ptr: int) -> None:
    """dla_host_round_finish: wait for the reduce, then unpack the result into out_ptrs."""
    L = lib()
    _check_tables("host_round_finish", 0, len(numels), out_ptrs=out_ptrs)
    if not isinstance(numels, ctypes.Array):
        numels = (ctypes.c_int64 * len(numels))(*numels)
    rc = L.so.dla_host_round_finish(dtype_code, len(numels), numels, result_ptr,
                                    (ctypes.c_void_p * len(out_ptrs))(*out_ptrs), stream_ptr)
    if rc != 0:
        L.check(rc, "dla_host_round_finish")


def wsum_sharded_ptrs(dtype_code: int, dev_ids: Sequence[int], peer_ptrs: Sequence[int], weights: Sequence[float],
                      n_elems: int, out_ptrs: Sequence[int], gather: int, stream_ptrs: Sequence[int]) -> None:
    """dla_wsum_sharded: bucket s of every peer reduced on dev_ids[s] into out_ptrs[s]."""
    L = lib()
    g = len(dev_ids)
    if len(out_ptrs) != g or len(stream_ptrs) != g:
        raise ValueError("one out pointer and one stream per shard")
    _check_tables("wsum_sharded", len(peer_ptrs), 1, weights=weights)
    rc = L.so.dla_wsum_sharded(dtype_code, g, (ctypes.c_int * g)(*dev_ids), _ptr_array(peer_ptrs),
                               _dbl_array(weights), len(peer_ptrs), n_elems, _ptr_array(out_ptrs), gather,
                               _ptr_array(stream_ptrs))
    L.check(rc, "dla_wsum_sharded")


def wsum_slab_tiled_ptr(dtype_code: int, base_ptr: int, tile_elems: int, slab_rows: int, weights: Sequence[float],
                        n_elems: int, out_ptr: int, stream_ptr: int, cfg: Optional[LaunchCfg] = None) -> None:
    """dla_wsum_slab_tiled: FedAvg of rows 0..len(weights)-1 of a tile-interleaved slab."""
    L = lib()
    rc = L.so.dla_wsum_slab_tiled(dtype_code, base_ptr, tile_elems, slab_rows, _dbl_array(weights), len(weights),
                                  n_elems, out_ptr, stream_ptr, ctypes.byref(cfg) if cfg is not None else None)
    L.check(rc, "dla_wsum_slab_tiled")


def slab_stage(dtype_code: int, base_ptr: int, tile_elems: int, slab_rows: int, n_tiles: int, row: int, dst_elem: int,
               src_ptr: int, n_elems: int, stream_ptr: int) -> None:
    """dla_slab_stage: n_elems elements at src_ptr (host or device) -> row `row` of a tile-interleaved
    slab of n_tiles tiles from flat element dst_elem on (one 2D copy for the whole tiles)."""
    L = lib()
    L.check(L.so.dla_slab_stage(dtype_code, base_ptr, tile_elems, slab_rows, n_tiles, row, dst_elem, src_ptr,
                                n_elems, stream_ptr), "dla_slab_stage")


def host_in_place_rounds() -> int:
    """dla_host_in_place_rounds: host rounds whose page-locked peer rows the kernel read in place."""
    return int(lib().so.dla_host_in_place_rounds())


def slab_tile_elems(dtype_code: int, slab_rows: int, n_elems: int) -> int:
    """dla_slab_tile_elems: the recommended tile of a tile-interleaved slab."""
    return int(lib().so.dla_slab_tile_elems(dtype_code, slab_rows, n_elems))


def shard_range(dtype_code: int, n_elems: int, n_shards: int, shard: int):
    """dla_shard_range: (start, end) of a shard's bucket."""
    L = lib()
    a, b = ctypes.c_int64(), ctypes.c_int64()
    L.check(L.so.dla_shard_range(dtype_code, n_elems, n_shards, shard, ctypes.byref(a), ctypes.byref(b)),
            "dla_shard_range")
    return a.value, b.value


def shutdown() -> None:
    """dla_shutdown: release the sharded reduce's events and the peer access it enabled."""
    L = lib()
    L.check(L.so.dla_shutdown(), "dla_shutdown")


class Plan:
    """dla_plan_t: a prepared reduce over fixed device buffers (launch-only per call)."""

    def __init__(self, dtype_code: int, peer_ptrs: Sequence[int], weights: Sequence[float], n_elems: int,
                 out_ptr: int, cfg: Optional[LaunchCfg] = None):
        L = lib()
        self._so = L.so
        self._check = L.check
        self.n_peers = len(peer_ptrs)
        h = ctypes.c_void_p()
        rc = L.so.dla_plan_create(ctypes.byref(h), dtype_code, _ptr_array(peer_ptrs), _dbl_array(weights),
                                  self.n_peers, n_elems, out_ptr, ctypes.byref(cfg) if cfg is not None else None)
        L.check(rc, "dla_plan_create")
        self._h = h

    def set_weights(self, weights: Sequence[float]) -> None:
        if len(weights) != self.n_peers:
            raise AssertionError("len(weights) != n_peers")
        self._check(self._so.dla_plan_set_weights(self._h, _dbl_array(weights)), "dla_plan_set_weights")

    def launch(self, stream_ptr: int) -> None:
        rc = self._so.dla_plan_launch(self._h, stream_ptr)
        if rc != 0:
            self._check(rc, "dla_plan_launch")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._so.dla_plan_destroy(h)
            self._h = None


class TiledPlan:
    """A prepared dla_wsum_slab_tiled call: the argument arrays are built once, so a round
    that reduces the same tiled slab again pays only the call (the tiled counterpart of Plan)."""

    def __init__(self, dtype_code: int, base_ptr: int, tile_elems: int, slab_rows: int, weights: Sequence[float],
                 n_elems: int, out_ptr: int, cfg: Optional[LaunchCfg] = None):
        L = lib()
        self._so = L.so
        self._check = L.check
        self.n_peers = len(weights)
        self._args = [dtype_code, base_ptr, tile_elems, slab_rows, _dbl_array(weights), self.n_peers, n_elems,
                      out_ptr]
        self._cfg = ctypes.byref(cfg) if cfg is not None else None
        self._keep = cfg

    def set_weights(self, weights: Sequence[float]) -> None:
        if len(weights) != self.n_peers:
            raise AssertionError("len(weights) != n_peers")
        self._args[4] = _dbl_array(weights)

    def launch(self, stream_ptr: int) -> None:
        rc = self._so.dla_wsum_slab_tiled(*self._args, stream_ptr, self._cfg)
        if rc != 0:
            self._check(rc, "dla_wsum_slab_tiled")
