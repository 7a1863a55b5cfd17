"""CPU oracle for the accdfl FedAvg aggregation reduce.  TEST INFRASTRUCTURE ONLY.

Nothing in the product path (``decentralized-learning_amd/``) imports this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg do, and only as the checker / the timed CPU baseline.

Two restatements of the reference algorithm
(/root/reference/accdfl/core/gradient_aggregation/fedavg.py:12-26):

* :func:`fedavg_bits` — a NumPy bit-model of the arithmetic, per element::

      acc = p_0 * 0                                      # fedavg.py:21-22  p.mul_(0)
      for k in list order:                               # fedavg.py:23
          acc = R(acc + R(W(w_k) * p_k))                 # fedavg.py:25     c1.add_(w * p1)

  with W() = weight rounded from the Python double to the op-math type (float32 for
  f32/bf16/f16, float64 for f64) and R() = RNE rounding to the storage dtype after
  every product and every sum (no FMA).  bf16 is carried as uint16 bit patterns.

* :func:`fedavg_modules_torch` — the reference's own torch-CPU op sequence
  (deepcopy -> ``mul_(0)`` -> ``add_(w * p)`` in list order), restated.  This is
  the "reference CPU path" timed by ``bench.py`` as ``cpu_baseline`` (kind
  "port": the reference source never travels to the GPU box).

Parity pinning: both are checked bit-for-bit against golden vectors that
``tests/golden/make_golden.py`` generated in the build container by importing the
reference ``FedAvg`` itself.  See tests/test_oracle_golden.py.
"""
from __future__ import annotations

import copy
from typing import List, Sequence

import numpy as np

DTYPES = ("f32", "bf16", "f16", "f64")


def default_weights(n: int, weights):
    """fedavg.py:14-17 — falsy weights -> uniform float(1./N); else length must match."""
    if not weights:
        return [float(1.0 / n) for _ in range(n)]
    assert len(weights) == n
    return list(weights)


# ----------------------------------------------------------------- bf16 bit model
def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << np.uint32(16)).view(np.float32)


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    """RNE float32 -> bf16 bits, as c10::BFloat16 round_to_nearest_even (NaN -> 0x7FC0)."""
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)).astype(np.uint16)
    r[np.isnan(x)] = np.uint16(0x7FC0)
    return r


def _op32(w) -> np.float32:
    return np.float32(float(w))


def fedavg_bits(peers: Sequence[np.ndarray], weights, dtype: str) -> np.ndarray:
    """Bit-model of FedAvg over flat peer buffers.

    ``peers``: N arrays of equal length — float32 / float64 / float16 arrays, or
    uint16 bit patterns for bf16.  ``weights``: N Python numbers (already defaulted).
    Returns the averaged buffer in the same representation.
    """
    if dtype not in DTYPES:
        raise ValueError(dtype)
    n = len(peers)
    if n < 1:
        raise IndexError("list index out of range")  # fedavg.py:20 models[0]
    if len(weights) != n:
        raise AssertionError
    with np.errstate(all="ignore"):
        if dtype == "f32":
            acc = np.asarray(peers[0], np.float32) * np.float32(0)
            for p, w in zip(peers, weights):
                acc = acc + _op32(w) * np.asarray(p, np.float32)
            return acc.astype(np.float32)
        if dtype == "f64":
            acc = np.asarray(peers[0], np.float64) * 0.0
            for p, w in zip(peers, weights):
                acc = acc + float(w) * np.asarray(p, np.float64)
            return acc
        if dtype == "f16":
            acc = (np.asarray(peers[0], np.float16).astype(np.float32) * np.float32(0)).astype(np.float16)
            for p, w in zip(peers, weights):
                prod = (_op32(w) * np.asarray(p, np.float16).astype(np.float32)).astype(np.float16)
                acc = (acc.astype(np.float32) + prod.astype(np.float32)).astype(np.float16)
            return acc
        # bf16
        acc = f32_to_bf16(bf16_to_f32(np.asarray(peers[0], np.uint16)) * np.float32(0))
        for p, w in zip(peers, weights):
            prod = f32_to_bf16(_op32(w) * bf16_to_f32(np.asarray(p, np.uint16)))
            acc = f32_to_bf16(bf16_to_f32(acc) + bf16_to_f32(prod))
        return acc


def _as_f64(p, dt: str) -> np.ndarray:
    if dt == "bf16":
        return bf16_to_f32(np.asarray(p, np.uint16)).astype(np.float64)
    return np.asarray(p, {"f32": np.float32, "f16": np.float16, "f64": np.float64}[dt]).astype(np.float64)


def _round32(x32: np.ndarray, dt: str) -> np.ndarray:
    """An f32 op-math result rounded RNE to dtype dt, returned as float64 (exact)."""
    if dt == "bf16":
        return bf16_to_f32(f32_to_bf16(x32)).astype(np.float64)
    if dt == "f16":
        return x32.astype(np.float16).astype(np.float64)
    return x32.astype(np.float64)


def _round64(x64: np.ndarray, dt: str) -> np.ndarray:
    """An f64 op-math result cast to dtype dt as torch does (to 16-bit types through float)."""
    return x64 if dt == "f64" else _round32(x64.astype(np.float32), dt)


def fedavg_bits_mixed(peers: Sequence[np.ndarray], dtypes: Sequence[str], weights) -> np.ndarray:
    """Bit-model of fedavg.py:20-25 for one parameter whose peers have several dtypes (peer k in
    ``dtypes[k]``, represented as in :func:`fedavg_bits`); the result has dtypes[0] (the deepcopy of
    models[0], :20).  ``c1.add_(w * p1)`` (:25) rounds ``w * p1`` in p1's dtype (op-math f32, or f64
    for an f64 peer), then adds in the promoted type's op-math (f64 if either side is f64, else f32)
    and rounds the sum to the centre's dtype; an f64 sum reaches a 16-bit centre through float
    (c10::BFloat16 / c10::Half take a float).  Pinned by the reference: tests/golden/mixed_*."""
    n = len(peers)
    if n < 1:
        raise IndexError("list index out of range")
    if len(weights) != n or len(dtypes) != n:
        raise AssertionError
    d0 = dtypes[0]
    with np.errstate(all="ignore"):
        x0 = _as_f64(peers[0], d0)
        acc = x0 * 0.0 if d0 == "f64" else (x0.astype(np.float32) * np.float32(0)).astype(np.float64)
        for p, dk, w in zip(peers, dtypes, weights):
            x = _as_f64(p, dk)
            prod = float(w) * x if dk == "f64" else _round32(_op32(w) * x.astype(np.float32), dk)
            if d0 == "f64" or dk == "f64":
                acc = _round64(acc + prod, d0)
            else:
                acc = _round32(acc.astype(np.float32) + prod.astype(np.float32), d0)
    if d0 == "bf16":
        return f32_to_bf16(acc.astype(np.float32))
    return acc.astype({"f32": np.float32, "f16": np.float16, "f64": np.float64}[d0])


def fedavg_param_lists(param_lists: List[List[np.ndarray]], weights, dtype: str) -> List[np.ndarray]:
    """FedAvg over per-model parameter lists with the reference's zip truncation
    (fedavg.py:24: parameter i gets a term from every model that has >= i+1 params)."""
    n = len(param_lists)
    weights = default_weights(n, weights)
    if n < 1:
        raise IndexError("list index out of range")
    outs = []
    for i, p0 in enumerate(param_lists[0]):
        ks = [k for k in range(n) if len(param_lists[k]) > i]
        flat = [np.asarray(param_lists[k][i]).reshape(-1) for k in ks]
        outs.append(fedavg_bits(flat, [weights[k] for k in ks], dtype).reshape(np.asarray(p0).shape))
    return outs


# ------------------------------------------------------- torch op-sequence port
def fedavg_modules_torch(models, weights):
    """The reference op sequence on torch-CPU (fedavg.py:13-26), restated for timing."""
    import torch

    if not weights:
        weights = [float(1.0 / len(models)) for _ in range(len(models))]
    else:
        assert len(weights) == len(models)
    with torch.no_grad():
        center = copy.deepcopy(models[0])
        for p in center.parameters():
            p.mul_(0)
        for m, w in zip(models, weights):
            for c1, p1 in zip(center.parameters(), m.parameters()):
                c1.add_(w * p1)
        return center


def fedavg_flat_torch(peers, weights, out=None):
    """Same op sequence on flat CPU tensors (one parameter tensor per peer)."""
    import torch

    with torch.no_grad():
        acc = peers[0].clone() if out is None else out.copy_(peers[0])
        acc.mul_(0)
        for p, w in zip(peers, weights):
            acc.add_(w * p)
        return acc


def fedavg_flat_torch_warm(peers, weights, out, tmp):
    """fedavg_flat_torch with the product temporary of ``c1.add_(w * p1)`` (fedavg.py:25) in a
    caller-held buffer: the same op sequence and bits (``torch.mul(p, w, out=tmp)`` is ``w * p``),
    without a fresh allocation per peer.  In a fresh process each ``w * p`` of a 25 M model maps and
    page-faults 100 MB (glibc serves requests above its 32 MB mmap ceiling with a new mapping unless
    its heap already holds a free region that large), which makes the literal sequence 5-30x
    slower than its arithmetic; this is the sequence at its best, the stricter CPU baseline."""
    import torch

    with torch.no_grad():
        out.copy_(peers[0])
        out.mul_(0)
        for p, w in zip(peers, weights):
            torch.mul(p, w, out=tmp)
            out.add_(tmp)
        return out


# ------------------------------------------------------------ comparison helper
def same_bits(a: np.ndarray, b: np.ndarray, dtype: str) -> bool:
    """Bit equality, with every NaN equal to every NaN (payloads are not contract:
    torch-CPU emits 0x7FC0 or 0xFFFF for bf16 NaN depending on vector position)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if dtype == "bf16":
        fa, fb = bf16_to_f32(a.view(np.uint16)), bf16_to_f32(b.view(np.uint16))
        ua, ub = a.view(np.uint16), b.view(np.uint16)
    else:
        ftype = {"f32": np.float32, "f64": np.float64, "f16": np.float16}[dtype]
        utype = {"f32": np.uint32, "f64": np.uint64, "f16": np.uint16}[dtype]
        fa, fb = a.view(ftype), b.view(ftype)
        ua, ub = a.view(utype), b.view(utype)
    na, nb = np.isnan(fa), np.isnan(fb)
    if not np.array_equal(na, nb):
        return False
    return bool(np.array_equal(ua[~na], ub[~nb]))


def first_mismatch(a: np.ndarray, b: np.ndarray, dtype: str):
    """Index and values of the first differing element (for error messages)."""
    a = np.asarray(a).reshape(-1)
    b = np.asarray(b).reshape(-1)
    for i in range(a.size):
        if not same_bits(a[i : i + 1], b[i : i + 1], dtype):
            return i, a[i], b[i]
    return None
