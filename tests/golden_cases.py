"""Loader for the golden FedAvg vectors in tests/golden/*.npz (made by make_golden.py
from the reference implementation)."""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NP_FLOAT = {"f32": np.float32, "f16": np.float16, "f64": np.float64}


@dataclass
class Case:
    name: str
    dtype: str
    weights: Optional[list]
    params: List[List[np.ndarray]]      # [peer][param] raw bits, shaped
    buffers: List[List[np.ndarray]]     # [peer][buffer]
    out: List[np.ndarray]               # reference output params (raw bits)
    out_buffers: List[np.ndarray]
    requires_grad: List[bool]
    in_requires_grad: List[bool]


def case_names() -> List[str]:
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith(("wire_", "mixed_")))


def load(name: str) -> Case:
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))
    meta = json.loads(str(z["meta"]))
    n = meta["n_peers"]
    params = [[z["p_%d_%d" % (k, i)].reshape(s) for i, s in enumerate(meta["shapes"][k])] for k in range(n)]
    nb = len(meta["buffers"])
    buffers = [[z["b_%d_%d" % (k, j)] for j in range(nb)] for k in range(n)]
    n_out = len(meta["shapes"][0])
    out = [z["out_%d" % i].reshape(meta["shapes"][0][i]) for i in range(n_out)]
    out_buffers = [z["outb_%d" % j] for j in range(nb)]
    return Case(meta["name"], meta["dtype"], meta["weights"], params, buffers, out, out_buffers,
                meta["requires_grad"], meta.get("in_requires_grad", meta["requires_grad"]))


def as_float(bits: np.ndarray, dtype: str) -> np.ndarray:
    """Raw bits -> float array (bf16 stays as uint16 bits: the oracle's representation)."""
    if dtype == "bf16":
        return bits.view(np.uint16)
    return bits.view(NP_FLOAT[dtype])


def to_torch(bits: np.ndarray, dtype: str):
    import torch

    tdt = {"f32": torch.int32, "bf16": torch.int16, "f16": torch.int16, "f64": torch.int64}[dtype]
    fdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}[dtype]
    sdt = {"f32": np.int32, "bf16": np.int16, "f16": np.int16, "f64": np.int64}[dtype]
    return torch.from_numpy(np.ascontiguousarray(bits).view(sdt).copy()).view(tdt).view(fdt)


def from_torch(t, dtype: str) -> np.ndarray:
    import torch

    tdt = {"f32": torch.int32, "bf16": torch.int16, "f16": torch.int16, "f64": torch.int64}[dtype]
    udt = {"f32": np.uint32, "bf16": np.uint16, "f16": np.uint16, "f64": np.uint64}[dtype]
    return t.detach().cpu().contiguous().view(tdt).numpy().view(udt)


def build_models(case: Case, device="cpu"):
    """Reconstruct the peer nn.Modules of a case (same parameter order / buffers)."""
    import torch
    from torch import nn

    class Peer(nn.Module):
        def __init__(self, ps, bs):
            super().__init__()
            rg = list(case.in_requires_grad) + [True] * max(0, len(ps) - len(case.in_requires_grad))
            self.ps = nn.ParameterList([nn.Parameter(to_torch(p, case.dtype), requires_grad=r)
                                        for p, r in zip(ps, rg)])
            for j, b in enumerate(bs):
                self.register_buffer("b%d" % j, torch.from_numpy(b.copy()))

    return [Peer(case.params[k], case.buffers[k]).to(device) for k in range(len(case.params))]


@dataclass
class MixedCase:
    """A round whose models do not share one dtype (make_golden.save_mixed_cases)."""
    name: str
    dtypes: List[List[str]]             # [peer][param]
    weights: Optional[list]
    params: List[List[np.ndarray]]      # [peer][param] raw bits, shaped
    out: List[np.ndarray]               # reference output params (raw bits, models[0]'s dtypes)

    @property
    def out_dtypes(self) -> List[str]:
        return self.dtypes[0]


def mixed_case_names() -> List[str]:
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "mixed_*.npz")))


def load_mixed(name: str) -> MixedCase:
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))
    meta = json.loads(str(z["meta"]))
    n = meta["n_peers"]
    params = [[z["p_%d_%d" % (k, i)].reshape(s) for i, s in enumerate(meta["shapes"][k])] for k in range(n)]
    out = [z["out_%d" % i].reshape(s) for i, s in enumerate(meta["shapes"][0])]
    return MixedCase(meta["name"], meta["dtypes"], meta["weights"], params, out)


def build_mixed_models(case: MixedCase, device="cpu"):
    """The peer nn.Modules of a mixed case (parameter i of peer k in case.dtypes[k][i])."""
    from torch import nn

    class Peer(nn.Module):
        def __init__(self, ps, dts):
            super().__init__()
            self.ps = nn.ParameterList([nn.Parameter(to_torch(p, d)) for p, d in zip(ps, dts)])

    return [Peer(case.params[k], case.dtypes[k]).to(device) for k in range(len(case.params))]
