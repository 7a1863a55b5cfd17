"""How fast can N GNLeNet CPU models be packed into one pinned slab? (diagnostic, GPU box)"""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
from torch import nn

torch.set_grad_enabled(False)
shapes = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,), (64,),
          (64,), (10, 576), (10,)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
models = [nn.ParameterList([nn.Parameter(torch.randn(s) * 0.05) for s in shapes]) for _ in range(n)]
params = [[p.detach() for p in m.parameters()] for m in models]
total = sum(torch.Size(s).numel() for s in shapes)
numels = [torch.Size(s).numel() for s in shapes]
pinned = torch.empty((n, total), pin_memory=True)
pageable = torch.empty((n, total))
libc = ctypes.CDLL(None)
libc.memcpy.restype = ctypes.c_void_p
libc.memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]


def t(fn, reps=500):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def cat_into(buf):
    def f():
        for k in range(n):
            torch.cat([p.view(-1) for p in params[k]], out=buf[k])
    return f


def foreach_into(buf):
    views = [list(torch.split(buf[k], numels)) for k in range(n)]

    def f():
        for k in range(n):
            torch._foreach_copy_(views[k], [p.view(-1) for p in params[k]])
    return f


def memcpy_into(buf):
    def f():
        for k in range(n):
            dst = buf[k].data_ptr()
            for p in params[k]:
                nb = p.numel() * 4
                libc.memcpy(dst, p.data_ptr(), nb)
                dst += nb
    return f


def np_into(buf):
    arr = buf.numpy()

    def f():
        for k in range(n):
            np.concatenate([p.numpy().reshape(-1) for p in params[k]], out=arr[k])
    return f


res = {}
for name, buf in (("pinned", pinned), ("pageable", pageable)):
    res["cat_" + name] = t(cat_into(buf))
    res["foreach_" + name] = t(foreach_into(buf))
    res["memcpy_" + name] = t(memcpy_into(buf))
    res["numpy_" + name] = t(np_into(buf))
torch.set_num_threads(1)
res["cat_pinned_1thread"] = t(cat_into(pinned))
print(json.dumps({"n": n, "bytes": n * total * 4, "us": res}))
