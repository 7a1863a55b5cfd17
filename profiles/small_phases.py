"""Phases of the small-round host path (GNLeNet, N peers, CPU modules) timed apart
(diagnostic, GPU box).  Usage: python profiles/small_phases.py [N]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402

shapes = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,), (64,),
          (64,), (10, 576), (10,)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
models = [nn.ParameterList([nn.Parameter(torch.randn(s) * 0.05) for s in shapes]) for _ in range(n)]
w = [1.0 / n] * n
dev = torch.device("cuda", 0)
total = sum(torch.Size(s).numel() for s in shapes)
numels = [torch.Size(s).numel() for s in shapes]
pitch = (total + 63) // 64 * 64
st = fa._HostStaging(dev, torch.float32)
st.ensure(n, pitch)
params = [list(m.parameters()) for m in models]
center = fa._center_copy(models[0], pin=False)
cparams = list(center.parameters())
cur = torch.cuda.current_stream(dev)


def t(fn, reps=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def pack():
    for k in range(n):
        torch.cat([p.detach().view(-1) for p in params[k]], out=st.h_in[k, :total])


def gpu():
    st.d_in[:n].copy_(st.h_in[:n], non_blocking=True)
    st.plan_for(n, total, w).launch(int(cur.cuda_stream))
    st.h_out[:total].copy_(st.d_out[:total], non_blocking=True)
    cur.synchronize()


def launch_only():
    st.plan_for(n, total, w).launch(int(cur.cuda_stream))
    cur.synchronize()


def unpack():
    torch._foreach_copy_([c.view(-1) for c in cparams], list(torch.split(st.h_out[:total], numels)))


from types import SimpleNamespace  # noqa: E402

from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod  # noqa: E402
from accdfl_amd.core.model_manager import DeviceModelManager  # noqa: E402

mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0, capacity=n)


def dmm_round():
    mm.reset_incoming_trained_models()
    for k, m in enumerate(models):
        mm.process_incoming_trained_model(k, m)
    return mm.aggregate_trained_models(w)


torch.set_grad_enabled(False)
res = {
    "device_model_manager_round_us": t(dmm_round),
    "aggregate_us": t(lambda: fa.FedAvg.aggregate(models, w)),
    "parameters_lists_us": t(lambda: [list(m.parameters()) for m in models]),
    "center_copy_us": t(lambda: fa._center_copy(models[0], pin=False)),
    "pack_us": t(pack),
    "h2d_launch_d2h_sync_us": t(gpu),
    "launch_sync_us": t(launch_only),
    "unpack_us": t(unpack),
    "deepcopy_plain_us": t(lambda: __import__("copy").deepcopy(models[0])),
}
print(json.dumps({"n": n, "params": total, **res}))
