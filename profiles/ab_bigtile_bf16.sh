# Probe: bf16 big tiles (8 chunks per lane, forced variants 16 / 17) vs the default stream,
# with a bit-exactness check of the forced launches.
# (The forced bf16 big-tile path this measured was removed after the probe; on the current
# build variants 16 / 17 fall back to the stream for bf16.)
set -e
timeout -k 10 120 python - <<'PY'
import sys, torch
sys.path.insert(0, "decentralized-learning_amd")
from accdfl_amd import _lib
for n, p in ((8, 3_000_003), (4, 1_000_001)):
    slab = (torch.randn(n, (p + 127) // 128 * 128, device="cuda") * 0.05).to(torch.bfloat16)
    w = [float(x) for x in torch.rand(n, dtype=torch.float64)]
    ptrs = [slab[k].data_ptr() for k in range(n)]
    outs = []
    for cfg in (None, _lib.LaunchCfg(16, 0, 0, 0), _lib.LaunchCfg(17, 0, 0, 0)):
        o = torch.empty(p, device="cuda", dtype=torch.bfloat16)
        _lib.wsum_ptrs(1, ptrs, w, p, o.data_ptr(), torch.cuda.current_stream().cuda_stream, cfg)
        outs.append(o)
    torch.cuda.synchronize()
    print("parity n=%d p=%d bit_exact=%s" % (n, p, all(torch.equal(outs[0].view(torch.int16), o.view(torch.int16)) for o in outs[1:])))
PY
for cfg in "8 50000000" "8 40000000" "4 50000000" "6 50000000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 bf16"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype bf16 --sweep-cfgs "0,0,0,0;16,0,0,0;17,0,0,0"
done
