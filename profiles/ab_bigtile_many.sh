# A/B: default kernel (stream / wide) vs the peer-major big-tile kernel (forced variant 16)
# for fp32 shares of 16 and 32 peers, plus a bit-exactness check of the forced launch.
set -e
timeout -k 10 120 python - <<'PY'
import sys, torch
sys.path.insert(0, "decentralized-learning_amd")
from accdfl_amd import _lib
for n, p in ((16, 3_000_001), (32, 1_690_046)):
    slab = torch.randn(n, (p + 127) // 128 * 128, device="cuda") * 0.05
    w = [float(x) for x in torch.rand(n, dtype=torch.float64)]
    ptrs = [slab[k].data_ptr() for k in range(n)]
    outs = []
    for cfg in (None, _lib.LaunchCfg(16, 0, 0, 0)):
        o = torch.empty(p, device="cuda")
        _lib.wsum_ptrs(0, ptrs, w, p, o.data_ptr(), torch.cuda.current_stream().cuda_stream, cfg)
        outs.append(o)
    torch.cuda.synchronize()
    print("parity n=%d p=%d bit_exact=%s" % (n, p, torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))))
PY
for cfg in "16 12500000" "16 21296355" "32 1690046" "32 6250000" "16 3000000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 f32"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype f32 --sweep-cfgs "0,0,0,0;16,0,0,0"
done
