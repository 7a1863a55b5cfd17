# Probe: big tile with buffer loads and amdgpu_waves_per_eu(2) (variant 18: 256 VGPRs, two
# waves per SIMD) vs the big tile (16, 270 VGPRs, one wave per SIMD) and the stream (4).
# (The variant-18 kernel this measured was removed after the probe: see DESIGN §9.)
set -e
timeout -k 10 120 python - <<'PY'
import sys, torch
sys.path.insert(0, "decentralized-learning_amd")
from accdfl_amd import _lib
for p in (4_194_304 + 4096 * 5 + 3, 1_000_003):
    n = 8
    slab = torch.randn(n, (p + 127) // 128 * 128, device="cuda") * 0.05
    w = [float(x) for x in torch.rand(n, dtype=torch.float64)]
    ptrs = [slab[k].data_ptr() for k in range(n)]
    outs = []
    for cfg in (None, _lib.LaunchCfg(18, 0, 0, 0)):
        o = torch.empty(p, device="cuda")
        _lib.wsum_ptrs(0, ptrs, w, p, o.data_ptr(), torch.cuda.current_stream().cuda_stream, cfg)
        outs.append(o)
    torch.cuda.synchronize()
    print("parity p=%d bit_exact=%s" % (p, torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))))
PY
for cfg in "8 25000000" "8 12500000" "8 21300000" "8 16000000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 f32"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype f32 --sweep-cfgs "0,0,0,0;16,0,0,0;18,0,0,0;4,1,0,64"
done
