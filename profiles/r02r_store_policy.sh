set -o pipefail
mkdir -p gpurun_out
run() { echo "## $*"; timeout -k 10 200 python -u bench.py --sweep --no-ceilings "$@" 2>&1 | grep -v amdgpu.ids; }
{
run --peers 32 --params 1690046 --dtype f32 --tile-bytes 1024 --sweep-cfgs 9,21 &&
run --peers 64 --params 1233086 --dtype f32 --tile-bytes 4096 --sweep-cfgs 9,21 &&
run --peers 128 --params 2662045 --dtype bf16 --tile-bytes 4096 --sweep-cfgs 9,21 &&
run --peers 128 --params 85354 --dtype f32 --tile-bytes 1024 --sweep-cfgs 9,21 &&
run --peers 64 --params 4932344 --dtype f32 --tile-bytes 4096 --sweep-cfgs 9,21 &&
run --peers 128 --params 21296355 --dtype bf16 --tile-bytes 4096 --sweep-cfgs 9,21 &&
run --peers 8 --params 25000000 --dtype f32 --tile-bytes 16384 --sweep-cfgs 9,21 &&
echo "## separate buffers (row-major), cfg variant 9 vs 21" &&
run --peers 32 --params 1690046 --dtype f32 --sweep-cfgs "9,0,0,0;21,0,0,0" &&
run --peers 64 --params 1233086 --dtype f32 --sweep-cfgs "9,0,0,0;21,0,0,0" &&
run --peers 128 --params 2662045 --dtype bf16 --sweep-cfgs "9,0,0,0;21,0,0,0" &&
run --peers 128 --params 665511 --dtype bf16 --sweep-cfgs "9,0,0,0;21,0,0,0" &&
run --peers 128 --params 21296355 --dtype bf16 --sweep-cfgs "9,0,0,0;21,0,0,0"
} > gpurun_out/r02r_sweep_store_policy.log
