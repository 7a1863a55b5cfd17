mkdir -p gpurun_out/r02zf
timeout -k 10 500 python bench.py > gpurun_out/r02zf/bench.log 2>&1 || exit 1
bash profiles/collect.sh r02zf --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small || exit 1
cp gpurun_out/prof_r02zf/summary/* gpurun_out/prof_r02zf/trace.log gpurun_out/r02zf/
rm -rf gpurun_out/prof_r02zf
