mkdir -p gpurun_out/r02zu
bash profiles/collect.sh r02zu --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small || exit 1
cp gpurun_out/prof_r02zu/summary/* gpurun_out/prof_r02zu/trace.log gpurun_out/r02zu/
rm -rf gpurun_out/prof_r02zu
