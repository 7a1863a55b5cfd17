mkdir -p gpurun_out/r02zh
bash profiles/collect.sh r02zh_c4 --peers 128 --params 2662045 --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small --no-strong || exit 1
cp gpurun_out/prof_r02zh_c4/summary/* gpurun_out/prof_r02zh_c4/trace.log gpurun_out/r02zh/
rm -rf gpurun_out/prof_r02zh_c4
