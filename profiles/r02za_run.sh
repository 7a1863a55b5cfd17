mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 python profiles/cpu_baseline_probe.py 4 > gpurun_out/r02za_cpu_$i.log 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02za_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02za_bench.log 2>&1
