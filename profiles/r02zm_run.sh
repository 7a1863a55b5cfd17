mkdir -p gpurun_out/r02zm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zm/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python profiles/small_round_crossover.py > gpurun_out/r02zm/crossover.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --host-configs-only > gpurun_out/r02zm/hostcfg.log 2>&1
