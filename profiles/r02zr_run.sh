mkdir -p gpurun_out/r02zr
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zr/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --host-configs-only > gpurun_out/r02zr/hostcfg.log 2>&1
