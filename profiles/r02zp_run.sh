mkdir -p gpurun_out/r02zp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zp/gpu_tests.log 2>&1 || exit 1
timeout -k 10 500 python profiles/host_path_layout_probe.py > gpurun_out/r02zp/layout_paths.log 2>&1
