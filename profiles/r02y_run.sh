mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_c_abi_demo.py tests/test_call_sites.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02y_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --host-configs-only > gpurun_out/r02y_hostcfg_native.log 2>&1 &&
ACCDFL_AMD_HOST_PATH=pipelined timeout -k 10 300 python bench.py --host-configs-only > gpurun_out/r02y_hostcfg_pipelined.log 2>&1 &&
timeout -k 10 200 python bench.py --sweep --tile-bytes 16384 --sweep-cfgs 9,22,23,24 --no-ceilings > gpurun_out/r02y_sweep_ns.log 2>&1 &&
timeout -k 10 200 python bench.py --sweep --peers 128 --params 2662045 --dtype bf16 --tile-bytes 4096,16384 --sweep-cfgs 21,9,22,23,24 --no-ceilings > gpurun_out/r02y_sweep_c4.log 2>&1
