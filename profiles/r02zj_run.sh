mkdir -p gpurun_out/r02zj
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_c_abi_demo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02zj/tests.log 2>&1 || exit 1
export DLA_HOST_REDUCE_STATS=1 PROBE_BIND=gpu
for i in 1 2; do timeout -k 10 200 python profiles/host_reduce_probe.py "ns,configs[2],configs[3'],configs[4]" > gpurun_out/r02zj/probe_$i.log 2>&1 || exit 1; done
