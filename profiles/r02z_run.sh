mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_c_abi_demo.py tests/test_call_sites.py tests/test_gpu_dfl_round.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02z_tests.log 2>&1 || exit 1
export DLA_HOST_REDUCE_STATS=1
for th in 8 16; do for mb in 32 64; do
  DLA_COPY_THREADS=$th ACCDFL_AMD_HOST_CHUNK_MB=$mb timeout -k 10 200 python profiles/host_reduce_probe.py "ns,configs[2],configs[3'],configs[4]" > gpurun_out/r02z_probe_t${th}_c${mb}.log 2>&1 || exit 1
done; done
