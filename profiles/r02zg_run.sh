mkdir -p gpurun_out/r02zg
export DLA_HOST_REDUCE_STATS=1 PROBE_BIND=gpu
for mb in 8 16 32; do
  ACCDFL_AMD_HOST_CHUNK_MB=$mb timeout -k 10 200 python profiles/host_reduce_probe.py "ns,configs[2],configs[3'],configs[4]" > gpurun_out/r02zg/probe_c${mb}.log 2>&1 || exit 1
done
