mkdir -p gpurun_out
export DLA_HOST_REDUCE_STATS=1
for th in 8 16; do for mb in 32 96; do
  DLA_COPY_THREADS=$th ACCDFL_AMD_HOST_CHUNK_MB=$mb timeout -k 10 200 python profiles/host_reduce_probe.py "ns,configs[3'],configs[4]" > gpurun_out/r02z_probe_t${th}_c${mb}.log 2>&1 || exit 1
done; done
