mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --host-configs-only > gpurun_out/r02zd_bound_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --host-configs-only --no-numa-bind > gpurun_out/r02zd_unbound_$i.log 2>&1 || exit 1
done
