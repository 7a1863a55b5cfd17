mkdir -p gpurun_out/r02zq
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02zq/smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r02zq/bench.log 2>&1
