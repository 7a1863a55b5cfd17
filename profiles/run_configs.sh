mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --configs-only > gpurun_out/configs.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run -- python bench.py --configs-only > gpurun_out/configs_prof.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
