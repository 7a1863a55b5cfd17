#!/bin/bash
# r03ab: (1) SQ counters of the north-star kernel capped at 14 workgroups per CU (the policy) and
# uncapped (DLA_VEC_WGS_PER_CU=0); (2) the cap on the strong-scaling shares of the north star
# (8 x 12.5 / 6.25 / 3.125 M f32: the policy caps launches of >= 256 MiB of input only), forced on
# (W=14) and off against the base build.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ab
mkdir -p $out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d $out/pmc_capped -o run -- python3 profiles/pmc_driver.py ns > $out/pmc_capped.log 2>&1 &&
DLA_VEC_WGS_PER_CU=0 timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d $out/pmc_uncapped -o run -- python3 profiles/pmc_driver.py ns > $out/pmc_uncapped.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_capped_fetch -o run -- python3 profiles/pmc_driver.py ns > $out/pmc_capped_fetch.log 2>&1 &&
for w in 0 14; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns_2,ns_4,ns_8 --stages "" --rounds 7 \
    > $out/shares_w${w}.log 2>&1 || exit $?
done
timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns_2,ns_4,ns_8 --stages "" --rounds 7 > $out/shares_policy.log 2>&1
