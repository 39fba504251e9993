#!/bin/bash
# SQ stall breakdown and L2 hit rate of the in-CG SpMV (one counter set per pass).
set -u
export TMPDIR=/tmp; OUT=gpurun_out/pmc_sq; rm -rf $OUT; mkdir -p $OUT
pass() {  # pass <name> <counters> <workload args>
    local name=$1 ctr=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -- python tools/pmc_workload.py "$@" > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass sq200 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" --n 200
pass tcc200 "TCC_HIT_sum TCC_MISS_sum" --n 200
pass sq7 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" --n 256 --stencil 7
pass tcc7 "TCC_HIT_sum TCC_MISS_sum" --n 256 --stencil 7
