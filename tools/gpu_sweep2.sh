#!/bin/bash
# NT vs default-policy loads for the LDS SpMV across sizes; 7-pt at 256^3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
step() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    case $rc in 124|134|137|139) echo "fatal in $name, stopping"; exit $rc;; esac
    return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -q
step sweep_sizes 400 python tools/spmv_sweep.py --n 64 100 128 150 176 200 --variants 2000 2100 2000 2100 1000
step sweep_7pt 300 python tools/spmv_sweep.py --n 256 --stencil 7 --variants 1000 1001 2000 2100 2001 2000 2100
step bench_7pt 300 python bench.py --n 256 --stencil 7 --steps 3 --warmup 1 --no-cpu-baseline
