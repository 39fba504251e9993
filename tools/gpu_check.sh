#!/bin/bash
# One GPU-box pass: parity tests, kernel sweep, bench (events + graph), CLI.
# Every GPU step has its own time limit; the script stops at the first
# crash/timeout (exit codes 124/134/137/139) and never retries.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    case $rc in 124|134|137|139) echo "fatal in $name, stopping"; exit $rc;; esac
    return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -q
[ -n "${SKIP_SWEEP:-}" ] || step sweep 300 python tools/spmv_sweep.py
step bench_events 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline
step bench_nofold 300 python bench.py --steps 5 --warmup 1 --fold 0 --no-cpu-baseline
step bench_nofuse 300 python bench.py --steps 5 --warmup 1 --fuse-p 0 --no-cpu-baseline
step bench_7pt 300 python bench.py --n 256 --stencil 7 --steps 3 --warmup 1 --no-cpu-baseline
step bench_7pt_nodefer 300 python bench.py --n 256 --stencil 7 --steps 3 --warmup 1 --x-defer 0 --no-cpu-baseline
step bench_100 300 python bench.py --n 100 --steps 5 --warmup 1 --no-cpu-baseline
step bench_100_nofold 300 python bench.py --n 100 --steps 5 --warmup 1 --fold 0 --no-cpu-baseline
step bench_100_fold2 300 python bench.py --n 100 --steps 5 --warmup 1 --fold 2 --no-cpu-baseline
step bench_100_fold3 300 python bench.py --n 100 --steps 5 --warmup 1 --fold 3 --no-cpu-baseline
step bench_fold2 300 python bench.py --steps 5 --warmup 1 --fold 2 --no-cpu-baseline
step bench_fold3 300 python bench.py --steps 5 --warmup 1 --fold 3 --no-cpu-baseline
step bench_7pt_nofold 300 python bench.py --n 256 --stencil 7 --steps 3 --warmup 1 --fold 0 --no-cpu-baseline
step cli_100 120 hpccg-sycl_amd/bin/test_HPCCG 100 100 100
HPCCG_DEVICE_GENERATE=1 step cli_200dev 120 hpccg-sycl_amd/bin/test_HPCCG 200 200 200
step cli_10 60 hpccg-sycl_amd/bin/test_HPCCG 10 10 10
