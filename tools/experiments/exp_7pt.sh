#!/bin/bash
# 7-pt 256^3 and 27-pt 200^3 A/B: fused p via LDS windows (SELL-512-P LDS), fused p in
# the plain gather, in-kernel dot completion. One bench line per case.
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out/exp7
run() {  # run <name> <args...>
    local name=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 "$@" \
        > gpurun_out/exp7/$name.log 2> gpurun_out/exp7/$name.err
    local rc=$?
    echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/exp7/$name.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" 2>/dev/null)"
    case $rc in 124|134|137|139) exit $rc;; esac
}
S7="--n 256 --stencil 7"
run 7_def $S7
run 7_8507_fuse $S7 --variant 8507 --fuse-p 1
run 7_8226 $S7 --variant 8226
run 7_8200 $S7 --variant 8200
run 7_8000 $S7 --variant 8000
run 7_8208 $S7 --variant 8208
run 7_fold2 $S7 --fold 2
run 7_8226_fold2 $S7 --variant 8226 --fold 2
run 200_fold2 --fold 2
run 200_fold3 --fold 3
run 200_def
