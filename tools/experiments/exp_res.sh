#!/bin/bash
# resident_mb sweep at 100^3 with SELL-512-P (MB of the image on default-policy loads).
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out/expr
run() {
    local name=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 4 --warmup 1 "$@" \
        > gpurun_out/expr/$name.log 2> gpurun_out/expr/$name.err
    local rc=$?
    echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/expr/$name.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" 2>/dev/null)"
    case $rc in 124|134|137|139) exit $rc;; esac
}
for rep in 1 2; do
for r in 0 64 128 176 224 400; do run 100_r${r}_$rep --n 100 --resident-mb $r --variant 8226; done
run 100_def_$rep --n 100
run 100_x8_$rep --n 100 --x-ring 8
done
