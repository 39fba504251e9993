#!/bin/bash
# Batched window staging (84xx) vs the per-window loop (8226 / 8300).
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out/exps
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fusion_options or tiny_and_thin or csr_entry" -x -q --timeout 240 --timeout-method thread > gpurun_out/exps/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/exps/pt.log; exit 1; }
tail -1 gpurun_out/exps/pt.log
run() {
    local name=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 4 --warmup 1 "$@" \
        > gpurun_out/exps/$name.log 2> gpurun_out/exps/$name.err
    local rc=$?
    echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/exps/$name.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" 2>/dev/null)"
    case $rc in 124|134|137|139) exit $rc;; esac
}
for rep in 1 2; do
for v in 8226 8426 8446; do run 200_${v}_$rep --variant $v; done
for v in 8300 8423 8443; do run 100_${v}_$rep --n 100 --variant $v; done
done
