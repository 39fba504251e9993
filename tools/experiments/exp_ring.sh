#!/bin/bash
# x-deferral ring length and fold A/B (bench lines), after the bitwise option test.
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fusion_options or folded" -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/pt.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/exp/pt.log; exit 1; }
tail -2 gpurun_out/exp/pt.log
run() {
    local name=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 4 --warmup 1 "$@" \
        > gpurun_out/exp/$name.log 2> gpurun_out/exp/$name.err
    local rc=$?
    echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/exp/$name.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" 2>/dev/null)"
    case $rc in 124|134|137|139) exit $rc;; esac
}
S7="--n 256 --stencil 7"
for rep in 1 2; do
run 7_def_$rep $S7
run 7_r16_$rep $S7 --x-ring 16
run 7_r32_$rep $S7 --x-ring 32
run 7_r32f2_$rep $S7 --x-ring 32 --fold 2
run 200_def_$rep
run 200_r16_$rep --x-ring 16
run 200_r32_$rep --x-ring 32
run 200_r32f2_$rep --x-ring 32 --fold 2
run 100_def_$rep --n 100
run 100_r32_$rep --n 100 --x-ring 32
done
