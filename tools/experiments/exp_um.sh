#!/bin/bash
# Several slices per update workgroup (update_slices) with r.r folded (fold 1) or
# finalized (fold 2), after the bitwise option test.
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out/expu
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fusion_options or folded or tiny_and_thin" -x -q --timeout 240 --timeout-method thread > gpurun_out/expu/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/expu/pt.log; exit 1; }
tail -1 gpurun_out/expu/pt.log
run() {
    local name=$1; shift
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 4 --warmup 1 "$@" \
        > gpurun_out/expu/$name.log 2> gpurun_out/expu/$name.err
    local rc=$?
    echo "$name rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/expu/$name.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" 2>/dev/null)"
    case $rc in 124|134|137|139) exit $rc;; esac
}
for rep in 1 2; do
for cfg in "200:" "100:--n 100" "7:--n 256 --stencil 7"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  run ${tag}_u1f2_$rep $args
  run ${tag}_u1f1_$rep $args --fold 1
  run ${tag}_u4f1_$rep $args --fold 1 --update-slices 4
  run ${tag}_u8f1_$rep $args --fold 1 --update-slices 8
  run ${tag}_u4f2_$rep $args --update-slices 4
done
done
