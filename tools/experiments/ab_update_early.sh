#!/bin/bash
# Loop update with Ap and r loaded before the iteration test, and the
# early-load SELL-512-P LDS SpMV (8236), at the three single-GPU configs.
export TMPDIR=/tmp
O=gpurun_out/ue; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fusion_options" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -n 5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']} ue {d['config']['options']['update_early']}")
PY
}
B="--steps 3 --warmup 1 --no-secondary"
for r in 1 2; do
  run u200_0_$r --variant 8236 --update-early 0 $B
  run u200_1_$r --variant 8236 --update-early 1 $B
  run u100_0_$r --n 100 --update-early 0 $B
  run u100_1_$r --n 100 --update-early 1 $B
  run u7_0_$r --n 256 --stencil 7 --update-early 0 $B
  run u7_1_$r --n 256 --stencil 7 --update-early 1 $B
done
