#!/bin/bash
# Pair kernel: batched staging loads (8972/8973), 64-VGPR cap (8974, 8966) vs 8963.
export TMPDIR=/tmp
O=gpurun_out/pair3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "variants_agree" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -n 5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']}")
PY
}
B="--steps 3 --warmup 1 --no-secondary"
for r in 1 2 3; do
  run d_$r $B
  for v in 8972 8973 8974 8966; do run v${v}_$r --variant $v $B; done
done
