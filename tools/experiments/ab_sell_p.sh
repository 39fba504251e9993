#!/bin/bash
# SELL-512-P (per-row pattern ids) against SELL-512-C in the CG bench, plus the
# 100^3 regression check (4200 vs 2200, resident_mb 0 / 128).
export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "variants_agree or fusion or sell_p or group_kernel or sell_v or value_codes" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us  upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']}")
PY
}
for v in 4200 8208 8216 8219 8226; do run n200_$v --n 200 --variant $v; done
for v in 4200 4300 8300 8308 8316 8208; do run n100_$v --n 100 --variant $v; done
run n100_8308_r0 --n 100 --variant 8308 --resident-mb 0
run n100_8308_r200 --n 100 --variant 8308 --resident-mb 200
for v in 3000 8500 8501; do run s7_$v --n 256 --stencil 7 --variant $v; done
