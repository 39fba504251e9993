#!/bin/bash
# Full GPU suite, default bench lines, then SELL-512-P variant A/B.
export TMPDIR=/tmp
O=gpurun_out/p2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = d.get("value_coded_secondary") or {}
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us frac {d['roofline']['frac']} upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']} | V {sec.get('value')} {sec.get('spmv_avg_us')}")
PY
}
run d200
run d100 --n 100
run d7 --n 256 --stencil 7 --steps 3
for v in 8226 8216; do run n200_$v --variant $v --steps 3 --warmup 1 --no-secondary; done
for v in 8300 8326; do run n100_$v --n 100 --variant $v --steps 3 --warmup 1 --no-secondary; done
for v in 8500 8507 8607; do run s7_$v --n 256 --stencil 7 --variant $v --steps 3 --warmup 1 --no-secondary; done
