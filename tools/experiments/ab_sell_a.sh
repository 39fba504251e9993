#!/bin/bash
# SELL-512-A (offset-aligned slots, direct x loads) vs the defaults, with the
# p update separate or formed per x load (fuse_p 1): parity first, then bench.
export TMPDIR=/tmp
O=gpurun_out/sa; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants_agree or fusion_options" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us frac {d['roofline']['frac']} upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']}")
PY
}
B="--steps 3 --warmup 1 --no-secondary"
run d200 $B
run a200_8700 --variant 8700 $B
run a200_8700f --variant 8700 --fuse-p 1 $B
run a200_8727f --variant 8727 --fuse-p 1 $B
run d100 --n 100 $B
run a100_8800 --n 100 --variant 8800 $B
run a100_8800f --n 100 --variant 8800 --fuse-p 1 $B
run d7 --n 256 --stencil 7 $B
run a7_8707 --n 256 --stencil 7 --variant 8707 $B
run a7_8707f --n 256 --stencil 7 --variant 8707 --fuse-p 1 $B
