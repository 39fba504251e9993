#!/bin/bash
# SELL-512-A pair windows (two slices per block) vs the defaults.
export TMPDIR=/tmp
O=gpurun_out/pair; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants_agree or fusion_options or sell_a or variants_bitwise" > $O/pytest.log 2>&1
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
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']} fuse {d['config']['options']['fuse_p']}")
PY
}
B="--steps 3 --warmup 1 --no-secondary"
for r in 1 2; do
  run d200_$r $B
  run p200_8960_$r --variant 8960 $B
  run p200_8962_$r --variant 8962 $B
done
run d100 --n 100 $B
run p100_8970 --n 100 --variant 8970 $B
run p100_8960 --n 100 --variant 8960 $B
