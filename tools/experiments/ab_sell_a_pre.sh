#!/bin/bash
# SELL-512-A with the value slots and offsets loaded before the run test.
export TMPDIR=/tmp
O=gpurun_out/sap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants_agree or sell_a" > $O/pytest.log 2>&1
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
print(f"{sys.argv[2]:>14} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:8.2f} us frac {d['roofline']['frac']} upd {d['update_kernel_avg_us']} variant {d['config']['spmv_variant']} fuse {d['config']['options']['fuse_p']}")
PY
}
B="--steps 3 --warmup 1 --no-secondary"
S7="--n 256 --stencil 7"
run d7 $S7 $B
run p7_8717f $S7 --variant 8717 $B
run p7_8717 $S7 --variant 8717 --fuse-p 0 $B
run p7_8817f $S7 --variant 8817 $B
run d7b $S7 $B
run d100 --n 100 $B
for v in 8837 8857 8737; do run p100_$v --n 100 --variant $v $B; done
run d100b --n 100 $B
