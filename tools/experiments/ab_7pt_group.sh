#!/bin/bash
# 7-pt 256^3: group windows (pair / quad, p fused in the staging) vs SELL-512-A direct (8707).
export TMPDIR=/tmp
O=gpurun_out/g7; mkdir -p $O
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --n 256 --stencil 7 "$@" > $O/$tag.json 2>$O/$tag.err
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
  run d_$r $B
  for v in 8963 8962 8983; do run v${v}_$r --variant $v $B; done
done
