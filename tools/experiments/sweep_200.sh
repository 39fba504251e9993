#!/bin/bash
# 200^3 with the pair-window SpMV: ring, fold, update shape, order, residency.
export TMPDIR=/tmp
O=gpurun_out/s200; mkdir -p $O
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-secondary "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -n 5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d['config']['options']
print(f"{sys.argv[2]:>10} {d['value']:8.1f} it/s spmv {d['roofline']['avg_launch_us']:6.2f} upd {d['update_kernel_avg_us']} fold {o['fold']} um {o['update_slices']} ring {o['x_ring']} rev {o['rev_update']} res {o['resident_mb']}")
PY
}
for r in 1 2; do
  run d_$r
  run r16_$r --x-ring 16
  run r64_$r --x-ring 64
  run f1u4_$r --fold 1 --update-slices 4
  run rev0_$r --rev-update 0
  run res128_$r --resident-mb 128
  run g32_$r --graph-chunk 32
done
