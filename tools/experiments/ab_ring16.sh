#!/bin/bash
# x_ring 16 vs the auto 32 at 200^3 (pair windows) and 7-pt 256^3.
export TMPDIR=/tmp
O=gpurun_out/ring16; mkdir -p $O
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-secondary "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -n 5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d['config']['options']
print(f"{sys.argv[2]:>10} {d['value']:8.1f} it/s spmv {d['roofline']['avg_launch_us']:6.2f} upd {d['update_kernel_avg_us']} ring {o['x_ring']}")
PY
}
for r in 1 2 3 4; do run d_$r; run r16_$r --x-ring 16; run r24_$r --x-ring 24; done
for r in 1 2 3; do run d7_$r --n 256 --stencil 7; run r7_16_$r --n 256 --stencil 7 --x-ring 16; done
