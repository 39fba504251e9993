#!/bin/bash
# 100^3 (launch- and latency-bound): dot completion, update shape, ring and
# graph chunk options around the SELL-512-A default.
export TMPDIR=/tmp
O=gpurun_out/s100; mkdir -p $O
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline --n 100 --steps 5 --warmup 1 --no-secondary "$@" > $O/$tag.json 2>$O/$tag.err
  local rc=$?
  case $rc in 0) ;; *) echo "$tag rc=$rc"; tail -n 5 $O/$tag.err; exit $rc;; esac
  python - "$O/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
o = d['config']['options']
print(f"{sys.argv[2]:>12} {d['value']:9.1f} it/s spmv {d['roofline']['avg_launch_us']:6.2f} upd {d['update_kernel_avg_us']} fold {o['fold']} um {o['update_slices']} ring {o['x_ring']} med {d['solve_ms']['median_graph_replay']}")
PY
}
run d1
run f1u4 --fold 1 --update-slices 4
run f1u8 --fold 1 --update-slices 8
run f3u4 --fold 3 --update-slices 4
run f0 --fold 0
run r16 --x-ring 16
run r32 --x-ring 32
run g64 --graph-chunk 64
run g499 --graph-chunk 499
run red --redund 1
run d2
