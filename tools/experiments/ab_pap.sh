#!/bin/bash
# p.Ap summed by every update workgroup (pap_in_update) vs folded in the SpMV.
export TMPDIR=/tmp
O=gpurun_out/pap; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fusion_options or tiny_and_thin or edge" > $O/pytest.log 2>&1
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
o = d['config']['options']
print(f"{sys.argv[2]:>12} {d['value']:9.1f} it/s spmv {d['roofline']['avg_launch_us']:6.2f} upd {d['update_kernel_avg_us']} pap {o['pap_in_update']} fold {o['fold']} med {d['solve_ms']['median_graph_replay']}")
PY
}
B="--n 100 --steps 5 --warmup 1 --no-secondary"
for r in 1 2 3; do
  run d_$r $B
  run p_$r --pap-in-update 1 $B
  run pf1_$r --pap-in-update 1 --fold 3 --update-slices 1 $B
done
