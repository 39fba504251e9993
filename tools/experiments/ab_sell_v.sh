#!/bin/bash
# SELL-512-V / -V4 kernels against SELL-512-C in the CG bench (200^3, 100^3, 7-pt 256^3).
export TMPDIR=/tmp
O=gpurun_out/v1; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log
run() {  # run <args> <variants...>
 local a=$1; shift
 for v in "$@"; do
  timeout -k 10 200 python bench.py $a --steps 3 --warmup 1 --no-cpu-baseline --variant $v > $O/b.json 2>$O/b.err; rc=$?
  echo "$a v=$v rc=$rc $(python -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['roofline']['avg_launch_us'], d['check']['x_minus_xexact_inf'], d['config']['options'])" 2>&1 | tail -1)"
  case $rc in 124|134|137|139) exit $rc;; esac
 done
}
for o in "--resident-mb 0" "--resident-mb 256" "--resident-mb 1000" "--fold 1" "--fold 2" "--fold 3" "--redund 1"; do
 run "--n 200 $o" 7201
done
for o in "--resident-mb 0" "--resident-mb 256" "--resident-mb 1000" "--fold 1" "--fold 0" "--fold 3"; do
 run "--n 256 --stencil 7 $o" 7201
done
