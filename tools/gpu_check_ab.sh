#!/bin/bash
# One GPU call after a kernel change: the guard tests, the whole -m gpu suite,
# then a process-level A/B of the working tree against lib_base/
# (tools/build_base.sh) on the three single-GPU configs. Stops at the first
# failure. Usage: REPS=3 bash tools/gpu_check_ab.sh [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/chk
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/chk/guard.log 2>&1 || { tail -40 gpurun_out/chk/guard.log; exit 1; }
tail -3 gpurun_out/chk/guard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${1:+-k "$1"} \
    > gpurun_out/chk/pytest.log 2>&1 || { tail -40 gpurun_out/chk/pytest.log; exit 1; }
tail -2 gpurun_out/chk/pytest.log
[ -n "$NO_AB" ] && exit 0
: > gpurun_out/chk/ab.log
for cfg in "--n 200" "--n 100" "--n 256 --stencil 7"; do
  for rep in $(seq ${REPS:-3}); do
    for which in new base; do
      if [ $which = base ]; then export HPCCG_HIP_LIB=$PWD/lib_base/libhpccg_hip.so; else unset HPCCG_HIP_LIB; fi
      timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --no-trace-check --steps ${STEPS:-10} > gpurun_out/chk/one.json \
          2>> gpurun_out/chk/err.log || { tail -20 gpurun_out/chk/err.log; exit 1; }
      python3 -c "
import json; d = json.load(open('gpurun_out/chk/one.json'))
print('$cfg', '$which', d['value'], d['roofline']['avg_launch_us'])" | tee -a gpurun_out/chk/ab.log
    done
  done
done
