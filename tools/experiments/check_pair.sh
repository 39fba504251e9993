#!/bin/bash
# Full GPU suite with the pair-window default, then the 200^3 evidence
# (rocprofv3 stats + FETCH/WRITE passes) and the default bench line with the
# CPU baseline; stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pt.log
case $rc in 0) ;; *) exit $rc;; esac
N=200 bash tools/gpu_profile.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/fb200.log 2> gpurun_out/fb200.err || exit $?
for i in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-secondary --variant 8236 > gpurun_out/c8236_$i.log 2>&1 || exit $?; timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-secondary > gpurun_out/c8963_$i.log 2>&1 || exit $?; done
