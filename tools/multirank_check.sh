#!/bin/bash
# Multi-rank path on one GPU: the group / RCCL / guard tests, then the
# in-process group and the emulated RCCL rank against single-rank solves.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mr
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "group or rccl or guard or fuzz" > gpurun_out/mr/pytest.log 2>&1 || { tail -40 gpurun_out/mr/pytest.log; exit 1; }
tail -2 gpurun_out/mr/pytest.log
for n in 100 200; do
  timeout -k 10 300 python tools/group_bench.py --n $n --P 2 --variants 1:0 > gpurun_out/mr/group$n.log 2>&1 \
      || { tail -20 gpurun_out/mr/group$n.log; exit 1; }
  cat gpurun_out/mr/group$n.log
done
timeout -k 10 300 python tools/group_bench.py --n 256 --7pt --P 2 --variants 1:0 > gpurun_out/mr/group7.log 2>&1 \
    || { tail -20 gpurun_out/mr/group7.log; exit 1; }
cat gpurun_out/mr/group7.log
timeout -k 10 300 python tools/comm_bench.py --n 100 --variants 0:0:1,1:0:1,2:0:1 > gpurun_out/mr/comm100.log 2>&1 \
    || { tail -20 gpurun_out/mr/comm100.log; exit 1; }
cat gpurun_out/mr/comm100.log
