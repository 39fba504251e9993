#!/bin/bash
# Multi-rank evidence on one GPU for the round: the emulated RCCL rank
# (force_comm 1: scalars through RCCL; 2: also the r-halo as a self
# send/recv) and the peer-memory all-reduce against the single-rank solve, at
# 100^3, 200^3 and 7-pt 256^3; then the in-process two-rank group. Output:
# gpurun_out/mrev/*.log (copied to profiles/r03_multirank by hand).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mrev
V="0:0:1,1:0:1,2:0:1:-1:1:0:0,2:0:1:-1:1:0:-1,2:0:1:-1:1:-1:1,2:0:1:-1:1:-1:-1,2:0:1:-1:1:-1:3,0:0:1"
for cfg in "--n 100" "--n 200" "--n 256 --7pt"; do
  tag=$(echo "$cfg" | tr -d ' -' )
  timeout -k 10 300 python tools/comm_bench.py $cfg --variants $V > gpurun_out/mrev/comm_$tag.log 2>&1 \
      || { tail -20 gpurun_out/mrev/comm_$tag.log; exit 1; }
  grep '^{' gpurun_out/mrev/comm_$tag.log
done
for cfg in "--n 100" "--n 200" "--n 256 --7pt"; do
  tag=$(echo "$cfg" | tr -d ' -' )
  timeout -k 10 300 python tools/group_bench.py $cfg --P 2 --variants 1:0 > gpurun_out/mrev/group_$tag.log 2>&1 \
      || { tail -20 gpurun_out/mrev/group_$tag.log; exit 1; }
  grep '^{' gpurun_out/mrev/group_$tag.log
done
