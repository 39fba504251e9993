#!/bin/bash
# Round evidence in one GPU call: rocprofv3 kernel stats + FETCH/WRITE passes
# for the three single-GPU configs (tools/gpu_profile.sh), then the default
# bench lines with the CPU baseline. Stops at the first fatal step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
N=200 bash tools/gpu_profile.sh || exit $?
N=100 bash tools/gpu_profile.sh || exit $?
N=256 STENCIL=7 bash tools/gpu_profile.sh || exit $?
bash tools/final_bench.sh
