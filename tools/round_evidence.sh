#!/bin/bash
# Round evidence in one GPU call: for the three single-GPU configs, the
# default bench line (CPU baseline included) under rocprofv3 kernel stats,
# then the FETCH/WRITE passes (tools/gpu_profile.sh). Stops at the first fatal
# step. Summaries: tools/pmc_summary.py gpurun_out/prof_<n> <tag> <n>
# gpurun_out/prof_<n>/stats.log <stencil>.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
N=200 bash tools/gpu_profile.sh || exit $?
N=100 bash tools/gpu_profile.sh || exit $?
N=256 STENCIL=7 bash tools/gpu_profile.sh || exit $?
