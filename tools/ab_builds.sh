# Process-level A/B of the working-tree library against lib_base/ (see
# tools/build_base.sh): bench lines alternating A B A B ..., $REPS rounds.
# Usage: BENCH_ARGS="--n 100" REPS=3 bash tools/ab_builds.sh
export TMPDIR=/tmp; mkdir -p gpurun_out/abb; : > gpurun_out/abb/summary.log
for rep in $(seq ${REPS:-3}); do
  for which in new base; do
    if [ $which = base ]; then export HPCCG_HIP_LIB=$PWD/lib_base/libhpccg_hip.so; else unset HPCCG_HIP_LIB; fi
    timeout -k 10 200 python bench.py $BENCH_ARGS --no-cpu-baseline --no-trace-check --steps ${STEPS:-10} > gpurun_out/abb/one.json 2>> gpurun_out/abb/err.log || exit 1
    python3 -c "
import json; d = json.load(open('gpurun_out/abb/one.json'))
print('$which', d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" >> gpurun_out/abb/summary.log
  done
done
cat gpurun_out/abb/summary.log
