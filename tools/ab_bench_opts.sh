# Process-level A/B of bench.py option sets (each run a fresh process, so the
# per-process placement spread averages out over REPS rounds, A B A B ...).
# Usage: BENCH_ARGS="--n 100" A="" B="--x-ring 8" REPS=4 bash tools/ab_bench_opts.sh
export TMPDIR=/tmp; mkdir -p gpurun_out/abo; : > gpurun_out/abo/summary.log
for rep in $(seq ${REPS:-4}); do
  for which in A B; do
    if [ $which = A ]; then OPTS="$A"; else OPTS="$B"; fi
    timeout -k 10 200 python bench.py $BENCH_ARGS $OPTS --no-cpu-baseline --no-trace-check --no-host-boundary --steps ${STEPS:-10} > gpurun_out/abo/one.json 2>> gpurun_out/abo/err.log || exit 1
    python3 -c "
import json; d = json.load(open('gpurun_out/abo/one.json'))
print('$which', d['value'], d['roofline']['avg_launch_us'], d['update_kernel_avg_us'])" >> gpurun_out/abo/summary.log
  done
done
cat gpurun_out/abo/summary.log
