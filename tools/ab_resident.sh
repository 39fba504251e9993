# Round-robin A/B of the launch forms at 100^3 (option resident_update 0 = the
# unit + update-block launch, 1 = the per-iteration resident k_spmv_ar, -1 =
# auto: the persistent k_cg_persist), fresh process per line.
export TMPDIR=/tmp; mkdir -p gpurun_out/abr; : > gpurun_out/abr/summary.log
for rep in $(seq ${REPS:-2}); do
  for v in ${SHAPES:-0 1 -1}; do
    timeout -k 10 200 python bench.py --n ${N:-100} --no-cpu-baseline --no-trace-check --no-host-boundary --no-secondary --steps ${STEPS:-10} \
        --set resident_update=$v > gpurun_out/abr/one.json 2>> gpurun_out/abr/err.log || exit 1
    python3 -c "
import json; d = json.load(open('gpurun_out/abr/one.json'))
print('shape $v', d['value'], d['roofline']['avg_launch_us'], d['config']['options'].get('resident_update'))" >> gpurun_out/abr/summary.log
  done
done
cat gpurun_out/abr/summary.log
