# Same-box A/B of bench options: AB_CASES is a ;-separated list of
# "<bench args>" lines, each run twice in ABAB order (no CPU baseline).
# Prints value and SpMV/update launch averages per run.
export TMPDIR=/tmp; mkdir -p gpurun_out/abo; : > gpurun_out/abo/bench.log
IFS=';' read -ra CASES <<< "$AB_CASES"
for rep in 1 2; do
  for c in "${CASES[@]}"; do
    timeout -k 10 200 python bench.py $c --no-cpu-baseline --no-trace-check --no-host-boundary --steps ${STEPS:-10} > gpurun_out/abo/one.json 2>> gpurun_out/abo/bench.err || exit 1
    python3 - "$c" <<'PY' >> gpurun_out/abo/bench.log
import json, sys
d = json.load(open("gpurun_out/abo/one.json"))
print(f"{sys.argv[1]:<40s} {d['value']:10.1f} it/s  spmv {d['roofline']['avg_launch_us']:7.2f} us  update {d['update_kernel_avg_us']:6.2f} us")
PY
  done
done
cat gpurun_out/abo/bench.log
