#!/bin/bash
# Process-level A/B of several library builds: "new" (the working tree) and
# lib_<name>/ directories (tools/build_base.sh, or patched copies), bench lines
# round-robin. Usage: LIBS="base noguard" CFGS="--n 100|--n 256 --stencil 7"
#                     REPS=5 bash tools/ab_libs.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
: > gpurun_out/abl/ab.log
IFS='|' read -ra cfgs <<< "${CFGS:---n 100}"
for cfg in "${cfgs[@]}"; do
  for rep in $(seq ${REPS:-3}); do
    for which in new ${LIBS:-base}; do
      if [ $which = new ]; then unset HPCCG_HIP_LIB; else export HPCCG_HIP_LIB=$PWD/lib_$which/libhpccg_hip.so; fi
      timeout -k 10 200 python bench.py $cfg --no-cpu-baseline --no-trace-check --no-host-boundary --steps ${STEPS:-10} $EXTRA > gpurun_out/abl/one.json \
          2>> gpurun_out/abl/err.log || { tail -20 gpurun_out/abl/err.log; exit 1; }
      python3 -c "
import json; d = json.load(open('gpurun_out/abl/one.json'))
print('$cfg', '$which', d['value'], d['roofline']['avg_launch_us'], d.get('update_kernel_avg_us'))" | tee -a gpurun_out/abl/ab.log
    done
  done
done
