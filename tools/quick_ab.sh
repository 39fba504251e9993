# Quick A/B after a kernel change: targeted parity tests, then bench lines
# (no CPU baseline) for the three configs with fold 2 (default) vs fold 1,
# then the in-process group overhead at P=2. Stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "agree or fusion or folded or solve_vs or reproducible" > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
for cfg in "--n 100" "--n 200" "--n 256 --stencil 7"; do
  for fold in 2 1; do
    timeout -k 10 200 python bench.py $cfg --fold $fold --no-cpu-baseline >> gpurun_out/ab/bench.log 2>> gpurun_out/ab/bench.err || exit 1
  done
done
timeout -k 10 300 python tools/group_bench.py --n 200 --P 2 > gpurun_out/ab/group200.log 2>&1 || { tail -20 gpurun_out/ab/group200.log; exit 1; }
timeout -k 10 300 python tools/group_bench.py --n 100 --P 2 > gpurun_out/ab/group100.log 2>&1 || { tail -20 gpurun_out/ab/group100.log; exit 1; }
cat gpurun_out/ab/group200.log gpurun_out/ab/group100.log
