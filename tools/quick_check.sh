#!/bin/bash
# GPU parity tests, then the default bench lines (no CPU baseline) for the
# three single-GPU configs. Stops at the first failure; no retries.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q200.log 2> gpurun_out/q200.err &&
timeout -k 10 300 python bench.py --n 100 --no-cpu-baseline > gpurun_out/q100.log 2> gpurun_out/q100.err &&
timeout -k 10 300 python bench.py --n 256 --stencil 7 --steps 3 --no-cpu-baseline > gpurun_out/q7.log 2> gpurun_out/q7.err
