export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q200.log 2>&1 &&
timeout -k 10 300 python bench.py --n 100 --no-cpu-baseline > gpurun_out/q100.log 2>&1 &&
timeout -k 10 300 python bench.py --n 256 --stencil 7 --steps 3 --no-cpu-baseline > gpurun_out/q7.log 2>&1
