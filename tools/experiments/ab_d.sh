export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt.log 2>&1 || exit $?
for v in 1000 3000 3100 1000 3000; do run --n 256 --stencil 7 --steps 3 --variant $v; done
run --n 256 --stencil 7 --steps 3 --variant 3000 --fuse-p 1
timeout -k 10 300 python tools/spmv_sweep.py --n 256 --stencil 7 --variants 1000 3000 3001 3002 3100 0 > gpurun_out/sweep_d.log 2>&1
