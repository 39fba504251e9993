export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt.log 2>&1 || exit $?
for v in 2200 4200 2200 4200; do run --variant $v --steps 10; done
for v in 2200 4200 4300; do run --n 100 --variant $v --steps 10; done
for v in 1000 3000 3100 1000 3000; do run --n 256 --stencil 7 --steps 3 --variant $v; done
run --n 256 --stencil 7 --steps 3 --variant 3000 --fuse-p 1
