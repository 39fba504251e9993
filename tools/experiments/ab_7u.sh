export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pt.log 2>&1 || exit $?
for i in 1 2; do for v in 3000 3007; do run --n 256 --stencil 7 --steps 3 --variant $v; done; done
