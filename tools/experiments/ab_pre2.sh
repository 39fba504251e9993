export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for i in 1 2; do for v in 4200 4202 4206 4208 4000; do run --variant $v --steps 10; done; done
for v in 4200 4206; do run --n 100 --variant $v --steps 10; done
