export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for i in 1 2 3; do for v in 2000 2200 2208; do run --variant $v --steps 10; done; done
for i in 1 2; do for v in 2100 2300 2000 2200; do run --n 100 --variant $v --steps 10; done; done
