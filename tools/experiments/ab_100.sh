export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for i in 1 2; do run --n 100 --steps 10; done
run --n 100 --steps 10 --fold 0
run --steps 10
