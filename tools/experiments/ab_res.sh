export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for mb in 0 64 128 160 192 224 0; do run --n 100 --variant 2200 --resident-mb $mb --steps 10; done
run --n 100 --variant 2300 --steps 10
for mb in 0 96 160 224 0 160; do run --variant 2200 --resident-mb $mb --steps 10; done
