export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for mb in 64 128 160 192 256 128 192; do run --n 100 --resident-mb $mb --steps 10; done
for f in 0 2; do run --n 100 --fold $f --steps 10; done
