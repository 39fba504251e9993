export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/pre.jsonl
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/pre_one.log 2>&1 || exit $?; echo "$* $(tail -n1 gpurun_out/pre_one.log)" >> gpurun_out/pre.jsonl; }
for i in 1 2; do for c in 8 32 128 499; do run --n 100 --graph-chunk $c --steps 10; done; done
for c in 8 64; do run --graph-chunk $c --steps 10; done
