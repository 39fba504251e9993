export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 100 200; do for f in 0 1 2 3; do
timeout -k 10 300 python bench.py --n $n --fold $f --no-cpu-baseline > gpurun_out/f_${n}_${f}.log 2>&1 || exit $?
done; done
