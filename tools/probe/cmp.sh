set -u
export TMPDIR=/tmp
O=gpurun_out/cmp; mkdir -p $O
timeout -k 10 120 ./tools/probe/spmv_probe 200 20 > $O/probe.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 120 ./tools/probe/spmv_probe 200 20 > $O/probe2.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_prof.json 2> $O/bench_prof.err || exit 4
