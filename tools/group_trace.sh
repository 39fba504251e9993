#!/bin/bash
# Kernel + copy timeline of the in-process group (tools/group_bench.py) for
# one use_graph:fold variant per pass; read with tools/trace_gaps.py.
set -u
export TMPDIR=/tmp
N=${N:-100}
for v in ${VARIANTS:-0:1 0:0 1:0}; do
    tag=${v/:/_}
    OUT=gpurun_out/gtrace_${N}_$tag
    rm -rf $OUT; mkdir -p $OUT
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -- \
        python tools/group_bench.py --n $N --P 2 --steps 1 --max-iter ${MAXIT:-20} --variants $v --no-single \
        > $OUT/run.log 2>&1
    rc=$?
    echo "$v rc=$rc"
    case $rc in 0) ;; *) tail -20 $OUT/run.log; exit $rc;; esac
done
