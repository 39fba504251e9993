#!/bin/bash
# Round-end check: smoke(), then the default bench lines with the CPU baseline
# for 100^3 and 7-pt 256^3 (the PMC-traffic field reads the committed summaries).
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -n 20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --n 100 > gpurun_out/fb100.log 2> gpurun_out/fb100.err || exit $?
timeout -k 10 400 python bench.py --n 256 --stencil 7 --steps 3 > gpurun_out/fb7.log 2> gpurun_out/fb7.err || exit $?
timeout -k 10 400 python bench.py > gpurun_out/fb200b.log 2> gpurun_out/fb200b.err || exit $?
