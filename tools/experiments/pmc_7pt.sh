#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of the 7-pt 256^3 SELL-512-A
# SpMV with the p update separate and formed per load.
export TMPDIR=/tmp
O=gpurun_out/pmc7; rm -rf $O; mkdir -p $O
for f in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/f${f}_$c -- python tools/pmc_workload.py --n 256 --stencil 7 --variant 8707 --fuse-p $f > $O/f${f}_$c.log 2>&1
    rc=$?; echo "fuse $f $c rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
