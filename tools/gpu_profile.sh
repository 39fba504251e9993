#!/bin/bash
# rocprofv3 evidence for the round: kernel-trace stats of the default bench
# command (its JSON line lands in $OUT/stats.log),
# then FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM
# section) over the SpMV and the known-bytes streaming kernel used to
# calibrate them. Stops at the first crash/timeout; no retries.
set -u
export TMPDIR=/tmp
N=${N:-200}
OUT=gpurun_out/prof_$N${STENCIL:+_$STENCIL}
rm -rf $OUT; mkdir -p $OUT
step() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name rc=$rc"
    case $rc in 124|134|137|139) echo "fatal in $name, stopping"; exit $rc;; esac
    return 0
}

S=${STENCIL:-27}
# the committed bench line comes from this same process (same allocations as
# the kernel stats: the per-process placement spread, DESIGN.md 4, cannot
# separate the two), CPU baseline included
# (the headline config's line carries the secondary configs, as the driver's does)
SEC=""; [ "$N" = 200 ] && [ "$S" = 27 ] || SEC="--no-secondary"
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -- python bench.py --n $N --stencil $S $SEC
step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python tools/pmc_workload.py --n $N --stencil $S
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python tools/pmc_workload.py --n $N --stencil $S
find $OUT -name "*.csv" | head -20
