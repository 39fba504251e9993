# the GPU suite once with every device buffer fenced by
# canaries (HPCCG_CANARY=1, checked after every solve), then the round-3
# contiguous-candidate placement probe once under the same canaries, with the
# diagnostics variant of the library (-DHPCCG_DIAG_CONTIG: the only build with
# a path to physically contiguous memory):
#   bash tools/build_variant.sh contig -DHPCCG_DIAG_CONTIG   (on the CPU side)
#   gpurun -- bash tools/canary_run.sh
# Stops at the first step that faults, aborts or times out.
mkdir -p gpurun_out/canary
export HPCCG_CANARY=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/canary/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> gpurun_out/canary/suite.log
tail -5 gpurun_out/canary/suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
HPCCG_HIP_LIB=lib_contig/libhpccg_hip.so HPCCG_PROBE_ALLOC=4 timeout -k 10 600 python -u tools/diag_carry.py 1 \
    > gpurun_out/canary/contig_probe.log 2>&1
rc2=$?
echo "probe rc=$rc2" >> gpurun_out/canary/contig_probe.log
tail -30 gpurun_out/canary/contig_probe.log
exit $rc2
