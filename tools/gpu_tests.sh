set -o pipefail
mkdir -p gpurun_out/t1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t1/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/t1/smoke.log; exit 1; }
tail -2 gpurun_out/t1/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t1/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/t1/pytest.log
exit $rc
