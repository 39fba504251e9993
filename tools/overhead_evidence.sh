# Multi-rank overhead evidence on one GPU: the RCCL rank path emulated with a
# 1-rank communicator (tools/comm_bench.py) and the in-process group
# (tools/group_bench.py), 200^3 and 100^3. Stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out/ovh
timeout -k 10 300 python tools/comm_bench.py --n 200 > gpurun_out/ovh/comm200.log 2>&1 &&
timeout -k 10 200 python tools/comm_bench.py --n 100 > gpurun_out/ovh/comm100.log 2>&1 &&
timeout -k 10 300 python tools/group_bench.py --n 200 --P 2 --variants 1:0,0:0,0:1 > gpurun_out/ovh/group200.log 2>&1 &&
timeout -k 10 200 python tools/group_bench.py --n 100 --P 2 --variants 1:0,0:0,0:1 > gpurun_out/ovh/group100.log 2>&1
