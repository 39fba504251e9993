set -o pipefail
mkdir -p gpurun_out/t5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_group.py -k "kernels_agree or fusion_options or group_kernel" > gpurun_out/t5/pytest.log 2>&1 || { tail -30 gpurun_out/t5/pytest.log; exit 1; }
tail -2 gpurun_out/t5/pytest.log
timeout -k 10 200 python tools/ab_inproc.py --n 256 --stencil 7 --variants "x_defer=1;x_defer=2" --reps 4 > gpurun_out/t5/ab7.log 2>&1 || { tail -20 gpurun_out/t5/ab7.log; exit 1; }
grep it_per_s gpurun_out/t5/ab7.log
timeout -k 10 200 python tools/ab_inproc.py --n 100 --variants "x_defer=1;x_defer=2;x_defer=2,x_ring=9;x_defer=2,x_ring=17" --reps 4 > gpurun_out/t5/ab100.log 2>&1 || { tail -20 gpurun_out/t5/ab100.log; exit 1; }
grep it_per_s gpurun_out/t5/ab100.log
