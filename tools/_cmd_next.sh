mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests2.log 2>&1; echo rc=$? >> gpurun_out/gpu_tests2.log
LIBS="prev" CFGS="--n 100|--n 200|--n 256 --stencil 7" REPS=3 STEPS=10 bash tools/ab_libs.sh > gpurun_out/ab_rec.log 2>&1
