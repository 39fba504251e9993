# Default bench lines (with the CPU baseline) for the three single-GPU configs.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/fb200.log 2> gpurun_out/fb200.err &&
timeout -k 10 300 python bench.py --n 100 > gpurun_out/fb100.log 2> gpurun_out/fb100.err &&
timeout -k 10 400 python bench.py --n 256 --stencil 7 > gpurun_out/fb7.log 2> gpurun_out/fb7.err
