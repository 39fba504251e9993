mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_direct_pairs.py > gpurun_out/dp_tests.log 2>&1; echo rc=$? >> gpurun_out/dp_tests.log
for v in 2 1 2 1; do timeout -k 10 200 python bench.py --n 100 --no-cpu-baseline --steps 20 --set direct_spu=$v > gpurun_out/dp_$v.json 2>/dev/null; python3 -c "import json;d=json.load(open('gpurun_out/dp_$v.json'));print('spu $v', d['value'], d['roofline']['avg_launch_us'])" >> gpurun_out/dp_ab.log; done
