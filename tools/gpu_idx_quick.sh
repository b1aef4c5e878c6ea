set -e
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bruteforce or c4 or index or sharded" 2>&1 | tail -15
timeout -k 10 120 python -u tools/time_index.py 1000000 100 2 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --index-mode sharded > gpurun_out/bench_sh.json 2> gpurun_out/bench_sh.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_sh.json')); print(json.dumps(d['index'])[:900])"
