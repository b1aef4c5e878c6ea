set -e
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "global or sharded" 2>&1 | tail -15
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-index --steps 30 --warmup 5 --train-mode sharded > gpurun_out/bench_sh.json 2> gpurun_out/bench_sh.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_sh.json')); print(d['value'], d['ms_per_step'], d['scaling'], d['config'])"
