set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bruteforce or c4 or index" 2>&1 | tail -3
VARIANTS="stats nowait noins nofilt nosync" bash tools/gpu_probe2.sh
timeout -k 10 120 python -u tools/time_index.py 1000000 100 2 2>&1 | grep -v amdgpu.ids
