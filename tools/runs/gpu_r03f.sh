set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r03f.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03f.log | tail -12; tail -1 gpurun_out/t_r03f.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03f.log; exit $rc; }
bash tools/gpu_sharded_ab.sh
bash tools/profile_round.sh r03a
