set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -x -v -s --timeout 280 --timeout-method thread -k train_steps > gpurun_out/t_r03o_cfg.log 2>&1; rc=$?
grep -E "PASS|FAIL|\{" gpurun_out/t_r03o_cfg.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh r03o tests bench
