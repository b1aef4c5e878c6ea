set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "wgrad" > gpurun_out/t_r03p_wg.log 2>&1 || { tail -20 gpurun_out/t_r03p_wg.log; exit 1; }
tail -1 gpurun_out/t_r03p_wg.log
timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "wgrad tt"
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -x -v -s --timeout 280 --timeout-method thread -k train_steps > gpurun_out/t_r03p_cfg.log 2>&1; rc=$?
grep -E "PASS|FAIL|\{" gpurun_out/t_r03p_cfg.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh r03p tests bench
