set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -x -v --timeout 200 --timeout-method thread -k "inbatch or xent or train_step or wgrad or c3 or c2" > gpurun_out/t_r03v.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03v.log | tail -12; tail -1 gpurun_out/t_r03v.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03v.log; exit $rc; }
bash tools/gpu_step_ab.sh 3 blas:TT_WGRAD=blas: tt:TT_WGRAD=tt: tt512:TT_WGRAD=tt,TT_WGRAD_WGS=512:
