set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r03e4.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03e4.log | tail -12; tail -1 gpurun_out/t_r03e4.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03e4.log; exit $rc; }
bash tools/gpu_trace_step.sh e4 > /dev/null; sed -n '/inbatch_pass_kernel<128, 1>/,$p' gpurun_out/trace_e4/timeline.txt; grep -o '"ms_per_step[^,]*' gpurun_out/trace_e4/line.json
bash tools/gpu_step_ab.sh 3 early:-: late:TT_SPARSE_EARLY=0:
