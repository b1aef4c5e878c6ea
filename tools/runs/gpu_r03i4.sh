set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r03i4.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03i4.log | tail -12; tail -1 gpurun_out/t_r03i4.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03i4.log; exit $rc; }
bash tools/gpu_trace_step.sh i4 > /dev/null; sed -n 1,12p gpurun_out/trace_i4/timeline.txt; grep -E "block_sum|join|gather" gpurun_out/trace_i4/timeline.txt; grep -o '"ms_per_step[^,]*' gpurun_out/trace_i4/line.json
