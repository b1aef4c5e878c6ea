set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread -k "sparse or sort or dedup or adagrad or adam or train_step or c3 or c2 or scatter or c5" > gpurun_out/t_r03i2.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03i2.log | tail -12; tail -1 gpurun_out/t_r03i2.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03i2.log; exit $rc; }
bash tools/gpu_trace_step.sh i2 > /dev/null; grep -E "block_sum|join|gather" gpurun_out/trace_i2/timeline.txt; grep -o '"ms_per_step[^,]*' gpurun_out/trace_i2/line.json
