set -o pipefail
mkdir -p gpurun_out
TT_SPARSE_INLINE=1 timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r03j.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03j.log | tail -12; tail -1 gpurun_out/t_r03j.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03j.log; exit $rc; }
TT_SPARSE_INLINE=1 bash tools/gpu_trace_step.sh j > /dev/null; sed -n '/combine_cols/,$p' gpurun_out/trace_j/timeline.txt | cut -c1-90; grep -o '"ms_per_step[^,]*' gpurun_out/trace_j/line.json
bash tools/gpu_step_ab.sh 3 inline:TT_SPARSE_INLINE=1: after:TT_SPARSE_INLINE=0:
