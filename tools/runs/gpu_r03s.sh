set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread -k "sharded or integration or c4 or sparse or dedup or sort or adagrad or train_step or inbatch or xent" > gpurun_out/t_r03s.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03s.log | tail -12; tail -1 gpurun_out/t_r03s.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03s.log; exit $rc; }
for m in chunk region; do echo "== sort $m"; TT_SPARSE_SORT=$m timeout -k 10 120 python -u tools/time_sort.py || exit 1; done
bash tools/gpu_step_ab.sh 2 new:-: sep:TT_INBATCH_COMBINE=separate: region:TT_SPARSE_SORT=region:
