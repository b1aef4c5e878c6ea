set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread -k "inbatch or xent or train_step or sort or sparse or dedup" > gpurun_out/t_r03u.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03u.log | tail -12; tail -1 gpurun_out/t_r03u.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03u.log; exit $rc; }
for m in chunk region; do echo "== sort $m"; TT_SPARSE_SORT=$m timeout -k 10 120 python -u tools/time_sort.py | grep -E "1371981x1|132x2|5x1|all" || exit 1; done
bash tools/gpu_step_ab.sh 2 fused:-: sep:TT_INBATCH_COMBINE=separate: fused256:TT_INBATCH_WGS=256: sep256:TT_INBATCH_COMBINE=separate,TT_INBATCH_WGS=256: sepregion:TT_INBATCH_COMBINE=separate,TT_SPARSE_SORT=region:
