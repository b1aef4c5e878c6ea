set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread -k "inbatch or xent or train_step" > gpurun_out/t_r03t.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03t.log | tail -12; tail -1 gpurun_out/t_r03t.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03t.log; exit $rc; }
bash tools/gpu_step_ab.sh 2 new:-: sep:TT_INBATCH_COMBINE=separate:
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03t -o sort -- python3 tools/time_sort.py > gpurun_out/prof_r03t_sort.log 2>&1 || exit 1
find gpurun_out/prof_r03t -name "*kernel_stats.csv" | head -3
