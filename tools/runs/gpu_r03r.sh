set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_kernels_gpu.py tests/test_configs_gpu.py -x -v --timeout 200 --timeout-method thread -k "sharded or rccl or global or integration or bruteforce or c4 or index or topk" > gpurun_out/t_r03r.log 2>&1; rc=$?
grep -E "FAIL|Error" gpurun_out/t_r03r.log | tail -12; tail -1 gpurun_out/t_r03r.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03r.log; exit $rc; }
for n in iprobe8_base iprobe9_base; do echo "== $n"; timeout -k 10 60 ./tools/pbin/$n 131072 | tail -2 | head -1 || exit 1; done
bash tools/gpu_step_ab.sh 2 blas:TT_WGRAD=blas: tt:TT_WGRAD=tt:
MATCH=mlp_wgrad bash tools/gpu_pmc_py.sh wg tools/time_mlp.py
