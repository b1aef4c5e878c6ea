# Round 4: scan with staggered waves 4-7 (filter-first halves) vs lockstep; early
# backward (query tower beside the cols pass) vs after; MFMA calibration.
set -e
mkdir -p gpurun_out/s04g
timeout -k 10 60 ./tools/pbin/mfma_peak
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -q -k "bruteforce or index or c4 or train_step or fit or graph or early" --timeout 300 --timeout-method thread -rf > gpurun_out/s04g/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/s04g/tests.log | head -40; exit 1; }
tail -1 gpurun_out/s04g/tests.log
for rep in 1 2; do
for v in stag lock; do
  if [ $v = lock ]; then export TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/v1/libtt.so; else unset TT_LIB_PATH; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/time_index.py 1000000 100 3
  timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
done
done
unset TT_LIB_PATH
bash tools/gpu_step_ab.sh 3 early:TT_EARLY_BACKWARD=1: late:TT_EARLY_BACKWARD=0:
