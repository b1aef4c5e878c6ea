# Round 4: finalize with NW waves per query (TT_FINAL_WAVES 1/2/4): index tests per group size, timing.
set -e
mkdir -p gpurun_out/s04h
for nw in 4 2 0; do
  TT_FINAL_WAVES=$nw timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "bruteforce or index or c4 or topk or retriever or export" --timeout 300 --timeout-method thread -rf > gpurun_out/s04h/tests_$nw.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/s04h/tests_$nw.log | head -40; exit 1; }
  echo "nw=$nw $(tail -1 gpurun_out/s04h/tests_$nw.log)"
done
for nw in 1 2 4; do
  echo "== NW=$nw"
  TT_FINAL_WAVES=$nw timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
  TT_FINAL_WAVES=$nw timeout -k 10 120 python -u tools/time_index.py 2048 100 10
  TT_FINAL_WAVES=$nw timeout -k 10 120 python -u tools/time_index.py 262144 100 3
done
for lf in 2304 3200 4096; do
  echo "== NW=4 LF=$lf"; TT_FINAL_WAVES=4 TT_FINAL_LF=$lf timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
done
