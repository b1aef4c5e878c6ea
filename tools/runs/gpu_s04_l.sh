# Round 4: index tests after the big-k list target, then the full bench (runner point with 256 checked rows, e2e recall leg).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "bruteforce or index or c4 or topk or retriever or export or recall" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); i=d['index']
print('value', d['value'], 'ms', d['ms_per_step'])
print('index', {k: i[k] for k in ('qps','seconds','exact_match_rows','checked_rows')})
print('runner', {k: i['runner_point'][k] for k in ('ms_per_batch','qps','exact_match_rows','checked_rows')})
print('e2e', i['runner_recall_e2e'])
"
