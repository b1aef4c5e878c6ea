# Round 4: scan running threshold (levels) + branch-free flush stores: index tests, probe A/B, stats.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04j; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py tests/test_pipeline_gpu.py -q -k "bruteforce or index or c4 or topk or retriever or export" --timeout 300 --timeout-method thread -rf > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $OUT/tests.log | head -40; exit 1; }
tail -1 $OUT/tests.log
for v in stats oldstats; do echo "== $v"; timeout -k 10 60 ./tools/pbin/probe_$v 131072 | tail -3; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in base nolv old; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v$rep -o t -- ./tools/pbin/probe_$v 131072 > $OUT/$v$rep.log 2>&1
  echo "== $v $(grep nq= $OUT/$v$rep.log | tail -1)"
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$OUT/$v$rep/*kernel_stats.csv')[0])):
  if 'scan' in r['Name'] or 'finalize' in r['Name'] or 'sample' in r['Name']: print('   ', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -f $OUT/$v$rep/*kernel_trace.csv
done
done
timeout -k 10 120 python -u tools/time_index.py 1000000 100 3
timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
bash tools/gpu_trace_step.sh s04
