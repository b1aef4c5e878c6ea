# Round 4: scan4 (one wave per SIMD, 4 query sets per wave) vs scan v1: index tests, timing A/B, rocprof.
set -e
mkdir -p gpurun_out/s04f
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_distributed_gpu.py -q -k "bruteforce or index or c4" --timeout 300 --timeout-method thread -rf > gpurun_out/s04f/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" gpurun_out/s04f/tests.log | head -40; exit 1; }
tail -2 gpurun_out/s04f/tests.log
for rep in 1 2; do
for v in new v1; do
  if [ $v = v1 ]; then export TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/v1/libtt.so; else unset TT_LIB_PATH; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/time_index.py 1000000 100 3
  timeout -k 10 120 python -u tools/time_index.py 2048 1000 10
done
done
unset TT_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s04f/prof -o run -- python3 tools/time_index.py 262144 100 3 > gpurun_out/s04f/prof.log 2>&1
f=$(find gpurun_out/s04f/prof -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
