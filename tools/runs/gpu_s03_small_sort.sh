# Finalize: one bitonic sort of small cuts (TT_FINAL_SMALL_SORT) vs select + sort; index parity tests.
set -e
mkdir -p gpurun_out/ss
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base ss base ss ssst; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ss/$v -o run -- ./tools/pbin/probe_$v 131072 > gpurun_out/ss/$v.log 2>&1
  f=$(find gpurun_out/ss/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v $(grep nq= gpurun_out/ss/$v.log | tail -1) | $(grep top5 gpurun_out/ss/$v.log) $(grep 'list entries' gpurun_out/ss/$v.log | tail -1)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'finalize' in n or 'fallback' in n: print('   ', n[:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  rm -rf gpurun_out/ss/$v
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bruteforce or index or c4 or sharded or topk or recall or retriever or export" > gpurun_out/ss_tests.log 2>&1 || { tail -40 gpurun_out/ss_tests.log; exit 1; }
tail -2 gpurun_out/ss_tests.log
timeout -k 10 120 python -u tools/time_index.py 1000000 100 3 2>&1 | grep -v amdgpu.ids
