set -o pipefail
mkdir -p gpurun_out
for n in iprobe2_base iprobe2_stats; do echo "== $n"; timeout -k 10 60 ./tools/pbin/$n 131072 || exit 1; done > gpurun_out/iprobe_r03d.log 2>&1; rc=$?
cat gpurun_out/iprobe_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "bruteforce or index or c4 or topk or retriev or recall or smoke or sharded" > gpurun_out/t_r03d.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/t_r03d.log | tail -40; tail -3 gpurun_out/t_r03d.log; exit $rc
