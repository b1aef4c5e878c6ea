set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_r03w.log 2>&1; rc=$?
grep -E "FAIL|Error|first-step update" gpurun_out/t_r03w.log | tail -30; grep -E "passed|failed" gpurun_out/t_r03w.log | tail -1; [ $rc -eq 0 ] || { tail -30 gpurun_out/t_r03w.log; exit $rc; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r03w.json 2> gpurun_out/bench_r03w.err || { tail -20 gpurun_out/bench_r03w.err; exit 1; }
cat gpurun_out/bench_r03w.json
