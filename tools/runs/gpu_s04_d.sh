# Round 4: contract train-step tests on the GPU's activations, wgrad fix, C5 8-rank test, C5 bench leg.
set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 400 --timeout-method thread -rf -s > gpurun_out/gputests_s04d.log 2>&1 || { grep -E "^E |FAILED|passed|failed|@0" gpurun_out/gputests_s04d.log | head -60; exit 1; }
tail -3 gpurun_out/gputests_s04d.log
grep -E "'loss@0'|first-step" gpurun_out/gputests_s04d.log | head -20 || true
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s04d.json 2> gpurun_out/bench_s04d.err || { tail -30 gpurun_out/bench_s04d.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s04d.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['cols_pass']['ms_per_launch'], d['roofline']['ms_fused_entry']); print(json.dumps(d.get('c5_sharded_table')))"
