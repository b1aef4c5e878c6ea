# Round 4: in-batch contract (exact positive pair, integer-log2 running max), shard chunk ABI, status fixes.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -rf > gpurun_out/gputests_s04b.log 2>&1 || { tail -80 gpurun_out/gputests_s04b.log; exit 1; }
tail -3 gpurun_out/gputests_s04b.log
grep -E "rel err|contract|@" gpurun_out/gputests_s04b.log | head -40 || true
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s04b.json 2> gpurun_out/bench_s04b.err || { tail -30 gpurun_out/bench_s04b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s04b.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['cols_pass']['ms_per_launch'], d['roofline']['ms_fused_entry'])"
