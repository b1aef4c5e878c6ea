# Round 4: C2/C3 train-step tests (gradients recovered from Adagrad), bench with the C5 sharded-table leg.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -q --timeout 400 --timeout-method thread -rf -s -k "train_steps" > gpurun_out/gputests_s04e.log 2>&1 || { grep -E "^E |FAILED|passed|failed|@0" gpurun_out/gputests_s04e.log | head -60; exit 1; }
tail -3 gpurun_out/gputests_s04e.log
grep -E "'fwd@0'" gpurun_out/gputests_s04e.log | head -4 || true
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s04e.json 2> gpurun_out/bench_s04e.err || { tail -30 gpurun_out/bench_s04e.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s04e.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['cols_pass']['ms_per_launch'], d['roofline']['ms_fused_entry']); print(json.dumps(d.get('c5_sharded_table'))); print(json.dumps(d['index']['runner_point']))"
