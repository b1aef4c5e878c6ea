# Final check of the round-3 tree: GPU suite, smoke, bench line (with the runner's k=1000 index point).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_s04a.log 2>&1 || { tail -40 gpurun_out/gputests_s04a.log; exit 1; }
tail -2 gpurun_out/gputests_s04a.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
timeout -k 10 500 python -u bench.py > gpurun_out/bench_s04a.json 2> gpurun_out/bench_s04a.err || { tail -30 gpurun_out/bench_s04a.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s04a.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['index'].get('runner_point')))"
