# Re-entry check: GPU suite, smoke, TT_TOWER_PAIR A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03k.log 2>&1 || { tail -40 gpurun_out/gputests_r03k.log; exit 1; }
tail -2 gpurun_out/gputests_r03k.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3
bash tools/gpu_step_ab.sh 3 base:TT_TOWER_PAIR=0: pair:TT_TOWER_PAIR=1:
