# Round 6 check: the -m gpu suite, smoke(), the default bench line and the
# round profile (kernel stats + PMC traffic) -> gpurun_out/ (copied into profiles/).
set -e
TAG=${1:-r06b}
bash tools/gpu_round.sh $TAG tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/gpu_round.sh $TAG bench prof
