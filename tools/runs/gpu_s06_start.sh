# Round 6 start: the -m gpu suite, smoke(), the default bench line on this round's first box.
set -e
TAG=${1:-r06a}
bash tools/gpu_round.sh $TAG tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/gpu_round.sh $TAG bench
