# Round 4 check: the -m gpu suite, smoke(), the default bench line, the round
# profile (kernel stats + PMC traffic) -> gpurun_out/, copied into profiles/.
set -e
bash tools/gpu_round.sh r04z tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/gpu_round.sh r04z bench prof
