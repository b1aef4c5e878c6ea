# Round 4: cProfile of the sharded step's host side at world 1, 2048 rows.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04cp; mkdir -p $OUT
timeout -k 10 300 python -u -m cProfile -o $OUT/prof.out bench.py --train-mode sharded --batch 2048 --steps 300 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/line.json 2> $OUT/err.txt
python -c "import json; d=json.load(open('$OUT/line.json')); print(round(d['ms_per_step'],4))"
