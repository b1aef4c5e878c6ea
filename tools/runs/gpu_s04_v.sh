# Round 4: kernel trace of the sharded (data-parallel) step at world 1, per-rank
# batch 2048 (an 8-way split of C3) and 16384.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04v; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for B in 2048 16384; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$B -o t -- python3 $GRAFT_REPO_ROOT/bench.py --train-mode sharded --batch $B --steps 30 --warmup 5 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/line$B.json 2> $OUT/err$B.txt
  python3 -c "import json; d=json.load(open('$OUT/line$B.json')); print('B=$B', round(d['ms_per_step'],4))"
done
