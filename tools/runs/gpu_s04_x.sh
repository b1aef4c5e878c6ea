# Round 4: host time per phase of the sharded step at world 1 (TT_HOST_PROFILE).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04x; mkdir -p $OUT
for B in 2048 16384; do
  TT_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --train-mode sharded --batch $B --steps 100 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/h$B.json 2> $OUT/h$B.err
  python -c "import json; d=json.load(open('$OUT/h$B.json')); print('B=$B', round(d['ms_per_step'],4))"
  grep "host ms" $OUT/h$B.err
done
