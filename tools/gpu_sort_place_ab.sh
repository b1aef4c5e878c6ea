# A/B of the embedding-sort capture point (TT_SORT_AFTER), interleaved, train leg only.
#   bash tools/gpu_sort_place_ab.sh "<modes>" <rounds>   -> gpurun_out/sortplace/
set -e
MODES=${1:-"loss mid gather"}; ROUNDS=${2:-3}
OUT=gpurun_out/sortplace; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for m in $MODES; do
    TT_SORT_AFTER=$m timeout -k 10 120 python -u bench.py --steps 300 --warmup 30 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > $OUT/$m.$r.json 2> $OUT/$m.$r.err
    python3 -c "import json,sys; d=json.load(open('$OUT/$m.$r.json')); print('$m', $r, round(d['ms_per_step'],4))"
  done
done
