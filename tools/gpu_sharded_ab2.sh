# Interleaved same-box A/B of the sharded step's tower streams at world 1.
set -e
mkdir -p gpurun_out
for r in 1 2; do for B in 16384 2048; do for v in 1 0; do
  TT_GLOBAL_TOWER_STREAMS=$v timeout -k 10 300 python -u bench.py --train-mode sharded --batch $B --steps 100 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > gpurun_out/sh2_${B}_$v.json 2> gpurun_out/sh2_${B}_$v.err
  python -c "import json; d=json.load(open('gpurun_out/sh2_${B}_$v.json')); print('round $r B=$B streams=$v', round(d['ms_per_step'],4))"
done; done; done
