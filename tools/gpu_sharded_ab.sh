# Sharded (data-parallel) step at world 1: graphed vs eager middle, at the
# single-GPU batch and at the per-rank batch of an 8-way split (2048).
set -e
mkdir -p gpurun_out
for B in 16384 2048; do
  for mode in graph eager; do
    if [ $mode = eager ]; then export TT_SHARDED_EAGER=1; else unset TT_SHARDED_EAGER; fi
    timeout -k 10 300 python -u bench.py --train-mode sharded --batch $B --steps 100 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > gpurun_out/sh_${B}_$mode.json 2> gpurun_out/sh_${B}_$mode.err
    python -c "import json; d=json.load(open('gpurun_out/sh_${B}_$mode.json')); print('B=$B $mode', round(d['ms_per_step'],4))"
    grep "host ms" gpurun_out/sh_${B}_$mode.err || true
  done
done
