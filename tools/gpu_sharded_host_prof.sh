# cProfile of the world-1 sharded step (host time per phase) at 2048 rows.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m cProfile -o gpurun_out/sh_prof.out bench.py --train-mode sharded --batch 2048 --steps 200 --warmup 10 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > gpurun_out/sh_prof.json 2> gpurun_out/sh_prof.err
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/sh_prof.out")
p.sort_stats("tottime").print_stats(35)
PY
