# Interleaved A/B of train-step variants (train leg only).  Each variant is
# "NAME:ENV=VAL,ENV=VAL:bench flags" (ENV part may be empty, '-' for none).
#   bash tools/gpu_step_ab.sh <rounds> <variant>...   -> gpurun_out/step_ab/
set -e
ROUNDS=$1; shift
OUT=gpurun_out/step_ab; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; flags=${rest#*:}
    [ "$envs" = "-" ] && envs=""
    env ${envs//,/ } timeout -k 10 120 python -u bench.py --steps 300 --warmup 30 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather $flags > $OUT/$name.$r.json 2> $OUT/$name.$r.err
    python3 -c "import json; d=json.load(open('$OUT/$name.$r.json')); print('$name', $r, round(d['ms_per_step'],4))"
  done
done
