# C5 leg (bench.py --c5-only) at world 1: the route forked onto a side
# stream beside the fetch (fork, default), the fetch captured first (first),
# or both on the origin stream (serial), interleaved; then a kernel trace.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05c5ab; mkdir -p $OUT
for r in 1 2 3 4; do
  for v in fork first serial; do
    TT_C5_ORDER=$v timeout -k 10 150 python -u bench.py --c5-only --steps 50 --warmup 5 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -5 $OUT/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json'))['c5_sharded_table']; print('$v', $r, round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
TT_C5_ORDER=${C5_TRACE_ORDER:-serial} bash tools/runs/gpu_s05_c5_trace.sh > /dev/null
