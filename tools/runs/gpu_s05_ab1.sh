# Round 5: in-batch passes with one split per XCD group (TT_INBATCH_XCD,
# default on) vs the (blocks, S) grid: interleaved train-step A/B + the
# passes' own event timings from the bench line.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05ab1; mkdir -p $OUT
for r in 1 2 3; do
  for v in xcd1 xcd0; do
    E=""; [ $v = xcd0 ] && E="TT_INBATCH_XCD=0"
    env $E timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --no-index --no-cpu-baseline --pipeline-rows 0 \
      --no-uniform-gather --no-c5 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || exit 0
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json')); r=d['roofline']; print('$v', $r, round(d['ms_per_step'],4), 'rows', round(r['ms_per_launch']*1e3,1), 'cols', round(r['cols_pass']['ms_per_launch']*1e3,1), 'entry', round(r['ms_fused_entry']*1e3,1))"
  done
done
exit 0
