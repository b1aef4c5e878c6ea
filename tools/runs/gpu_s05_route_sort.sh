# Route sort configurations (rocPRIM merge-sort path, block sort of BS x IPT
# keys; variant builds tools/vlib/rs_*): route tests per variant, then the C5
# leg interleaved against the default configuration.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rs2; mkdir -p $OUT
V="rs_b1024i4 rs_b512i8 rs_b1024i8 rs_b256i16"
for v in $V; do
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "route" > $OUT/t_$v.log 2>&1 && echo "$v tests: $(tail -1 $OUT/t_$v.log)" || echo "$v tests FAILED: $(grep -E 'Error|error' $OUT/t_$v.log | head -3)"
done
for r in 1 2 3; do
  for v in base $V; do
    L=""; [ $v != base ] && L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so
    TT_LIB_PATH=$L timeout -k 10 150 python -u bench.py --c5-only --steps 50 --warmup 5 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { echo "$v failed"; tail -3 $OUT/$v.$r.err; continue; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json'))['c5_sharded_table']; print('$v', $r, round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
