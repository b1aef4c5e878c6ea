# Runner point (2048 queries x 105,542 x k = 1000): list target 1.5k + 100
# (tree) vs 1.3k / 1.2k (variant builds rm13 / rm12), each with the default
# finalize staging capacity and with TT_FINAL_LF=2368 (20 KB of LDS per
# query: 8 queries per CU, the whole batch in one round), interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rlf; mkdir -p $OUT
for r in 1 2 3; do
  for v in new rm13 rm12; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so
    for lf in 0 2368; do
      E=""; [ $lf != 0 ] && E="TT_FINAL_LF=$lf"
      env TT_LIB_PATH=$L $E timeout -k 10 120 python -u tools/time_index.py 2048 1000 20 > $OUT/$v.$lf.$r.log 2>&1 || { echo "$v lf=$lf FAILED"; tail -3 $OUT/$v.$lf.$r.log; exit 1; }
      echo "$v lf=$lf r$r: $(tail -1 $OUT/$v.$lf.$r.log)"
    done
  done
done
