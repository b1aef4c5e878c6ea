# Round 5: the screen's list-size target with the per-row certificate:
# k=100 R = 3k+100 (this tree) vs 2.5k+75 (r25) vs 2k+50 (r20); k=1000
# R = 1.5k+100 (this tree) vs 1.25k+100 (big125); interleaved timings.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rs; mkdir -p $OUT
for r in 1 2 3; do
  for v in new r25 r20 big125; do
    L=""; [ $v != new ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $OUT/$v.$r.log 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $OUT/$v.$r.log; exit 1; }
      echo "$v r$r [$cfg]: $(tail -1 $OUT/$v.$r.log)"
    done
  done
done
