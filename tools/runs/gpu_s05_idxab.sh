# Round 5: per-row residual screen bound — interleaved index timing, this
# tree's libtt vs the same sources with the round-start tt_index.hip.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05idxab; mkdir -p $OUT
for r in 1 2 3; do
  for v in new base; do
    L=""; [ $v = base ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/r05base/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      f=$OUT/$v.$r.$(echo $cfg | tr ' ' _).log
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $f 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $f; exit 0; }
      echo "$v r$r [$cfg]: $(tail -1 $f)"
    done
  done
done
exit 0
