# Round 5: sample tiles per split (TT_INDEX_MAX_SAMPLE 128 = this tree, 96, 80).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05sm; mkdir -p $OUT
for r in 1 2 3; do
  for v in new s96 s80; do
    L=""; [ $v != new ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $OUT/$v.$r.log 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $OUT/$v.$r.log; exit 1; }
      echo "$v r$r [$cfg]: $(tail -1 $OUT/$v.$r.log)"
    done
  done
done
