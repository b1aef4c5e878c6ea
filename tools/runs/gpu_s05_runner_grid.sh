# Runner point: list target (tree 1.2k + 100; rm11 / rm10 variant builds)
# x finalize staging capacity (default 3.5k + 128 = 30.8 KB per query; or
# TT_FINAL_LF = 3136 / 2624 / 2368: 26 / 22 / 20 KB, 6 / 7 / 8 queries per CU).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05rg; mkdir -p $OUT
for r in 1 2; do
  for v in rm11 rm10; do
    L=""; [ $v != new ] && L=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so
    for lf in 0 3136 2624 2368; do
      E=""; [ $lf != 0 ] && E="TT_FINAL_LF=$lf"
      env TT_LIB_PATH=$L $E timeout -k 10 120 python -u tools/time_index.py 2048 1000 20 > $OUT/$v.$lf.$r.log 2>&1 || { echo "$v lf=$lf FAILED"; tail -3 $OUT/$v.$lf.$r.log; exit 1; }
      echo "$v lf=$lf r$r: $(tail -1 $OUT/$v.$lf.$r.log | cut -c1-60)"
    done
  done
done
