# Round 4: the full -m gpu suite on the clean in-tree build; if it dies, the
# same suite on a library built from the last tree that passed (98aaefd).
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04suite2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/cur.log 2>&1
rc=$?
echo "current tree rc=$rc: $(tail -1 $OUT/cur.log)"
grep -n "Fatal" $OUT/cur.log | head -2
if [ $rc -ne 0 ]; then
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/pbin/lib_r04y/libtt.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r04y.log 2>&1
  echo "r04y lib rc=$?: $(tail -1 $OUT/r04y.log)"
  grep -n "Fatal" $OUT/r04y.log | head -2
fi
exit 0
