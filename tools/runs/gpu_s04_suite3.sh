# Round 4: the full -m gpu suite with the capture-time events held for the
# graphs' lifetime.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04suite3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/cur.log 2>&1
rc=$?
echo "rc=$rc: $(tail -1 $OUT/cur.log)"
grep -n "Fatal" -A22 $OUT/cur.log | grep -v "^.*dist-packages/_pytest\|pluggy" | head -24
exit 0
