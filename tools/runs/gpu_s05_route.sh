OUT=$GRAFT_REPO_ROOT/gpurun_out/s05route; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -k "route" --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "route tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL\|Error\|assert" $OUT/t.log | head -20
exit 0
