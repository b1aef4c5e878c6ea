# Round 5: index scan with one 32-query set per wave, 16 waves (4 per SIMD;
# TT_SCAN_ONESET=1, tools/vlib/idx_oneset) — the bit-exact index tests on
# that library, then interleaved timing against this tree (two sets per wave).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05b8; mkdir -p $OUT
TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/idx_oneset/libtt.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -v \
  -k "index or bruteforce or topk or candidate" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "FAIL|Error" $OUT/t.log | head; tail -3 $OUT/t.log; exit 1; }
echo "oneset index tests: $(tail -1 $OUT/t.log)"
for r in 1 2 3; do
  for v in new idx_oneset; do
    L=""; [ $v != new ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $OUT/$v.$r.log 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $OUT/$v.$r.log; exit 1; }
      echo "$v r$r [$cfg]: $(tail -1 $OUT/$v.$r.log)"
    done
  done
done
