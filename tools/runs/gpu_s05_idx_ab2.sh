# Round 5: index scan A/B — bit-exact index tests on this tree's libtt, then
# interleaved timings of this tree (new) against variant builds under
# tools/vlib/<name>/ (built beforehand by tools/build_variant.sh).
#   bash tools/runs/gpu_s05_idx_ab2.sh <tag> <variant> [<variant> ...]
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -m gpu -v \
  -k "index or bruteforce or topk or candidate" --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "index tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL" $OUT/t.log | head; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in new "$@"; do
    L=""; [ $v != new ] && L="TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/$v/libtt.so"
    for cfg in "1048576 100 2" "2048 1000 20"; do
      f=$OUT/$v.$r.$(echo $cfg | tr ' ' _).log
      env $L timeout -k 10 120 python -u tools/time_index.py $cfg > $f 2>&1 || { echo "$v r$r [$cfg] FAILED"; tail -3 $f; exit 1; }
      echo "$v r$r [$cfg]: $(tail -1 $f)"
    done
  done
done
