# Round 5: tt_route_fixed — fused one-workgroup kernel phase times (stamps
# build) and the call's cost fused vs multi-launch; route parity tests; C5.
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05r2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -k "route or routed" --timeout 120 \
  --timeout-method thread > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/t.log)"; grep -n "FAIL\|Error" $OUT/t.log | head; [ $rc -ne 0 ] && exit 0
for B in 1024 2048 5461; do
  TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/vlib/r05stamps/libtt.so timeout -k 10 120 python -u tools/time_route.py $B > $OUT/st$B.log 2>&1 || { tail -5 $OUT/st$B.log; exit 0; }
  cat $OUT/st$B.log | grep -v amdgpu.ids
  TT_ROUTE_FUSED=0 timeout -k 10 120 python -u tools/time_route.py $B > $OUT/nf$B.log 2>&1 || { tail -5 $OUT/nf$B.log; exit 0; }
  cat $OUT/nf$B.log | grep -v amdgpu.ids
done
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --c5-only --steps 50 > $OUT/c5_$i.json 2> $OUT/c5_$i.err; rc=$?
echo "c5 $i rc=$rc: $(python3 -c "import json;d=json.load(open('$OUT/c5_$i.json'))['c5_sharded_table'];print(d['ms_per_step'], d['roofline']['frac'])" 2>&1 | tail -1)"
[ $rc -ne 0 ] && exit 0
done
exit 0
