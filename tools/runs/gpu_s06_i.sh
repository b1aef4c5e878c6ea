# Round 6: the towers' weight images packed by the train step's gather launch
# (tt_gather_multi_pack) — bit-identity tests, then interleaved step A/B.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -k "pack or graph or train_step or fit or bit_identical" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_step_ab.sh 4 "pack1:TT_PACK_WITH_GATHER=1:" "pack0:TT_PACK_WITH_GATHER=0:"
