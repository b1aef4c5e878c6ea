# Round 5: is the round-4 crash the one-rank route group sharing the step's
# communicator (routing all_to_alls on a side stream while the step's
# all_reduce is captured on the compute stream)?  The pre-round-5
# distributed.py with its own route communicator at world 1 (expected: no
# crash), then as it was (expected: crash, last step).
# The two old revisions are not in the tree any more; before the gpurun call,
# extract them here (the GPU box has no .git):
#   mkdir -p tools/runs/s05_old && for f in distributed_old distributed_old_routegroup; do
#     git show 7f08554:tools/runs/s05_old/$f.py > tools/runs/s05_old/$f.py; done
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05seg5; mkdir -p $OUT
D=hm-retrieval-two-tower_amd/pkg/modelling/distributed.py
T="tests/test_model_gpu.py tests/test_pipeline_gpu.py::test_graphed_device_fit_equals_eager_host_fit"
cp tools/runs/s05_old/distributed_old_routegroup.py $D
TT_SEGV_BT=$OUT/bt_rg.txt timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/routegroup.log 2>&1; rc=$?
echo "own route group rc=$rc: $(tail -1 $OUT/routegroup.log)"; [ $rc -ne 0 ] && exit 0
cp tools/runs/s05_old/distributed_old.py $D
TT_SEGV_BT=$OUT/bt_old.txt timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/old.log 2>&1; rc=$?
echo "old rc=$rc: $(tail -1 $OUT/old.log)"
exit 0
