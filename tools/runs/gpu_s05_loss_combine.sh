# The step's loss summed inside the loss entry's last launch (default) vs a
# tt_sum launch after it (TT_LOSS_IN_COMBINE=0): the in-batch / model tests,
# then an interleaved step A/B.
set -e
mkdir -p gpurun_out/s05lc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "inbatch or model or graph or step or bit_identical or loss" > gpurun_out/s05lc/tests.log 2>&1 || { tail -40 gpurun_out/s05lc/tests.log; exit 1; }
tail -1 gpurun_out/s05lc/tests.log
bash tools/gpu_step_ab.sh 4 base:TT_LOSS_IN_COMBINE=0: lc:-:
