# Split in-batch prep (TT_SPLIT_PREP): bit-identity tests, then an
# interleaved step A/B against the one-call loss entry.
set -e
mkdir -p gpurun_out/s05sp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "split_prep or inbatch_fused_entry or igrad_first" > gpurun_out/s05sp/tests.log 2>&1 || { tail -40 gpurun_out/s05sp/tests.log; exit 1; }
tail -2 gpurun_out/s05sp/tests.log
bash tools/gpu_step_ab.sh 5 base:-: split:TT_SPLIT_PREP=1:
