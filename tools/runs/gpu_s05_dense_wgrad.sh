# Each layer's Adagrad step inside its weight-gradient launches (default,
# TT_FUSED_DENSE_WGRAD=1) vs one dense_adagrad launch per tower (=0): model /
# config / MLP tests, then an interleaved step A/B.
set -e
mkdir -p gpurun_out/s05dw
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "model or step or bit_identical or mlp or c2 or c3 or graph" > gpurun_out/s05dw/tests.log 2>&1 || { tail -40 gpurun_out/s05dw/tests.log; exit 1; }
tail -1 gpurun_out/s05dw/tests.log
bash tools/gpu_step_ab.sh 4 base:TT_FUSED_DENSE_WGRAD=0: dw:-:
