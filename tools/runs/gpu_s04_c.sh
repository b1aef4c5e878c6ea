# Round 4: contract diagnosis at C2 / C3 train steps + the wgrad empty-split fix check.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_contract.py 4096 64 > gpurun_out/diag_c2.log 2>&1 || { tail -30 gpurun_out/diag_c2.log; exit 1; }
cat gpurun_out/diag_c2.log | grep -v INFO
timeout -k 10 400 python -u tools/diag_contract.py 16384 128 > gpurun_out/diag_c3.log 2>&1 || { tail -30 gpurun_out/diag_c3.log; exit 1; }
cat gpurun_out/diag_c3.log | grep -v INFO
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "mlp or inbatch" > gpurun_out/gpt_s04c.log 2>&1 || { tail -40 gpurun_out/gpt_s04c.log; exit 1; }
tail -2 gpurun_out/gpt_s04c.log
