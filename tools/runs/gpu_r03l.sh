set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/t_r03l.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/t_r03l.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep -v "^W2\|amdgpu.ids" | tail -12
timeout -k 10 60 ./tools/pbin/iprobe6_stats 131072 | tail -3 && bash tools/gpu_idx_prof.sh iprobe6_base r03l
