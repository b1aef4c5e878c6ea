set -o pipefail
mkdir -p gpurun_out
for n in base stats noins; do echo "== $n"; timeout -k 10 60 ./tools/pbin/iprobe_$n 131072 || exit 1; done > gpurun_out/iprobe_r03b.log 2>&1
cat gpurun_out/iprobe_r03b.log
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_configs_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_r03b.log 2>&1; rc=$?
tail -30 gpurun_out/t_r03b.log; exit $rc
