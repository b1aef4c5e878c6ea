# Full GPU check: -m gpu suite, index probe, 1M index timing, bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
VARIANTS="stats noins" bash tools/gpu_probe2.sh
timeout -k 10 120 python -u tools/time_index.py 1000000 100 2 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
