set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sharded_ab.sh
bash tools/gpu_trace_sharded.sh 16384 > /dev/null; grep "host ms" gpurun_out/trace_sh16384/err.txt; cat gpurun_out/trace_sh16384/timeline.txt | awk '{print}' | head -80
for v in nested_join; do AMD_LOG_LEVEL=3 timeout -k 10 60 python3 -X faulthandler tools/graph_fork_probe.py $v > gpurun_out/fork_$v.out 2> gpurun_out/fork_$v.err; echo "$v exit $?"; cat gpurun_out/fork_$v.out; grep -v "^$" gpurun_out/fork_$v.err | tail -25; done
