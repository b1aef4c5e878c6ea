# Kernel trace of a short bench run (train leg only) for step timelines:
#   bash tools/gpu_trace_step.sh <tag>    -> gpurun_out/trace_<tag>/
set -e
TAG=${1:-step}
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 > $OUT/line.json 2> $OUT/err.txt
python3 $GRAFT_REPO_ROOT/tools/step_timeline.py $OUT/t_kernel_trace.csv > $OUT/timeline.txt
cat $OUT/timeline.txt
