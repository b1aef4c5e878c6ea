# Kernel trace of the sharded step at world 1 (per-rank batch B), step timeline
set -e
B=${1:-2048}
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_sh$B
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
TT_HOST_PROFILE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 $GRAFT_REPO_ROOT/bench.py --train-mode sharded --batch $B --steps 30 --warmup 5 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > $OUT/line.json 2> $OUT/err.txt
python3 $GRAFT_REPO_ROOT/tools/step_timeline.py $OUT/t_kernel_trace.csv > $OUT/timeline.txt
grep "host ms" $OUT/err.txt || true
cat $OUT/timeline.txt
