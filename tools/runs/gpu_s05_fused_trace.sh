# Round 5: kernel timeline of the C3 step with the fused per-tower apply
# (--fused-apply), to see why it is slower than the default.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_fused; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather --no-c5 --fused-apply > $OUT/line.json 2> $OUT/err.txt
cd $GRAFT_REPO_ROOT
python3 -c "import json; d=json.load(open('$OUT/line.json')); print('fused ms/step', round(d['ms_per_step'],4))"
python3 tools/step_timeline.py $OUT/t_kernel_trace.csv > $OUT/timeline.txt && cat $OUT/timeline.txt
rm -f $OUT/t_kernel_trace.csv
