# Same-box comparison of the in-batch split target: step timelines + interleaved step A/B.
set -e
for w in 256 512; do TT_INBATCH_WGS=$w bash tools/gpu_trace_step.sh wgs$w > /dev/null; echo "== WGS $w"; grep -E "inbatch|combine|prep_kernel|sum_kernel|block_sum|gather" gpurun_out/trace_wgs$w/timeline.txt; grep -o '"ms_per_step[^,]*' gpurun_out/trace_wgs$w/line.json; done
bash tools/gpu_step_ab.sh 3 w256:TT_INBATCH_WGS=256: w512:TT_INBATCH_WGS=512:
