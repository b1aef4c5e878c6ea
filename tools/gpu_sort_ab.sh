# A/B of the embedding-update id sort: where it starts in the step (after the
# forward and captured after the backward, "loss"; captured between forward
# and backward, "mid"; ordered after the gather but captured late, "gather";
# issued and captured right after the gather, "early") x which sort runs
# (LDS region sort "lds" or key build + rocPRIM "device").
set -e
mkdir -p gpurun_out
for sort in ${SORTS:-lds device}; do
  for after in ${AFTER:-loss mid}; do
    TT_SPARSE_SORT=$sort TT_SORT_AFTER=$after timeout -k 10 200 python -u bench.py --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > gpurun_out/ab_${sort}_${after}.json 2>gpurun_out/ab_${sort}_${after}.err
    python -c "import json; d=json.load(open('gpurun_out/ab_${sort}_${after}.json')); print('$sort $after', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
  done
done
