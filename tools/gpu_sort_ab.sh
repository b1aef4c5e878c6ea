# A/B of where the embedding-update id sort starts in the step: after the
# forward ("loss"), ordered after the gather but captured late ("gather"),
# or issued and captured right after the gather ("early").
set -e
mkdir -p gpurun_out
for after in ${AFTER:-loss gather early}; do
  TT_SORT_AFTER=$after timeout -k 10 200 python -u bench.py --no-index --no-cpu-baseline --pipeline-rows 0 > gpurun_out/ab_${after}.json 2>gpurun_out/ab_${after}.err
  python -c "import json; d=json.load(open('gpurun_out/ab_${after}.json')); print('$after', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
done
