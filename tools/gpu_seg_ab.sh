# A/B: global rocPRIM radix sort vs one segment per table for the embedding-update id sort
set -e
mkdir -p gpurun_out
TT_LIB_PATH=$PWD/tools/pbin/libtt_seg.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "sparse or adagrad or train_steps or dedup or fused or stale" 2>&1 | tail -2
for v in base seg; do
  if [ $v = seg ]; then export TT_LIB_PATH=$PWD/tools/pbin/libtt_seg.so; else unset TT_LIB_PATH; fi
  timeout -k 10 200 python -u bench.py --no-index --no-cpu-baseline --pipeline-rows 0 --no-uniform-gather > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'])"
done
