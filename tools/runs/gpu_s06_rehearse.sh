# Round 6: dry run of bench.py's N > 1 path on the one-GPU box: 2 and 3
# ranks sharing cuda:0 over gloo (TT_BENCH_REHEARSE=1; not a measurement).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s06reh; mkdir -p $OUT
for N in 2 3; do
  TT_BENCH_REHEARSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --batch $([ $N = 3 ] && echo 16383 || echo 16384) --steps 5 --warmup 2 --index-queries 16384 --no-cpu-baseline > $OUT/line$N.json 2> $OUT/err$N.txt || { echo "N=$N failed"; tail -30 $OUT/err$N.txt; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/line$N.json'))
print('N=$N', d['n_gpus'], round(d['ms_per_step'],3), d['config']['global_batch'], d.get('rehearsal','')[:20], 'index qps', round(d['index']['qps']), 'c5', round(d['c5_sharded_table']['ms_per_step'],3))"
done
