# Round 4: SQ counters of the tower MLP kernels (tools/time_mlp.py shapes).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04pm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/sq -o sq -- python3 $GRAFT_REPO_ROOT/tools/time_mlp.py > $OUT/sq.log 2>&1
python3 - <<PY
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob('$OUT/sq/*counter_collection.csv')[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    n = r['Kernel_Name']
    if 'mlp_' not in n: continue
    key = n.replace('void ', '').replace('tt::(anonymous namespace)::', '').split('(')[0][:40] + ' grid=' + r.get('Grid_Size', '?')
    agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, len(next(iter(d.values()))), {c.replace('SQ_', ''): round(sum(v) / len(v) / 1e6, 3) for c, v in sorted(d.items())})
PY
rm -f $OUT/sq/*counter_collection.csv
