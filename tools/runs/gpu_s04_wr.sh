# Round 4: HBM write / fetch bytes of the index kernels at one 131k-query
# chunk of C4 (probe build), separate --pmc passes.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s04wr; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o w -- ./tools/pbin/probe_new 131072 105542 100 > /dev/null 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o f -- ./tools/pbin/probe_new 131072 105542 100 > /dev/null 2>&1
python3 - <<PY
import csv, glob, collections
for tag in ('w', 'f'):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob('$OUT/%s/*counter_collection.csv' % tag)[0])):
        n = r['Kernel_Name']
        if any(x in n for x in ('scan_kernel', 'finalize', 'sample_kernel', 'query_prep')):
            agg[n.replace('void ', '').replace('tt::(anonymous namespace)::', '').split('(')[0]].append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(tag, k, len(v), 'KiB/launch', round(sum(v) / len(v)), 'KB/query', round(sum(v) / len(v) * 1.024 / 131072, 2))
PY
rm -f $OUT/*/*counter_collection.csv
