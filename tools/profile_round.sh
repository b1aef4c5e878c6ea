#!/bin/bash
# Round profile on the GPU box (run from the repo root under gpurun):
#   1. kernel trace + stats (csv) of the default bench command
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) of a short bench run, each its own run
# Outputs under gpurun_out/prof_<tag>/.
set -e
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 $GRAFT_REPO_ROOT/bench.py > $OUT/bench_line.txt 2> $OUT/bench_stderr.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --index-queries 65536 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --index-queries 65536 > /dev/null 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $OUT/pmc_fetch/fetch_counter_collection.csv $OUT/pmc_write/write_counter_collection.csv --note "rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB per dispatch) from separate --pmc passes of bench.py --steps 5 --warmup 2 --no-cpu-baseline --index-queries 65536." > $OUT/pmc_traffic.json
# keep what is committed (stats, PMC summary); the raw traces exceed what gpurun copies back
rm -f $OUT/trace/bench_kernel_trace.csv $OUT/pmc_fetch/fetch_counter_collection.csv $OUT/pmc_write/write_counter_collection.csv
echo profile-ok
