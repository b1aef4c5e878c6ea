# Index probe under rocprofv3 + the index tests.  usage: bash tools/gpu_idx_prof.sh <probe> [tag]
set -o pipefail
P=${1:-iprobe3_base}; TAG=${2:-x}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG/$P -o run -- $R/tools/pbin/$P 131072 > $R/gpurun_out/prof_$TAG/$P.log 2>&1 || { tail $R/gpurun_out/prof_$TAG/$P.log; exit 1; }
cat $R/gpurun_out/prof_$TAG/$P.log | grep -v "^W2\|rocprof"
cd $R
python3 tools/rocpd_summary.py gpurun_out/prof_$TAG/$P/run_results.db | head -8
if [ -n "$3" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "bruteforce or index or c4 or topk or retriev or recall or smoke or sharded" > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log; exit $rc
fi
