# Kernel-trace stats of tools/gemm_probe.py (GPU box, repo root)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/gemmtrace${GEMM_PROBE:-0}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 $GRAFT_REPO_ROOT/tools/gemm_probe.py ${KINDS:-fwd,dx,dw} ${PRECS:-x3,bf16} > /dev/null 2>&1
python3 - <<'PY'
import csv, os
for r in csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/gemmtrace" + os.environ.get("GEMM_PROBE", "0") + "/t_kernel_stats.csv")):
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:110]}")
PY
