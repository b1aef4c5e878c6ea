# C5 leg at world 1: route + fetch + routed apply (serial, default) vs fetch +
# the single-device sparse Adagrad (direct probe: its own id sort), interleaved;
# then a kernel trace of the direct form.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05c5d; mkdir -p $OUT
for r in 1 2 3; do
  for v in serial direct; do
    TT_C5_ORDER=$v timeout -k 10 150 python -u bench.py --c5-only --steps 50 --warmup 5 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -5 $OUT/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$r.json'))['c5_sharded_table']; print('$v', $r, round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
C5_TRACE_ORDER=direct TT_C5_ORDER=direct bash tools/runs/gpu_s05_c5_trace.sh > /dev/null
python3 - gpurun_out/s05c5/t_kernel_trace.csv <<'PY'
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if 'gather_grouped' in r['Kernel_Name']]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3; e = (int(r["End_Timestamp"]) - t0) / 1e3
    n = re.sub(r"^void ", "", r["Kernel_Name"]).replace("tt::(anonymous namespace)::", "")
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} {n[:90]}")
PY
