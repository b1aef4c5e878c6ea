# Kernel trace of the C5 leg alone (bench.py --c5-only): the last replays'
# kernels with their queues and durations.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/s05c5; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 $GRAFT_REPO_ROOT/bench.py --c5-only --steps 20 --warmup 2 > $OUT/line.json 2> $OUT/err.txt
python3 - $OUT/t_kernel_trace.csv <<'PY' > $OUT/timeline.txt
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-60:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3; e = (int(r["End_Timestamp"]) - t0) / 1e3
    n = re.sub(r"^void ", "", r["Kernel_Name"]).replace("tt::(anonymous namespace)::", "")
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} {n[:110]}")
PY
cat $OUT/timeline.txt
