# The captured nested-fork probe, one process per variant; stops at the first crash.
for v in origin_join nested_join nested_twice; do
  timeout -k 10 60 python3 tools/graph_fork_probe.py $v; rc=$?
  [ $rc -eq 0 ] || { echo "$v: process exit $rc"; exit $rc; }
done
