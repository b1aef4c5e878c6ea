# Round 4: finalize group size and staged-list size at the two index points
# (TT_FINAL_WAVES, TT_FINAL_LF env knobs), same box.
set -e
for v in "0 0" "2 0" "1 768" "1 1536" "0 0"; do
  set -- $v
  echo "NW=$1 LF=$2 $(TT_FINAL_WAVES=$1 TT_FINAL_LF=$2 timeout -k 10 120 python -u tools/time_index.py 1000000 100 3 2>&1 | tail -1)"
done
for v in "0 0" "2 0" "4 4096" "0 0"; do
  set -- $v
  echo "NW=$1 LF=$2 $(TT_FINAL_WAVES=$1 TT_FINAL_LF=$2 timeout -k 10 120 python -u tools/time_index.py 2048 1000 10 2>&1 | tail -1)"
done
