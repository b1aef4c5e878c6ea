# Index scan priority variants (prebuilt in tools/pbin): time_index 1M x k=100.
set -e
for v in base prio1 prio2 noins noins1 noins2 probe1 probe2 probe2p; do
  echo "== $v"
  TT_LIB_PATH=$PWD/tools/pbin/libtt_$v.so timeout -k 10 120 python3 -u tools/time_index.py 1000000 100 3 2>&1 | grep -v amdgpu.ids
done
