# tt_mlp_rows timing + probe variants (tools/pbin/libtt_mlp*.so)
set -e
timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep " us " 
for v in ${VARIANTS:-mlpnoout mlpnob mlpnoa}; do
  echo "== $v"; TT_LIB_PATH=$PWD/tools/pbin/libtt_$v.so timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep " us "
done
