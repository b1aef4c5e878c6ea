# Round 4: knob sweeps — in-batch fragment reads in flight (TT_IB_AHEAD, probe
# builds) and the weight-gradient workgroup target (TT_WGRAD_WGS), same box.
set -e
for r in 1 2; do
  for v in a3 a2 a4 a5; do echo "$v $(timeout -k 10 60 ./tools/pbin/inb_$v 16384 100)"; done
done
for w in 1024 512 2048 768; do echo "== WGS=$w"; TT_WGRAD_WGS=$w timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "wgrad tt"; done
