set -o pipefail
for n in f0 f1 f2 f4; do echo "== $n"; timeout -k 10 60 ./tools/pbin/iprobe7_$n 131072 | tail -2 | head -1 || exit 1; done
for w in 512 1024 2048; do echo "== wgrad WGS $w"; TT_WGRAD_WGS=$w timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "wgrad tt"; done
