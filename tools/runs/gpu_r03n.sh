set -o pipefail
for n in noins base f2 f8; do echo "== $n"; timeout -k 10 60 ./tools/pbin/iprobe8_$n 131072 | tail -2 | head -1 || exit 1; done
bash tools/gpu_idx_prof.sh iprobe8_base r03n
