# Index probe: timing (base), list statistics (stats), no list stores (noins), at 131072 queries
set -e
for v in base stats noins; do echo "== $v"; timeout -k 10 60 ./tools/pbin/probe_$v ${NQ:-131072} 2>&1 | grep -v amdgpu.ids; done
