# Screen probe variants on the GPU box (binaries built in tools/pbin).
set -e
mkdir -p gpurun_out
O=gpurun_out/probe2.log
: > $O
for v in ${VARIANTS:-stats pipe noins nofilt nosync}; do echo "== $v" >> $O; timeout -k 10 60 ./tools/pbin/probe_$v ${NQ:-131072} >> $O 2>&1; done
grep -v amdgpu.ids $O
