# In-batch development loop on the GPU box: parity tests, then the timing probes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "inbatch" > gpurun_out/ib_tests.log 2>&1; rc=$?; tail -5 gpurun_out/ib_tests.log; [ $rc -eq 0 ] || exit $rc
for p in tools/bin/ibp_*; do echo "== $p"; timeout -k 10 120 ./$p || exit 1; done
