# Index development loop on the GPU box: parity tests, probes, timing, profile.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "bruteforce or c4 or index" > gpurun_out/idx_tests.log 2>&1 || { tail -40 gpurun_out/idx_tests.log; exit 1; }
tail -2 gpurun_out/idx_tests.log
O=gpurun_out/probe.log
: > $O
timeout -k 10 120 ./tools/pbin/probe_stats 131072 >> $O 2>&1
timeout -k 10 120 ./tools/pbin/probe_noins 131072 >> $O 2>&1
grep -v amdgpu.ids $O
timeout -k 10 120 python -u tools/time_index.py 1000000 100 2 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_probe
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_probe -o noins -- $GRAFT_REPO_ROOT/tools/pbin/probe_noins 131072 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_probe -o stats -- $GRAFT_REPO_ROOT/tools/pbin/probe_stats 131072 > /dev/null 2>&1
