timeout -k 10 60 ./tools/pbin/iprobe5_stats 131072 | tail -3 && bash tools/gpu_idx_prof.sh iprobe5_base r03i tests
