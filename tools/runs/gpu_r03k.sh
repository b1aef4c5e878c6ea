timeout -k 10 60 ./tools/pbin/iprobe6_stats 131072 | tail -3 && bash tools/gpu_idx_prof.sh iprobe6_base r03k tests && bash tools/gpu_pmc_scan.sh iprobe6_base
