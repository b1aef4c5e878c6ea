# Combined: scan probes, GPU suite, smoke, TT_TOWER_PAIR A/B.
set -e
bash tools/runs/gpu_s03_scan_probes.sh
bash tools/runs/gpu_s03_suite_pair_ab.sh
