# Combined: scan probes, GPU suite, smoke, TT_TOWER_PAIR A/B.
set -e
bash tools/runs/gpu_r03m.sh
bash tools/runs/gpu_r03k.sh
