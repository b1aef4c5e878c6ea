set -e
bash tools/runs/gpu_s03_small_sort.sh
bash tools/runs/gpu_s03_final.sh
