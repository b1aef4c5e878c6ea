bash tools/runs/gpu_r03e2.sh || exit 1
bash tools/runs/gpu_r03z.sh
