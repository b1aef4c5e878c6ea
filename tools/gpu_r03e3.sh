bash tools/gpu_r03e2.sh || exit 1
bash tools/gpu_r03z.sh
