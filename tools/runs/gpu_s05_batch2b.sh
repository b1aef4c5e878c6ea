bash tools/runs/gpu_s05_ovl2.sh
bash tools/runs/gpu_s05_batch2.sh
exit 0
