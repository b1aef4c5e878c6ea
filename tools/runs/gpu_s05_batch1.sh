# Round 5 batch: route kernel tests, the captured sharded step + C5 leg
# measurements, the in-batch XCD-split A/B.
bash tools/runs/gpu_s05_route.sh
bash tools/runs/gpu_s05_sharded.sh
bash tools/runs/gpu_s05_ab1.sh
exit 0
