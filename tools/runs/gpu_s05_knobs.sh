# Round 5: launch-size knobs of the C3 step (tt_mlp_wgrad and in-batch pass
# workgroup targets), interleaved step-time A/B.
set -e
bash tools/gpu_step_ab.sh 3 "def:-:--no-c5" "wg512:TT_WGRAD_WGS=512:--no-c5" "wg2048:TT_WGRAD_WGS=2048:--no-c5" "ib768:TT_INBATCH_WGS=768:--no-c5" "ib1024:TT_INBATCH_WGS=1024:--no-c5"
