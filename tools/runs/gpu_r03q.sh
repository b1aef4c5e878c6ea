set -o pipefail
MATCH=mlp_wgrad bash tools/gpu_pmc_py.sh wg tools/time_mlp.py
bash tools/gpu_step_ab.sh 2 blas:TT_WGRAD=blas: tt:TT_WGRAD=tt:
