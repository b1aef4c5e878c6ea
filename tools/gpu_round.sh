# Round check on the GPU box: -m gpu suite, default bench line, round profile.
#   bash tools/gpu_round.sh <tag> [tests|bench|prof ...]   (default: all three)
set -e
TAG=${1:-r02}; shift || true
STEPS=${*:-tests bench prof}
mkdir -p gpurun_out
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -40 gpurun_out/gputests_$TAG.log; exit 1; }
      tail -3 gpurun_out/gputests_$TAG.log ;;
    bench)
      timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
      cat gpurun_out/bench_$TAG.json ;;
    prof)
      bash tools/profile_round.sh $TAG ;;
  esac
done
