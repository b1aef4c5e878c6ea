# Build libtt variants (compile-time knobs; default: the index screen's
# warm-up length; VARIANTS="name:-DFLAG=..|..." and SCRIPT=tools/x.py override):
#   bash tools/index_variants.sh build
# and time them on the GPU box:
#   bash tools/index_variants.sh run
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS=${VARIANTS:-"base:|warm128:-DTT_WARM_TILES=128|warm256:-DTT_WARM_TILES=256|warm32:-DTT_WARM_TILES=32"}
SCRIPT=${SCRIPT:-tools/time_index.py}
if [ "$1" = build ]; then
  mkdir -p $ROOT/tools/bin
  IFS='|'; for v in $VARIANTS; do
    name=${v%%:*}; flags=${v#*:}
    out=$ROOT/tools/bin/obj_$name; mkdir -p $out
    unset IFS
    make -s -j8 -C $ROOT/hm-retrieval-two-tower_amd/csrc OUTDIR=$out HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics $flags"
    cp $out/libtt.so $ROOT/tools/bin/libtt_$name.so
    IFS='|'
  done
else
  IFS='|'; for v in $VARIANTS; do
    name=${v%%:*}; unset IFS
    echo "== $name"
    TT_LIB_PATH=$ROOT/tools/bin/libtt_$name.so timeout -k 10 120 python3 $ROOT/$SCRIPT
    IFS='|'
  done
fi
