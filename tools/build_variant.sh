#!/bin/bash
# Builds a variant libtt.so into tools/vlib/<name>/ (for same-box A/B timing
# through TT_LIB_PATH), from this tree's csrc/ with some sources replaced.
#   bash tools/build_variant.sh <name> [<src>=<git-rev> | <src>=<path> ...] [-- <extra hipcc flags>]
# e.g. bash tools/build_variant.sh base tt_index.hip=HEAD
#      bash tools/build_variant.sh nostats -- -DTT_SCAN_PROBE=1
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
TMP=$(mktemp -d /tmp/vsrc_XXXX)
SRC=$TMP/pkg/csrc   # the Makefile names ../../include
mkdir -p "$SRC" "$TMP/include"
cp "$ROOT"/include/* "$TMP/include/"
cp "$ROOT"/hm-retrieval-two-tower_amd/csrc/* "$SRC"/
EXTRA=""
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; EXTRA="$*"; break; fi
  f=${1%%=*}; v=${1#*=}
  if [ -f "$v" ]; then cp "$v" "$SRC/$f"
  else git -C "$ROOT" show "$v:hm-retrieval-two-tower_amd/csrc/$f" > "$SRC/$f"; fi
  shift
done
OUT="$ROOT/tools/vlib/$NAME"
mkdir -p "$OUT"
make -s -j 8 -C "$SRC" OUTDIR="$OUT" INCLUDE="-I$TMP/include -I$SRC" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics $EXTRA" 2>&1 | grep -E "error|Error|No rule" || true
rm -rf "$OUT/obj" "$TMP"
ls -la "$OUT/libtt.so"
