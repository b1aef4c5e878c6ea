# Round 4: probe — mlp_wgrad with the bf16 hi/lo split of its staged operands
# replaced by a truncation (results wrong): the split's share of the kernel.
set -e
for v in base nosplit; do
  if [ $v = nosplit ]; then export TT_LIB_PATH=$GRAFT_REPO_ROOT/tools/pbin/libnosplit/libtt.so; else unset TT_LIB_PATH; fi
  echo "== $v"; timeout -k 10 120 python -u tools/time_mlp.py 2>&1 | grep "wgrad tt"
done
