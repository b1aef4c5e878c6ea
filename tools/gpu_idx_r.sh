# List-size target sweep of the index screen (tools/pbin/iprobeR_*: TT_INDEX_R_MUL/ADD builds with stats)
for n in r300 r200 r150 r120; do echo "== $n"; timeout -k 10 60 ./tools/pbin/iprobeR_$n 131072 || exit 1; done
