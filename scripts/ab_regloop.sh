# r02 A/B: ragged decrypt regular groups in their own loop with incremental positions (rl1,
# CYAES_RAGGED_REGULAR_LOOP=1) vs the shared per-row loop (rl0); default kernel choice.
set -u
for v in rl1 rl0 rl1 rl0; do
  echo "== $v"
  timeout -k 10 120 python tools/ab_ragged.py --rounds 7 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,65536:65280 || exit 1
done
