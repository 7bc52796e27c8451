# r02 A/B: ragged lane encrypt with aligned-slot stores (sl: chain->payload tiles + wave-uniform
# misalignment, CYAES_ALIGNED_SLOTS=1) vs unaligned 16-B stores (nosl), lane kernel forced; then auto choice.
set -u
for v in sl nosl sl nosl; do
  echo "== $v (lane kernel)"
  CYAES_QUAD_MAX_CHAINS=0 timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,65536:65280 || exit 1
done
echo "== sl (auto kernel choice)"
timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/sl.so --sizes 1048576:1472,262144:1472,21000:1472 || exit 1
