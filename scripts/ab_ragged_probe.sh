set -u
for v in as noas as noas; do
  echo "== $v (lane kernel)"
  CYAES_QUAD_MAX_CHAINS=0 timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,65536:65280 || exit 1
done
echo "== as (auto: quad for ragged < 2M chains)"
timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/as.so --sizes 1048576:1472,262144:1472
