# r02 A/B: ragged decrypt with the progress atomic after the step's loads (pl1) vs before (pl0).
set -u
for v in pl1 pl0 pl1 pl0; do
  echo "== $v"
  timeout -k 10 120 python tools/ab_ragged.py --rounds 7 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,65536:65280 || exit 1
done
