set -u
for v in qu nqu qu nqu; do
  echo "== $v"
  timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,21000:1472,65536:65280 || exit 1
done
