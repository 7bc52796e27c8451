set -u
L="build/variants/qbase.so build/variants/qdpp.so"
for sz in "4096 1024" "65536 1472" "16384 65536" "1 1472"; do
  set -- $sz
  echo "== $1 x $2"
  timeout -k 10 120 python tools/ab.py $L --rounds 8 --payloads $1 --payload-bytes $2 || exit 1
done
for v in qbase qdpp qbase qdpp; do
  echo "== relay $v"
  timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/$v.so --sizes 1048576:1472,21000:1472 || exit 1
done
