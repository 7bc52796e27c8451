set -u
L="build/variants/tp1.so build/variants/tp0.so"
echo "== config C"
timeout -k 10 200 python tools/ab.py $L --rounds 8 || exit 1
echo "== config B"
timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config C again"
timeout -k 10 200 python tools/ab.py build/variants/tp0.so build/variants/tp1.so --rounds 8 || exit 1
