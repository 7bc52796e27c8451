set -u
L="build/variants/med.so build/variants/nomed.so"
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config D"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 --ppk 256 || exit 1
echo "== 2M x 1024"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1572864 --payload-bytes 1024 || exit 1
echo "== config B again (reversed)"; timeout -k 10 200 python tools/ab.py build/variants/nomed.so build/variants/med.so --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
