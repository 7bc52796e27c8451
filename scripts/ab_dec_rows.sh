# r02 A/B: flat/ragged decrypt rows per step (R-way ILP per LDS round trip): 4 (dr4, kept) vs 6 (dr6, a few VGPR spills).
set -u
L="build/variants/dr4.so build/variants/dr6.so"
echo "== config C"; timeout -k 10 200 python tools/ab.py $L --rounds 6 || exit 1
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config C again"; timeout -k 10 200 python tools/ab.py build/variants/dr6.so build/variants/dr4.so --rounds 6 || exit 1
