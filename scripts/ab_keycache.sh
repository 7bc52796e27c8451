# r02 A/B: lane encrypt keeps the last key schedule in SGPRs across chains (kc1,
# CYAES_ENC_KEY_CACHE=1) vs a schedule load per chain (kc0). Lane kernel above 131,072 chains.
set -u
L="build/variants/kc1.so build/variants/kc0.so"
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config D"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 --ppk 256 || exit 1
echo "== config C"; timeout -k 10 200 python tools/ab.py $L --rounds 6 || exit 1
echo "== config B again"; timeout -k 10 200 python tools/ab.py build/variants/kc0.so build/variants/kc1.so --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
