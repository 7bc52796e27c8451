# r02: pair encrypt on relay streams: two dword loads + two dword stores per block (pl1) vs unaligned dwordx2 loads and stores (pl0: dwordx2 both); quad for reference.
set -u
for v in pl1 pl0 pl1 pl0; do
  echo "== pair $v"
  CYAES_ENC_KERNEL=pair timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472 || exit 1
done
echo "== quad"
CYAES_ENC_KERNEL=quad timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --lib build/variants/pl1.so --sizes 1048576:1472,262144:1472 || exit 1
