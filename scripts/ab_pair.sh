# r02: two-lanes-per-chain encrypt (k_encrypt_pair) -- parity under the GPU suite with every
# encrypt forced onto it, then times against the lane and quad kernels (CYAES_ENC_KERNEL).
set -u
CYAES_ENC_KERNEL=pair timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_sweep.py tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pair.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_pair.txt; [ $rc -ne 0 ] && exit $rc
for k in pair lane quad pair lane quad; do
  echo "== $k"
  CYAES_ENC_KERNEL=$k timeout -k 10 120 python tools/ab_ragged.py --rounds 5 --sizes 1048576:1472,262144:1472,131072:1472,21000:1472,65536:65280 || exit 1
done
