# r02 A/B: ragged decrypt regular groups software-pipelined (next step's loads before this
# step's stores) with 2 rows per step (rp2, default) or 4 (rp4, VGPR spills) vs the shared loop (rp0).
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_sweep.py tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rpipe.txt 2>&1
rc=$?; tail -1 gpurun_out/pytest_rpipe.txt; [ $rc -ne 0 ] && exit $rc
for v in rp2 rp0 rp4 rp2 rp0; do
  echo "== $v"
  timeout -k 10 120 python tools/ab_ragged.py --rounds 7 --lib build/variants/$v.so --sizes 1048576:1472,262144:1472,65536:65280 || exit 1
done
