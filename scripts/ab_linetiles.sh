# r02 A/B: uniform lane encrypt with line tiles + head (lt1, CYAES_LINE_TILES=1: every 8-block chunk
# stores whole 128-B lines) vs chunks from the payload start (lt0).  GPU suite on the default build first.
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_sweep.py tests/test_config_e.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lt.txt 2>&1
rc=$?; tail -1 gpurun_out/pytest_lt.txt; [ $rc -ne 0 ] && exit $rc
L="build/variants/lt1.so build/variants/lt0.so"
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config D"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 --ppk 256 || exit 1
echo "== 1 M x 1488 B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1488 || exit 1
echo "== config C"; timeout -k 10 200 python tools/ab.py $L --rounds 4 || exit 1
echo "== config B again"; timeout -k 10 200 python tools/ab.py build/variants/lt0.so build/variants/lt1.so --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
