# r02 A/B: flat decrypt for 64 <= bpp < 256 (config B/D's 92-block payloads) with row positions
# by add+compare (fm1, CYAES_FLAT_MID=1) vs a fastdiv per row (fm0); GPU suite on the default build first.
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_flatmid.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_flatmid.txt; [ $rc -ne 0 ] && exit $rc
L="build/variants/fm1.so build/variants/fm0.so"
echo "== config B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
echo "== config D"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1472 --ppk 256 || exit 1
echo "== 1 M x 1024 B"; timeout -k 10 200 python tools/ab.py $L --rounds 10 --payloads 1048576 --payload-bytes 1024 || exit 1
echo "== config B again"; timeout -k 10 200 python tools/ab.py build/variants/fm0.so build/variants/fm1.so --rounds 10 --payloads 1048576 --payload-bytes 1472 || exit 1
