# r04: strided decrypt rows as 32-bit byte offsets (scalar base + lane offset loads and stores),
# under max ILP (libcyaes.so) and iterative ILP (off32itl.so), against HEAD's 64-bit rows (head.so).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batcher.py tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "strided or relay_stream or relay_loop" > $O/pytest_strided.txt 2>&1
CYAES_LIBRARY=build/variants/bounds.so timeout -k 10 300 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 150 --timeout-method thread -k "strided or relay_stream" > $O/pytest_strided_bounds.txt 2>&1
CYAES_LIBRARY=build/variants/off32itl.so timeout -k 10 300 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 150 --timeout-method thread -k "strided or relay_stream" > $O/pytest_strided_itl.txt 2>&1
H=build/variants/head.so
L=cyclone_amd/libcyaes.so
I=build/variants/off32itl.so
timeout -k 10 300 python tools/ab.py $H $L $I --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 16 > $O/ab_relay.txt 2>&1
timeout -k 10 300 python tools/ab.py $H $L $I --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 16 > $O/ab_relay2.txt 2>&1
echo done
