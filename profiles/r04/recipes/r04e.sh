# r04: the shipped decrypt policy (auto: dynamic pool for long launches, short-launch
# divisor 4) vs forced static / forced dynamic; then the GPU suite and the bench.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j
mkdir -p $O
L=cyclone_amd/libcyaes.so
V="$L $L:CYAES_DEC_DYN=0 $L:CYAES_DEC_DYN=1"
timeout -k 10 150 python tools/ab.py $V --payloads 1048576 --payload-bytes 1472 --rounds 8 > $O/ab_B.txt 2>&1
timeout -k 10 150 python tools/ab.py $V --payloads 1048576 --payload-bytes 1472 --ppk 256 --rounds 8 > $O/ab_D.txt 2>&1
timeout -k 10 250 python tools/ab.py $V --rounds 4 > $O/ab_C.txt 2>&1
timeout -k 10 150 python tools/ab.py $V --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 8 > $O/ab_relay_strided.txt 2>&1
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo done
