# r04: the strided flat decrypt under the iterative-ILP scheduler (its own TU part; hot block
# 54 waits vs 93 under max ILP).  split0.so: the same split, strided part under max ILP.
# decitl.so: the whole flat-decrypt TU under iterative ILP.  Outputs in gpurun_out/r04s/.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
L=cyclone_amd/libcyaes.so
S=build/variants/split0.so
V=build/variants/decitl.so
timeout -k 10 200 python tools/ab.py $S $L $V --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 12 > $O/ab_relay.txt 2>&1
timeout -k 10 200 python tools/ab.py $S $L $V --payloads 1048576 --payload-bytes 1472 --rounds 10 > $O/ab_B.txt 2>&1
timeout -k 10 300 python tools/ab.py $S $V --rounds 6 > $O/ab_C.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 150 --timeout-method thread -k "strided or relay_stream" > $O/pytest_strided.txt 2>&1
echo done
