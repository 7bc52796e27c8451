# r04: flat decrypt TU under the iterative-ILP scheduler (strided hot block 54 waits vs 93).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
L=cyclone_amd/libcyaes.so
V=build/variants/decitl.so
timeout -k 10 200 python tools/ab.py $L $V --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 12 > $O/ab_relay.txt 2>&1
timeout -k 10 200 python tools/ab.py $L $V --payloads 1048576 --payload-bytes 1472 --rounds 12 > $O/ab_B.txt 2>&1
timeout -k 10 300 python tools/ab.py $L $V --rounds 6 > $O/ab_C.txt 2>&1
echo done
