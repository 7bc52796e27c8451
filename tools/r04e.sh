# r04: per-workgroup decrypt tickets vs static ranges; schedulers; range sizes.  Outputs in gpurun_out/r04f/.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 60 build/hostreg_probe > $O/hostreg.txt 2>&1 || true
# the GPU suite; a failing test (exit 1) is recorded and the A/Bs still run, anything else stops here
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
set -e
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=cyclone_amd/libcyaes.so
V="$L $L:CYAES_DEC_DYN=0 build/variants/decitl.so build/variants/allitl.so build/variants/decnoprio.so build/variants/decahead.so"
timeout -k 10 150 python tools/ab.py $V $L:CYAES_DEC_RANGE_STEPS=1 $L:CYAES_DEC_RANGE_STEPS=4 --payloads 1048576 --payload-bytes 1472 --rounds 8 > $O/ab_B.txt 2>&1
timeout -k 10 200 python tools/ab.py $V --rounds 4 > $O/ab_C.txt 2>&1
timeout -k 10 150 python tools/ab.py $V --payloads 1048576 --payload-bytes 1472 --ppk 256 --rounds 8 > $O/ab_D.txt 2>&1
timeout -k 10 150 python tools/ab.py $V $L:CYAES_DEC_GROUPS_PER_WAVE=16 --payloads 1048576 --payload-bytes 1472 --relay --rounds 8 > $O/ab_relay_ragged.txt 2>&1
timeout -k 10 150 python tools/ab.py $V --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 8 > $O/ab_relay_strided.txt 2>&1
timeout -k 10 120 python tools/timeline.py --config B --reps 1 > $O/timeline_B.txt 2>&1
timeout -k 10 120 python tools/timeline.py --config relay --reps 1 > $O/timeline_relay.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo done
