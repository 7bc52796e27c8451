# r04 session experiments (one GPU call): HIP host-registration probe, wave
# timelines, decrypt A/Bs (dynamic vs static ranges; iterative vs max ILP
# scheduler; strided vs ragged relay streams).  Outputs in gpurun_out/r04d/.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 build/hostreg_probe > $O/hostreg.txt 2>&1 || true
L=cyclone_amd/libcyaes.so
timeout -k 10 150 python tools/ab.py $L $L:CYAES_DEC_DYN=0 build/variants/decitl.so --payloads 1048576 --payload-bytes 1472 --rounds 8 > $O/ab_B.txt 2>&1
timeout -k 10 150 python tools/ab.py $L $L:CYAES_DEC_DYN=0 build/variants/decitl.so --rounds 4 > $O/ab_C.txt 2>&1
timeout -k 10 150 python tools/ab.py $L $L:CYAES_DEC_DYN=0 build/variants/decitl.so --payloads 1048576 --payload-bytes 1472 --ppk 256 --rounds 8 > $O/ab_D.txt 2>&1
timeout -k 10 150 python tools/ab.py $L $L:CYAES_DEC_DYN=0 build/variants/decitl.so build/variants/allitl.so --payloads 1048576 --payload-bytes 1472 --relay --rounds 8 > $O/ab_relay_ragged.txt 2>&1
timeout -k 10 150 python tools/ab.py $L $L:CYAES_DEC_DYN=0 build/variants/decitl.so build/variants/allitl.so --payloads 1048576 --payload-bytes 1472 --relay --relay-api strided --rounds 8 > $O/ab_relay_strided.txt 2>&1
for cfg in B relay C D; do
  timeout -k 10 120 python tools/timeline.py --config $cfg --reps 2 > $O/timeline_$cfg.txt 2>&1
  timeout -k 10 120 python tools/timeline.py --config $cfg --reps 1 CYAES_DEC_DYN=0 > $O/timeline_${cfg}_static.txt 2>&1
done
timeout -k 10 200 python tools/ab_relay_layout.py --rounds 5 --layouts contig_inplace,hdr16_inplace,hdr12_s1488_inplace,relay_inplace,relay_out,s1536_off0_inplace > $O/relay_layout.txt 2>&1
echo done
