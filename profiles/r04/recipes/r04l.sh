# r04: what the strided decrypt pays for on relay streams: alignment or stride (layout sweep).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 400 python tools/ab_relay_layout.py --api strided --rounds 7 --layouts contig_inplace,hdr16_inplace,hdr12_s1488_inplace,relay_inplace,relay_out,contig_off4_inplace,s1536_off0_inplace,s1536_off12_inplace > $O/layout_strided.txt 2>&1
echo done
