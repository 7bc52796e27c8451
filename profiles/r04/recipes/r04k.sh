# r04: relay loop depth / looper sweep (1,472-B chunks).  Outputs in gpurun_out/r04k/.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k
mkdir -p $O
: > $O/relay_loop.jsonl
for t in 8 12; do
  for d in 3 4 6; do
    timeout -k 10 60 build/relay_loop --threads $t --size 1472 --seconds 4 --depth $d >> $O/relay_loop.jsonl 2>> $O/err.txt
  done
done
timeout -k 10 60 build/relay_loop --threads 8 --size 1472 --seconds 4 --depth 4 --chunks 128 >> $O/relay_loop.jsonl 2>> $O/err.txt
timeout -k 10 60 build/relay_loop --threads 8 --size 1472 --seconds 4 --depth 4 --chunks 512 >> $O/relay_loop.jsonl 2>> $O/err.txt
echo done
