# r04: relay loop depth and batcher loads on the current build.  Outputs in gpurun_out/r04g/.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
: > $O/relay_loop.jsonl
for d in 1 2 3; do
  for sz in 1472 rand:4000; do
    timeout -k 10 60 build/relay_loop --threads 8 --size $sz --seconds 4 --depth $d >> $O/relay_loop.jsonl 2> $O/relay_loop_err.txt
  done
done
: > $O/bench_batcher.jsonl
for cfg in "seal --pool 1" "open --pool 1"; do
  timeout -k 10 60 build/bench_batcher --op $cfg --threads 8 --window 16384 --seconds 4 --complete poll >> $O/bench_batcher.jsonl 2>> $O/bench_batcher_err.txt
done
echo done
