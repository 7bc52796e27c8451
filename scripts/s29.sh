mkdir -p gpurun_out/s29
timeout -k 10 300 python -u tools/ab_ragged.py > gpurun_out/s29/ab_ragged.txt 2>&1 || exit 1
for bk in 0 1; do timeout -k 10 60 build/bench_batcher --op open --threads 8 --window 8192 --seconds 3 --bulk $bk >> gpurun_out/s29/batcher.jsonl 2>>gpurun_out/s29/batcher.err || exit 1; done
echo done
