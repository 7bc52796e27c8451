# r04 last build: per-wave timelines (clock-probe build) of configs B, D and the relay stream,
# and a rocprof kernel-stats pass over the packet configs and the relay stream.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t
mkdir -p $O
for cfg in B D relay; do
  timeout -k 10 120 python tools/timeline.py --config $cfg --reps 2 > $O/timeline_$cfg.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rocprof_packets -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config B --steps 10 --warmup 3 --no-cpu --packet-configs D --relay-stream 1 --e2e-gib 0 --traffic none > $GRAFT_REPO_ROOT/$O/bench_packets.txt 2>&1
echo done
