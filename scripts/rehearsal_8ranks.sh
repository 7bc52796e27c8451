# r02: bench.py --config E as 8 torchrun ranks on the box's one GPU (gloo; ranks share the device):
# the N=8 pass split (one reduced pass per rank), key broadcast, max-over-ranks timing, per-rank
# pass digests against tests/golden/config_e_passes.json "reduced".
set -u
export CYAES_BENCH_SAME_DEVICE=1 CYAES_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --config E --e-pass-payloads 4096 --e-passes 8 --steps 3 --warmup 1 \
  --packet-configs B,D --packet-steps 3 --packet-warmup 2 --no-cpu --no-clock
