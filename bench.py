#!/usr/bin/env python3
"""bench.py -- device-resident AES-128-CBC encrypt+decrypt throughput on MI355X.

Metric (BASELINE.json): "AES encrypt+decrypt GiB/s device-resident (64 KiB
payloads); % HBM roofline @1/2/4/8 GPU".  One step = one CBC-encrypt pass
plus one CBC-decrypt pass over the per-GPU batch (config C of BASELINE.json:
1 key, 262,144 payloads x 65,536 B = 16 GiB per GPU; every payload an
independent chain from DefaultIV, the relay semantics of
relay_local.cpp:206 / relay_server.cpp:329).  value = 2 x bytes x steps x
ranks / max-over-ranks wall time, in GiB/s (2^30).

Multi-GPU (torchrun, one process per GPU): rank 0 holds the session key and
broadcasts it over RCCL (xGMI); every rank expands it on its device and
processes its own payload shard (weak scaling: per-GPU batch fixed, payload
indices [rank*P, (rank+1)*P) of the global stream).  No data-path collective.

packet_configs: the north star's other named sizes, measured after the
headline config at the same GPU count with the same timing rules: config B
(1 M x 1,472 B, MTU-sized) and config D (4,096 session keys x 256 x 1,472 B).
Reported beside `value`, never as it.

cpu_baseline: the oracle (a plain-C restatement of the reference's scalar
Rijndael, oracle/aes_oracle.c) timed on this host's cores on a bounded
sample of the same workload, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "AES encrypt+decrypt GiB/s device-resident (64 KiB payloads); % HBM roofline @1/2/4/8 GPU"
LOOKUPS_PER_BLOCK = 160      # 9 x 16 T-table + 16 S-box lookups (cyr_rijndael.cpp:659-704)
LDS_LANES_PER_CLK_CU = 32    # ds_read_b32: 2 x 32-lane groups, 1 cycle each (MI355X_MICROARCH.md, LDS)
NUM_CUS = 256
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
PLAINTEXT_SEED = 0x5EEDC1C1
CONFIGS = {
    # name: (payloads per GPU, payload bytes, payloads per session key (0 = one key))
    "C": (262144, 65536, 0),
    "B": (1048576, 1472, 0),
    "D": (1048576, 1472, 256),
    "A": (4096, 1024, 0),
}


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C", choices=sorted(CONFIGS))
    ap.add_argument("--payloads", type=int, default=0, help="override payloads per GPU")
    ap.add_argument("--cpu-sample", type=int, default=0, help="cpu baseline sample payloads (0 = auto)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--packet-configs", default="B,D",
                    help="other BASELINE.json packet configs measured after the headline one ('none' to skip)")
    ap.add_argument("--packet-steps", type=int, default=20)
    ap.add_argument("--packet-warmup", type=int, default=20,
                    help="untimed steps before each packet config (a 1,472-B step is ~2 ms; 20 cover the clock "
                         "ramp that 2 steps of the 23-ms headline step cover, profiles/r01/packet_warmup.txt)")
    return ap.parse_args()


def session_keys(n):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import struct
    seed = 0xC1C10E55D0000000

    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return x ^ (x >> 31)
    return b"".join(struct.pack("<QQ", sm(seed + 2 * s), sm(seed + 2 * s + 1)) for s in range(n))


def cpu_baseline(cfg_name, npay, pb, ppk, d_ct, torch, sample=0):
    """Oracle (scalar reference restatement) on the host cores; bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    # ~4 GiB of payload by default: ~20 s of CPU work over 16 threads
    sample = min(npay, sample if sample > 0 else int(max(1, (4 << 30) // pb)))
    keys = [bytes(range(16))] if not ppk else [session_keys(sample // ppk + 1)[16 * s:16 * s + 16]
                                              for s in range(sample // ppk + 1)]
    pt = oracle.synthetic(0, sample, pb)
    t0 = time.perf_counter()
    ct = oracle.batch(False, keys, ppk, pt, pb, nthreads=threads)
    t1 = time.perf_counter()
    rt = oracle.batch(True, keys, ppk, ct, pb, nthreads=threads)
    t2 = time.perf_counter()
    # single-core figure on a smaller slice
    s1 = max(1, sample // 32)
    t3 = time.perf_counter()
    ct1 = oracle.batch(False, keys, ppk, pt[:s1 * pb], pb, nthreads=1)
    t4 = time.perf_counter()
    oracle.batch(True, keys, ppk, ct1, pb, nthreads=1)
    t5 = time.perf_counter()
    torch.cuda.synchronize()
    gpu_sample = d_ct[: sample * pb].cpu().numpy()
    exact = bool(np.array_equal(gpu_sample, ct)) and bool(np.array_equal(rt, pt))
    gib = float(1 << 30)
    return {
        "value": round(2 * sample * pb / (t2 - t0) / gib, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": "config %s: first %d payloads x %d B (%.2f GiB), encrypt then decrypt, %d threads "
                  "(one Rijndael key schedule per thread, as relay's work threads); oracle/aes_oracle.c"
                  % (cfg_name, sample, pb, sample * pb / gib, threads),
        "single_core": round(2 * s1 * pb / ((t4 - t3) + (t5 - t4)) / gib, 4),
        "seconds": round(t2 - t0, 3),
        "matches_gpu": exact,
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    # Rehearsal knobs for a 1-GPU box (never used by the driver): run every rank
    # on device 0 and use gloo instead of RCCL.
    device = 0 if os.environ.get("CYAES_BENCH_SAME_DEVICE") else local
    backend = os.environ.get("CYAES_DIST_BACKEND", "nccl")
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    import cyclone_amd as ca
    from cyclone_amd import dist as cdist

    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    ctx = ca.GpuContext(device)
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "openssl_vectors.json")))["configs"]
    gib = float(1 << 30)

    def run_config(name, npay, steps, warmup, verify, keep_cipher=False):
        """One config, timed as the contract says; returns a result dict (rank-local
        kernel times, max-over-ranks wall time)."""
        _, pb, ppk = CONFIGS[name]
        nbytes = npay * pb
        # Session key(s): rank 0 owns them (the relay's DH secret), RCCL-broadcast
        # over xGMI straight into device memory; each GPU expands its own sessions.
        p0, npay = cdist.weak_shard(npay, rank)
        nkeys = cdist.session_range(0, npay * world, ppk)[1]
        d_keys = cdist.broadcast_keys((session_keys(nkeys) if ppk else bytes(range(16))) if rank == 0 else None,
                                      nkeys, "cuda")
        k0, nk = cdist.session_range(p0, npay, ppk)
        d_keys = d_keys[16 * k0: 16 * (k0 + nk)].contiguous()
        ctx.set_keys_device(d_keys, nk, sh)

        log("rank %d/%d: config %s, %d payloads x %d B = %.2f GiB per GPU, %d CUs"
            % (rank, world, name, npay, pb, nbytes / 2**30, ctx.num_cus))
        d_pt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        d_ct = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        d_rt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic(d_pt, p0, npay, pb, PLAINTEXT_SEED, sh)

        def enc():
            ctx.encrypt_uniform(d_pt, d_ct, npay, pb, payloads_per_key=ppk, stream=sh)

        def dec():
            ctx.decrypt_uniform(d_ct, d_rt, npay, pb, payloads_per_key=ppk, stream=sh)

        for _ in range(warmup):
            enc()
            dec()
        torch.cuda.synchronize()

        parity = None
        if verify:
            gname = name if rank == 0 else ("E_rank1" if (rank == 1 and name == "C") else None)
            dp = ctx.digest(d_pt, nbytes, sh)
            dc = ctx.digest(d_ct, nbytes, sh)
            dr = ctx.digest(d_rt, nbytes, sh)
            ok = dr == dp
            g = golden.get(gname) if gname else None
            if g and g["npayloads"] == npay and g["payload_bytes"] == pb and g["p0"] == p0:
                ok = ok and ["%016x" % v for v in dc] == g["cipher_digest"] and \
                    ["%016x" % v for v in dp] == g["plain_digest"]
            ok = ok and ctx.check() == ca.CYAES_OK
            flag = torch.tensor([0 if ok else 1], device="cuda")
            if world > 1:
                dist.all_reduce(flag)
            parity = "bit-exact" if int(flag.item()) == 0 else "MISMATCH"
            log("config %s parity: %s" % (name, parity))

        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            ev[i][0].record(stream)
            enc()
            ev[i][1].record(stream)
            dec()
            ev[i][2].record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        t = float(elapsed.item())
        res = {
            "name": name, "npay": npay, "pb": pb, "ppk": ppk, "nbytes": nbytes, "t": t, "steps": steps,
            "value": 2.0 * nbytes * steps * world / t / gib,
            "enc_ms": sum(a.elapsed_time(b) for a, b, _ in ev) / steps,
            "dec_ms": sum(b.elapsed_time(c) for _, b, c in ev) / steps,
            "parity": parity, "d_ct": d_ct if keep_cipher else None,
        }
        del d_pt, d_rt
        if not keep_cipher:
            del d_ct
        return res

    npay = args.payloads or CONFIGS[args.config][0]
    main_res = run_config(args.config, npay, args.steps, args.warmup, not args.no_verify, keep_cipher=True)
    nbytes, pb, ppk = main_res["nbytes"], main_res["pb"], main_res["ppk"]
    npay, t, value = main_res["npay"], main_res["t"], main_res["value"]
    enc_ms, dec_ms, parity = main_res["enc_ms"], main_res["dec_ms"], main_res["parity"]

    def roof(ms, nb=nbytes):
        ach = 2.0 * nb / (ms / 1e3) / 1e9  # algorithmic: read N + write N per launch
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4)}

    def lds(ms, nb=nbytes):
        # The binding on-chip resource: 160 conflict-free ds_read_b32
        # lookups per 16-B block; nominal LDS rate 32 lanes/clk/CU (2 cycles per wave64
        # ds_read_b32), here priced at the 2.4 GHz peak shader clock.  In-kernel clock
        # probes (tools/ab.py + CYAES_CLOCK_PROBE) show ~1.9 GHz under this load.
        look = LOOKUPS_PER_BLOCK * (nb / 16) / (ms / 1e3)
        peak = LDS_LANES_PER_CLK_CU * NUM_CUS * 2.4e9
        return {"lookups_per_s": float("%.4g" % look), "peak_at_2p4ghz": float("%.4g" % peak),
                "frac": round(look / peak, 4)}

    kern = {"encrypt": dict(roof(enc_ms), avg_ms=round(enc_ms, 4), lds=lds(enc_ms)),
            "decrypt": dict(roof(dec_ms), avg_ms=round(dec_ms, 4), lds=lds(dec_ms))}
    dom = "encrypt" if enc_ms >= dec_ms else "decrypt"
    roofline = dict(roof(enc_ms if dom == "encrypt" else dec_ms), kernel=dom, traffic=None)
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tfile):
        tr = json.load(open(tfile)).get(args.config, {}).get(dom)
        if tr:
            roofline["traffic"] = tr.get("bytes_per_launch")
            roofline["traffic_note"] = tr.get("note")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log("cpu baseline ...")
        cpu = cpu_baseline(args.config, npay, pb, ppk, main_res["d_ct"], torch, args.cpu_sample)
    main_res["d_ct"] = None
    torch.cuda.empty_cache()

    # The north star's other named packet sizes, at the same GPU count: MTU-sized
    # payloads (config B) and per-session keys (config D).  Reported beside the
    # headline config, never as `value`.
    packet_configs = {}
    for name in ([] if args.packet_configs == "none" else args.packet_configs.split(",")):
        if name == args.config or name not in CONFIGS:
            continue
        r = run_config(name, CONFIGS[name][0], args.packet_steps, args.packet_warmup, not args.no_verify)
        packet_configs[name] = {
            "value": round(r["value"], 2), "unit": "GiB/s", "ms_per_step": round(r["t"] / r["steps"] * 1e3, 4),
            "steps": r["steps"], "warmup": args.packet_warmup, "payloads_per_gpu": r["npay"], "payload_bytes": r["pb"],
            "payloads_per_key": r["ppk"], "encrypt_ms": round(r["enc_ms"], 4), "decrypt_ms": round(r["dec_ms"], 4),
            "hbm_frac_step": round(4.0 * r["nbytes"] / (r["t"] / r["steps"]) / 1e9 / HBM_PEAK_GBS, 4),
            "parity": r["parity"],
        }
        torch.cuda.empty_cache()

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "config %s: %d payloads x %d B per GPU (%.2f GiB), %s, encrypt+decrypt, "
                                   "device-resident, AES-128-CBC chain per payload from DefaultIV"
                                   % (args.config, npay, pb, nbytes / gib,
                                      ("%d payloads per session key" % ppk) if ppk else "1 key"),
                       "payloads_per_gpu": npay, "payload_bytes": pb, "parallelism": "payload shards x%d, "
                       "RCCL key broadcast" % world},
            "hbm_frac_step": round(4.0 * nbytes * world / (t / args.steps) / 1e9 / (HBM_PEAK_GBS * world), 4),
            "roofline": roofline, "kernels": kern, "cpu_baseline": cpu, "parity": parity,
            "packet_configs": packet_configs,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
