#!/usr/bin/env python3
"""bench.py -- device-resident AES-128-CBC encrypt+decrypt throughput on MI355X.

Metric (BASELINE.json): "AES encrypt+decrypt GiB/s device-resident (64 KiB
payloads); % HBM roofline @1/2/4/8 GPU".  Every payload is an independent
CBC chain from DefaultIV (the relay semantics of relay_local.cpp:206 /
relay_server.cpp:329,472).

Headline workload (default `--config E`, BASELINE.json configs[4], SURVEY.md
§8(d)): 8,388,608 payloads x 65,536 B = 512 GiB in total, processed in 32
fixed passes of 262,144 payloads (16 GiB, exactly config C's batch).  At N
GPUs, GPU g walks passes [g*32/N, (g+1)*32/N): the total is fixed and the
per-GPU pass size is the same at every N.  One step = one
walk of the whole E job: for each pass of the rank, the plaintext is written
into HBM (untimed: input staging, `fill_ms`), then one encrypt pass and one
decrypt pass run on it, timed between device synchronisations.
value = 2 x 512 GiB x steps / max over ranks of the summed timed seconds.
At N = 1 the rank walks all 32 passes, so the pass roofline is config C's.

Multi-GPU (torchrun, one process per GPU): rank 0 holds the session key and
broadcasts it over RCCL (xGMI); every rank expands it on its device and walks
its own passes.  No data-path collective.

`--config A|B|C|D` run one BASELINE.json config per GPU instead (weak
scaling: per-GPU batch fixed, payload range [rank*P, (rank+1)*P)).
packet_configs: configs A (the reference's own unit-test shape, 4,096 x
1,024 B, cyt_unit_crypt.cpp:173-248), B (1 M x 1,472 B) and D (4,096 session
keys x 256 x 1,472 B), measured after the headline at the same GPU count with
the same timing rules, each with its CPU baseline (all usable cores and one
core) at N = 1; reported beside `value`, never as it.

roofline: the kernels are bound by LDS gather issue, so
`bound` is "lds"; `frac` keeps the contract's definition (algorithmic bytes /
kernel time / 8 TB/s) and `ceiling` prices the binding unit: lookups per
clock per CU at the shader clock measured inside the kernels (a clock-probe
build of the same kernels, build/variants/clockprobe.so).

cpu_baseline: the oracle (a plain-C restatement of the reference's scalar
Rijndael, oracle/aes_oracle.c) on every usable host core (relay's
work_thread_counts = get_cpu_counts(), relay_local.cpp:475) on a bounded
sample of the same workload, rank 0 at N=1 only.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "AES encrypt+decrypt GiB/s device-resident (64 KiB payloads); % HBM roofline @1/2/4/8 GPU"
LOOKUPS_PER_BLOCK = 160      # 9 x 16 T-table + 16 S-box lookups (cyr_rijndael.cpp:659-704)
LDS_LANES_PER_CLK_CU = 32    # ds_read_b32: 2 cycles per wave64 instruction (MI355X_MICROARCH.md, LDS)
LDS_MEASURED_PEAK = 27.7     # back-to-back conflict-free ds_read_b32 microbench (profiles/r01/microbench.jsonl)
NUM_CUS = 256
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
HBM_COPY_CEILING_GBS = 6290.0  # measured float4 copy ceiling, same guide
PLAINTEXT_SEED = 0x5EEDC1C1
CONFIGS = {
    # name: (payloads per GPU, payload bytes, payloads per session key (0 = one key))
    "C": (262144, 65536, 0),
    "B": (1048576, 1472, 0),
    "D": (1048576, 1472, 256),
    "A": (4096, 1024, 0),
}
E_PASS_PAYLOADS, E_PASSES, E_PAYLOAD_BYTES = 262144, 32, 65536  # 32 x 2^18 = 2^23 payloads
MIXED_SEED = 0xFF00  # relay_stream.mixed layout (tests/golden/relay_mixed.json)
RELAY_MAX_CHUNK = 0xFF00


def mixed_stream_layout(total_bytes, seed=MIXED_SEED):
    """A relay tunnel stream of mixed packet sizes (relay_local.cpp:188-206):
    the client's socket delivers reads of r bytes (uniform in 1 .. 4 x 0xFF00,
    drawn with `seed`) until total_bytes are sent; each read goes out as chunks
    of min(rest, 0xFF00) bytes, each in a packet of a 4-B header, an 8-B
    RelayForwardMsg and the chunk rounded up to 16 B (encrypted in place),
    packets back to back.  Returns (payload offsets uint64, payload bytes
    uint32, stream bytes rounded up to 16)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    sizes, rest = [], total_bytes
    while rest > 0:
        r = min(rest, int(rng.integers(1, 4 * RELAY_MAX_CHUNK + 1)))
        rest -= r
        full, tail = divmod(r, RELAY_MAX_CHUNK)
        sizes += [RELAY_MAX_CHUNK] * full + ([tail] if tail else [])
    chunk = np.array(sizes, dtype=np.uint64)
    nbytes = ((chunk + 15) // 16 * 16).astype(np.uint32)
    pkt = nbytes.astype(np.uint64) + 12
    offsets = (np.cumsum(pkt) - pkt + 12).astype(np.uint64)
    return offsets, nbytes, int((int(pkt.sum()) + 15) // 16 * 16)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="E", choices=sorted(CONFIGS) + ["E"])
    ap.add_argument("--payloads", type=int, default=0, help="A-D: override payloads per GPU")
    ap.add_argument("--e-pass-payloads", type=int, default=E_PASS_PAYLOADS, help="E: payloads per pass")
    ap.add_argument("--e-passes", type=int, default=E_PASSES, help="E: passes in the whole job")
    ap.add_argument("--e-mode", default="duplex", choices=["duplex", "sequential"],
                    help="E: duplex = launch j encrypts pass j while it decrypts pass j-1 (cyaes_gpu_duplex_uniform); "
                         "sequential = an encrypt and a decrypt launch per pass")
    ap.add_argument("--cpu-sample", type=int, default=0, help="cpu baseline sample payloads (0 = auto)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-clock", action="store_true", help="skip the in-kernel clock measurement")
    ap.add_argument("--packet-configs", default="A,B,D",
                    help="other BASELINE.json packet configs measured after the headline one ('none' to skip)")
    ap.add_argument("--packet-steps", type=int, default=20)
    ap.add_argument("--relay-stream", type=int, default=1,
                    help="1: also time config B's payloads as an in-place relay packet stream (offset 12)")
    ap.add_argument("--packet-cpu-sample", type=int, default=0,
                    help="packet configs: payloads in the CPU-baseline sample (0 = auto: the whole 1,472-B batch)")
    ap.add_argument("--traffic", default="live", choices=["live", "file", "none"],
                    help="roofline.traffic: live = rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over config C "
                         "run as child processes in this run (rank 0, N=1); file = profiles/traffic.json")
    ap.add_argument("--e2e-gib", type=int, default=8,
                    help="rank 0 at N = 1, config E/C: GiB of 64 KiB payloads in pinned host memory streamed "
                         "H2D -> encrypt -> decrypt -> D2H for the `e2e` object (0 = skip)")
    ap.add_argument("--packet-warmup", type=int, default=20,
                    help="untimed steps before each packet config (a 1,472-B step is ~2 ms; 20 cover the clock "
                         "ramp, profiles/r01/packet_warmup.txt)")
    return ap.parse_args()


def traffic_plan(traffic, rank, world, config, environ):
    """(run the live traffic passes?, reason if not): rank 0 at N = 1 on the
    config C / E kernels, and never when this bench.py is itself being profiled
    (rocprofv3 sets ROCPROF_* for the program it runs): no nested passes."""
    if traffic != "live":
        return False, "not requested"
    if rank != 0 or world != 1 or config not in ("C", "E"):
        return False, "rank 0 at N = 1 on config C / E only"
    if any(k.startswith("ROCPROF_") for k in environ):
        return False, "running under rocprofv3: no nested profiler passes"
    return True, None


def live_traffic(timeout_s=150):
    """HBM bytes per AES launch, measured now: two rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE; one counter each, as MI355X_MICROARCH.md's
    HBM section prescribes) over `bench.py --config E --e-passes 2 --steps 1`
    (config C-sized passes: an encrypt launch, a duplex launch, a decrypt
    launch, plus the encrypt that leaves pass 0 for the e2e check), each a child
    process with its own time limit.  Corrections as tools/traffic.py: kB x1024,
    FETCH_SIZE x2 on gfx950.  Returns ({"encrypt": bytes, "decrypt": bytes,
    "duplex": bytes}, None) or (None, reason)."""
    import shutil
    import signal
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import traffic as tr
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    out = {}
    with tempfile.TemporaryDirectory(prefix="cyaes_pmc_") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            # rocprofv3 is a python script: run it with this interpreter, so the
            # only exec is rocprofv3's own of the profiled program
            cmd = [sys.executable, prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.join(ROOT, "bench.py"), "--config", "E", "--e-passes", "2", "--steps", "1",
                   "--warmup", "0", "--no-cpu", "--no-verify", "--no-clock", "--packet-configs", "none",
                   "--relay-stream", "0", "--e2e-gib", "0", "--traffic", "none"]
            env = dict(os.environ)
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                env.pop(k, None)
            proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=tmp, env=env,
                                    start_new_session=True)
            try:
                proc.wait(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
                return None, "rocprofv3 --pmc %s timed out" % counter
            if proc.returncode != 0:
                return None, "rocprofv3 --pmc %s exited %d" % (counter, proc.returncode)
            try:
                kb = tr.per_launch_kb(d, counter)
            except SystemExit as e:
                return None, str(e)
            for kind, v in kb.items():
                out.setdefault(kind, 0)
                out[kind] += int(round(v * 1024 * (2 if counter == "FETCH_SIZE" else 1)))
    return out, None


def session_keys(n):
    """Config D session keys: LE(splitmix64(S+2s)) || LE(splitmix64(S+2s+1))."""
    import struct
    seed = 0xC1C10E55D0000000

    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return x ^ (x >> 31)
    return b"".join(struct.pack("<QQ", sm(seed + 2 * s), sm(seed + 2 * s + 1)) for s in range(n))


def usable_cores():
    """(threads to use, facts): the CPUs this process may run on -- the affinity
    mask, capped by a cgroup CPU quota when one is set (a GPU box shares its
    host; nproc / os.cpu_count() show the whole machine)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return use, {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota}


def cpu_baseline(cfg_name, npay, pb, ppk, d_ct, torch, sample=0):
    """Oracle (scalar reference restatement) on the usable host cores; bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    threads, facts = usable_cores()
    # ~0.4 GiB of payload per thread (at most 8 GiB): ~2-4 s of CPU time per thread at ~0.2 GiB/s/core
    # per direction, a few seconds of wall time
    sample = min(npay, sample if sample > 0 else int(max(1, min(threads * (400 << 20), 8 << 30) // pb)))
    keys = [bytes(range(16))] if not ppk else [session_keys(sample // ppk + 1)[16 * s:16 * s + 16]
                                              for s in range(sample // ppk + 1)]
    pt = oracle.synthetic(0, sample, pb)
    # A small config (A: 4 MiB) is timed over repeats of the whole batch, at
    # least 256 MiB of payload per direction, so thread start-up does not dominate.
    reps = max(1, -(-(256 << 20) // (sample * pb)))
    t0 = time.perf_counter()
    for _ in range(reps):
        ct = oracle.batch(False, keys, ppk, pt, pb, nthreads=threads)
    t1 = time.perf_counter()
    for _ in range(reps):
        rt = oracle.batch(True, keys, ppk, ct, pb, nthreads=threads)
    t2 = time.perf_counter()
    # single-core figure on a smaller slice
    s1 = max(1, min(sample, (256 << 20) // pb))
    reps1 = max(1, -(-(32 << 20) // (s1 * pb)))
    t3 = time.perf_counter()
    for _ in range(reps1):
        ct1 = oracle.batch(False, keys, ppk, pt[:s1 * pb], pb, nthreads=1)
    t4 = time.perf_counter()
    for _ in range(reps1):
        oracle.batch(True, keys, ppk, ct1, pb, nthreads=1)
    t5 = time.perf_counter()
    torch.cuda.synchronize()
    gpu_sample = d_ct[: sample * pb].cpu().numpy()
    exact = bool(np.array_equal(gpu_sample, ct)) and bool(np.array_equal(rt, pt))
    gib = float(1 << 30)
    return dict({
        "value": round(2 * reps * sample * pb / (t2 - t0) / gib, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": "config %s: first %d payloads x %d B (%.2f GiB), encrypt then decrypt, %d threads = the usable "
                  "host cores (one Rijndael key schedule per thread, as relay's work threads, relay_local.cpp:475)%s; "
                  "oracle/aes_oracle.c" % (cfg_name, sample, pb, sample * pb / gib, threads,
                                           ", the whole batch %d times per direction" % reps if reps > 1 else ""),
        "single_core": round(2 * reps1 * s1 * pb / ((t4 - t3) + (t5 - t4)) / gib, 4),
        "repeats": reps,
        "seconds": round(t2 - t0, 3),
        "matches_gpu": exact,
    }, **facts)


LAUNCH_ENV = "CYAES_BENCH_LAUNCHER"          # set by the parent for the ranks it starts
TRAFFIC_ENV = "CYAES_BENCH_LIVE_TRAFFIC"     # the parent's live traffic result, JSON, for rank 0


def world_check(gpus, environ):
    """(world size, error): the ranks this process belongs to.  Under torchrun
    WORLD_SIZE must equal --gpus; without it the process is rank 0 of 1 (and
    for --gpus N > 1 it becomes the launcher of N ranks, see launcher_cmd)."""
    w = environ.get("WORLD_SIZE")
    if w is None:
        return 1, None
    if int(w) != gpus:
        return int(w), ("--gpus %d but WORLD_SIZE %s: refusing to time a different number of GPUs than "
                        "asked for" % (gpus, w))
    return int(w), None


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launcher_cmd(gpus, argv, port, python=sys.executable):
    """The child command `python bench.py --gpus N ...` runs when it is not
    already a torchrun rank: one process per GPU on this node, rendezvous on
    127.0.0.1, the same bench.py arguments."""
    return [python, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py")] + list(argv)


def launch_ranks(args, argv):
    """--gpus N > 1 without torchrun (the driver's `python3 bench.py --gpus N`):
    this process never touches the GPU.  It runs the live HBM-traffic passes
    first (child processes, one GPU), then starts torchrun with N ranks as a
    child process, hands the traffic result to rank 0 through the environment,
    forwards rank 0's JSON line (adding `launcher`) and exits with the child's
    return code."""
    import signal
    import subprocess
    env = dict(os.environ)
    run_passes, why = traffic_plan(args.traffic, 0, 1, args.config, os.environ)
    live = None
    if run_passes:
        log("hbm traffic: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (config C, one GPU) ...")
        live, why = live_traffic()
    env[TRAFFIC_ENV] = json.dumps({"traffic": live, "why": why})
    env[LAUNCH_ENV] = "bench.py"
    cmd = launcher_cmd(args.gpus, argv, free_port())
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True)

    def stop(signum, _frame):
        try:
            os.killpg(proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        raise SystemExit(128 + signum)
    old = {sig: signal.signal(sig, stop) for sig in (signal.SIGTERM, signal.SIGINT)}
    lines = 0
    for line in proc.stdout:
        text = line.strip()
        if text.startswith("{"):
            try:
                out = json.loads(text)
            except ValueError:
                out = None
            if isinstance(out, dict) and out.get("metric") == METRIC:
                out["launcher"] = {"kind": "bench.py -> torch.distributed.run child", "nproc_per_node": args.gpus}
                print(json.dumps(out), flush=True)
                lines += 1
                continue
        sys.stderr.write(line)
        sys.stderr.flush()
    rc = proc.wait()
    for sig, h in old.items():
        signal.signal(sig, h)
    if rc == 0 and lines != 1:
        log("error: the ranks exited 0 but printed %d result lines" % lines)
        rc = 1
    return rc


def run_e2e(ctx, torch, d_pt, d_ct, npay, pb, gib_cap, chunk=256 << 20):
    """`e2e` object: n = min(gib_cap GiB, this pass) payloads of pb bytes in
    pinned host memory (torch pin_memory = hipHostMalloc), streamed through
    cyaes_gpu_encrypt_host and cyaes_gpu_decrypt_host (H2D -> AES -> D2H on a
    ring of three device slot pairs), best of 3 after one untimed
    call; beside it the pinned copy ceilings of this box, measured in the same
    run (tools/linkprobe.py).  bit_exact: the host ciphertext equals the
    device-resident ciphertext of the same payloads (pass 0, checked against its
    OpenSSL digest earlier in this run) and the round trip restores the
    plaintext."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_e2e
    import linkprobe
    n = min(npay, max(1, (gib_cap << 30) // pb))
    nb = n * pb
    h_pt = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_ct = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_rt = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_pt.copy_(d_pt[:nb])
    t_e, t_d, ok = bench_e2e.measure(ctx, h_pt, h_ct, h_rt, n, pb, chunk, 3)
    piece = 1 << 30
    tmp = torch.empty(min(nb, piece), dtype=torch.uint8, device="cuda")
    for o in range(0, nb, piece):
        m = min(piece, nb - o)
        tmp[:m].copy_(h_ct[o:o + m])
        ok = ok and bool(torch.equal(tmp[:m], d_ct[o:o + m]))
    torch.cuda.synchronize()
    del tmp, h_pt, h_ct, h_rt
    link = linkprobe.measure(torch, min(nb, 4 << 30), chunk, 3)
    gib = float(1 << 30)
    encdec = 2 * nb / (t_e + t_d) / gib
    return {
        "unit": "GiB/s", "payloads": n, "payload_bytes": pb, "bytes": nb, "host_memory": "pinned",
        "path": "cyaes_gpu_encrypt_host then cyaes_gpu_decrypt_host: H2D -> AES -> D2H in %d MiB chunks, "
                "3 streams" % (chunk >> 20),
        "encrypt": round(nb / t_e / gib, 2), "decrypt": round(nb / t_d / gib, 2), "enc_plus_dec": round(encdec, 2),
        "link": link, "frac_of_duplex_link": round(encdec / link["duplex_gibs_per_direction"], 4),
        "bit_exact": ok,
    }


def main():
    args = parse()
    world, err = world_check(args.gpus, os.environ)
    if err:
        log("error: " + err)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.gpus < 1:
        log("error: --gpus must be >= 1")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # The traffic passes run first, before this process touches the GPU: each
    # is a child process (rocprofv3 starts the profiled bench.py by exec), and
    # no process that has initialised the GPU may be the parent of an exec chain.
    live, why = (None, "not requested")
    run_passes, why = traffic_plan(args.traffic, rank, world, args.config, os.environ)
    if TRAFFIC_ENV in os.environ:  # measured by the launching parent (launch_ranks)
        handed = json.loads(os.environ[TRAFFIC_ENV])
        run_passes = False
        if rank == 0:
            live, why = handed["traffic"], handed["why"] or "measured by the launching parent"
    if run_passes:
        log("hbm traffic: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (config C) ...")
        live, why = live_traffic()
    import torch
    import torch.distributed as dist

    # Rehearsal knobs for a 1-GPU box (never used by the driver): run every rank
    # on device 0 and use gloo instead of RCCL.
    device = 0 if os.environ.get("CYAES_BENCH_SAME_DEVICE") else local
    backend = os.environ.get("CYAES_DIST_BACKEND", "nccl")
    torch.cuda.set_device(device)
    # CYAES_BENCH_FORCE_DIST=1 initialises the process group even at world size 1,
    # so the driver's N>1 code path (RCCL init on the rank's device, key
    # broadcast, barriers, max-over-ranks all_reduce, shard all_gather) runs on a
    # one-GPU box (tests/test_config_e.py).
    dist_on = world > 1 or bool(os.environ.get("CYAES_BENCH_FORCE_DIST"))
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
        log("process group: backend %s, world %d, device %d" % (dist.get_backend(), dist.get_world_size(), device))
    # Which process group and which device each rank ran on, so the JSON line
    # alone shows RCCL (backend "nccl") saw N ranks on N distinct devices.
    props = torch.cuda.get_device_properties(device)
    dev_id = {"device": device, "pci": "%04x:%02x:%02x" % (props.pci_domain_id, props.pci_bus_id, props.pci_device_id),
              "uuid": str(getattr(props, "uuid", ""))}
    dist_info = {"backend": dist.get_backend() if dist_on else None,
                 "world_size": dist.get_world_size() if dist_on else 1}
    key_digest = {}  # digest of the session keys this rank received by broadcast (per config)

    import cyclone_amd as ca
    from cyclone_amd import dist as cdist

    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    ctx = ca.GpuContext(device)
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "openssl_vectors.json")))["configs"]
    gib = float(1 << 30)

    def max_over_ranks(x):
        v = torch.tensor([x], dtype=torch.float64, device="cuda")
        if dist_on:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v.item())

    def all_ok(ok):
        flag = torch.tensor([0 if ok else 1], device="cuda")
        if dist_on:
            dist.all_reduce(flag)
        return int(flag.item()) == 0

    def set_session_keys(p0, npay, ppk):
        # Session key(s): rank 0 owns them (the relay's DH secret), RCCL-broadcast
        # over xGMI straight into device memory; each GPU expands its own sessions.
        nkeys = cdist.session_range(0, npay * world, ppk)[1]
        d_keys = cdist.broadcast_keys((session_keys(nkeys) if ppk else bytes(range(16))) if rank == 0 else None,
                                      nkeys, "cuda")
        key_digest["last"] = hashlib.sha256(d_keys.cpu().numpy().tobytes()).hexdigest()[:16]
        k0, nk = cdist.session_range(p0, npay, ppk)
        ctx.set_keys_device(d_keys[16 * k0: 16 * (k0 + nk)].contiguous(), nk, sh)

    def digests_match(g, d_pt, d_ct, nbytes):
        return (["%016x" % v for v in ctx.digest(d_ct, nbytes, sh)] == g["cipher_digest"] and
                ["%016x" % v for v in ctx.digest(d_pt, nbytes, sh)] == g["plain_digest"])

    def run_config(name, npay, steps, warmup, verify, keep_cipher=False):
        """One config of A-D, timed as the contract says; returns a result dict
        (rank-local kernel times, max-over-ranks wall time)."""
        _, pb, ppk = CONFIGS[name]
        nbytes = npay * pb
        p0, npay = cdist.weak_shard(npay, rank)
        set_session_keys(p0, npay, ppk)
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
        shard = dict({"rank": rank, "p0": p0, "npayloads": npay, "keys_sha256_16": key_digest["last"]}, **dev_id)
        if verify:
            ok = ctx.digest(d_rt, nbytes, sh) == ctx.digest(d_pt, nbytes, sh)
            g = golden.get(name) if rank == 0 else None
            if g and g["npayloads"] == npay and g["payload_bytes"] == pb and g["p0"] == p0:
                ok = ok and digests_match(g, d_pt, d_ct, nbytes)
                shard["golden_verified"] = True
            ok = ok and ctx.check() == ca.CYAES_OK
            parity = "bit-exact" if all_ok(ok) else "MISMATCH"
            # this rank's cipher digest, for checks of shards no golden covers (tests/test_config_e.py)
            shard["cipher_digest"] = ["%016x" % v for v in ctx.digest(d_ct, nbytes, sh)]
            log("config %s parity: %s" % (name, parity))
        shards = [shard]
        if dist_on:
            shards = [None] * world
            dist.all_gather_object(shards, shard)

        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if dist_on:
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
        if dist_on:
            dist.barrier()
        t1 = time.perf_counter()
        t = max_over_ranks(t1 - t0)
        res = {
            "name": name, "npay": npay, "pb": pb, "ppk": ppk, "nbytes": nbytes, "t": t, "steps": steps,
            "value": 2.0 * nbytes * steps * world / t / gib,
            "enc_ms": sum(a.elapsed_time(b) for a, b, _ in ev) / steps,
            "dec_ms": sum(b.elapsed_time(c) for _, b, c in ev) / steps,
            "parity": parity, "d_ct": d_ct if keep_cipher else None, "d_pt": d_pt if keep_cipher else None,
            "shards": shards,
        }
        del d_rt
        if not keep_cipher:
            del d_ct, d_pt
        return res

    def run_mixed_stream():
        """relay_stream.mixed: config B's bytes as a relay tunnel stream of
        mixed packet sizes (mixed_stream_layout: full 0xFF00 chunks and the
        reads' tails, relay_local.cpp:188-206), encrypted then decrypted in
        place through the ragged entry points (device offset / size lists), as
        the relay's sender (relay_local.cpp:206) and receiver
        (relay_server.cpp:329) would hand a parsed stream over.  Every GPU the
        same stream (weak scaling).  Parity: digests of the whole stream buffer
        against tests/golden/relay_mixed.json (oracle-derived)."""
        import numpy as np
        offsets, nbytes, alloc = mixed_stream_layout(CONFIGS["B"][0] * CONFIGS["B"][1])
        n = int(offsets.size)
        payload = int(nbytes.sum())
        set_session_keys(0, 1, 0)
        mbuf = torch.empty(alloc, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(offsets.astype(np.int64)).to("cuda")
        d_nb = torch.from_numpy(nbytes.astype(np.int32)).to("cuda")
        ctx.fill_synthetic(mbuf, 0, alloc // 16, 16, PLAINTEXT_SEED, sh)

        def dig():
            return ["%016x" % v for v in ctx.digest(mbuf, alloc, sh)]

        def m_enc():
            ctx.encrypt_ragged(mbuf, mbuf, d_off, d_nb, n, stream=sh)

        def m_dec():
            ctx.decrypt_ragged(mbuf, mbuf, d_off, d_nb, n, stream=sh)
        mpar = None
        if not args.no_verify:
            gm = json.load(open(os.path.join(ROOT, "tests", "golden", "relay_mixed.json")))
            ok = gm["packets"] == n and gm["stream_bytes"] == alloc and dig() == gm["plain_digest"]
            m_enc()
            ok = ok and ctx.check() == ca.CYAES_OK and dig() == gm["cipher_digest"]
            m_dec()
            ok = ok and ctx.check() == ca.CYAES_OK and dig() == gm["plain_digest"]
            mpar = "bit-exact" if all_ok(ok) else "MISMATCH"
        for _ in range(args.packet_warmup):
            m_enc()
            m_dec()
        mev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                torch.cuda.Event(enable_timing=True)) for _ in range(args.packet_steps)]
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.packet_steps):
            mev[i][0].record(stream)
            m_enc()
            mev[i][1].record(stream)
            m_dec()
            mev[i][2].record(stream)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        mt = max_over_ranks(time.perf_counter() - t0)
        # duplex: this stream encrypted while a second one (its ciphertext) is
        # decrypted, cyaes_gpu_duplex_ragged, against the two calls back to back
        mbuf2 = torch.empty_like(mbuf)
        ctx.fill_synthetic(mbuf, 0, alloc // 16, 16, PLAINTEXT_SEED, sh)
        ctx.fill_synthetic(mbuf2, 0, alloc // 16, 16, PLAINTEXT_SEED, sh)
        ctx.encrypt_ragged(mbuf2, mbuf2, d_off, d_nb, n, stream=sh)

        def m_dup():
            ctx.duplex_ragged(mbuf, mbuf, d_off, d_nb, n, mbuf2, mbuf2, d_off, d_nb, n, stream=sh)
        dpar = None
        if not args.no_verify:
            m_dup()
            ok = ctx.check() == ca.CYAES_OK and dig() == gm["cipher_digest"]
            ok = ok and ["%016x" % v for v in ctx.digest(mbuf2, alloc, sh)] == gm["plain_digest"]
            dpar = "bit-exact" if all_ok(ok) else "MISMATCH"

        def two():
            m_enc()
            m_dec()
        dup_t = {}
        for _ in range(args.packet_warmup):
            m_dup()
        for rnd in range(2):  # alternate order against the clock ramp
            for name, fn in ((("two", two), ("duplex", m_dup)) if rnd == 0 else (("duplex", m_dup), ("two", two))):
                if dist_on:
                    dist.barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(args.packet_steps):
                    fn()
                torch.cuda.synchronize()
                dup_t.setdefault(name, []).append(max_over_ranks(time.perf_counter() - t1) / args.packet_steps)
        t_two, t_dup = min(dup_t["two"]), min(dup_t["duplex"])
        duplex = {"ms": round(1e3 * t_dup, 4), "two_calls_ms": round(1e3 * t_two, 4),
                  "value": round(2.0 * payload * world / t_dup / gib, 2), "unit": "GiB/s",
                  "speedup": round(t_two / t_dup, 4), "parity": dpar,
                  "note": "encrypt this stream while its ciphertext copy is decrypted (cyaes_gpu_duplex_ragged: packed "
                          "encrypt, decrypt on the context's second stream) vs encrypt_ragged + decrypt_ragged; "
                          "best of two rounds in alternating order, %d steps each" % args.packet_steps}
        del mbuf2
        out = {
            "value": round(2.0 * payload * args.packet_steps * world / mt / gib, 2), "unit": "GiB/s",
            "encrypt_ms": round(sum(a.elapsed_time(b) for a, b, _ in mev) / args.packet_steps, 4),
            "decrypt_ms": round(sum(b.elapsed_time(c) for _, b, c in mev) / args.packet_steps, 4),
            "parity": mpar, "packets": n, "payload_bytes": payload,
            "full_chunks": int((nbytes == RELAY_MAX_CHUNK).sum()),
            "layout": "config B's %d bytes as relay chunks: socket reads uniform in 1..4 x 0xFF00 B, each sent as "
                      "0xFF00-B chunks plus its tail, payload = chunk rounded to 16 at packet offset 12, packets back "
                      "to back, in place, cyaes_gpu_{en,de}crypt_ragged" % (CONFIGS["B"][0] * CONFIGS["B"][1]),
            "parity_note": "digest of the whole stream buffer vs tests/golden/relay_mixed.json (oracle)",
            "duplex": duplex,
        }
        del mbuf, d_off, d_nb
        torch.cuda.empty_cache()
        return out

    def run_e(steps, warmup, verify):
        """Config E: the whole job's fixed passes, this rank's share (see module doc)."""
        pp, passes, pb = args.e_pass_payloads, args.e_passes, E_PAYLOAD_BYTES
        if passes % world:
            raise SystemExit("config E: %d passes do not split over %d ranks" % (passes, world))
        mine = list(range(rank * passes // world, (rank + 1) * passes // world))
        nbytes = pp * pb
        duplex = args.e_mode == "duplex"
        set_session_keys(0, pp, 0)
        log("rank %d/%d: config E, passes %d..%d of %d, %d payloads x %d B = %.2f GiB per pass, %d CUs, %s launches"
            % (rank, world, mine[0], mine[-1], passes, pp, pb, nbytes / gib, ctx.num_cus, args.e_mode))
        d_pt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        d_cts = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(2 if duplex else 1)]
        d_rt = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        gfile = os.path.join(ROOT, "tests", "golden", "config_e_passes.json")
        gpass = {}
        if os.path.exists(gfile):
            for layout in json.load(open(gfile)).values():
                if isinstance(layout, dict) and layout.get("pass_payloads") == pp:
                    gpass = {g["pass"]: g for g in layout["passes"]}

        def fill(i):
            ctx.fill_synthetic(d_pt, i * pp, pp, pb, PLAINTEXT_SEED, sh)

        def walk(ev, verify_walk):
            """One walk of this rank's passes.  Sequential: per pass, an encrypt
            launch and a decrypt launch.  Duplex: launch j encrypts pass j while
            it decrypts pass j-1 (cyaes_gpu_duplex_uniform; the two directions of
            a relay pipe, relay_server.cpp:472 / :329), plus a decrypt-only
            launch after the last pass.  Each pass's plaintext is written into
            HBM first (untimed input staging); every launch is timed between
            device synchronisations.  Returns (timed s, fill s, verified passes, ok)."""
            t_aes = t_fill = 0.0
            verified, ok = [], True
            prev = None  # (pass, its ciphertext buffer, its plaintext digest)

            def timed(*launches):  # (kind, fn) ...: back to back, one timed segment
                nonlocal t_aes
                torch.cuda.synchronize()
                a0 = time.perf_counter()
                for rec, fn in launches:
                    if ev is not None:
                        ev.append((rec, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                        ev[-1][1].record(stream)
                    fn()
                    if ev is not None:
                        ev[-1][2].record(stream)
                torch.cuda.synchronize()
                t_aes += time.perf_counter() - a0

            for j, i in enumerate(mine):
                f0 = time.perf_counter()
                fill(i)  # input staging: the pass's payloads arrive in HBM (untimed)
                torch.cuda.synchronize()
                t_fill += time.perf_counter() - f0
                pdig = ctx.digest(d_pt, nbytes, sh) if verify_walk else None
                ct = d_cts[j % len(d_cts)]
                if duplex and prev is not None:
                    pct = prev[1]
                    timed(("duplex", lambda: ctx.duplex_uniform(d_pt, ct, pp, pb, pct, d_rt, pp, pb, stream=sh)))
                elif duplex:
                    timed(("encrypt", lambda: ctx.encrypt_uniform(d_pt, ct, pp, pb, stream=sh)))
                else:
                    timed(("encrypt", lambda: ctx.encrypt_uniform(d_pt, ct, pp, pb, stream=sh)),
                          ("decrypt", lambda: ctx.decrypt_uniform(ct, d_rt, pp, pb, stream=sh)))
                if verify_walk:
                    good = True
                    if duplex and prev is not None:  # the previous pass came back in this launch
                        good = ctx.digest(d_rt, nbytes, sh) == prev[2]
                    elif not duplex:
                        good = ctx.digest(d_rt, nbytes, sh) == pdig
                    if i in gpass:
                        good = good and digests_match(gpass[i], d_pt, ct, nbytes)
                        if good:
                            verified.append(i)
                    ok = ok and good
                prev = (i, ct, pdig)
            if duplex:  # the last pass's decrypt
                pct = prev[1]
                timed(("decrypt", lambda: ctx.decrypt_uniform(pct, d_rt, pp, pb, stream=sh)))
                if verify_walk:
                    ok = ok and ctx.digest(d_rt, nbytes, sh) == prev[2]
            return t_aes, t_fill, verified, ok

        verified, ok = [], True
        for w in range(max(warmup, 1 if verify else 0)):
            _, _, v, good = walk(None, verify and w == 0)
            if verify and w == 0:
                verified, ok = v, good
        torch.cuda.synchronize()
        parity = None
        if verify:
            ok = ok and ctx.check() == ca.CYAES_OK
            parity = "bit-exact" if all_ok(ok) else "MISMATCH"
            log("config E parity: %s (golden passes verified on rank %d: %s)" % (parity, rank, verified))

        ev = []
        t_aes, t_fill = 0.0, 0.0
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t_begin = time.perf_counter()
        for _ in range(steps):
            ta, tf, _, _ = walk(ev, False)
            t_aes += ta
            t_fill += tf
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        t_wall = time.perf_counter() - t_begin
        t = max_over_ranks(t_aes)
        shard = dict({"rank": rank, "passes": mine, "golden_verified": verified,
                      "keys_sha256_16": key_digest["last"]}, **dev_id)
        shards = [shard]
        if dist_on:
            shards = [None] * world
            dist.all_gather_object(shards, shard)

        def avg(kind):
            v = [a.elapsed_time(b) for k, a, b in ev if k == kind]
            return sum(v) / len(v) if v else None
        res = {
            "name": "E", "npay": pp, "pb": pb, "ppk": 0, "nbytes": nbytes, "t": t, "steps": steps,
            "value": 2.0 * nbytes * passes * steps / t / gib,
            "enc_ms": avg("encrypt"), "dec_ms": avg("decrypt"), "duplex_ms": avg("duplex"),
            "launches": {k: sum(1 for e in ev if e[0] == k) // steps for k in ("encrypt", "decrypt", "duplex")},
            "parity": parity, "d_ct": d_cts[0], "d_pt": d_pt, "passes_per_gpu": len(mine), "passes": passes,
            "fill_ms": max_over_ranks(t_fill) / steps * 1e3, "wall_ms": max_over_ranks(t_wall) / steps * 1e3,
            "shards": shards,
        }
        # leave pass 0's plaintext and cipher in d_pt / d_cts[0] for the e2e check and the cpu
        # baseline sample (rank 0 walks pass 0 at every N)
        if rank == 0 and mine[0] == 0:
            fill(0)
            ctx.encrypt_uniform(d_pt, d_cts[0], pp, pb, stream=sh)
        del d_rt
        return res

    if args.config == "E":
        main_res = run_e(args.steps, args.warmup, not args.no_verify)
    else:
        main_res = run_config(args.config, args.payloads or CONFIGS[args.config][0], args.steps, args.warmup,
                              not args.no_verify, keep_cipher=True)
    nbytes, pb, ppk = main_res["nbytes"], main_res["pb"], main_res["ppk"]
    npay, t, value = main_res["npay"], main_res["t"], main_res["value"]
    enc_ms, dec_ms, parity = main_res["enc_ms"], main_res["dec_ms"], main_res["parity"]
    dup_ms = main_res.get("duplex_ms")  # config E in duplex mode: the launches that hold 32/N - 1 of the passes

    # In-kernel shader clock under this load: the clock-probe build of the same
    # kernels on the same buffers (s_memtime cycles / s_memrealtime 100 MHz ticks
    # per wave, tools/clockcal.hip).  Untimed; measurement only.
    clock = None
    probe_path = os.path.join(ROOT, "build", "variants", "clockprobe.so")
    if not args.no_clock and os.path.exists(probe_path) and main_res.get("d_pt") is not None:
        import ctypes
        plib = ca.load_library(probe_path)
        pctx = ca.GpuContext(device, lib=plib)
        if ppk:
            pctx.set_keys(session_keys((npay + ppk - 1) // ppk))
        else:
            pctx.set_keys(bytes(range(16)))
        d_tmp = torch.empty_like(main_res["d_ct"])
        buf = (ctypes.c_ulonglong * 8)()
        for r in range(4):
            pctx.encrypt_uniform(main_res["d_pt"], d_tmp, npay, pb, payloads_per_key=ppk, stream=sh)
            pctx.decrypt_uniform(d_tmp, d_tmp, npay, pb, payloads_per_key=ppk, stream=sh)
            torch.cuda.synchronize()
            if r == 0:
                plib.cyaes_debug_probe(buf)  # first launch: clock ramp; discard
        plib.cyaes_debug_probe(buf)
        clock = {k: (buf[4 * i] / buf[4 * i + 1] * 0.1 if buf[4 * i + 1] else None)
                 for i, k in enumerate(("encrypt", "decrypt"))}
        if dup_ms:  # the duplex launch: its encrypt and decrypt phases together, cycles over ticks
            d_ct2 = torch.empty_like(d_tmp)
            for r in range(3):
                pctx.encrypt_uniform(main_res["d_pt"], d_tmp, npay, pb, stream=sh)  # the decrypt half's input
                torch.cuda.synchronize()
                plib.cyaes_debug_probe(buf)  # (discarded)
                pctx.duplex_uniform(main_res["d_pt"], d_ct2, npay, pb, d_tmp, d_tmp, npay, pb, stream=sh)
                torch.cuda.synchronize()
                plib.cyaes_debug_probe(buf)  # this duplex launch: kind 0 its encrypt phase, kind 1 its decrypt
            cyc, tick = buf[0] + buf[4], buf[1] + buf[5]
            clock["duplex"] = cyc / tick * 0.1 if tick else None
            del d_ct2
        pctx.close()
        del d_tmp

    def roof(ms, nb=nbytes):
        ach = 2.0 * nb / (ms / 1e3) / 1e9  # algorithmic: read N + write N per launch
        return {"bound": "lds", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "frac_vs_copy_ceiling": round(ach / HBM_COPY_CEILING_GBS, 4)}

    def ceiling(ms, ghz, nb=nbytes):
        # The binding on-chip resource: 160 conflict-free
        # ds_read_b32 lookups per 16-B block, issued at 32 lanes/clk/CU.
        look = LOOKUPS_PER_BLOCK * (nb / 16) / (ms / 1e3)
        out = {"unit": "LDS lookups/clk/CU", "lookups_per_s": float("%.4g" % look),
               "peak_nominal": LDS_LANES_PER_CLK_CU, "peak_microbench": LDS_MEASURED_PEAK,
               "frac_at_2p4ghz": round(look / (LDS_LANES_PER_CLK_CU * NUM_CUS * 2.4e9), 4)}
        if ghz:
            per_clk = look / (NUM_CUS * ghz * 1e9)
            out.update(clock_ghz=round(ghz, 3), clock_source="in-kernel s_memtime/s_memrealtime, clockprobe.so",
                       achieved=round(per_clk, 2), frac=round(per_clk / LDS_LANES_PER_CLK_CU, 4))
        return out

    # Per kernel: algorithmic bytes per launch (encrypt / decrypt: N read + N
    # written; duplex: both, 4N) over its average launch time (HIP events on the
    # launch stream).  Config E in duplex mode: the duplex launches carry 31 of
    # 32 passes' work, so they are the dominant kernel.
    launches = [("encrypt", enc_ms, 1), ("decrypt", dec_ms, 1)] + ([("duplex", dup_ms, 2)] if dup_ms else [])
    kern = {k: dict(roof(ms, nbytes * m), avg_ms=round(ms, 4), algorithmic_bytes=int(2 * nbytes * m),
                    ceiling=ceiling(ms, (clock or {}).get(k), nbytes * m))
            for k, ms, m in launches if ms}
    dom = "duplex" if dup_ms else ("encrypt" if enc_ms >= dec_ms else "decrypt")
    roofline = dict(roof(kern[dom]["avg_ms"], nbytes * (2 if dup_ms else 1)), kernel=dom, traffic=None,
                    ceiling=kern[dom]["ceiling"])
    tfile = os.path.join(ROOT, "profiles", "traffic.json")
    ftr = None
    if os.path.exists(tfile):
        ftr = json.load(open(tfile)).get("C" if args.config == "E" else args.config, {}).get(dom)
    if live and dom in live:
        algo1 = 2.0 * CONFIGS["C"][0] * CONFIGS["C"][1]  # the passes profile config C-sized launches (live_traffic)
        algo = {"duplex": 2 * algo1}
        roofline["traffic"] = live[dom]
        roofline["traffic_note"] = ("measured in this run: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate "
                                    "child processes, bench.py --config E --e-passes 2, i.e. config C-sized launches: "
                                    "an encrypt, a duplex, a decrypt), FETCH_SIZE x2 per the gfx950 calibration, "
                                    "x1024 kB->B; per launch of the dominant kernel")
        roofline["traffic_ratio"] = round(live[dom] / algo.get(dom, algo1), 4)
        for k in kern:
            if k in live:
                kern[k]["traffic"] = live[k]
                kern[k]["traffic_ratio"] = round(live[k] / algo.get(k, algo1), 4)
    elif ftr and args.traffic != "none":
        roofline["traffic"] = ftr.get("bytes_per_launch")
        roofline["traffic_note"] = "committed profiles/traffic.json (%s); " % (why,) + str(ftr.get("note"))

    # End to end, PCIe-inclusive (north_star: "the end-to-end rate including
    # hipMemcpyAsync to and from the device over pinned staging buffers"):
    # the path starts and ends in host memory (relay_local.cpp:188-217: socket
    # buffer -> encrypt -> send).  Rank 0 at N = 1, after the timed region.
    e2e = None
    if (rank == 0 and world == 1 and args.e2e_gib > 0 and pb == E_PAYLOAD_BYTES and not ppk
            and main_res.get("d_ct") is not None):
        log("e2e: host -> device -> host ...")
        e2e = run_e2e(ctx, torch, main_res["d_pt"], main_res["d_ct"], npay, pb, args.e2e_gib)

    cpu = None
    if rank == 0 and not args.no_cpu:
        log("cpu baseline ...")
        cpu = cpu_baseline("C (= config E pass 0)" if args.config == "E" else args.config, npay, pb, ppk,
                           main_res["d_ct"], torch, args.cpu_sample)
    main_res["d_ct"] = main_res["d_pt"] = None
    torch.cuda.empty_cache()

    # The other BASELINE.json configs, at the same GPU count: the reference's
    # unit-test shape (config A), MTU-sized payloads (config B) and per-session
    # keys (config D).  Reported beside the
    # headline config, never as `value`.
    packet_configs = {}
    for name in ([] if args.packet_configs == "none" else args.packet_configs.split(",")):
        if name == args.config or name not in CONFIGS:
            continue
        want_cpu = rank == 0 and world == 1 and not args.no_cpu
        r = run_config(name, CONFIGS[name][0], args.packet_steps, args.packet_warmup, not args.no_verify,
                       keep_cipher=want_cpu)
        pcpu = None
        if want_cpu:  # the same config on the host cores, same run, a bounded sample
            log("cpu baseline %s ..." % name)
            pcpu = cpu_baseline(name, r["npay"], r["pb"], r["ppk"], r["d_ct"], torch, args.packet_cpu_sample)
            r["d_ct"] = r["d_pt"] = None
        packet_configs[name] = {
            "value": round(r["value"], 2), "unit": "GiB/s", "ms_per_step": round(r["t"] / r["steps"] * 1e3, 4),
            "steps": r["steps"], "warmup": args.packet_warmup, "payloads_per_gpu": r["npay"], "payload_bytes": r["pb"],
            "payloads_per_key": r["ppk"], "encrypt_ms": round(r["enc_ms"], 4), "decrypt_ms": round(r["dec_ms"], 4),
            "hbm_frac_step": round(4.0 * r["nbytes"] / (r["t"] / r["steps"]) / 1e9 / HBM_PEAK_GBS, 4),
            "parity": r["parity"], "shards": r["shards"], "cpu_baseline": pcpu,
        }
        torch.cuda.empty_cache()

    # Relay packet stream in HBM: config B's payloads at
    # packet offset 12 with a 12-B gap per packet (stride 1,484 B, 4-B aligned
    # payloads, relay_local.cpp:189-206), encrypted then decrypted in place with
    # the runtime's default kernel choice, through the strided entry points (the
    # payloads are equally strided) and, as `ragged`, the ragged ones.  Reported
    # beside the headline, never as `value`.
    relay = None
    if args.relay_stream and "B" in CONFIGS:
        rn, rpb, _ = CONFIGS["B"]
        hdr, stride = 12, CONFIGS["B"][1] + 12
        p0, rn = cdist.weak_shard(rn, rank)
        set_session_keys(p0, rn, 0)
        d_pt = torch.empty(rn * rpb, dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic(d_pt, p0, rn, rpb, PLAINTEXT_SEED, sh)
        buf = torch.full((rn * stride + 16,), 0xA5, dtype=torch.uint8, device="cuda")
        view = buf[: rn * stride].view(rn, stride)
        view[:, hdr:hdr + rpb] = d_pt.view(rn, rpb)
        d_off = torch.arange(rn, dtype=torch.int64, device="cuda") * stride + hdr
        d_nb = torch.full((rn,), rpb, dtype=torch.int32, device="cuda")

        # The receiver's integration: parse the stream (cyaes_relay_parse /
        # cyaes_relay_payloads) and, when the payloads are equally strided, as a
        # stream of MTU packets is, run the strided entry points; the ragged ones
        # (device offset and size lists) otherwise.  Both are timed.
        apis = {
            "strided": (lambda: ctx.encrypt_strided(buf, buf, hdr, stride, rn, rpb, stream=sh),
                        lambda: ctx.decrypt_strided(buf, buf, hdr, stride, rn, rpb, stream=sh)),
            "ragged": (lambda: ctx.encrypt_ragged(buf, buf, d_off, d_nb, rn, stream=sh),
                       lambda: ctx.decrypt_ragged(buf, buf, d_off, d_nb, rn, stream=sh)),
        }
        relay = {}
        for api, (r_enc, r_dec) in apis.items():
            rpar = None
            if not args.no_verify:
                view[:, hdr:hdr + rpb] = d_pt.view(rn, rpb)
                r_enc()
                ok = ctx.check() == ca.CYAES_OK
                g = golden.get("B") if rank == 0 else None
                if g and g["npayloads"] == rn and g["p0"] == p0:
                    ct = view[:, hdr:hdr + rpb].contiguous()
                    ok = ok and ["%016x" % v for v in ctx.digest(ct, rn * rpb, sh)] == g["cipher_digest"]
                    del ct
                r_dec()
                ok = ok and ctx.check() == ca.CYAES_OK and bool(torch.equal(view[:, hdr:hdr + rpb].reshape(-1), d_pt))
                ok = ok and bool((view[:, :hdr] == 0xA5).all())
                rpar = "bit-exact" if all_ok(ok) else "MISMATCH"
            for _ in range(args.packet_warmup):
                r_enc()
                r_dec()
            rev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                    torch.cuda.Event(enable_timing=True)) for _ in range(args.packet_steps)]
            if dist_on:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.packet_steps):
                rev[i][0].record(stream)
                r_enc()
                rev[i][1].record(stream)
                r_dec()
                rev[i][2].record(stream)
            torch.cuda.synchronize()
            if dist_on:
                dist.barrier()
            rt = max_over_ranks(time.perf_counter() - t0)
            relay[api] = {
                "value": round(2.0 * rn * rpb * args.packet_steps * world / rt / gib, 2), "unit": "GiB/s",
                "encrypt_ms": round(sum(a.elapsed_time(b) for a, b, _ in rev) / args.packet_steps, 4),
                "decrypt_ms": round(sum(b.elapsed_time(c) for _, b, c in rev) / args.packet_steps, 4),
                "parity": rpar,
            }
        # Both directions of a relay end at once (relay_server.cpp:472 encrypts
        # target -> tunnel while :329 decrypts tunnel -> target): the sent stream
        # encrypted while the received one is decrypted, one launch per step
        # (cyaes_gpu_duplex_strided) against the two strided calls above.
        buf2 = torch.full_like(buf, 0xA5)
        view2 = buf2[: rn * stride].view(rn, stride)
        view2[:, hdr:hdr + rpb] = d_pt.view(rn, rpb)
        ctx.encrypt_strided(buf2, buf2, hdr, stride, rn, rpb, stream=sh)  # the received stream: ciphertext

        def r_dup():
            ctx.duplex_strided(buf, buf, hdr, stride, rn, rpb, buf2, buf2, hdr, stride, rn, rpb, stream=sh)
        dpar = None
        if not args.no_verify:
            view[:, hdr:hdr + rpb] = d_pt.view(rn, rpb)
            ct2 = view2[:, hdr:hdr + rpb].contiguous()
            r_dup()
            ok = ctx.check() == ca.CYAES_OK and bool(torch.equal(view[:, hdr:hdr + rpb], ct2))
            ok = ok and bool(torch.equal(view2[:, hdr:hdr + rpb].reshape(-1), d_pt))
            ok = ok and bool((view[:, :hdr] == 0xA5).all()) and bool((view2[:, :hdr] == 0xA5).all())
            g = golden.get("B") if rank == 0 else None
            if g and g["npayloads"] == rn and g["p0"] == p0:
                ok = ok and ["%016x" % v for v in ctx.digest(ct2, rn * rpb, sh)] == g["cipher_digest"]
            del ct2
            dpar = "bit-exact" if all_ok(ok) else "MISMATCH"
        for _ in range(args.packet_warmup):
            r_dup()
        dev_ = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.packet_steps)]
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.packet_steps):
            dev_[i][0].record(stream)
            r_dup()
            dev_[i][1].record(stream)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        dt = max_over_ranks(time.perf_counter() - t0)
        relay["duplex"] = {
            "value": round(2.0 * rn * rpb * args.packet_steps * world / dt / gib, 2), "unit": "GiB/s",
            "ms_per_step": round(sum(a.elapsed_time(b) for a, b in dev_) / args.packet_steps, 4),
            "parity": dpar,
            "api": "cyaes_gpu_duplex_strided: one stream of the layout encrypted while a second one is decrypted, "
                   "one launch (+ its prepass) per step; compare encrypt_ms + decrypt_ms of the strided calls",
        }
        del buf2, view2
        relay = dict(relay["strided"], ragged=relay["ragged"], duplex=relay["duplex"],
                     api="cyaes_gpu_{en,de}crypt_strided "
                     "(cyaes_relay_stride finds the stream equally strided); `ragged`: the same stream through "
                     "cyaes_gpu_{en,de}crypt_ragged with device offset / size lists",
                     layout="config B payloads (%d x %d B per GPU) at packet offset %d, packet stride %d B, in place"
                            % (rn, rpb, hdr, stride),
                     steps=args.packet_steps, warmup=args.packet_warmup,
                     parity_note="gathered ciphertext digest vs config B's OpenSSL digest (rank 0 shard); "
                                 "headers untouched; decrypt restores the plaintext")
        del buf, view, d_pt, d_off, d_nb
        torch.cuda.empty_cache()
        relay["mixed"] = run_mixed_stream()

    if rank == 0:
        if args.config == "E":
            P = main_res["passes"]
            workload = ("config E: %d payloads x %d B in total (%.0f GiB), %d fixed passes of %d payloads "
                        "(%.2f GiB%s); %d GPU(s) x %d passes each, 1 key RCCL-broadcast, "
                        "encrypt+decrypt, device-resident, AES-128-CBC chain per payload from DefaultIV"
                        % (P * npay, pb, P * nbytes / gib, P, npay, nbytes / gib,
                           ", config C's batch" if npay == E_PASS_PAYLOADS else ", reduced", world, P // world))
            step_bytes = P * nbytes
        else:
            workload = ("config %s: %d payloads x %d B per GPU (%.2f GiB), %s, encrypt+decrypt, device-resident, "
                        "AES-128-CBC chain per payload from DefaultIV"
                        % (args.config, npay, pb, nbytes / gib,
                           ("%d payloads per session key" % ppk) if ppk else "1 key"))
            step_bytes = nbytes * world
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if args.config == "E" else "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": workload, "payloads_per_pass" if args.config == "E" else "payloads_per_gpu": npay,
                       "payload_bytes": pb, "parallelism": "payload shards x%d, RCCL key broadcast" % world},
            "hbm_frac_step": round(4.0 * step_bytes / (t / args.steps) / 1e9 / (HBM_PEAK_GBS * world), 4),
            "roofline": roofline, "kernels": kern, "cpu_baseline": cpu, "parity": parity,
            "packet_configs": packet_configs, "relay_stream": relay, "e2e": e2e,
        }
        out["shards"] = main_res["shards"]
        out["dist"] = dict(dist_info, ranks_reporting=len(main_res["shards"]),
                           distinct_devices=len({(sh["pci"], sh["uuid"]) for sh in main_res["shards"]}),
                           same_keys_all_ranks=len({sh["keys_sha256_16"] for sh in main_res["shards"]}) == 1)
        if args.config == "E":
            out["config"].update(passes=main_res["passes"], passes_per_gpu=main_res["passes_per_gpu"])
            out["config"].update(launches=args.e_mode)
            timed = ("per pass: the pass's launches between device synchronisations (duplex: launch j encrypts "
                     "pass j and decrypts pass j-1, plus one decrypt launch after the last pass), summed; max over "
                     "ranks" if args.e_mode == "duplex" else
                     "per pass: encrypt + decrypt between device synchronisations, summed; max over ranks")
            out["timing"] = {"timed": timed, "fill_ms_per_step": round(main_res["fill_ms"], 3),
                             "wall_ms_per_step_incl_fill": round(main_res["wall_ms"], 3),
                             "launches_per_step": main_res.get("launches")}
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
