"""Host-side measurement plumbing (no GPU): the rocprofv3 counter parsing that
bench.py's live roofline.traffic and tools/traffic.py share, and the
corrections MI355X_MICROARCH.md's HBM section prescribes for gfx950
(counters in kB, FETCH_SIZE counting half the bytes)."""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import traffic  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def write_counters(d, rows):
    os.makedirs(os.path.join(d, "host", "1234"), exist_ok=True)
    with open(os.path.join(d, "host", "1234", "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))


def test_per_launch_kb_averages_per_dispatch_and_kernel(tmp_path):
    enc = "void cyaes::(anonymous namespace)::k_encrypt<false, false, false, false>(cyaes::EncArgs)"
    dec = "void cyaes::(anonymous namespace)::k_decrypt_flat<false, true, false, false>(cyaes::DecArgs)"
    rows = [
        # two encrypt launches, each reported as two per-XCD rows that sum
        (1, enc, "FETCH_SIZE", 100.0), (1, enc, "FETCH_SIZE", 50.0),
        (3, enc, "FETCH_SIZE", 200.0), (3, enc, "FETCH_SIZE", 250.0),
        (2, dec, "FETCH_SIZE", 80.0),
        (4, "k_fill_synthetic", "FETCH_SIZE", 1e9),  # not an AES kernel: ignored
        (2, dec, "WRITE_SIZE", 5.0),                 # another counter: ignored here
    ]
    write_counters(str(tmp_path), rows)
    kb = traffic.per_launch_kb(str(tmp_path), "FETCH_SIZE")
    assert kb == {"encrypt": pytest.approx(300.0), "decrypt": pytest.approx(80.0)}


def test_missing_counter_file_is_reported(tmp_path):
    with pytest.raises(SystemExit):
        traffic.per_launch_kb(str(tmp_path), "FETCH_SIZE")


def test_traffic_json_corrections(tmp_path):
    enc = "k_encrypt<false, false, false, false>"
    dec = "k_decrypt_flat<false, true, false, false>"
    fdir, wdir = str(tmp_path / "f"), str(tmp_path / "w")
    algo_kb = traffic.ALGO / 1024
    # FETCH reads half the bytes on gfx950: N/2 kB read + N kB written = the algorithmic 2N
    write_counters(fdir, [(1, enc, "FETCH_SIZE", algo_kb / 4), (2, dec, "FETCH_SIZE", algo_kb / 4)])
    write_counters(wdir, [(1, enc, "WRITE_SIZE", algo_kb / 2), (2, dec, "WRITE_SIZE", algo_kb / 2)])
    out = str(tmp_path / "traffic.json")
    sys.argv = ["traffic.py", fdir, wdir, "--out", out]
    traffic.main()
    import json
    t = json.load(open(out))["C"]
    for k in ("encrypt", "decrypt"):
        assert t[k]["bytes_per_launch"] == traffic.ALGO
        assert t[k]["ratio"] == 1.0
        assert t[k]["fetch_bytes"] == traffic.ALGO // 2


def test_bench_traffic_plan_and_pass_command(monkeypatch):
    """bench.py's live HBM-traffic passes: only rank 0 at N = 1 on config C / E,
    never nested under rocprofv3, and each pass is the rocprofv3 script run by
    this interpreter (no exec hop through `env`) over a bench.py that runs no
    passes of its own."""
    import shutil
    import subprocess
    sys.path.insert(0, ROOT)
    import bench
    assert bench.traffic_plan("live", 0, 1, "E", {}) == (True, None)
    assert bench.traffic_plan("live", 0, 1, "C", {"PATH": "/bin"})[0] is True
    assert bench.traffic_plan("file", 0, 1, "E", {})[0] is False
    assert bench.traffic_plan("live", 1, 2, "E", {})[0] is False
    assert bench.traffic_plan("live", 0, 1, "B", {})[0] is False
    run, why = bench.traffic_plan("live", 0, 1, "E", {"ROCPROF_COUNTER_COLLECTION": "1"})
    assert run is False and "rocprofv3" in why
    if not shutil.which("rocprofv3"):
        pytest.skip("rocprofv3 not on PATH")
    seen = []

    class Fake:
        returncode = 3

        def __init__(self, cmd, **kw):
            seen.append((cmd, kw))

        def wait(self, timeout=None):
            return self.returncode
    monkeypatch.setattr(subprocess, "Popen", Fake)
    live, why = bench.live_traffic(timeout_s=5)
    assert live is None and "exited 3" in why
    cmd, kw = seen[0]
    assert cmd[0] == sys.executable and cmd[1].endswith("rocprofv3") and cmd[2:4] == ["--pmc", "FETCH_SIZE"]
    assert cmd[cmd.index("--") + 1] == sys.executable
    assert cmd[-2:] == ["--traffic", "none"] and cmd[cmd.index("--e2e-gib") + 1] == "0" and "RANK" not in kw["env"] and kw["start_new_session"]


def test_bench_world_size_must_match_gpus():
    """--gpus N under torchrun must agree with WORLD_SIZE: a
    mismatch is an error, not a note, so a scaling run cannot silently time a
    different number of GPUs than it is labelled with."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.world_check(1, {}) == (1, None)
    assert bench.world_check(8, {}) == (1, None)  # not a rank: bench.py launches the 8 ranks itself
    assert bench.world_check(4, {"WORLD_SIZE": "4"}) == (4, None)
    w, err = bench.world_check(8, {"WORLD_SIZE": "1"})
    assert w == 1 and "--gpus 8 but WORLD_SIZE 1" in err


def test_bench_mismatch_exits_nonzero():
    """The real entry point: WORLD_SIZE=2 with --gpus 1 exits 2 before it
    imports torch or touches a GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2, p.stderr
    assert "refusing" in p.stderr and p.stdout == ""


def test_bench_launcher_command():
    """`python bench.py --gpus N` (no torchrun) starts torchrun as a child: N
    processes on this node, rendezvous on 127.0.0.1, the same arguments."""
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "3"], 29555, python="/py")
    assert cmd[:3] == ["/py", "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8" and cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_launcher_forwards_rank0_line(monkeypatch, capsys):
    """launch_ranks: forwards exactly the rank-0 result line (with `launcher`
    added), sends everything else to stderr, hands the traffic result to the
    ranks through the environment, and returns the child's exit code."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench
    script = ("import json, os, sys; print('noise'); print('{not json'); "
              "t = json.loads(os.environ['%s']); "
              "print(json.dumps({'metric': %r, 'value': 1.0, 'why': t['why'], 'launched': os.environ['%s']})); "
              "sys.exit(int(sys.argv[1]))" % (bench.TRAFFIC_ENV, bench.METRIC, bench.LAUNCH_ENV))
    args = argparse.Namespace(gpus=2, traffic="none", config="E")
    for rc in (0, 5):
        monkeypatch.setattr(bench, "launcher_cmd", lambda g, argv, port, _rc=rc: [sys.executable, "-c", script, str(_rc)])
        assert bench.launch_ranks(args, []) == rc
        out, err = capsys.readouterr()
        lines = out.splitlines()
        assert len(lines) == 1, out
        d = json.loads(lines[0])
        assert d["launcher"]["nproc_per_node"] == 2 and d["launched"] == "bench.py" and d["why"] == "not requested"
        assert "noise" in err and "{not json" in err
    # ranks that exit 0 without a result line are a failure
    monkeypatch.setattr(bench, "launcher_cmd", lambda g, argv, port: [sys.executable, "-c", "print('x')"])
    assert bench.launch_ranks(args, []) == 1
