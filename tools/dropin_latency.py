import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import cyclone_amd as ca
aes = ca.Rijndael(bytes(range(16)))
for size in (16, 1472, 65280):
    buf = bytes(size)
    for op in ("encrypt", "decrypt"):
        f = getattr(aes, op)
        for _ in range(20): f(buf)
        n = 300
        t0 = time.perf_counter()
        for _ in range(n): f(buf)
        dt = (time.perf_counter() - t0) / n
        print(f"{op} {size} B: {dt*1e6:.1f} us/call")
