#!/usr/bin/env python3
"""tools/e2e_pins_probe.py -- host batches over torch pinned memory: time per
call and what the registration registry did (cyaes_debug_pins deltas), for
encrypt_host / decrypt_host as bench.py's e2e object runs them."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import cyclone_amd as ca
    n, pb = int(sys.argv[1]) if len(sys.argv) > 1 else 131072, 65536
    c = ca.GpuContext(0)
    c.set_keys(bytes(range(16)))
    nb = n * pb
    h = [torch.empty(nb, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    d = torch.empty(nb, dtype=torch.uint8, device="cuda")
    c.fill_synthetic(d, 0, n, pb, 0x5EEDC1C1)
    h[0].copy_(d)
    for rep in range(3):
        for name, fn in (("encrypt", lambda: c.encrypt_host(h[0], h[1], n, pb)),
                         ("decrypt", lambda: c.decrypt_host(h[1], h[2], n, pb))):
            p0 = ca.debug_pins()
            t0 = time.perf_counter()
            fn()
            t1 = time.perf_counter()
            p1 = ca.debug_pins()
            print("%s rep %d: %.1f ms, %.2f GiB/s, pins %s" % (name, rep, (t1 - t0) * 1e3, nb / (t1 - t0) / 2**30,
                                                               {k: p1[k] - p0[k] for k in p1 if p1[k] != p0[k]}))
    print("round trip ok:", bool(torch.equal(h[2], h[0])))
    c.close()


if __name__ == "__main__":
    main()
