#!/usr/bin/env python3
"""bench_adler.py -- Adler-32 on the MI355X (include/cyaes_adler32.h,
SURVEY.md §8(f) row 4): one JSON line per mode.

  big:   one 16 GiB device buffer reduced by the whole GPU (cyaes_gpu_adler32)
  batch: 262,144 buffers x 64 KiB (RingBuf / filetransfer fragment shape),
         one wave per buffer (cyaes_gpu_adler32_batch)

Roofline: HBM, algorithmic bytes = the buffer bytes read once.  Checked
against the oracle on a sampled slice.
usage: python bench_adler.py [--gib 16] [--steps 5]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import cyclone_amd as ca
    import oracle

    lib = ca.load_library()
    n = args.gib << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx = ca.GpuContext(0)
    ctx.fill_synthetic(buf, 0, n // 65536, 65536, oracle.PLAINTEXT_SEED)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    out = ctypes.c_uint32()

    # big: whole-GPU reduction of one buffer
    times = []
    for i in range(args.steps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert lib.cyaes_gpu_adler32(buf.data_ptr(), n, 1, ctypes.byref(out), s.cuda_stream) == 0
        e1.record(s)
        torch.cuda.synchronize()
        if i:
            times.append(e0.elapsed_time(e1))
    ms = sorted(times)[len(times) // 2]
    # parity: chain the first 256 MiB through the oracle vs the device on the same slice
    sl = 256 << 20
    dev_sl = ctypes.c_uint32()
    assert lib.cyaes_gpu_adler32(buf.data_ptr(), sl, 1, ctypes.byref(dev_sl), s.cuda_stream) == 0
    ok = dev_sl.value == oracle.adler32(1, buf[:sl].cpu().numpy())
    print(json.dumps({"metric": "Adler-32 GB/s, one device buffer", "mode": "big", "bytes": n,
                      "ms": round(ms, 3), "gbs": round(n / ms / 1e6, 1),
                      "roofline": {"bound": "hbm", "achieved": round(n / ms / 1e6, 1), "peak": HBM_PEAK / 1e9,
                                   "unit": "GB/s", "frac": round(n / ms / 1e-3 / HBM_PEAK, 4)},
                      "adler32": "%08x" % out.value, "parity": "bit-exact" if ok else "MISMATCH"}))

    # batch: fragments of 64 KiB
    pb = 65536
    cnt = n // pb
    offs = torch.arange(cnt, dtype=torch.int64, device="cuda") * pb
    lens = torch.full((cnt,), pb, dtype=torch.int64, device="cuda")
    res = torch.empty(cnt, dtype=torch.int32, device="cuda")
    times = []
    for i in range(args.steps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert lib.cyaes_gpu_adler32_batch(buf.data_ptr(), offs.data_ptr(), lens.data_ptr(), None, res.data_ptr(),
                                           cnt, s.cuda_stream) == 0
        e1.record(s)
        torch.cuda.synchronize()
        if i:
            times.append(e0.elapsed_time(e1))
    ms = sorted(times)[len(times) // 2]
    host = buf[:64 * pb].cpu().numpy()
    got = res[:64].cpu().numpy().view("uint32")
    ok = all(int(got[k]) == oracle.adler32(1, host[k * pb:(k + 1) * pb]) for k in range(64))
    print(json.dumps({"metric": "Adler-32 GB/s, batch of fragments", "mode": "batch", "buffers": cnt,
                      "buffer_bytes": pb, "ms": round(ms, 3), "gbs": round(n / ms / 1e6, 1),
                      "roofline": {"bound": "hbm", "achieved": round(n / ms / 1e6, 1), "peak": HBM_PEAK / 1e9,
                                   "unit": "GB/s", "frac": round(n / ms / 1e-3 / HBM_PEAK, 4)},
                      "parity": "bit-exact (64 sampled buffers)" if ok else "MISMATCH"}))


if __name__ == "__main__":
    main()
