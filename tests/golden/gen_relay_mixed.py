#!/usr/bin/env python3
"""Writes tests/golden/relay_mixed.json: the digests of bench.py's mixed-size
relay stream (relay_stream.mixed) before and after encryption, computed with
the oracle (oracle/aes_oracle.c, cyo_batch_ragged: each payload an
independent chain from DefaultIV, as relay_local.cpp:206 encrypts a packet).

Layout: bench.mixed_stream_layout(config B's bytes), the whole stream buffer
filled as cyaes_gpu_fill_synthetic(buf, 0, bytes / 16, 16, PLAINTEXT_SEED)
(headers included; encryption leaves them untouched).  Digest: cyaes_gpu_digest
of the whole stream buffer.  Run: python tests/golden/gen_relay_mixed.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import bench
    import oracle
    n_b, pb_b, _ = bench.CONFIGS["B"]
    offsets, nbytes, alloc = bench.mixed_stream_layout(n_b * pb_b)
    buf = oracle.synthetic(0, alloc // 16, 16, bench.PLAINTEXT_SEED)
    plain = oracle.digest(buf)
    oracle.batch_ragged(False, bytes(range(16)), buf, offsets, nbytes, nthreads=os.cpu_count() or 1)
    cipher = oracle.digest(buf)
    out = {
        "generator": "tests/golden/gen_relay_mixed.py (oracle/aes_oracle.c cyo_batch_ragged)",
        "layout": "bench.mixed_stream_layout(%d), seed %#x" % (n_b * pb_b, bench.MIXED_SEED),
        "chunk_bytes": n_b * pb_b, "packets": int(offsets.size), "payload_bytes": int(nbytes.sum()),
        "stream_bytes": alloc, "full_chunks": int((nbytes == bench.RELAY_MAX_CHUNK).sum()),
        "layout_sha256_16": hashlib.sha256(offsets.tobytes() + nbytes.tobytes()).hexdigest()[:16],
        "key": bytes(range(16)).hex(),
        "plain_digest": ["%016x" % v for v in plain], "cipher_digest": ["%016x" % v for v in cipher],
    }
    path = os.path.join(ROOT, "tests", "golden", "relay_mixed.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
