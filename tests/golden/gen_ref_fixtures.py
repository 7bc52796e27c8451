#!/usr/bin/env python3
"""Generate golden fixtures from the reference's own test and table data.

Runs ONLY in the build container, where /root/reference exists (read as text,
nothing is compiled, imported or executed).  Writes data, not source:

  ref_kat.json / ref_kat.txt  -- the Rijndael known-answer vector of
      test/unit/cyt_unit_crypt.cpp:177-186 (key, plaintext, ciphertext,
      iv_check), as hex; and (ref_kat.json "adler32") the Adler-32 known
      answers of cyt_unit_crypt.cpp:18-50, and ("ringbuf_checksum") the
      RingBuf::checksum answers of cyt_unit_ring_buf.cpp:370-385.
  ref_tables.json             -- SHA-256 of each static table of
      source/cyCrypt/crypt/cyr_rijndael.cpp:25-501 (S, Si, T1..T8, U1..U4,
      rcon), serialised as little-endian u8/u32 arrays, plus DefaultIV
      (:503-504).  The oracle regenerates the tables from GF(2^8) arithmetic
      and tests/test_oracle.py pins them against these digests.
"""
import hashlib
import json
import os
import re
import struct
import sys

REF = os.environ.get("CYCLONE_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def _ints(body):
    return [int(t, 16) for t in re.findall(r"0x[0-9a-fA-F]+", body)]


def tables():
    src = open(os.path.join(REF, "source/cyCrypt/crypt/cyr_rijndael.cpp"), encoding="utf-8-sig").read()
    out = {}
    for name in ["sm_S", "sm_Si", "sm_T1", "sm_T2", "sm_T3", "sm_T4", "sm_T5", "sm_T6", "sm_T7", "sm_T8",
                 "sm_U1", "sm_U2", "sm_U3", "sm_U4", "sm_rcon"]:
        m = re.search(r"static const (uint8_t|uint32_t) " + name + r"\[(\d+)\]\s*=\s*\{(.*?)\};", src, re.S)
        kind, n, body = m.group(1), int(m.group(2)), m.group(3)
        vals = _ints(body)
        assert len(vals) == n, (name, len(vals), n)
        fmt = "<%d%s" % (n, "B" if kind == "uint8_t" else "I")
        out[name] = {"n": n, "bytes": struct.calcsize(fmt), "sha256": hashlib.sha256(struct.pack(fmt, *vals)).hexdigest()}
    m = re.search(r"Rijndael::DefaultIV\s*=\s*\{(.*?)\};", src, re.S)
    out["DefaultIV"] = bytes(_ints(m.group(1))).hex()
    return out


def kat():
    src = open(os.path.join(REF, "test/unit/cyt_unit_crypt.cpp"), encoding="utf-8-sig").read()
    body = src[src.index('TEST_CASE("Crypto algorithm(Rijndael) test"'):]
    key = bytes(_ints(re.search(r"BLOCK key\s*=\s*\{(.*?)\};", body, re.S).group(1)))
    plain = re.search(r'plain_text\s*=\s*"(.*?)";', body).group(1).encode()
    cipher = bytes(_ints(re.search(r"encrypt_text\[\]\s*=\s*\{(.*?)\};", body, re.S).group(1)))
    iv_check = bytes(_ints(re.search(r"iv_check\s*=\s*\{(.*?)\};", body, re.S).group(1)))
    assert len(key) == 16 and len(plain) == 64 and len(cipher) == 64 and len(iv_check) == 16
    return {"source": "test/unit/cyt_unit_crypt.cpp:177-186", "key": key.hex(), "plaintext": plain.hex(),
            "ciphertext": cipher.hex(), "iv_check": iv_check.hex(), "random_roundtrips": 20,
            "random_roundtrip_bytes": 128}


def adler_kat():
    """Adler-32 known answers of test/unit/cyt_unit_crypt.cpp:18-50 (strings,
    the 64-byte data_buf, its split point) as data."""
    src = open(os.path.join(REF, "test/unit/cyt_unit_crypt.cpp"), encoding="utf-8-sig").read()
    body = src[src.index('TEST_CASE("Crypto algorithm(Adler32) basic test"'):]
    body = body[:body.index("TEST_CASE", 10)]
    strings = re.findall(r'const char\* \w+ = "(.*?)";\s*(?:uint32_t )?adler = adler32\(INITIAL_ADLER.*?\);\s*'
                         r'REQUIRE_EQ\((0x[0-9a-fA-F]+)ul, adler\);', body, re.S)
    data = bytes(_ints(re.search(r"data_buf\[\]\s*=\s*\{(.*?)\};", body, re.S).group(1)))
    expect = int(re.search(r"REQUIRE_EQ\((0x[0-9a-fA-F]+)ul, adler1\)", body).group(1), 16)
    first = int(re.search(r"size_t first = (\d+);", body).group(1))
    assert len(strings) == 2 and len(data) == 64
    return {"source": "test/unit/cyt_unit_crypt.cpp:18-50",
            "strings": [{"text": t, "adler": int(a, 16)} for t, a in strings],
            "data_buf": data.hex(), "data_adler": expect, "split": first,
            "null_or_empty": 1, "random_cases": 100, "random_cap": 257}


def ringbuf_checksum_kat():
    """RingBuf::checksum known answers of test/unit/cyt_unit_ring_buf.cpp:370-385
    (Adler-32 over byte ranges of the buffer holding text_pattern, :48-49) and
    its empty / out-of-range rules (cyc_ring_buf.cpp:365-373), as data."""
    src = open(os.path.join(REF, "test/unit/cyt_unit_ring_buf.cpp"), encoding="utf-8-sig").read()
    text = re.search(r'const char\* text_pattern = "(.*?)";', src).group(1)
    body = src[src.index("//checksum"):]
    body = body[:body.index("//make wrap condition and checksum")]
    cases = [{"off": 0 if o == "0" else int(o), "count": int(c), "adler": int(a, 16)}
             for a, o, c in re.findall(r"REQUIRE_EQ\((0x[0-9a-fA-F]+)ul, rb1\.checksum\((\w+), (\d+)\)\)", body)]
    full = int(re.search(r"REQUIRE_EQ\((0x[0-9a-fA-F]+)ul, rb1\.checksum\(0, text_length\)\)", body).group(1), 16)
    hdr = open(os.path.join(REF, "source/cyCore/core/cyc_ring_buf.h"), encoding="utf-8-sig").read()
    a, b = re.search(r"kDefaultCapacity = (\d+) - (\d+)", hdr).groups()
    cap = int(a) - int(b)
    assert len(cases) == 2
    return {"source": "test/unit/cyt_unit_ring_buf.cpp:370-385; cyc_ring_buf.cpp:365-387", "text": text,
            "full": full, "ranges": cases, "capacity": cap, "wrap_size": 32}


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are committed, nothing to do")
    k = kat()
    with open(os.path.join(HERE, "ref_kat.json"), "w") as f:
        json.dump(k, f, indent=1)
    with open(os.path.join(HERE, "ref_kat.txt"), "w") as f:
        for name in ["key", "plaintext", "ciphertext", "iv_check"]:
            f.write("%s=%s\n" % (name, k[name]))
    k["adler32"] = adler_kat()
    k["ringbuf_checksum"] = ringbuf_checksum_kat()
    with open(os.path.join(HERE, "ref_kat.json"), "w") as f:
        json.dump(k, f, indent=1)
    t = tables()
    t["source"] = "source/cyCrypt/crypt/cyr_rijndael.cpp:25-504"
    with open(os.path.join(HERE, "ref_tables.json"), "w") as f:
        json.dump(t, f, indent=1)
    print("wrote ref_kat.json, ref_kat.txt, ref_tables.json")


if __name__ == "__main__":
    main()
