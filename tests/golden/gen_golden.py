"""Regenerates the committed golden fixtures in tests/golden/.

Run in the build container (needs OpenSSL 3's legacy provider for MD4):
    python tests/golden/gen_golden.py

Independence: every expected value here is computed WITHOUT the C oracle
(oracle/rsg_oracle.c) so that tests/test_oracle.py pins the oracle against
outside arithmetic:
  * MD4 comes from OpenSSL's legacy provider (libcrypto.so.3, via ctypes);
  * the weak sum comes from a numpy restatement of Checksum1
    (internal/rsyncchecksum/rsyncchecksum.go:29-51);
  * hash-search token streams come from the pure-Python transcription
    oracle.py:py_hash_search (internal/sender/match.go:21-282) fed with the
    OpenSSL MD4.
The weak known-answer values are copied as DATA from the reference's own test
(internal/rsyncchecksum/checksum_test.go:38-52); the RFC 1320 vectors are the
published appendix A.5 values.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cases  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (only py_hash_search, pure Python)

# ---------------------------------------------------------------- OpenSSL MD4
_ssl = ctypes.CDLL(ctypes.util.find_library("crypto"))
_ssl.OSSL_PROVIDER_load.restype = ctypes.c_void_p
_ssl.OSSL_PROVIDER_load.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
assert _ssl.OSSL_PROVIDER_load(None, b"legacy")
assert _ssl.OSSL_PROVIDER_load(None, b"default")
_ssl.EVP_MD_fetch.restype = ctypes.c_void_p
_ssl.EVP_MD_fetch.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
_MD4 = _ssl.EVP_MD_fetch(None, b"MD4", None)
assert _MD4
_ssl.EVP_Digest.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                            ctypes.POINTER(ctypes.c_uint), ctypes.c_void_p, ctypes.c_void_p]


def ssl_md4(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    n = ctypes.c_uint(0)
    assert _ssl.EVP_Digest(data, len(data), out, ctypes.byref(n), ctypes.c_void_p(_MD4), None) == 1
    return out.raw


def ssl_checksum2(seed: int, data) -> bytes:
    return ssl_md4(bytes(data) + struct.pack("<i", orc._i32(seed)))


# ---------------------------------------------------------------- numpy weak
def np_checksum1(buf: np.ndarray) -> int:
    x = buf.astype(np.int8).astype(np.int64)
    n = x.size
    s1 = int(x.sum()) & 0xFFFFFFFF
    s2 = int(((n - np.arange(n, dtype=np.int64)) * x).sum()) & 0xFFFFFFFF
    return ((s1 & 0xFFFF) + (s2 << 16)) & 0xFFFFFFFF


def head_for(n: int, blen: int):
    if blen <= 0:
        b = max(int(np.sqrt(float(n))), 700)
    else:
        b = blen
    return ((n + b - 1) // b, b, 16, n % b)


def block_records(data: np.ndarray, blen: int, seed: int) -> bytes:
    count, b, _, _ = head_for(data.size, blen)
    out = bytearray()
    for i in range(count):
        blk = data[i * b: min((i + 1) * b, data.size)]
        out += struct.pack("<I", np_checksum1(blk))
        out += ssl_checksum2(seed, blk.tobytes())
    return bytes(out)


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


# ---------------------------------------------------------------- fixtures
def gen_md4():
    rfc = [b"", b"a", b"abc", b"message digest", b"abcdefghijklmnopqrstuvwxyz",
           b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
           b"1234567890" * 8]
    rfc_expected = ["31d6cfe0d16ae931b73c59d7e0c089c0", "bde52cb31de33e46245e05fbdbd6fb24",
                    "a448017aaf21d8525fc10ae87aa6729d", "d9130a8164549fe818874806e1c7014b",
                    "d79e1c308aa5bbcdeea8ed63df412da9", "043f8582f241db351ce627e153e7f0e4",
                    "e33b4ddc9c38f2199c3e7b164fcc0536"]
    vec = []
    for m, e in zip(rfc, rfc_expected):
        got = ssl_md4(m).hex()
        assert got == e, (m, got, e)
        vec.append({"msg_hex": m.hex(), "md4": e})
    c2 = []
    data = cases.splitmix64_bytes(7, 131072 + 64)
    for n in [0, 1, 3, 4, 51, 52, 55, 56, 59, 60, 63, 64, 119, 120, 676, 700, 1024, 1773, 131072]:
        for seed in [cases.SEED, 0, -1]:
            c2.append({"len": n, "seed": seed,
                       "sum2": ssl_checksum2(seed, data[:n].tobytes()).hex()})
    # the SURVEY.md §8(c) spot value
    spot = bytes(range(256)) * 2 + bytes(188)
    spot_sum = ssl_checksum2(0x12345678, spot).hex()
    assert spot_sum == "1a4950903b7341bcb2dbc9b44ae740fa"
    return {"rfc1320": vec, "checksum2": {"data": "splitmix64(seed=7)", "cases": c2},
            "spot": {"seed": 0x12345678, "msg": "bytes(range(256))*2+bytes(188)", "sum2": spot_sum}}


def gen_weak_kat():
    # internal/rsyncchecksum/checksum_test.go:39-52 (values as data)
    runs = [[0, 592, 0xA5D47568], [593, 593, 0x23645688], [594, 1185, 0x8C1C2378],
            [1186, 1186, 0x12504720], [1187, 1778, 0x7D9883B0], [1779, 1779, 0x61B8DFF0]]
    f = cases.weak_kat_file()
    k = 1768
    for lo, hi, v in runs:
        for i in range(lo, hi + 1):
            assert np_checksum1(f[i * k: (i + 1) * k]) == v, i
    return {"source": "internal/rsyncchecksum/checksum_test.go:32-73", "chunk": k,
            "file": "0x11*1MiB || 0xbb*1MiB || 0xee*1MiB", "runs": runs}


def gen_block_sums():
    out = {}
    cfg1 = cases.splitmix64_bytes(1, 1 << 20)
    assert cfg1[:16].tobytes().hex() == "c15c0289ec2d0a9167ec8e65a18debbe"
    for blen in (1024, 700):
        head = head_for(cfg1.size, blen if blen != 1024 else 0)
        rec = block_records(cfg1, blen if blen != 1024 else 0, cases.SEED)
        out[f"cfg1_B{blen}"] = {
            "data": "splitmix64(seed=1, 1048576)", "seed": cases.SEED, "block_len_arg":
            (0 if blen == 1024 else blen), "head": head,
            "sha256_head_records": sha(struct.pack("<4i", *head) + rec),
            "first": rec[:20].hex(), "last": rec[-20:].hex()}
    rag = []
    for i, n in enumerate(cases.ragged_lengths()):
        d = cases.splitmix64_bytes(1000 + i, n)
        for blen, seed in ((700, cases.SEED), (1773, -1), (64, 0), (1, 5), (0, cases.SEED)):
            rec = block_records(d, blen, seed)
            rag.append({"data_seed": 1000 + i, "len": n, "block_len": blen, "seed": seed,
                        "head": head_for(n, blen), "sha256_records": sha(rec),
                        "first": rec[:20].hex()})
    out["ragged"] = rag
    return out


def gen_match():
    res = {}
    for name, (src, basis, blen, seed) in cases.match_cases().items():
        head = head_for(basis.size, blen)
        rec = block_records(basis, blen, seed)
        if head[0]:
            a = np.frombuffer(rec, dtype=np.uint8).reshape(-1, 20)
            sum1 = a[:, :4].copy().view("<u4").reshape(-1)
            sum2 = a[:, 4:].copy()
        else:
            sum1 = np.zeros(0, np.uint32)
            sum2 = np.zeros((0, 16), np.uint8)
        tg = orc.stable_targets(sum1)
        matches, tokens = orc.py_hash_search(src.tobytes(), head, sum1, sum2, tg, seed,
                                             c2=ssl_checksum2)
        fsum = ssl_md4(struct.pack("<i", orc._i32(seed)) + src.tobytes())
        res[name] = {"src_len": int(src.size), "basis_len": int(basis.size), "head": head,
                     "seed": seed, "n_matches": len(matches), "matches": matches,
                     "tokens_len": len(tokens), "tokens_sha256": sha(tokens),
                     "file_sum": fsum.hex()}
        print(f"  {name}: head={head} matches={len(matches)} tokens={len(tokens)}")
    return res


def gen_file_sums():
    """Whole-file sums: MD4(file) and MD4(int32_LE(seed) || file), by OpenSSL."""
    data = cases.splitmix64_bytes(11, 300_001)
    out = []
    for n in [0, 1, 3, 4, 5, 55, 56, 59, 60, 61, 63, 64, 65, 119, 120, 123, 124, 127, 128, 700, 4096,
              65_537, 300_001]:
        m = data[:n].tobytes()
        e = {"len": n, "plain": ssl_md4(m).hex(), "seeded": {}}
        for seed in [cases.SEED, 0, -1]:
            e["seeded"][str(seed)] = ssl_md4(struct.pack("<i", seed) + m).hex()
        out.append(e)
    return {"data": "splitmix64(seed=11)", "cases": out}


def main():
    w = lambda name, obj: json.dump(obj, open(os.path.join(HERE, name), "w"), indent=1)
    w("md4_vectors.json", gen_md4())
    print("md4 ok")
    w("weak_kat.json", gen_weak_kat())
    print("weak kat ok")
    w("block_sums.json", gen_block_sums())
    print("block sums ok")
    w("match_cases.json", gen_match())
    print("match ok")
    w("file_sums.json", gen_file_sums())
    print("file sums ok")


if __name__ == "__main__":
    main()
