"""Pins the CPU oracle (oracle/rsg_oracle.c) against the committed golden
fixtures, which were computed without it (tests/golden/gen_golden.py)."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import cases
from oracle import oracle as orc

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_splitmix_numpy_matches_c():
    for seed, n in [(1, 4096), (3, 1001), (0, 7), (2**63 + 5, 64)]:
        assert cases.splitmix64_bytes(seed, n).tobytes() == orc.splitmix64_bytes(seed, n).tobytes()
    assert cases.splitmix64_bytes(1, 16).tobytes().hex() == "c15c0289ec2d0a9167ec8e65a18debbe"


def test_md4_rfc1320():
    for v in load("md4_vectors.json")["rfc1320"]:
        assert orc.md4(bytes.fromhex(v["msg_hex"])).hex() == v["md4"]


def test_checksum2_edge_lengths():
    g = load("md4_vectors.json")
    data = cases.splitmix64_bytes(7, 131072 + 64)
    for c in g["checksum2"]["cases"]:
        assert orc.checksum2(c["seed"], data[: c["len"]]).hex() == c["sum2"], c
    spot = bytes(range(256)) * 2 + bytes(188)
    assert orc.checksum2(g["spot"]["seed"], spot).hex() == g["spot"]["sum2"]


def test_file_sums_golden():
    """Whole-file sums (rsyncchecksum.go:60-66 plain; match.go:52-53 /
    receiver.go:117-120 seed-prefixed) against OpenSSL MD4 fixtures."""
    g = load("file_sums.json")
    data = cases.splitmix64_bytes(11, 300_001)
    for c in g["cases"]:
        m = data[: c["len"]]
        assert orc.file_sum(0, 0, m).hex() == c["plain"], c["len"]
        for seed, want in c["seeded"].items():
            assert orc.file_sum(1, int(seed), m).hex() == want, (c["len"], seed)


def test_weak_kat_reference():
    """internal/rsyncchecksum/checksum_test.go:32-73: all 1780 values."""
    g = load("weak_kat.json")
    f = cases.weak_kat_file()
    k = g["chunk"]
    n = 0
    for lo, hi, v in g["runs"]:
        for i in range(lo, hi + 1):
            assert orc.checksum1(f[i * k:(i + 1) * k]) == v, i
            n += 1
    assert n == 1780


def test_checksum1_matches_python_literal():
    d = cases.splitmix64_bytes(9, 3000)
    for n in [0, 1, 2, 3, 4, 5, 7, 8, 9, 700, 1773, 3000]:
        assert orc.checksum1(d[:n]) == orc.py_checksum1(d[:n].tobytes())


def test_sum_sizes_sqroot():
    """rsynccommon.go:14-37, SURVEY.md F5."""
    assert orc.sum_sizes_sqroot(1 << 20) == (1024, 1024, 16, 0)
    assert orc.sum_sizes_sqroot(490000) == (700, 700, 16, 0)
    assert orc.sum_sizes_sqroot(490001) == (701, 700, 16, 1)
    assert orc.sum_sizes_sqroot(1 << 30) == (32768, 32768, 16, 0)
    assert orc.sum_sizes_sqroot(32 << 30)[1] == 185363
    assert orc.sum_sizes_sqroot(0) == (0, 700, 16, 0)


def test_block_sums_cfg1():
    g = load("block_sums.json")
    data = cases.splitmix64_bytes(1, 1 << 20)
    for key in ("cfg1_B1024", "cfg1_B700"):
        e = g[key]
        rec = orc.block_sums(data, e["block_len_arg"], e["seed"])
        head = orc.sum_head(data.size, e["block_len_arg"])
        assert list(head) == e["head"]
        assert rec[:20].hex() == e["first"] and rec[-20:].hex() == e["last"]
        assert hashlib.sha256(orc.head_bytes(head) + rec).hexdigest() == e["sha256_head_records"]


def test_block_sums_cfg1_survey_anchors():
    """SURVEY.md appendix anchor values (B=1024 and B=700)."""
    g = load("block_sums.json")
    assert g["cfg1_B1024"]["sha256_head_records"] == \
        "210a8f890dbcf14483e828dc4e9c345f698634c1c3e0e1940bf4c5bae12309e6"
    assert g["cfg1_B700"]["sha256_head_records"] == \
        "cc94b704a1944aa2cf66ffec6215337fc1b0cab3022aa071d79718324dd7ae4b"


def test_block_sums_ragged():
    for e in load("block_sums.json")["ragged"]:
        d = cases.splitmix64_bytes(e["data_seed"], e["len"])
        rec = orc.block_sums(d, e["block_len"], e["seed"])
        assert list(orc.sum_head(e["len"], e["block_len"])) == e["head"]
        assert hashlib.sha256(rec).hexdigest() == e["sha256_records"], e


def _basis_sums(basis, blen, seed):
    head = orc.sum_head(basis.size, blen)
    rec = orc.block_sums(basis, blen, seed)
    if head[0]:
        s1, s2 = orc.parse_records(rec)
    else:
        s1, s2 = np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8)
    return head, s1, s2


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
def test_hash_search_golden(name):
    g = load("match_cases.json")[name]
    src, basis, blen, seed = cases.match_cases()[name]
    head, s1, s2 = _basis_sums(basis, blen, seed)
    assert list(head) == g["head"]
    matches, tokens, fsum = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    assert [list(m) for m in matches] == g["matches"]
    assert len(tokens) == g["tokens_len"]
    assert hashlib.sha256(tokens).hexdigest() == g["tokens_sha256"]
    assert fsum.hex() == g["file_sum"]


def test_hash_search_c_equals_python_random():
    rng = np.random.default_rng(5)
    for t in range(6):
        basis = cases.splitmix64_bytes(500 + t, int(rng.integers(1000, 20000)))
        src = cases.mutate(basis, 600 + t, 0.3, 1, 900, n_ins=2, n_del=2)
        blen = int(rng.choice([64, 100, 333, 700]))
        head, s1, s2 = _basis_sums(basis, blen, t)
        tg = orc.stable_targets(s1)
        m1, t1, _ = orc.hash_search(src, head, s1, s2, tg, t)
        m2, t2 = orc.py_hash_search(src.tobytes(), head, s1, s2, tg, t)
        assert m1 == m2 and t1 == t2


def test_tokens_terminate_and_decode():
    """Token stream decodes (receiver.go:123-166 / token.go) back to the source."""
    src, basis, blen, seed = cases.match_cases()["shifted_700"]
    head, s1, s2 = _basis_sums(basis, blen, seed)
    _, tokens, _ = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    out = bytearray()
    p = 0
    while True:
        (tok,) = struct.unpack_from("<i", tokens, p)
        p += 4
        if tok == 0:
            break
        if tok > 0:
            out += tokens[p:p + tok]
            p += tok
        else:
            i = -(tok + 1)
            ln = head[3] if (i == head[0] - 1 and head[3]) else head[1]
            out += basis[i * head[1]: i * head[1] + ln].tobytes()
    assert p == len(tokens)
    assert bytes(out) == src.tobytes()


# ---- receiver token application (receiver.go:98-188)
def _stream(name):
    src, basis, blen, seed = cases.match_cases()[name]
    head, s1, s2 = _basis_sums(basis, blen, seed)
    _, tokens, fsum = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    return src, basis, head, seed, tokens + fsum


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
def test_receive_data_rebuilds_golden(name):
    """Every golden search's token stream + whole-file sum rebuilds the source
    from the basis and passes the seeded MD4 check (receiver.go:166-173)."""
    src, basis, head, seed, stream = _stream(name)
    out, used = orc.receive_data(stream, head, basis, seed)
    assert out == src.tobytes()
    assert used == len(stream)


def test_receive_data_errors():
    src, basis, head, seed, stream = _stream("shifted_700")
    bad = bytearray(stream)
    bad[-1] ^= 1  # sender's sum differs -> "file corruption"
    with pytest.raises(ValueError, match="-3"):
        orc.receive_data(bytes(bad), head, basis, seed)
    with pytest.raises(ValueError, match="-3"):  # wrong seed
        orc.receive_data(stream, head, basis, seed + 1)
    with pytest.raises(ValueError, match="-1"):  # stream cut inside the sum
        orc.receive_data(stream[:-3], head, basis, seed)
    with pytest.raises(ValueError, match="-1"):  # cut before the terminator
        orc.receive_data(stream[:20], head, basis, seed)
    with pytest.raises(ValueError, match="-2"):  # basis shorter than a matched block
        orc.receive_data(stream, head, basis[:1000], seed)
    with pytest.raises(ValueError, match="-2"):  # match token, no basis
        orc.receive_data(stream, head, None, seed)
