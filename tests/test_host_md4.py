"""The product's host MD4 (rsync_amd/csrc/rsg_md4_host.cpp, through the
rsg_testing_md4 hook): RFC 1320's test suite and the oracle's whole-file
sums (plain and seeded, match.go:52-53) at lengths around every padding
boundary, fed in pieces of every size class.  This MD4 serves whole-file
sums whose bytes stream through host memory; block checksums never use it."""
import ctypes

import numpy as np
import pytest

import cases
from oracle import oracle as orc
from rsync_amd import _lib

RFC1320 = {
    b"": "31d6cfe0d16ae931b73c59d7e0c089c0",
    b"a": "bde52cb31de33e46245e05fbdbd6fb24",
    b"abc": "a448017aaf21d8525fc10ae87aa6729d",
    b"message digest": "d9130a8164549fe818874806e1c7014b",
    b"abcdefghijklmnopqrstuvwxyz": "d79e1c308aa5bbcdeea8ed63df412da9",
    b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789": "043f8582f241db351ce627e153e7f0e4",
    b"1234567890" * 8: "e33b4ddc9c38f2199c3e7b164fcc0536",
}


def md4(data, seeded=False, seed=0, piece=0):
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    out = np.zeros(16, np.uint8)
    _lib.check(_lib.lib.rsg_testing_md4(a.ctypes.data if a.size else None, a.size, int(seeded), seed, piece,
                                        out.ctypes.data))
    return out.tobytes()


@pytest.mark.parametrize("msg", sorted(RFC1320))
def test_rfc1320(msg):
    assert md4(msg).hex() == RFC1320[msg]


@pytest.mark.parametrize("n", [0, 1, 3, 4, 51, 52, 55, 56, 59, 60, 63, 64, 65, 119, 120, 127, 128, 700, 4097, 100_003])
@pytest.mark.parametrize("piece", [0, 1, 7, 64, 1000])
def test_matches_oracle_file_sums(n, piece):
    d = cases.splitmix64_bytes(n + 17, n)
    assert md4(d, piece=piece) == orc.file_sum(0, 0, d)
    for seed in (cases.SEED, 0, -1):
        assert md4(d, True, seed, piece) == orc.file_sum(1, seed, d)


def test_large_buffer():
    d = cases.splitmix64_bytes(5, 9 << 20)
    assert md4(d, True, cases.SEED, 1 << 20) == orc.file_sum(1, cases.SEED, d)
