"""GPU parity of the whole-file MD4 sums through the
C-ABI: RSG_FILESUM_PLAIN = rsyncchecksum.ReaderChecksum (rsyncchecksum.go:60-66),
RSG_FILESUM_SEEDED = MD4(int32_LE(seed) || file) (match.go:52-53,
receiver.go:117-120).  Checked against the OpenSSL fixtures and the oracle."""
import json
import os

import numpy as np
import pytest

import cases
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def eng():
    import rsync_amd
    e = rsync_amd.Engine(0)
    yield e
    e.close()


def test_file_sums_golden(eng):
    import rsync_amd
    g = json.load(open(os.path.join(GOLD, "file_sums.json")))
    data = cases.splitmix64_bytes(11, 300_001)
    files = [data[: c["len"]] for c in g["cases"]]
    plain = eng.file_sums(files, rsync_amd.FILESUM_PLAIN)
    assert [p.hex() for p in plain] == [c["plain"] for c in g["cases"]]
    for seed in (cases.SEED, 0, -1):
        got = eng.file_sums(files, rsync_amd.FILESUM_SEEDED, seed)
        assert [p.hex() for p in got] == [c["seeded"][str(seed)] for c in g["cases"]], seed


def test_file_sums_device_unaligned_and_arena_end(eng):
    """Files at every byte alignment, zero-length files, a file ending exactly
    at the arena's end (the guarded loads), in one batch."""
    import rsync_amd
    rng = np.random.default_rng(21)
    lens = [int(x) for x in rng.integers(0, 3000, 700)] + [0, 0, 1, 59, 60, 64, 65, 100_003]
    offs, o = [], 0
    for n in lens:
        o += int(rng.integers(0, 8))  # any alignment
        offs.append(o)
        o += n
    arena_bytes = offs[-1] + lens[-1]  # last file ends at the arena end
    host = cases.splitmix64_bytes(22, arena_bytes)
    arena = eng.alloc(arena_bytes)
    arena.upload(host)
    for mode, seed in ((rsync_amd.FILESUM_PLAIN, 0), (rsync_amd.FILESUM_SEEDED, cases.SEED)):
        out = eng.file_sums_device(arena, list(zip(offs, lens)), mode, seed)
        got = out.download(16 * len(lens)).reshape(-1, 16)
        for i, (off, n) in enumerate(zip(offs, lens)):
            assert got[i].tobytes() == orc.file_sum(mode, seed, host[off:off + n]), (i, off, n, mode)


def test_file_sums_many_files(eng):
    """cfg4-shaped batch (lengths 4-64 KiB), scaled down: 3000 files."""
    import rsync_amd
    rng = np.random.default_rng(4)
    lens = [int(x) for x in rng.integers(4096, 65537, 3000)]
    files = [cases.splitmix64_bytes(100 + i, n) for i, n in enumerate(lens)]
    got = eng.file_sums(files, rsync_amd.FILESUM_SEEDED, cases.SEED)
    for i in range(0, 3000, 7):
        assert got[i] == orc.file_sum(1, cases.SEED, files[i]), i


def test_checksum2_empty_and_reader_checksum():
    """Checksum2 of an empty buffer is MD4(seed) (rsyncchecksum.go:53-58);
    ReaderChecksum is the plain MD4."""
    import rsync_amd
    for seed in (0, -1, cases.SEED):
        assert rsync_amd.checksum2(seed, b"") == orc.checksum2(seed, b"")
    d = cases.splitmix64_bytes(5, 12345)
    assert rsync_amd.reader_checksum(d) == orc.md4(d)
    assert rsync_amd.reader_checksum(b"") == orc.md4(b"")


def test_file_sums_bad_mode(eng):
    from rsync_amd import _lib
    with pytest.raises(_lib.RsgError):
        eng.file_sums([b"abc"], 7)


def test_file_sums_device_aligned_segments(eng):
    """Every file 4-byte aligned (16-byte packed, as the library's arenas):
    the staged kernel's exact 256-byte segments (no funnel shift, no 17th
    unit), with lengths around the segment and MD4 padding boundaries, waves
    whose lanes run past each other's last segment, and a last file ending
    exactly at the arena end (the per-lane fallback for its wave)."""
    import rsync_amd
    rng = np.random.default_rng(23)
    lens = [int(x) for x in rng.integers(0, 70_000, 900)] + [0, 1, 55, 56, 63, 64, 251, 252, 255, 256, 257, 4096]
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o += (n + 15) & ~15
    arena_bytes = offs[-1] + lens[-1]
    host = cases.splitmix64_bytes(24, arena_bytes)
    arena = eng.alloc(arena_bytes)
    arena.upload(host)
    for mode, seed in ((rsync_amd.FILESUM_PLAIN, 0), (rsync_amd.FILESUM_SEEDED, -7)):
        out = eng.file_sums_device(arena, list(zip(offs, lens)), mode, seed)
        got = out.download(16 * len(lens)).reshape(-1, 16)
        for i, (off, n) in enumerate(zip(offs, lens)):
            assert got[i].tobytes() == orc.file_sum(mode, seed, host[off:off + n]), (i, off, n, mode)


@pytest.mark.parametrize("shift", [0, 8, 13, 40])
def test_file_sums_lane_orders(shift):
    """rsg_testing_search_option 6 (the lane order's length buckets: 1 byte,
    256 B, 8 KiB, one bucket = the callers' order) changes which lane hashes
    which file, never a digest; out-of-range values are refused."""
    import rsync_amd
    from rsync_amd import _lib
    e = rsync_amd.Engine(0)
    try:
        e.set_option("fs_key_shift", shift)
        for bad in (-1, 41):
            with pytest.raises(_lib.RsgError):
                e.set_option("fs_key_shift", bad)
        rng = np.random.default_rng(25)
        lens = [int(x) for x in rng.integers(0, 40_000, 300)]
        files = [cases.splitmix64_bytes(200 + i, n) for i, n in enumerate(lens)]
        got = e.file_sums(files, rsync_amd.FILESUM_SEEDED, cases.SEED)
        for i in range(0, 300, 3):
            assert got[i] == orc.file_sum(1, cases.SEED, files[i]), i
    finally:
        e.close()
