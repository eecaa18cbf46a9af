"""GPU parity of the receiver block-sum kernel (generator.go:325-350) against
the oracle and the golden fixtures.  Everything goes through the C-ABI."""
import hashlib
import json
import os
import struct

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


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_weak_kat_through_gpu(eng):
    """The reference's only pinned values (checksum_test.go:32-73): 1780 weak
    sums of 1768-byte chunks, computed as blocks by the GPU kernel."""
    g = load("weak_kat.json")
    f = cases.weak_kat_file()
    heads, rec, _ = eng.block_sums([f], 0, g["chunk"])
    assert heads[0].count == 1780
    s1 = np.frombuffer(rec, np.uint8).reshape(-1, 20)[:, :4].copy().view("<u4").reshape(-1)
    for lo, hi, v in g["runs"]:
        assert (s1[lo:hi + 1] == v).all(), (lo, hi)
    assert rec == orc.block_sums(f, g["chunk"], 0)


def test_cfg1_golden(eng):
    g = load("block_sums.json")
    data = cases.splitmix64_bytes(1, 1 << 20)
    for key in ("cfg1_B1024", "cfg1_B700"):
        e = g[key]
        heads, rec, _ = eng.block_sums([data], e["seed"], e["block_len_arg"])
        assert list(heads[0].astuple()) == e["head"]
        assert hashlib.sha256(struct.pack("<4i", *heads[0].astuple()) + rec).hexdigest() == e["sha256_head_records"]


def test_ragged_golden_host_path(eng):
    g = load("block_sums.json")["ragged"]
    for e in g:
        d = cases.splitmix64_bytes(e["data_seed"], e["len"])
        heads, rec, _ = eng.block_sums([d], e["seed"], e["block_len"])
        assert list(heads[0].astuple()) == e["head"]
        assert hashlib.sha256(rec).hexdigest() == e["sha256_records"], e


def test_ragged_batch_one_call(eng):
    """All ragged files in ONE batch (lanes of one wave straddle files)."""
    lens = cases.ragged_lengths()
    for blen, seed in ((700, cases.SEED), (1773, -1), (63, 7), (0, 0)):
        files = [cases.splitmix64_bytes(2000 + i, n) for i, n in enumerate(lens)]
        heads, rec, first = eng.block_sums(files, seed, blen)
        want = b"".join(orc.block_sums(f, blen, seed) for f in files)
        assert rec == want
        for i, f in enumerate(files):
            assert heads[i].astuple() == orc.sum_head(f.size, blen)


def _device_case(eng, offsets, lens, blens, seed, arena_bytes=None):
    end = max(o + n for o, n in zip(offsets, lens)) if lens else 0
    arena_bytes = arena_bytes or end
    host = np.zeros(arena_bytes, np.uint8)
    datas = []
    for i, (o, n) in enumerate(zip(offsets, lens)):
        d = cases.splitmix64_bytes(3000 + i, n)
        host[o:o + n] = d
        datas.append(d)
    arena = eng.alloc(arena_bytes)
    arena.upload(host)
    recs, total = eng.block_sums_device(arena, list(zip(offsets, lens, blens)), seed)
    got = recs.download(total * 20).tobytes()
    want = b"".join(orc.block_sums(d, b, seed) for d, b in zip(datas, blens))
    return got, want


def test_device_unaligned_offsets(eng):
    """Files at odd arena offsets and odd block lengths: the funnel-shift path."""
    lens = [5000, 701, 64, 3, 1773 * 3 + 2, 4096]
    offs, o = [], 1
    for n in lens:
        offs.append(o)
        o += n + 3
    got, want = _device_case(eng, offs, lens, [700, 701, 13, 700, 1773, 1001], cases.SEED)
    assert got == want


def test_device_file_ends_at_arena_end(eng):
    """The tail chunk's loads are guarded at the arena end (no over-read)."""
    for n in (1, 63, 64, 65, 700, 701, 1999):
        for off in (0, 1, 2, 3, 4):
            got, want = _device_case(eng, [off], [n], [700], -1, arena_bytes=off + n)
            assert got == want, (n, off)


def test_device_aligned_multi_file(eng):
    lens = [1 << 20] * 8 + [12345, 0, 77]
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o += (n + 15) & ~15
    got, want = _device_case(eng, offs, lens, [700] * len(lens), cases.SEED)
    assert got == want


@pytest.mark.parametrize("variant", [-1, 7])
def test_planned_cfg2_full(eng, variant):
    """cfg2 at full size (1024 x 1 MiB @ B=700, generated on the device):
    every one of the 1 533 952 records bit-exact vs the oracle (~1.5 s of
    oracle time), record count and layout exact -- the automatic choice
    (park) and the pipelined staged kernel."""
    n_files, size = 1024, 1 << 20
    arena = eng.alloc(n_files * size)
    for f in range(n_files):
        eng.fill_splitmix64(arena, size, f + 1, offset=f * size)
    plan = eng.plan([(f * size, size, 700) for f in range(n_files)], n_files * size)
    assert plan.total_records == n_files * 1498
    recs = eng.alloc(plan.total_records * 20)
    try:
        eng.set_block_sums_kernel(variant)
        plan.run(arena, cases.SEED, recs)
        eng.synchronize()
    finally:
        eng.set_block_sums_kernel(-1)
    allrec = recs.download(plan.total_records * 20).tobytes()
    for f in range(n_files):
        o = plan.first_record[f] * 20
        assert allrec[o:o + 1498 * 20] == orc.block_sums(cases.splitmix64_bytes(f + 1, size), 700, cases.SEED), f


def test_large_block_sampled(eng):
    """cfg5 shape (B = 128 KiB, 2049 MD4 compressions per lane) on a 1 GiB
    device file: sampled blocks, including the last, vs the oracle."""
    size, B = (1 << 30) + 1234, 131072
    arena = eng.alloc(size)
    eng.fill_splitmix64(arena, size, 55)
    recs, total = eng.block_sums_device(arena, [(0, size, B)], cases.SEED)
    assert total == (size + B - 1) // B
    rng = np.random.default_rng(0)
    picks = sorted(set(rng.integers(0, total, 24).tolist()) | {0, total - 1})
    all_rec = recs.download(total * 20).reshape(-1, 20)
    for b in picks:
        n = min(B, size - b * B)
        blk = cases.splitmix64_range(55, b * B, n)
        assert all_rec[b].tobytes() == orc.block_sums(blk, B, cases.SEED), b


def test_host_path_splits_large_file(eng):
    """A file larger than one staging batch (64 MiB) is cut at block boundaries."""
    d = cases.splitmix64_bytes(77, (150 << 20) + 333)
    heads, rec, _ = eng.block_sums([d, d[:1000]], 5, 700)
    assert rec == orc.block_sums(d, 700, 5) + orc.block_sums(d[:1000], 700, 5)


def test_checksum_api(eng):
    import rsync_amd
    d = cases.splitmix64_bytes(9, 5000)
    for n in (1, 3, 4, 55, 56, 64, 700, 5000):
        assert rsync_amd.checksum1(d[:n]) == orc.checksum1(d[:n])
        assert rsync_amd.checksum2(-7, d[:n]) == orc.checksum2(-7, d[:n])


def test_generate_and_send_sums_wire(eng):
    import rsync_amd
    d = cases.splitmix64_bytes(1, 1 << 20)
    conn = rsync_amd.Conn()
    eng.generate_and_send_sums(conn, d, d.size, cases.SEED)
    want = orc.head_bytes(orc.sum_sizes_sqroot(d.size)) + orc.block_sums(d, 0, cases.SEED)
    assert bytes(conn.buf) == want


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6, 7])
@pytest.mark.parametrize("blen", [700, 64, 1024, 1400, 1773, 4096, 131072])
def test_kernel_variants_match(eng, variant, blen):
    """Every kernel variant (direct / staged / park / long / staged with 128-
    and 512-byte segments) gives the oracle's
    records, including waves and park tiles that straddle files; unaligned
    arenas make the LDS-DMA variants fall back to direct."""
    from rsync_amd import _lib
    lens = [1 << 20, 700 * 64 * 3 + 5, 12345, 64, 1, 0, 300_001]
    files = [cases.splitmix64_bytes(4000 + i, n) for i, n in enumerate(lens)]
    want = b"".join(orc.block_sums(f, blen, cases.SEED) for f in files)
    try:
        eng.set_block_sums_kernel(variant)
        _, rec, _ = eng.block_sums(files, cases.SEED, blen)
        arena = eng.alloc(sum(lens))
        offs = np.cumsum([0] + lens[:-1]).tolist()
        arena.upload(np.concatenate(files))
        recs, total = eng.block_sums_device(arena, [(o, n, blen) for o, n in zip(offs, lens)], cases.SEED)
        rec_dev = recs.download(total * 20).tobytes()
    finally:
        eng.set_block_sums_kernel(-1)
    assert rec == want
    assert rec_dev == want


@pytest.mark.parametrize("blen", [2000, 2289, 3504, 6000, 1773, 4222, 5882, 1448])
def test_line_windows_piece_strides(eng, blen):
    """Variant 7 (line windows) at block lengths whose launch takes 10-unit
    pieces (2000 / 2289 / 3504 / 6000: the bank-conflict choice) and 9-unit
    ones (1773 / 4222 / 5882 / 1448), on the sweep's layout (files back to
    back, every block off the 128-byte lines) and on ragged files, through
    the host path and a device arena; every record equal to the oracle's."""
    lens = [1 << 20, (1 << 20) - 1, blen * 64 * 2 + 7, blen, 1, 12345, 0, 300_001]
    files = [cases.splitmix64_bytes(8100 + i, n) for i, n in enumerate(lens)]
    want = b"".join(orc.block_sums(f, blen, cases.SEED) for f in files)
    try:
        eng.set_block_sums_kernel(7)
        _, rec, _ = eng.block_sums(files, cases.SEED, blen)
        arena = eng.alloc(sum(lens))
        offs = np.cumsum([0] + lens[:-1]).tolist()
        arena.upload(np.concatenate(files))
        recs, total = eng.block_sums_device(arena, [(o, n, blen) for o, n in zip(offs, lens)], cases.SEED)
        rec_dev = recs.download(total * 20).tobytes()
    finally:
        eng.set_block_sums_kernel(-1)
    assert rec == want
    assert rec_dev == want


@pytest.mark.parametrize("variant", [-1, 3, 6, 7])
@pytest.mark.parametrize("blen", [700, 32768, 8192, 131072])
def test_unaligned_windows(eng, variant, blen):
    """The sender's confirmation shape: windows of one block each at random
    byte offsets of a source (plus windows cut short by the source's end and
    one ending exactly there), enough for full 64-window waves of the
    unaligned staged kernel (variant 6, the automatic choice for every
    unaligned batch in a 4-byte aligned arena) and of the deep-prefetch
    kernel (3)."""
    from rsync_amd import _lib
    size = 24 << 20
    src = cases.splitmix64_bytes(777, size)
    arena = eng.alloc(size)
    arena.upload(src)
    rng = np.random.default_rng(blen)
    offs = sorted(int(x) for x in rng.integers(0, size - blen, 300))
    wins = [(o, blen) for o in offs] + [(size - blen // 3, blen // 3), (size - blen, blen), (size - 1, 1)]
    want = b"".join(orc.block_sums(src[o:o + n], blen, cases.SEED) for o, n in wins)
    try:
        eng.set_block_sums_kernel(variant)
        recs, total = eng.block_sums_device(arena, [(o, n, blen) for o, n in wins], cases.SEED)
        got = recs.download(total * 20).tobytes()
    finally:
        eng.set_block_sums_kernel(-1)
    assert got == want


@pytest.mark.parametrize("variant", [1, 3, 4, 6, 7])
def test_variants_long_blocks_full_waves(eng, variant):
    """cfg5's block length with full 64-block waves (the staged LDS-DMA path
    of variants 1/4/5, not only their direct fallback): a 24 MiB file at
    B = 128 KiB plus a ragged second file."""
    from rsync_amd import _lib
    lens = [24 << 20, (3 << 20) + 777]
    datas = [cases.splitmix64_bytes(6000 + i, n) for i, n in enumerate(lens)]
    offs = [0, lens[0]]
    arena = eng.alloc(sum(lens))
    arena.upload(np.concatenate(datas))
    want = b"".join(orc.block_sums(d, 131072, cases.SEED) for d in datas)
    try:
        eng.set_block_sums_kernel(variant)
        recs, total = eng.block_sums_device(arena, [(o, n, 131072) for o, n in zip(offs, lens)], cases.SEED)
        got = recs.download(total * 20).tobytes()
    finally:
        eng.set_block_sums_kernel(-1)
    assert got == want


@pytest.mark.parametrize("variant,blen", [(2, 64), (7, 64), (7, 1400)])
def test_persistent_waves_many_groups(eng, variant, blen):
    """Many more 64-block groups than resident waves: the persistent park
    grid (one workgroup per CU, tiles handed round) and the line-window
    kernel over files of ragged lengths straddling groups, one ending
    exactly at the arena end (the last group takes the per-lane path)."""
    rng = np.random.default_rng(blen)
    # B = 64: 6 k groups, more than the resident waves of every variant (4096
    # at 128-byte segments); B = 1400: 3.7 k groups (more than 2048 / 1024
    # resident waves at 256 / 512-byte segments).  B = 4096 on a 5 GiB arena:
    # tests/test_gpu_large.py
    total = (24 << 20) if blen == 64 else (320 << 20)
    lens = []
    while sum(lens) < total:
        lens.append(int(rng.integers(1, 6 << 20)))
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o += (n + 15) & ~15
    arena_bytes = offs[-1] + lens[-1]
    host = np.zeros(arena_bytes, np.uint8)
    host[:] = cases.splitmix64_bytes(31337, arena_bytes)
    want = b"".join(orc.block_sums(host[o:o + n], blen, cases.SEED) for o, n in zip(offs, lens))
    arena = eng.alloc(arena_bytes)
    arena.upload(host)
    try:
        eng.set_block_sums_kernel(variant)
        recs, total_recs = eng.block_sums_device(arena, [(o, n, blen) for o, n in zip(offs, lens)], cases.SEED)
        got = recs.download(total_recs * 20).tobytes()
    finally:
        eng.set_block_sums_kernel(-1)
    assert got == want


@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3, 4, 6, 7])
def test_variants_device_aligned_arena(eng, variant):
    """Aligned device arena (the staged / park fast paths), files straddling
    waves and tiles, a file ending exactly at the arena end (park's direct
    tiles), blocks of 700/64/703 bytes (64: park with tiny blocks, ragged
    tails hashed by the predicated path) and the automatic choice's
    boundaries (-1: 703 park, 704..4096 128-byte segments, 4097 and up
    256-byte segments)."""
    from rsync_amd import _lib
    lens = [1 << 20, 700 * 64 * 3 + 5, 12344, 64, 4, 0, 300_000, 70_000 * 3]
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o += (n + 15) & ~15
    arena_bytes = offs[-1] + lens[-1]
    host = np.zeros(arena_bytes, np.uint8)
    datas = []
    for i, (off, n) in enumerate(zip(offs, lens)):
        d = cases.splitmix64_bytes(5000 + i, n)
        host[off:off + n] = d
        datas.append(d)
    arena = eng.alloc(arena_bytes)
    arena.upload(host)
    for blen in (700, 64, 703, 704, 1024, 1536, 1537, 4096, 4097):
        want = b"".join(orc.block_sums(d, blen, cases.SEED) for d in datas)
        try:
            eng.set_block_sums_kernel(variant)
            recs, total = eng.block_sums_device(arena, [(o, n, blen) for o, n in zip(offs, lens)], cases.SEED)
            got = recs.download(total * 20).tobytes()
        finally:
            eng.set_block_sums_kernel(-1)
        assert got == want, blen


SEED_T = 0x1BADB002


def test_pinned_sources_direct_dma(eng):
    """Files that already sit in rsg_alloc_pinned memory skip the staging copy
    (per-piece DMA from the caller's buffer); records must be identical to the
    staged path and to the oracle, including ragged lengths and a file that
    spans several 64 MiB batches."""
    rng = np.random.default_rng(21)
    lens = [0, 1, 700, 701, 5000, 1 << 20, (96 << 20) + 13]
    total = sum((n + 63) & ~63 for n in lens)
    pin = eng.alloc_pinned(total)
    try:
        views, at = [], 0
        for n in lens:
            v = pin[at:at + n]
            v[:] = rng.integers(0, 256, n, dtype=np.uint8)
            views.append(v)
            at += (n + 63) & ~63
        heads_p, rec_p, _ = eng.block_sums(views, SEED_T, 700)
        heads_s, rec_s, _ = eng.block_sums([v.copy() for v in views], SEED_T, 700)
        assert rec_p == rec_s
        assert [h.astuple() for h in heads_p] == [h.astuple() for h in heads_s]
        exp = b"".join(orc.block_sums(v.copy(), 700, SEED_T) for v in views[:-1])
        assert rec_p[: len(exp)] == exp
    finally:
        eng.free_pinned(pin)


def test_kernel_knobs_are_per_context():
    """The kernel variant set on one context leaves another context's choice
    alone (process-global switches could affect a concurrent
    caller), and only the shipped variants are accepted."""
    import rsync_amd
    a, b = rsync_amd.Engine(0), rsync_amd.Engine(0)
    try:
        files = [cases.splitmix64_bytes(60 + i, 1 << 20) for i in range(8)]
        want = b"".join(orc.block_sums(f, 700, cases.SEED) for f in files)
        a.set_block_sums_kernel(0)
        a.block_sums_fallbacks(reset=True)
        _, rec, _ = b.block_sums(files, cases.SEED, 700)  # b: automatic (park)
        assert rec == want
        _, rec_a, _ = a.block_sums(files, cases.SEED, 700)  # a: direct
        assert rec_a == want
        a.set_block_sums_kernel(-1)
        for bad in (99, 5, 8, 12, 14, 15, -2):
            with pytest.raises(rsync_amd.RsgError):
                a.set_block_sums_kernel(bad)
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("blen", [2176, 16384, 32768, 32769, 1224, 1280, 24576, 24577, 703, 704])
def test_automatic_rule_library_packed(eng, blen):
    """The automatic rule at its boundaries on the library's own packing
    (rsg_block_sums_host packs files at 128-byte offsets, so blocks whose
    length is a multiple of 128 start on 128-byte lines: variant 4 up to
    32 KiB, else 14 up to 24 KiB when 512-byte segments read <= 1.2 B, else
    1): ragged file lengths, every record equal to the oracle's."""
    rng = np.random.default_rng(blen)
    lens = [int(x) for x in rng.integers(1, 3 << 20, 5)] + [blen * 64 + 3, blen, 1]
    files = [cases.splitmix64_bytes(7000 + i, n) for i, n in enumerate(lens)]
    _, rec, _ = eng.block_sums(files, cases.SEED, blen)
    assert rec == b"".join(orc.block_sums(f, blen, cases.SEED) for f in files)


SQRT_LENS_MIB = [1, 2, 3, 5, 9, 17, 33, 64]


def test_reference_sizing_sqrt_lengths(eng):
    """The reference's own block length B = isqrt(len) (rsynccommon.go:22) for
    files of 1, 2, 3, 5, 9, 17, 33 and 64 MiB -- B = 1024, 1448, 1773, 2289,
    3072, 4222, 5882, 8192, most not a multiple of 128 or even of 4 -- on the
    device arena the sweep measures (tools/blocklen_sweep.py SWEEP_SQRT=1:
    files packed at 128-byte offsets, two per length, the second one byte
    short) through the automatic rule, and through the host path with the
    default sizing (block_len 0); every record equal to the oracle's."""
    import math
    lens = [x for m in SQRT_LENS_MIB for x in ((m << 20), (m << 20) - 1)]
    blens = [math.isqrt(m << 20) for m in SQRT_LENS_MIB for _ in range(2)]
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o += (n + 127) & ~127
    host = np.zeros(o, np.uint8)
    datas = []
    for i, (off, n) in enumerate(zip(offs, lens)):
        d = cases.splitmix64_bytes(9100 + i, n)
        host[off:off + n] = d
        datas.append(d)
    want = b"".join(orc.block_sums(d, b, cases.SEED) for d, b in zip(datas, blens))
    arena = eng.alloc(o)
    arena.upload(host)
    recs, total = eng.block_sums_device(arena, [(a, n, b) for a, n, b in zip(offs, lens, blens)], cases.SEED)
    assert recs.download(total * 20).tobytes() == want
    # host path, reference sizing chosen by the library (block_len 0 -> isqrt for len > 490000)
    heads, rec, _ = eng.block_sums(datas[::2], cases.SEED, 0)
    assert [h.block_len for h in heads] == blens[::2]
    assert rec == b"".join(orc.block_sums(d, b, cases.SEED) for d, b in zip(datas[::2], blens[::2]))
