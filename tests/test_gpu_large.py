"""GPU parity on multi-GiB arenas: file offsets and block offsets past 2 GiB
and 4 GiB, cfg4's full 100 000-file set and cfg5's 32 GiB file.

The reference takes int64 lengths and offsets everywhere
(internal/receiver/generator.go:325 `fileLen int64`, rsynccommon.go:14,
rsyncwire/wire.go:144 WriteInt64 past 2 GiB), so the kernels must give the
same records wherever a block sits in the arena -- and, since the records are
identical either way, the fallback census (rsg_block_sums_fallbacks) shows
that the LDS-DMA fast path was taken for every full wave / tile instead of
the per-lane fallback (the round-2 readfirstlane sign-extension bug sent
every wave with bit 31 of its offset set to the fallback).

Arenas are filled on the device with ONE splitmix64 stream, so any window of
them is regenerated on the host with cases.splitmix64_range; the oracle
checks every record of the small files near the 2/4 GiB boundaries and
sampled block ranges of the big files.
"""
import numpy as np
import pytest

import cases
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GIB = 1 << 30
STREAM_SEED = 0xC0FFEE
PAD = 1 << 20  # bytes after the last file: no wave reads past the arena, so no fallback is legitimate


@pytest.fixture(scope="module")
def eng():
    import rsync_amd
    e = rsync_amd.Engine(0)
    yield e
    e.close()


def _layout(unaligned: bool):
    """Files tiling [0, ~5 GiB): a big file up to 2 GiB - 8 MiB, ~16 MiB of
    4-64 KiB files across 2 GiB (irregular park tiles, waves straddling many
    files), a big file up to 4 GiB - 8 MiB, small files across 4 GiB, a big
    file of 1 GiB past it.  -> ([(offset, len)], kinds, arena_bytes)."""
    rng = np.random.default_rng(31)
    files, kinds, at = [], [], 0

    def add(n, kind):
        nonlocal at
        off = at
        if unaligned:  # odd offsets; the length shrinks so files never overlap
            sh = 1 + len(files) % 3
            files.append((off + sh, n - sh))
        else:
            files.append((off, n))
        kinds.append(kind)
        at = (off + n + 15) & ~15

    add(2 * GIB - (8 << 20) - 777, "big")
    while at < 2 * GIB + (8 << 20):
        add(int(rng.integers(4096, 65537)), "small")
    add(4 * GIB - (8 << 20) - at - 333, "big")
    while at < 4 * GIB + (8 << 20):
        add(int(rng.integers(4096, 65537)), "small")
    add(GIB + 12345, "big")
    return files, kinds, at + PAD


_ARENAS = {}


def _arena(eng, unaligned):
    """One device arena per layout for the whole module (5 GiB each)."""
    if unaligned not in _ARENAS:
        files, kinds, nbytes = _layout(unaligned)
        a = eng.alloc(nbytes)
        eng.fill_splitmix64(a, nbytes, STREAM_SEED)
        eng.synchronize()
        _ARENAS[unaligned] = (a, files, kinds)
    return _ARENAS[unaligned]


def _ranges(files, kinds, B, rng):
    """(file, b0, b1) block ranges to check: every block of the small files,
    and of each big file its first and last 64 blocks, 64 blocks around each
    of 2 GiB and 4 GiB when inside it, and 16 random blocks."""
    out = []
    for i, ((off, n), kind) in enumerate(zip(files, kinds)):
        nb = (n + B - 1) // B
        if kind == "small":
            out.append((i, 0, nb))
            continue
        out += [(i, 0, min(64, nb)), (i, max(0, nb - 64), nb)]
        for x in (2 * GIB, 4 * GIB):
            if off <= x < off + n:
                b = (x - off) // B
                out.append((i, max(0, b - 32), min(nb, b + 32)))
        out += [(i, int(b), int(b) + 1) for b in rng.integers(0, nb, 16)]
    return out


def _check(files, kinds, B, seed, rec, first):
    rng = np.random.default_rng(B)
    bad = []
    for i, b0, b1 in _ranges(files, kinds, B, rng):
        off, n = files[i]
        lo, hi = b0 * B, min(b1 * B, n)
        win = cases.splitmix64_range(STREAM_SEED, off + lo, hi - lo)
        want = orc.block_sums(win, B, seed)
        got = rec[(first[i] + b0) * 20:(first[i] + b1) * 20].tobytes()
        if got != want:
            bad.append((i, off, b0, b1))
    return bad


def _run(eng, unaligned, variant, B, seed=cases.SEED):
    from rsync_amd import _lib
    arena, files, kinds = _arena(eng, unaligned)
    desc = [(o, n, B) for o, n in files]
    plan = eng.plan(desc, arena.nbytes)
    recs = eng.alloc(plan.total_records * 20)
    eng.block_sums_fallbacks(reset=True)
    try:
        eng.set_block_sums_kernel(variant)
        plan.run(arena, seed, recs)
        eng.synchronize()
    finally:
        eng.set_block_sums_kernel(-1)
    fb = eng.block_sums_fallbacks(reset=True)
    rec = recs.download(plan.total_records * 20)
    recs.free()
    first = plan.first_record
    plan.close()
    return files, kinds, rec, first, fb


@pytest.mark.parametrize("variant,B", [(-1, 700), (2, 700), (1, 700), (4, 700), (4, 1024), (1, 131072),
                                       (-1, 131072), (-1, 4096), (7, 1000), (7, 4096), (7, 131072)])
def test_aligned_arena_past_4gib(eng, variant, B):
    """Aligned batch on a 5 GiB arena: park (regular and irregular tiles) and
    the staged kernels, every checked record equal to the oracle's and not one
    full wave or tile on the per-lane fallback."""
    files, kinds, rec, first, fb = _run(eng, False, variant, B)
    assert _check(files, kinds, B, cases.SEED, rec, first) == []
    assert fb == (0, 0), fb


@pytest.mark.parametrize("variant,B", [(-1, 700), (6, 700), (6, 32768), (6, 131072), (7, 32768), (-1, 131072)])
def test_unaligned_arena_past_4gib(eng, variant, B):
    """The same arena with every file at an odd offset (the unaligned staged
    kernel: pieces from the 4-byte aligned address below each block)."""
    files, kinds, rec, first, fb = _run(eng, True, variant, B, seed=-1)
    assert _check(files, kinds, B, -1, rec, first) == []
    assert fb == (0, 0), fb


def test_cfg4_full_set(eng):
    """BASELINE cfg4 at its real size: 100 000 files of uniform length in
    [4096, 65536] (PRNG seed 4, the bench's set), 3.48 GB arena at B = 700,
    automatic kernel (park; nearly every tile spans files).  256 random files
    plus the first and last against the oracle; no full tile on the fallback."""
    NF = 100_000
    lengths = np.random.default_rng(4).integers(4096, 65537, NF).tolist()
    offs, at = [], 0
    for n in lengths:
        offs.append(at)
        at += (n + 15) & ~15
    arena = eng.alloc(at + PAD)
    for f in range(NF):
        eng.fill_splitmix64(arena, lengths[f], f + 1, offset=offs[f])
    plan = eng.plan([(o, n, 700) for o, n in zip(offs, lengths)], arena.nbytes)
    recs = eng.alloc(plan.total_records * 20)
    eng.synchronize()
    eng.block_sums_fallbacks(reset=True)
    plan.run(arena, cases.SEED, recs)
    eng.synchronize()
    fb = eng.block_sums_fallbacks(reset=True)
    assert plan.total_records == sum((n + 699) // 700 for n in lengths)
    rng = np.random.default_rng(44)
    picks = sorted(set(rng.integers(0, NF, 256).tolist()) | {0, NF - 1})
    for f in picks:
        cnt = (lengths[f] + 699) // 700
        got = recs.download(cnt * 20, offset=plan.first_record[f] * 20).tobytes()
        assert got == orc.block_sums(cases.splitmix64_bytes(f + 1, lengths[f]), 700, cases.SEED), f
    assert fb == (0, 0), fb
    # the seeded whole-file sums of the same 100 000 files (match.go:52-53)
    import rsync_amd
    out = eng.file_sums_device(arena, list(zip(offs, lengths)), rsync_amd.FILESUM_SEEDED, cases.SEED)
    dig = out.download(16 * NF).reshape(-1, 16)
    for f in picks:
        assert dig[f].tobytes() == orc.file_sum(1, cases.SEED, cases.splitmix64_bytes(f + 1, lengths[f])), f
    out.free()
    arena.free()
    recs.free()
    plan.close()


def test_cfg5_32gib_file(eng):
    """BASELINE cfg5's per-GPU share at its real size: one 32 GiB file at
    B = 128 KiB (262 144 blocks of 2049 compressions).  Sampled blocks (48
    random, the blocks at every 2^31-byte boundary, the last) against the
    oracle; no full wave on the fallback."""
    size, B = 32 << 30, 131072
    arena = eng.alloc(size + PAD)
    eng.fill_splitmix64(arena, size, 5000)
    plan = eng.plan([(0, size, B)], arena.nbytes)
    nrec = plan.total_records
    assert nrec == size // B
    recs = eng.alloc(nrec * 20)
    eng.synchronize()
    eng.block_sums_fallbacks(reset=True)
    plan.run(arena, cases.SEED, recs)
    eng.synchronize()
    fb = eng.block_sums_fallbacks(reset=True)
    got = recs.download(nrec * 20).reshape(-1, 20)
    rng = np.random.default_rng(5)
    picks = set(rng.integers(0, nrec, 48).tolist()) | {nrec - 1}
    picks |= {(k << 31) // B for k in range(1, 16)} | {((k << 31) // B) - 1 for k in range(1, 17)}
    for b in sorted(picks):
        blk = cases.splitmix64_range(5000, b * B, B)
        assert got[b].tobytes() == orc.block_sums(blk, B, cases.SEED), b
    assert fb == (0, 0), fb
    arena.free()
    recs.free()
    plan.close()


@pytest.mark.parametrize("variant,kind", [(1, 0), (2, 1)])
def test_fallback_census_counts(eng, variant, kind):
    """The census is live: a file that ends exactly at the arena's end makes
    the last full wave (staged) / tile (park) read past the arena, so it must
    take the per-lane path -- and be counted -- with the records unchanged."""
    from rsync_amd import _lib
    n = 700 * 64 * 8
    d = cases.splitmix64_bytes(71, n)
    arena = eng.alloc(n)
    arena.upload(d)
    eng.block_sums_fallbacks(reset=True)
    try:
        eng.set_block_sums_kernel(variant)
        recs, total = eng.block_sums_device(arena, [(0, n, 700)], cases.SEED)
    finally:
        eng.set_block_sums_kernel(-1)
    fb = eng.block_sums_fallbacks(reset=True)
    assert recs.download(total * 20).tobytes() == orc.block_sums(d, 700, cases.SEED)
    assert fb[kind] >= 1 and fb[1 - kind] == 0, fb


@pytest.mark.parametrize("unaligned", [False, True])
def test_file_sums_past_4gib(eng, unaligned):
    """Whole-file MD4 (both modes, rsyncchecksum.go:60-66 and
    match.go:52-53) of the ~1000 small files around 2 GiB and 4 GiB of the
    5 GiB arena in one call: a wave's 64 files (longest first) lie on both
    sides of 4 GiB, so the staged kernel's per-lane 64-bit DMA addresses span
    more than 2 GiB."""
    import rsync_amd
    arena, files, kinds = _arena(eng, unaligned)
    small = [f for f, k in zip(files, kinds) if k == "small"]
    for mode, seed in ((rsync_amd.FILESUM_PLAIN, 0), (rsync_amd.FILESUM_SEEDED, cases.SEED)):
        out = eng.file_sums_device(arena, small, mode, seed)
        got = out.download(16 * len(small)).reshape(-1, 16)
        out.free()
        for i, (off, n) in enumerate(small):
            want = orc.file_sum(mode, seed, cases.splitmix64_range(STREAM_SEED, off, n))
            assert got[i].tobytes() == want, (i, off, n, mode)


def test_sender_search_past_4gib(eng):
    """The sender's rolling match (match.go:93-210) over a 5 GiB source: the
    reference's offsets are int64, so the packed roll's tiles past 2^32
    bytes, its carried start windows and the hand-off to roll_kernel's edge
    tiles must give the reference's walk.  The source is the basis with
    blocks overwritten on both sides of 4 GiB and at the remainder block:
    every other block matches at its own offset, in order (a modified block
    leaves the walk stepping byte by byte to the next block boundary)."""
    B = 131072
    size = 5 * GIB + 12345
    basis = eng.alloc(size)
    src = eng.alloc(size)
    try:
        eng.fill_splitmix64(basis, size, 77)
        eng.fill_splitmix64(src, size, 77)
        recs, total = eng.block_sums_device(basis, [(0, size, B)], cases.SEED)
        s1, s2 = orc.parse_records(recs.download(total * 20).tobytes())
        recs.free()
        head = orc.sum_head(size, B)
        assert head[0] == total == size // B + 1 and head[3] == 12345
        four = 4 * GIB // B
        bad = {four - 1, four, four + 1, total - 1}
        bad |= {int(x) for x in np.random.default_rng(5).integers(0, total - 1, 12)}
        for b in sorted(bad):
            eng.fill_splitmix64(src, 64, 1000 + b, offset=b * B + 100)
        eng.synchronize()
        got = eng.hash_search_device(src, size, head, s1, s2, orc.stable_targets(s1), cases.SEED)
        assert got == [(i * B, i) for i in range(total) if i not in bad]
    finally:
        src.free()
        basis.free()


def test_release_arenas(eng):
    """Frees the module's 5 GiB arenas (runs last in this file)."""
    for a, _, _ in _ARENAS.values():
        a.free()
    _ARENAS.clear()


def test_cfg3_batch_three_files_vs_oracle(eng):
    """The bench's call shape at real size: three cfg3 files (1 GiB bases,
    ~50 % overwritten sources with insertions and deletions, B = 32 768) in
    ONE rsg_hash_search_batch_device call, so the pipeline runs as in the
    bench -- each file's confirmation beside the next file's roll on the
    CUs the roll leaves free, the last one beside the previous one, the
    windows through the line-window kernel -- and every file's match list
    equals the oracle's hashSearch (~20 s of oracle time)."""
    size = 1 << 30
    rng = np.random.default_rng(33)
    jobs, want, bufs = [], [], []
    for f in range(3):
        basis = eng.alloc(size)
        src = eng.alloc(size + 4096)
        n = cases.make_cfg3_file(eng, basis, src, size, 40 + f, 32768, rng)
        eng.synchronize()
        rec = orc.block_sums(basis.download(size), 0, cases.SEED)
        basis.free()
        s1, s2 = orc.parse_records(rec)
        tg = orc.stable_targets(s1)
        head = orc.sum_head(size, 0)
        want.append(orc.hash_search(src.download(n), head, s1, s2, tg, cases.SEED)[0])
        jobs.append((src, n, head, s1, s2, tg))
        bufs.append(src)
    got = eng.hash_search_batch(jobs, cases.SEED)
    for f in range(3):
        assert len(want[f]) > 10_000
        assert got[f] == want[f], f
    for b in bufs:
        b.free()


def test_cfg3_real_size_vs_oracle(eng):
    """BASELINE cfg3 at its real size, one file: a 1 GiB basis and a source
    with ~50 % of its bytes overwritten plus insertions and deletions (the
    bench's recipe, tests/cases.make_cfg3_file), B = SumSizesSqroot(1 GiB) =
    32 768.  The basis sums come from the oracle (and equal the kernel's), and
    the batched device search -- the bench's call -- returns exactly the
    oracle's hashSearch match list (~7 s of oracle time)."""
    import rsync_amd
    size = 1 << 30
    rng = np.random.default_rng(3)
    basis = eng.alloc(size)
    src = eng.alloc(size + 4096)
    n = cases.make_cfg3_file(eng, basis, src, size, 3, 32768, rng)
    eng.synchronize()
    bh = basis.download(size)
    head = orc.sum_head(size, 0)
    assert head[1] == 32768
    rec = orc.block_sums(bh, 0, cases.SEED)
    recs, total = eng.block_sums_device(basis, [(0, size, 0)], cases.SEED)
    assert recs.download(total * 20).tobytes() == rec
    recs.free()
    s1, s2 = orc.parse_records(rec)
    tg = orc.stable_targets(s1)
    got = eng.hash_search_batch([(src, n, head, s1, s2, tg)], cases.SEED)[0]
    sh = src.download(n)
    want, _, _ = orc.hash_search(sh, head, s1, s2, tg, cases.SEED)
    assert len(want) > 10_000
    assert got == want
    basis.free()
    src.free()


