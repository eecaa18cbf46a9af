"""Deterministic input builders shared by the fixture generator and the tests.

Every byte comes from the splitmix64 stream, restated here
in numpy so the builders need neither the oracle nor a GPU.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
SEED = 0x1BADB002  # checksum seed used by the BASELINE configs


def splitmix64_bytes(seed: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        st = (np.uint64(seed & M64) + np.arange(1, words + 1, dtype=np.uint64)
              * np.uint64(0x9E3779B97F4A7C15))
        z = st
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def splitmix64_range(seed: int, start: int, n: int) -> np.ndarray:
    """Bytes [start, start+n) of the splitmix64(seed) stream (counter-based, so
    any window of a huge synthetic file is cheap to regenerate)."""
    w0 = start // 8
    w1 = (start + n + 7) // 8
    with np.errstate(over="ignore"):
        st = (np.uint64(seed & M64) + np.arange(w0 + 1, w1 + 1, dtype=np.uint64)
              * np.uint64(0x9E3779B97F4A7C15))
        z = st
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    o = start - 8 * w0
    return b[o:o + n].copy()


def weak_kat_file() -> np.ndarray:
    """internal/rsyncchecksum/checksum_test.go:12-18,36: 0x11 x 1 MiB || 0xbb x 1 MiB
    || 0xee x 1 MiB."""
    mib = 1 << 20
    return np.concatenate([np.full(mib, 0x11, np.uint8), np.full(mib, 0xBB, np.uint8),
                           np.full(mib, 0xEE, np.uint8)])


def ragged_lengths():
    """File lengths around every MD4/weak boundary the kernels special-case."""
    return [0, 1, 2, 3, 4, 5, 51, 52, 55, 56, 59, 60, 63, 64, 65, 119, 120, 127, 128,
            675, 676, 677, 699, 700, 701, 1023, 1024, 1400, 1401, 1773, 2047, 5000,
            65536 + 17]


def mutate(basis: np.ndarray, seed: int, frac: float, run_min: int, run_max: int,
           n_ins: int = 0, n_del: int = 0) -> np.ndarray:
    """Copy of `basis` with random runs overwritten until ~frac of the bytes are
    touched, plus n_ins insertions / n_del deletions at random unaligned offsets
    (the cfg3 recipe of SURVEY.md §8(d), scaled down)."""
    rng = np.random.default_rng(seed)
    out = basis.copy()
    target = int(frac * basis.size)
    touched = 0
    while touched < target and basis.size > run_max:
        ln = int(rng.integers(run_min, run_max + 1))
        pos = int(rng.integers(0, basis.size - ln))
        out[pos:pos + ln] = rng.integers(0, 256, ln, dtype=np.uint8)
        touched += ln
    for _ in range(n_ins):
        pos = int(rng.integers(0, out.size))
        ln = int(rng.integers(1, 64))
        out = np.concatenate([out[:pos], rng.integers(0, 256, ln, dtype=np.uint8), out[pos:]])
    for _ in range(n_del):
        if out.size < 128:
            break
        pos = int(rng.integers(0, out.size - 64))
        ln = int(rng.integers(1, 64))
        out = np.concatenate([out[:pos], out[pos + ln:]])
    return out


def match_cases():
    """name -> (src, basis, block_len (0 = sqrt sizing), seed)."""
    c = {}
    b = splitmix64_bytes(101, 50_000)
    c["aligned_700"] = (mutate(b, 1, 0.3, 700, 1400), b, 700, SEED)
    b = splitmix64_bytes(102, 80_000)
    c["shifted_700"] = (mutate(b, 2, 0.2, 1, 1400, n_ins=4, n_del=4), b, 700, SEED)
    b = splitmix64_bytes(103, 60_000)
    c["shifted_1773_seed0"] = (mutate(b, 3, 0.2, 1, 3000, n_ins=3, n_del=3), b, 1773, 0)
    b = splitmix64_bytes(104, 70_001)
    c["sqrt_sizing_seedm1"] = (mutate(b, 4, 0.25, 100, 900, n_ins=2, n_del=2), b, 0, -1)
    blk = splitmix64_bytes(105, 700)
    b = np.concatenate([blk, splitmix64_bytes(106, 1400), blk, blk, splitmix64_bytes(107, 333)])
    s = np.concatenate([splitmix64_bytes(108, 50), blk, blk, splitmix64_bytes(109, 10), b])
    c["dup_blocks"] = (s, b, 700, SEED)
    b = splitmix64_bytes(110, 7_777)
    c["tail_block"] = (np.concatenate([splitmix64_bytes(111, 123), b[-(7_777 % 700):]]), b, 700, SEED)
    c["empty_src"] = (np.zeros(0, np.uint8), splitmix64_bytes(112, 3000), 700, SEED)
    c["empty_basis"] = (splitmix64_bytes(113, 3000), np.zeros(0, np.uint8), 700, SEED)
    c["periodic_bb"] = (np.full(10_000, 0xBB, np.uint8), np.full(5_000, 0xBB, np.uint8), 700, SEED)
    c["src_shorter_than_block"] = (splitmix64_bytes(114, 300), splitmix64_bytes(115, 2000), 700, SEED)
    b = splitmix64_bytes(116, 1_000)
    c["src_equals_short_tail"] = (b[700:].copy(), b, 700, SEED)
    # a literal run long enough for the -2 flush (match.go:198-204)
    b = splitmix64_bytes(117, 4_000)
    s = np.concatenate([b[:1400], splitmix64_bytes(118, 600_000), b[1400:]])
    c["long_literal_flush"] = (s, b, 700, SEED)
    b = splitmix64_bytes(119, 200_000)
    c["identical_sqrt"] = (b.copy(), b, 0, SEED)
    return c


def make_cfg3_file(eng, basis, src, size, seed, B, rng):
    """Source = the basis with random runs (1 B .. 2B long) overwritten until
    ~50% of the bytes differ, plus a few insertions/deletions so matches fall at
    offsets that are not multiples of B.  Built on the
    device with splitmix64 fills and device copies; returns the source length."""
    import rsync_amd
    from rsync_amd import _lib
    eng.fill_splitmix64(basis, size, seed)
    # shifts: copy basis pieces with small gaps/overlaps into src
    cuts = sorted(rng.choice(np.arange(1, size - 1), 8, replace=False).tolist())
    pos_src, prev = 0, 0
    for i, c in enumerate(cuts + [size]):
        n = max(0, c - prev)
        _lib.check(_lib.lib.rsg_memcpy_d2d(eng.ctx, rsync_amd.engine.ctypes.c_void_p(src.ptr + pos_src),
                                            rsync_amd.engine.ctypes.c_void_p(basis.ptr + prev), n), eng.ctx)
        pos_src += n
        if i % 2 == 0 and c < size:  # insertion of random bytes
            k = int(rng.integers(1, 64))
            eng.fill_splitmix64(src, k, seed * 7919 + i, offset=pos_src)
            pos_src += k
        elif c < size:  # deletion
            prev = c + int(rng.integers(1, 64))
            continue
        prev = c
    total = pos_src
    touched, run_seed = 0, 1
    while touched < total // 2:
        ln = int(rng.integers(1, 2 * B))
        at = int(rng.integers(0, total - ln))
        eng.fill_splitmix64(src, ln, seed * 104729 + run_seed, offset=at)
        run_seed += 1
        touched += ln
    return total
