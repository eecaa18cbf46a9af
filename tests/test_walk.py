"""The sender's greedy walk (the host half of hashSearch, match.go:93-210)
through the rsg_testing_walk hook: the GPU confirmation is replaced by a table
of answers, so the walk's result and the number of confirmation round trips it
would issue are checked on the CPU.

Round 3's stall (a 1 GiB source whose candidates were dense and mostly false)
came from the walk confirming ~2 candidates per GPU round trip; the bound
tested here is what keeps such a stretch to a few dozen round trips."""
import ctypes

import numpy as np
import pytest

from rsync_amd import _lib


def walk(cand, truth, size, head, spec=0):
    """spec: 1 = speculative selection of sparse batches, 2 = every pending
    candidate, 0 = the library's default (RSG_CONFIRM_SPEC)."""
    cand = np.ascontiguousarray(cand, np.uint64)
    truth = np.ascontiguousarray(truth, np.int32)
    h = _lib.SumHead(*head)
    cap = max(1, cand.size)
    out = (_lib.Match * cap)()
    n = ctypes.c_uint64()
    stats = (ctypes.c_uint64 * 2)(spec, 0)
    _lib.check(_lib.lib.rsg_testing_walk(cand.ctypes.data, cand.size, truth.ctypes.data, size,
                                         ctypes.byref(h), out, cap, ctypes.byref(n), stats))
    return [(out[k].offset, out[k].index) for k in range(n.value)], stats[0], stats[1]


def reference_walk(cand, truth, size, head):
    """match.go's greedy order over the candidate offsets: visit q, a block
    b >= 0 moves to q + Len_b (match.go:158), a miss to the next offset."""
    count, blen, _, rem = head
    last = rem if rem else blen
    end = max(size + 1 - last, 1)  # match.go:70
    pos, out = 0, []
    for q, b in zip(cand.tolist(), truth.tolist()):
        if q >= end:
            break
        if q < pos or b < 0:
            continue
        out.append((q, b))
        pos = q + (rem if (b == count - 1 and rem) else blen)
    return out


def head_for(size, blen):
    count = -(-size // blen)
    return (count, blen, 16, size % blen)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("density", [0.0005, 0.02, 0.3, 1.0])
def test_walk_equals_greedy_reference(seed, density):
    rng = np.random.default_rng(seed)
    blen = int(rng.choice([700, 1024, 4096]))
    size = int(rng.integers(blen, 3_000_000))
    head = head_for(size, blen)
    n = max(1, int(size * density))
    cand = np.unique(rng.integers(0, size, n)).astype(np.uint64)
    p_true = rng.choice([0.0, 0.05, 0.5, 1.0])
    truth = np.where(rng.random(cand.size) < p_true, rng.integers(0, head[0], cand.size), -1).astype(np.int32)
    got, trips, windows = walk(cand, truth, size, head)
    assert got == reference_walk(cand, truth, size, head)
    assert windows <= cand.size * 2


def test_dense_false_candidates_bounded_round_trips():
    """Every offset of a 600 000-byte stretch is a candidate whose weak sum hits
    but whose MD4 does not (truth -1), then true matches follow.  The walk must
    get through it in a bounded number of confirmation batches."""
    blen = 32768
    size = 64 << 20
    head = head_for(size, blen)
    dense = np.arange(100_000, 700_000, dtype=np.uint64)
    tail = np.arange(1 << 20, size - blen, blen, dtype=np.uint64)
    cand = np.concatenate([dense, tail])
    truth = np.concatenate([np.full(dense.size, -1, np.int32),
                            (np.arange(tail.size) % head[0]).astype(np.int32)])
    got, trips, windows = walk(cand, truth, size, head)
    assert got == reference_walk(cand, truth, size, head)
    # 600 000 dense false candidates: widths 2, 8, 32, ... then full 65 536
    # windows per batch -> about 20 batches, not ~300 000
    assert trips <= 40, trips
    assert windows <= 4 * cand.size


def test_dense_true_periodic_bounded_round_trips():
    """Periodic data: every offset is a candidate and every visited one matches
    (the walk visits one offset per block).  The chain confirms about two
    windows per visited offset and 4096 visited offsets per round trip; the
    reach set adds at most 16 384 windows per round trip."""
    blen = 4096
    size = 32 << 20
    head = head_for(size, blen)
    cand = np.arange(0, size - blen + 1, dtype=np.uint64)
    truth = np.zeros(cand.size, np.int32)
    got, trips, windows = walk(cand, truth, size, head)
    want = reference_walk(cand, truth, size, head)
    assert got == want
    assert windows <= 2 * len(want) + trips * 16384 + 4096
    assert trips <= len(want) // 4096 + 4


def test_dense_alternating_failures():
    """A dense stretch where each chain step's first two candidates fail and
    the third matches: the chain guess is wrong at every step."""
    blen = 1024
    size = 8 << 20
    head = head_for(size, blen)
    cand = np.arange(0, size - blen + 1, dtype=np.uint64)
    truth = np.where(cand % 3 == 2, 5, -1).astype(np.int32)
    got, trips, windows = walk(cand, truth, size, head)
    assert got == reference_walk(cand, truth, size, head)
    # ~64 visited matches per round trip once the reach set is 8 wide
    assert trips <= len(got) // 32 + 8, trips


def _cfg3_like(seed, blen=32768, size=256 << 20, false_hits=2048):
    """Runs of consecutive matched blocks at shifted offsets (cfg3: a basis
    with half its blocks modified and a few insertions), plus random false
    weak hits (equal Sum1, different MD4) everywhere, inside matched spans too."""
    rng = np.random.default_rng(seed)
    head = head_for(size, blen)
    cand, truth, q = [], [], int(rng.integers(0, blen))
    while q + blen <= size:
        run = int(rng.integers(1, 12))
        b0 = int(rng.integers(0, head[0] - run))
        for k in range(run):
            if q + blen > size:
                break
            cand.append(q)
            truth.append(b0 + k)
            q += blen
        q += int(rng.integers(1, 6 * blen))  # a modified stretch, not a multiple of B
    fh = rng.integers(0, size - blen, false_hits)
    cand += fh.tolist()
    truth += [-1] * false_hits
    c = np.asarray(cand, np.uint64)
    t = np.asarray(truth, np.int32)
    order = np.argsort(c, kind="stable")
    c, t = c[order], t[order]
    keep = np.concatenate([[True], c[1:] != c[:-1]])
    return c[keep], t[keep], size, head


@pytest.mark.parametrize("seed", range(6))
def test_sparse_speculative_selection(seed):
    """cfg3's shape: the sparse batch confirms only the windows the walk
    visits if chained candidates (another candidate B before or after) match
    -- the false hits inside matched spans are never hashed -- and the match
    list is the greedy walk's.  Isolated true matches (one-block runs) and
    false hits that happen to be chained cost at most a few extra trips."""
    cand, truth, size, head = _cfg3_like(seed)
    got, trips, windows = walk(cand, truth, size, head, spec=1)
    want = reference_walk(cand, truth, size, head)
    assert got == want
    # visited offsets: every match plus the false hits outside matched spans
    pos, visited = 0, 0
    for q, b in zip(cand.tolist(), truth.tolist()):
        if q < pos:
            continue
        visited += 1
        if b >= 0:
            pos = q + head[1]
    assert trips <= 4, trips
    assert windows <= visited + 64 * trips, (windows, visited, cand.size)
    assert windows < cand.size


def test_sparse_speculation_wrong_chains():
    """Chained false hits (a pair of candidates B apart, both failing MD4)
    sends the speculative walk past candidates the real walk visits; those
    are confirmed in later round trips and the result is still exact."""
    blen = 4096
    size = 16 << 20
    head = head_for(size, blen)
    rng = np.random.default_rng(5)
    base = np.sort(rng.choice(np.arange(0, size - 2 * blen, 3 * blen), 600, replace=False)).astype(np.uint64)
    pairs = np.concatenate([base, base + blen])
    inner = base + 17  # visited after the pair's first candidate fails
    cand = np.unique(np.concatenate([pairs, inner])).astype(np.uint64)
    truth = np.where(np.isin(cand, inner), 3, -1).astype(np.int32)
    got, trips, windows = walk(cand, truth, size, head, spec=1)
    assert got == reference_walk(cand, truth, size, head)
    assert windows <= 2 * cand.size


@pytest.mark.parametrize("seed", range(3))
def test_sparse_every_candidate_one_round_trip(seed):
    """The default sparse batch (no speculation): every candidate of the
    stretch is confirmed in the one round trip, so the walk never waits for
    another, and the match list is the greedy walk's."""
    cand, truth, size, head = _cfg3_like(seed)
    got, trips, windows = walk(cand, truth, size, head, spec=2)
    assert got == reference_walk(cand, truth, size, head)
    assert trips == 1
    assert windows == cand.size
