"""GPU parity of the small-file sender (rsync_amd/csrc/rsg_search_small.hip,
rsg_sender_small.cpp): SendFiles' per-file hashSearch (sender.go:19-115,
match.go:21-230) for many small sources, one wave per file, against the C
oracle.  Every job's match list must equal orc.hash_search's; files whose
candidates overflow the kernel's LDS list (periodic data) fall back to the
large-file pipeline and must equal it too."""
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


def basis_sums(basis, blen, seed):
    head = orc.sum_head(basis.size, blen)
    if head[0]:
        s1, s2 = orc.parse_records(orc.block_sums(basis, blen, seed))
    else:
        s1, s2 = np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8)
    return head, s1, s2


@pytest.mark.parametrize("path", [0, 1], ids=["small_kernel", "pipeline"])
def test_golden_cases_both_paths(eng, path):
    """The 13 golden searches (aligned, shifted, B % 4 != 0, sqrt sizing,
    duplicate blocks, tail block, empty source / basis, periodic data, source
    shorter than a block, the -2 flush) through the one-wave-per-file kernel
    (0) and through the large-file pipeline (1)."""
    gold = json.load(open(os.path.join(GOLD, "match_cases.json")))
    try:
        eng.set_search_path(path)
        for name, (src, basis, blen, seed) in sorted(cases.match_cases().items()):
            head, s1, s2 = basis_sums(basis, blen, seed)
            got = eng.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
            assert [list(m) for m in got] == gold[name]["matches"], name
    finally:
        eng.set_search_path(0)


def _job(k, seed, rng):
    kind = k % 11
    n = int(rng.integers(1, 120_000))
    blen = int(rng.choice([0, 0, 1, 7, 64, 333, 700, 700, 1024, 4096, 8192]))
    if kind == 0:
        n = int(rng.integers(1, 64))            # tiny source (per-byte path only)
    elif kind == 1:
        blen = 4096
        n = int(rng.integers(100, 4095))        # basis shorter than one block
    basis = cases.splitmix64_bytes(20_000 + k, n)
    if kind == 2:
        src = cases.splitmix64_bytes(30_000 + k, int(rng.integers(1, 3000)))  # source shorter than B
    elif kind == 3:
        src = basis.copy()                      # identical: every block matches in order
    elif kind == 4:
        blk = cases.splitmix64_bytes(40_000 + k, 700)  # duplicate-content blocks
        basis = np.concatenate([blk, basis[:2000], blk, blk])
        src = np.concatenate([basis[:50], blk, blk, basis])
        blen = 700
    else:
        src = cases.mutate(basis, 50_000 + k, float(rng.uniform(0, 0.7)), 1, 3000,
                           n_ins=int(rng.integers(0, 4)), n_del=int(rng.integers(0, 4)))
    head, s1, s2 = basis_sums(basis, blen, seed)
    s2len = int(rng.choice([16, 16, 16, 3, 0]))
    head = (head[0], head[1], s2len, head[3])
    tg = orc.stable_targets(s1)
    if kind == 5 and tg.size > 1:  # another valid tie order among equal tags (Go's sort.Slice is unstable)
        tags = ((s1 & 0xFFFF) + (s1 >> 16)) & 0xFFFF
        tg = np.lexsort((rng.random(tg.size), tags)).astype(np.int32)
    return src, head, s1, s2, tg


@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_random_jobs_vs_oracle(eng, device):
    """600 small jobs of every shape in one batch call -- tiny sources, bases
    shorter than a block, sources shorter than B, identical and duplicate
    blocks, other targets orders, truncated sum2 (s2len 0 / 3), B from 1 to
    8192 and reference sizing -- plus an empty source, a count-0 head
    (sendFile) and periodic sources whose candidates overflow the kernel's
    list; each job equals the oracle's hashSearch."""
    seed = int(np.int32(0x5EED1234))
    rng = np.random.default_rng(6060 + device)
    jobs, want, bufs = [], [], []
    for k in range(600):
        src, head, s1, s2, tg = _job(k, seed, rng)
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
        jobs.append([src, head, s1, s2, tg])
    # edge jobs: empty source, count 0, periodic (candidate overflow -> pipeline)
    src, head, s1, s2, tg = _job(5, seed, rng)
    jobs.append([np.zeros(0, np.uint8), head, s1, s2, tg])
    want.append([])
    jobs.append([src, (0, 700, 16, 0), np.zeros(0, np.uint32), np.zeros(0, np.uint8), np.zeros(0, np.int32)])
    want.append([])
    for n, blen in [(200_000, 700), (30_000, 64)]:
        p_src = np.full(n, 0xBB, np.uint8)
        head, s1, s2 = basis_sums(np.full(n // 2, 0xBB, np.uint8), blen, seed)
        tg = orc.stable_targets(s1)
        jobs.append([p_src, head, s1, s2, tg])
        want.append(orc.hash_search(p_src, head, s1, s2, tg, seed)[0])
    batch = []
    for src, head, s1, s2, tg in jobs:
        if device:
            buf = eng.alloc(max(src.size, 1))
            if src.size:
                buf.upload(src)
            bufs.append(buf)
            batch.append((buf, src.size, head, s1, s2, tg))
        else:
            batch.append((src, None, head, s1, s2, tg))
    got = eng.hash_search_batch(batch, seed, device=device)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g == w, k


def test_cfg4_shaped_sampled_vs_oracle(eng):
    """BASELINE cfg4's file shape for the sender: 1024 sources of 4-64 KiB
    against 50 %-modified bases (reference sizing: B = 700) in one batch call;
    every job equals the oracle's hashSearch, and the small-file kernel, not
    the pipeline, settled them (kernel timing: small-file launches count as
    rolls; the pipeline's confirmation batches would show, none does)."""
    seed = cases.SEED
    rng = np.random.default_rng(4)
    batch, want, bufs = [], [], []
    for k in range(1024):
        n = int(rng.integers(4096, 65537))
        basis = cases.splitmix64_bytes(100_000 + k, n)
        src = cases.mutate(basis, 200_000 + k, 0.5, 1, 1400, n_ins=1, n_del=1)
        head, s1, s2 = basis_sums(basis, 0, seed)
        tg = orc.stable_targets(s1)
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
        buf = eng.alloc(src.size)
        buf.upload(src)
        bufs.append(buf)
        batch.append((buf, src.size, head, s1, s2, tg))
    eng.set_kernel_timing(True)
    try:
        got = eng.hash_search_batch(batch, seed)
        t = eng.kernel_times()
    finally:
        eng.set_kernel_timing(False)
    assert sum(len(w) for w in want) > 15_000
    assert got == want
    assert 1 <= t["roll_launches"] <= 4 and t["confirm_batches"] == 0, t


@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_bad_targets_settled_in_small_path(eng, device):
    """A small job whose `targets` is not a permutation fails on its own
    (RSG_ERR_INVALID, checked when its sums are packed; the kernel skips it)
    while the jobs around it, in the same launch, equal the oracle."""
    import rsync_amd
    seed = cases.SEED
    rng = np.random.default_rng(77)
    jobs, want, bufs = [], [], []
    for k in range(5):
        src, head, s1, s2, tg = _job(7 + 11 * k, seed, rng)
        if head[0] == 0 or src.size == 0:
            continue
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
        jobs.append([src, head, s1, s2, tg])
    bad = jobs[1]
    jobs.insert(1, [bad[0], bad[1], bad[2], bad[3], np.zeros_like(bad[4])])
    want.insert(1, None)
    batch = []
    for src, head, s1, s2, tg in jobs:
        if device:
            buf = eng.alloc(max(src.size, 1))
            buf.upload(src)
            bufs.append(buf)
            batch.append((buf, src.size, head, s1, s2, tg))
        else:
            batch.append((src, None, head, s1, s2, tg))
    eng.set_kernel_timing(True)
    try:
        got = eng.hash_search_batch(batch, seed, device=device, raise_on_error=False)
        t = eng.kernel_times()
    finally:
        eng.set_kernel_timing(False)
    assert [st for st, _ in got] == [0 if w is not None else rsync_amd._lib.ERR_INVALID for w in want]
    for (st, m), w in zip(got, want):
        if w is not None:
            assert m == w
    assert t["roll_launches"] >= 1 and t["confirm_batches"] == 0, t


def test_two_contexts_concurrently():
    """Two contexts searching small-file batches from two threads at once:
    their parallel loops share the library's worker pool (one loop at a
    time), and each batch still equals the oracle job by job."""
    import threading
    import rsync_amd
    seed = cases.SEED
    rng = np.random.default_rng(91)
    sets = []
    for t in range(2):
        jobs, want = [], []
        for k in range(700):
            src, head, s1, s2, tg = _job(5000 * (t + 1) + k, seed, rng)
            jobs.append((src, None, head, s1, s2, tg))
            want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
        sets.append((jobs, want))
    engines = [rsync_amd.Engine(0), rsync_amd.Engine(0)]
    got = [None, None]
    err = []

    def run(t):
        try:
            for _ in range(3):
                got[t] = engines[t].hash_search_batch(sets[t][0], seed, device=False)
        except Exception as e:  # surfaced below
            err.append(e)

    try:
        th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(120)
        assert not err, err
        for t in range(2):
            assert got[t] == sets[t][1], t
    finally:
        for e in engines:
            e.close()
