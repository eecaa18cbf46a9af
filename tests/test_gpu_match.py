"""GPU parity of the sender search (match.go:21-230) against the golden
fixtures and the C oracle.  Everything goes through the C-ABI."""
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


def basis_sums(basis, blen, seed):
    head = orc.sum_head(basis.size, blen)
    if head[0]:
        s1, s2 = orc.parse_records(orc.block_sums(basis, blen, seed))
    else:
        s1, s2 = np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8)
    return head, s1, s2


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
def test_golden_cases(eng, name):
    import rsync_amd
    g = json.load(open(os.path.join(GOLD, "match_cases.json")))[name]
    src, basis, blen, seed = cases.match_cases()[name]
    head, s1, s2 = basis_sums(basis, blen, seed)
    got = eng.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    assert [list(m) for m in got] == g["matches"]
    tokens = rsync_amd.encode_tokens(src, head, got)
    assert len(tokens) == g["tokens_len"]
    assert hashlib.sha256(tokens).hexdigest() == g["tokens_sha256"]


@pytest.mark.parametrize("seed_case", range(8))
def test_random_vs_oracle(eng, seed_case):
    rng = np.random.default_rng(100 + seed_case)
    n = int(rng.integers(1, 300_000))
    basis = cases.splitmix64_bytes(700 + seed_case, n)
    src = cases.mutate(basis, 800 + seed_case, float(rng.uniform(0, 0.6)), 1, 3000,
                       n_ins=int(rng.integers(0, 5)), n_del=int(rng.integers(0, 5)))
    blen = int(rng.choice([0, 1, 7, 64, 333, 700, 1024, 4096, 40000]))
    seed = int(rng.integers(-2**31, 2**31))
    head, s1, s2 = basis_sums(basis, blen, seed)
    s2len = int(rng.choice([16, 16, 2, 0]))
    head = (head[0], head[1], s2len, head[3])
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    assert eng.hash_search(src, head, s1, s2, tg, seed) == want


def test_device_unaligned_source(eng):
    src, basis, blen, seed = cases.match_cases()["shifted_700"]
    head, s1, s2 = basis_sums(basis, blen, seed)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    buf = eng.alloc(src.size + 3)
    buf.upload(np.concatenate([np.zeros(3, np.uint8), src]))

    class View:  # the same buffer seen 3 bytes in: a misaligned device pointer
        ptr = buf.ptr + 3
    assert eng.hash_search_device(View, src.size, head, s1, s2, tg, seed) == want


def test_periodic_dense(eng):
    """Every offset is a weak and strong hit (the dense path of the walk)."""
    src = np.full(3 << 20, 0xBB, np.uint8)
    basis = np.full(1 << 20, 0xBB, np.uint8)
    head, s1, s2 = basis_sums(basis, 0, 7)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, 7)
    assert eng.hash_search(src, head, s1, s2, tg, 7) == want


@pytest.mark.gpu
def test_periodic_candidate_overflow(eng):
    """More candidates than one roll launch may append (kCandCap = 2^22): a
    6 MiB periodic source halves its scan range and rolls again, reading
    each range's candidates from the pinned host list the roll writes."""
    src = np.full(6 << 20, 0xBB, np.uint8)
    basis = np.full(1 << 20, 0xBB, np.uint8)
    head, s1, s2 = basis_sums(basis, 0, 11)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, 11)
    assert eng.hash_search(src, head, s1, s2, tg, 11) == want


def test_cfg3_shape_vs_oracle(eng):
    """cfg3 recipe at 64 MiB: a ~50%-modified basis with
    long runs plus shifts, reference block sizing (B = sqrt(len))."""
    basis = cases.splitmix64_bytes(3, 64 << 20)
    head, s1, s2 = basis_sums(basis, 0, cases.SEED)
    src = cases.mutate(basis, 33, 0.5, 1, 2 * head[1], n_ins=5, n_del=5)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, cases.SEED)
    got = eng.hash_search(src, head, s1, s2, tg, cases.SEED)
    assert len(want) > 100
    assert got == want


@pytest.mark.parametrize("blen", [700, 4097, 32768, 65539, 131072])
def test_packed_roll_runs_vs_oracle(eng, blen):
    """The packed roll (interior tiles, two offsets per VALU op) over sources
    of 12-20 MiB: every workgroup rolls a run of several 32 KiB tiles (the
    carried start window), block lengths with every shifted-byte alignment
    (B mod 4 = 0..3) up to kFusedMaxB, and the hand-off to roll_kernel's edge
    path for the source's last tiles (match.go:93-210)."""
    n = (12 << 20) + 12345 + 997 * (blen % 7)
    basis = cases.splitmix64_bytes(4000 + blen, n)
    src = cases.mutate(basis, 4100 + blen, 0.4, 1, 3 * blen, n_ins=6, n_del=6)
    seed = 1234567 + blen
    head, s1, s2 = basis_sums(basis, blen, seed)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    assert len(want) > 20
    assert eng.hash_search(src, head, s1, s2, tg, seed) == want


def test_packed_roll_tile_length_blocks_vs_oracle(eng):
    """B = 32768 = the roll's tile length (the reference's block length for a
    1 GiB file): the kernel carries each tile's shifted bytes and their sums
    into the next tile as its outgoing bytes (roll_packed_kernel's BT form).
    A 56 MiB source gives every workgroup a run of 7 tiles, i.e. 6 carries,
    against the oracle (match.go:93-210)."""
    blen = 32768
    n = (56 << 20) + 4321
    basis = cases.splitmix64_bytes(4500, n)
    src = cases.mutate(basis, 4501, 0.5, 1, 3 * blen, n_ins=7, n_del=7)
    seed = 7654321
    head, s1, s2 = basis_sums(basis, blen, seed)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    assert len(want) > 200
    assert eng.hash_search(src, head, s1, s2, tg, seed) == want


def test_identical_large_property(eng):
    """1 GiB source identical to its basis (B = 32768): every block matches at
    its own offset, in order (size-independent property at full cfg3 file size)."""
    size = 1 << 30
    dev = eng.alloc(size)
    eng.fill_splitmix64(dev, size, 11)
    recs, total = eng.block_sums_device(dev, [(0, size, 0)], cases.SEED)
    rec = recs.download(total * 20).tobytes()
    s1, s2 = orc.parse_records(rec)
    head = orc.sum_head(size, 0)
    assert head[0] == total == 32768
    got = eng.hash_search_device(dev, size, head, s1, s2, orc.stable_targets(s1), cases.SEED)
    assert got == [(i * head[1], i) for i in range(total)]


@pytest.mark.parametrize("seed_case", range(4))
@pytest.mark.parametrize("recv_md4", ["default", "gpu"])
def test_delta_round_trip_on_gpu(eng, seed_case, recv_md4):
    """The whole delta path through the C-ABI: receiver block sums of the
    basis (generator.go:325-350) -> sender search (match.go:21-230) -> tokens
    (token.go) + whole-file sum (GPU file-sum kernel) -> receiveData
    (receiver.go:98-188) rebuilds the source and passes the seeded MD4 check
    (default: the host MD4 fused with token application, one file being one
    serial chain; recv_md4 = gpu: the GPU's file-sum kernel, rsg_testing_search_option 5); a flipped sum
    byte is reported as corruption (receiver.go:171-173)."""
    import rsync_amd
    eng.set_option("recv_md4", 1 if recv_md4 == "gpu" else 0)
    rng = np.random.default_rng(900 + seed_case)
    basis = cases.splitmix64_bytes(910 + seed_case, int(rng.integers(50_000, 2_000_000)))
    src = cases.mutate(basis, 920 + seed_case, 0.4, 1, 5000, n_ins=3, n_del=3)
    blen = int(rng.choice([0, 700, 1773]))
    seed = int(rng.integers(-2**31, 2**31))
    heads, rec, _ = eng.block_sums([basis], seed, blen)
    head = heads[0].astuple()
    assert rec == orc.block_sums(basis, head[1], seed)
    s1, s2 = orc.parse_records(rec)
    tg = orc.stable_targets(s1)
    matches = eng.hash_search(src, head, s1, s2, tg, seed)
    fsum = eng.file_sums([src], rsync_amd.FILESUM_SEEDED, seed)[0]
    stream = rsync_amd.encode_tokens(src, head, matches) + fsum
    want, used_o = orc.receive_data(stream, head, basis, seed)
    got, used = eng.receive_data(stream, head, basis, seed)
    assert got == want == src.tobytes() and used == used_o == len(stream)
    bad = bytearray(stream)
    bad[-5] ^= 0x40
    with pytest.raises(rsync_amd.RsgError) as e:
        eng.receive_data(bytes(bad), head, basis, seed)
    assert e.value.status == rsync_amd._lib.ERR_CORRUPT
    eng.set_option("recv_md4", 0)


@pytest.mark.gpu
def test_receive_data_large_pipelined(eng):
    """A file past rsg_receive_data's pipeline threshold (8 MiB): tokens are
    applied on a worker thread while the caller's thread hashes behind it.
    Same bytes, same sum check (receiver.go:117-120,159-173), corruption
    still caught."""
    import rsync_amd
    basis = cases.splitmix64_bytes(931, (24 << 20) + 12345)
    src = cases.mutate(basis, 932, 0.3, 1, 200_000, n_ins=4, n_del=4)
    seed = -123456789
    heads, rec, _ = eng.block_sums([basis], seed, 0)
    head = heads[0].astuple()
    s1, s2 = orc.parse_records(rec)
    matches = eng.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    fsum = eng.file_sums([src], rsync_amd.FILESUM_SEEDED, seed)[0]
    stream = rsync_amd.encode_tokens(src, head, matches) + fsum
    want, used_o = orc.receive_data(stream, head, basis, seed)
    got, used = eng.receive_data(stream, head, basis, seed)
    assert len(got) >= (8 << 20)
    assert got == want == src.tobytes() and used == used_o == len(stream)
    bad = bytearray(stream)
    bad[-1] ^= 0x01
    with pytest.raises(rsync_amd.RsgError) as e:
        eng.receive_data(bytes(bad), head, basis, seed)
    assert e.value.status == rsync_amd._lib.ERR_CORRUPT


def _random_delta(k, seed):
    rng = np.random.default_rng(500 + k)
    n = int(rng.integers(1, 400_000))
    basis = cases.splitmix64_bytes(510 + k, n)
    src = cases.mutate(basis, 520 + k, float(rng.uniform(0, 0.6)), 1, 3000,
                       n_ins=int(rng.integers(0, 4)), n_del=int(rng.integers(0, 4)))
    blen = int(rng.choice([0, 7, 333, 700, 4096, 40000]))
    head, s1, s2 = basis_sums(basis, blen, seed)
    return src, basis, head, s1, s2, orc.stable_targets(s1)


def _random_job(k, seed):
    src, _, head, s1, s2, tg = _random_delta(k, seed)
    return src, head, s1, s2, tg


def test_batch_host_vs_oracle(eng):
    """rsg_hash_search_batch_host: several files of one transfer in one
    pipelined call equal the oracle file by file; an empty source, a count-0
    head (sendFile path) and a job with bad targets in the middle are settled
    on their own job without disturbing the others."""
    import rsync_amd
    seed = 0x1BADB002
    jobs, want = [], []
    for k in range(6):
        src, head, s1, s2, tg = _random_job(k, seed)
        jobs.append((src, None, head, s1, s2, tg))
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
    src, head, s1, s2, tg = _random_job(6, seed)
    jobs.insert(3, (src, None, head, s1, s2, np.zeros_like(tg)))  # not a permutation
    want.insert(3, None)
    jobs.append((np.zeros(0, np.uint8), None, head, s1, s2, tg))  # empty source
    want.append([])
    jobs.append((src, None, (0, 700, 16, 0), np.zeros(0, np.uint32), np.zeros(0, np.uint8),
                 np.zeros(0, np.int32)))  # count 0
    want.append([])
    got = eng.hash_search_batch(jobs, seed, device=False, raise_on_error=False)
    assert [st for st, _ in got] == [0, 0, 0, rsync_amd._lib.ERR_INVALID, 0, 0, 0, 0, 0]
    for k, (st, m) in enumerate(got):
        if want[k] is not None:
            assert m == want[k], k
    with pytest.raises(rsync_amd.RsgError) as e:
        eng.hash_search_batch(jobs, seed, device=False)
    assert "permutation" in str(e.value)
    good = [j for k, j in enumerate(jobs) if want[k] is not None]
    assert eng.hash_search_batch(good, seed, device=False) == [w for w in want if w is not None]


def test_batch_device_matches_single(eng):
    """Device-resident batch (one aligned and one misaligned source, two 64 MiB
    cfg3-shaped files) equals the single-file calls and the oracle."""
    seed = cases.SEED
    bufs, jobs, want = [], [], []
    for k in range(3):
        basis = cases.splitmix64_bytes(30 + k, (64 << 20) if k < 2 else 300_000)
        head, s1, s2 = basis_sums(basis, 0, seed)
        src = cases.mutate(basis, 40 + k, 0.5, 1, 2 * head[1], n_ins=3, n_del=3)
        tg = orc.stable_targets(s1)
        shift = 5 if k == 2 else 0
        buf = eng.alloc(src.size + 16)
        buf.upload(np.concatenate([np.zeros(shift, np.uint8), src]))

        class View:
            ptr = buf.ptr + shift
        bufs.append(buf)
        jobs.append((View, src.size, head, s1, s2, tg))
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
    got = eng.hash_search_batch(jobs, seed)
    assert got == want
    assert got == [eng.hash_search_device(*j, seed) for j in jobs]


@pytest.mark.parametrize("order", ["big_then_tiny", "tiny_big_tiny"])
def test_batch_last_confirmation_beside_previous(eng, order):
    """The last job's confirmation runs on the roll stream beside job n-2's on
    the confirmation stream (rsg_match.cpp search_batch, last_own): a large
    sparse confirmation (a 96 MiB cfg3-shaped source, thousands of windows)
    followed by a tiny last job whose confirmation is queued while the large
    one still runs.  Each job has its own confirmation scratch, so both match
    lists equal the oracle's (match.go:21-230)."""
    seed = cases.SEED
    sizes = [96 << 20, 30_000] if order == "big_then_tiny" else [20_000, 96 << 20, 25_000]
    bufs, jobs, want = [], [], []
    for k, n in enumerate(sizes):
        basis = cases.splitmix64_bytes(60 + k, n)
        head, s1, s2 = basis_sums(basis, 0, seed)
        src = cases.mutate(basis, 70 + k, 0.5, 1, 2 * head[1], n_ins=3, n_del=3)
        tg = orc.stable_targets(s1)
        buf = eng.alloc(src.size + 16)
        buf.upload(src)
        bufs.append(buf)
        jobs.append((buf, src.size, head, s1, s2, tg))
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
    assert max(len(w) for w in want) > 1000
    for _ in range(3):
        assert eng.hash_search_batch(jobs, seed) == want


@pytest.mark.parametrize("blen", [131073, 200000])
def test_long_blocks_prefix_pass(eng, blen):
    """B > 128 KiB: the roll kernel takes its window sums from the tile_agg /
    tile_scan prefix passes instead of deriving them itself (rsg_match.cpp
    enqueue_scan); both paths must give the oracle's matches."""
    rng = np.random.default_rng(blen)
    basis = cases.splitmix64_bytes(blen, 3 << 20)
    src = cases.mutate(basis, blen + 1, 0.3, 1, 2 * blen, n_ins=3, n_del=3)
    seed = int(rng.integers(-2**31, 2**31))
    head, s1, s2 = basis_sums(basis, blen, seed)
    tg = orc.stable_targets(s1)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    assert len(want) > 0
    assert eng.hash_search(src, head, s1, s2, tg, seed) == want


@pytest.mark.parametrize("mode", ["auto", "gpu", "host"])
def test_receive_data_batch(eng, mode):
    """rsg_receive_data_batch over a transfer's worth of files (RecvFiles'
    per-file receiveData, receiver.go:18-188): 48 random delta streams plus
    edge jobs -- a flipped whole-file sum byte (RSG_ERR_CORRUPT, receiver.go:
    171-173), a stream cut before its sum, a match token without a basis
    (RSG_ERR_INVALID), an empty file -- each job's status and bytes equal the
    oracle's receive_data; the good jobs are unaffected by the bad ones.
    mode: which side checks the whole-file sums (rsg_testing_search_option
    5; auto = the batch's cost split)."""
    import rsync_amd
    eng.set_option("recv_md4", {"auto": 0, "gpu": 1, "host": 2}[mode])
    from rsync_amd import _lib
    seed = 0x5EED
    jobs, want = [], []
    for k in range(48):
        src, basis, head, s1, s2, tg = _random_delta(700 + k, seed)
        _, tok, fsum = orc.hash_search(src, head, s1, s2, tg, seed)
        stream = tok + fsum
        jobs.append((stream, head, basis))
        want.append((_lib.OK,) + orc.receive_data(stream, head, basis, seed))
    # corrupt sum, short stream, match without basis, empty file
    src, basis, head, s1, s2, tg = _random_delta(800, seed)
    _, tok, fsum = orc.hash_search(src, head, s1, s2, tg, seed)
    bad = bytearray(tok + fsum)
    bad[-3] ^= 1
    jobs.append((bytes(bad), head, basis))
    want.append((_lib.ERR_CORRUPT, None, None))
    jobs.append(((tok + fsum)[:-4], head, basis))
    want.append((_lib.ERR_INVALID, None, None))
    jobs.append((struct.pack("<ii", -1, 0) + bytes(16), (1, 700, 16, 0), None))
    want.append((_lib.ERR_INVALID, None, None))
    empty_sum = orc.file_sum(1, seed, np.zeros(0, np.uint8))
    jobs.append((struct.pack("<i", 0) + empty_sum, (0, 700, 16, 0), None))
    want.append((_lib.OK, b"", 4 + 16))
    got = eng.receive_data_batch(jobs, seed, raise_on_error=False)
    for k, ((st, data, used), (wst, wdata, wused)) in enumerate(zip(got, want)):
        assert st == wst, k
        if wst == _lib.OK:
            assert data == wdata and used == wused, k
    with pytest.raises(rsync_amd.RsgError) as e:
        eng.receive_data_batch(jobs, seed)
    assert e.value.status == _lib.ERR_CORRUPT
    assert [r[:2] for r in eng.receive_data_batch([j for j, w in zip(jobs, want) if w[0] == _lib.OK], seed)] \
        == [(w[1], w[2]) for w in want if w[0] == _lib.OK]
    eng.set_option("recv_md4", 0)


def test_receive_data_batch_mixed_sizes(eng):
    """A batch of three 20 MiB files and 60 small ones: the cost split sends
    the large files' sums to host threads and the small ones' to the GPU
    (one lane each).  A corrupt sum in one large and one small file is
    reported on exactly those jobs; every other file equals the oracle's."""
    from rsync_amd import _lib
    seed = 0x1234
    jobs, want = [], []
    rng = np.random.default_rng(77)
    for k in range(63):
        n = (20 << 20) if k in (5, 30, 61) else int(rng.integers(1000, 300_000))
        basis = cases.splitmix64_bytes(3000 + k, n)
        src = cases.mutate(basis, 3100 + k, 0.3, 1, 5000, n_ins=2, n_del=2) if n < (1 << 20) else basis.copy()
        head = orc.sum_head(basis.size, 0)
        s1, s2 = orc.parse_records(orc.block_sums(basis, head[1], seed))
        _, tok, fsum = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
        stream = bytearray(tok + fsum)
        if k in (30, 40):
            stream[-1] ^= 0x80
        jobs.append((bytes(stream), head, basis))
        want.append(_lib.ERR_CORRUPT if k in (30, 40) else _lib.OK)
        if k not in (30, 40):
            assert orc.receive_data(bytes(stream), head, basis, seed)[0] == src.tobytes()
    got = eng.receive_data_batch(jobs, seed, raise_on_error=False)
    assert [g[0] for g in got] == want
    for k, (st, data, used) in enumerate(got):
        if st == _lib.OK:
            assert data == orc.receive_data(jobs[k][0], jobs[k][1], jobs[k][2], seed)[0], k


@pytest.mark.parametrize("option,value", [("host_tables", 1), ("force_table_ovf", 1), ("spec", 1), ("confirm_cus", 0),
                                          ("path", 1)])
def test_search_modes_vs_oracle(option, value):
    """The search's other modes, each on a fresh context
    (rsg_testing_search_option): roll tables built on the host; a GPU-built
    table reported incomplete, so the rolls pass every filter hit on as a
    candidate and the confirmation alone decides; the speculative
    confirmation batches; confirmations serialised behind the rolls; every
    source through the large-file pipeline.  Golden cases, random searches
    and a multi-job batch against the oracle in every mode."""
    import rsync_amd
    import search_modes
    eng = rsync_amd.Engine(0)
    try:
        eng.set_option(option, value)
        assert search_modes.check_all(eng) > 20
    finally:
        eng.close()
