"""The streaming sender (row a13: sendFile's mapFile / ptr window,
internal/sender/fileio.go:31-112): rsg_hash_search_fd reads the source from
a file descriptor in windows, each searched on the GPU with a B-1 byte halo
while the next one is read, the walk's position carried across windows.

Parity: the match list equals the oracle's hashSearch (match.go:21-230) and
the whole-file sum equals the oracle's MD4(int32_LE(seed) || source)
(match.go:52-53) on the golden search cases and on multi-window sources at
several block lengths, with windows far smaller than the source (so matches,
candidates and confirmation windows straddle window edges).  A file shorter
than its stated length is the reference's "file has changed mid-transfer"."""
import os

import numpy as np
import pytest

import cases
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import rsync_amd
    e = rsync_amd.Engine(0)
    yield e
    e.close()


def _file(tmp_path, name, data):
    p = tmp_path / name
    p.write_bytes(np.asarray(data, np.uint8).tobytes())
    return os.open(p, os.O_RDONLY)


def _sums(basis, blen, seed):
    head = orc.sum_head(basis.size, blen)
    if head[0]:
        s1, s2 = orc.parse_records(orc.block_sums(basis, blen, seed))
    else:
        s1, s2 = np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8)
    return head, s1, s2, orc.stable_targets(s1)


def _search(eng, tmp_path, src, basis, blen, seed, window_kb, name="src"):
    head, s1, s2, tg = _sums(basis, blen, seed)
    fd = _file(tmp_path, name, src)
    old = os.environ.get("RSG_SEARCH_WINDOW_KB")
    os.environ["RSG_SEARCH_WINDOW_KB"] = str(window_kb)
    try:
        got, dig = eng.hash_search_fd(fd, src.size, head, s1, s2, tg, seed, file_sum=True)
    finally:
        os.close(fd)
        if old is None:
            del os.environ["RSG_SEARCH_WINDOW_KB"]
        else:
            os.environ["RSG_SEARCH_WINDOW_KB"] = old
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
    assert got == want
    assert dig == orc.file_sum(1, seed, src)
    return got


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
@pytest.mark.parametrize("window_kb", [32, 64, 256 * 1024])
def test_golden_cases_streamed(eng, tmp_path, name, window_kb):
    src, basis, blen, seed = cases.match_cases()[name]
    _search(eng, tmp_path, src, basis, blen, seed, window_kb)


@pytest.mark.parametrize("blen,window_kb", [(700, 96), (1024, 64), (4096, 128), (32768, 256), (131072, 512),
                                            (4097, 1024)])
def test_multi_window_sources(eng, tmp_path, blen, window_kb):
    """6-8 MiB sources vs 50 %-modified bases (the cfg3 recipe, scaled down),
    windows of 64 KiB-1 MiB: tens of windows per source."""
    rng = np.random.default_rng(blen)
    basis = cases.splitmix64_bytes(500 + blen, int(rng.integers(6 << 20, 8 << 20)))
    src = cases.mutate(basis, blen, 0.5, 1, 2 * blen, n_ins=8, n_del=8)
    m = _search(eng, tmp_path, src, basis, blen, cases.SEED, window_kb)
    assert len(m) > 0


def test_periodic_source_across_windows(eng, tmp_path):
    """Every offset a weak and strong hit (the dense walk), 40 windows."""
    basis = np.full(300_000, 0xBB, np.uint8)
    src = np.full(1_300_003, 0xBB, np.uint8)
    _search(eng, tmp_path, src, basis, 700, cases.SEED, 32)


def test_send_file_path_and_empty(eng, tmp_path):
    """count == 0 (sendFile, sender.go:86-88): no matches, the file sum still
    covers the whole file; an empty source: no matches, MD4(seed) only."""
    src = cases.splitmix64_bytes(7, 3_000_000)
    _search(eng, tmp_path, src, np.zeros(0, np.uint8), 700, cases.SEED, 64, "a")
    _search(eng, tmp_path, np.zeros(0, np.uint8), cases.splitmix64_bytes(8, 5000), 700, cases.SEED, 64, "b")


@pytest.mark.parametrize("short_by", [1, 700, 500_000])
def test_file_changed_mid_transfer(eng, tmp_path, short_by):
    import rsync_amd
    basis = cases.splitmix64_bytes(9, 2_000_000)
    src = basis.copy()
    head, s1, s2, tg = _sums(basis, 700, cases.SEED)
    fd = _file(tmp_path, "short", src[: src.size - short_by])
    os.environ["RSG_SEARCH_WINDOW_KB"] = "256"
    try:
        with pytest.raises(rsync_amd.RsgError) as e:
            eng.hash_search_fd(fd, src.size, head, s1, s2, tg, cases.SEED, file_sum=True)
    finally:
        os.close(fd)
        del os.environ["RSG_SEARCH_WINDOW_KB"]
    assert e.value.status == -7
    assert "file has changed mid-transfer" in str(e.value)
    # the context is usable afterwards
    _search(eng, tmp_path, src, basis, 700, cases.SEED, 256, "ok")


def test_offset_into_descriptor(eng, tmp_path):
    """The source at a byte offset of the descriptor (rsg_fd_file-style
    offset): the same matches as the source alone."""
    basis = cases.splitmix64_bytes(10, 1_000_000)
    src = cases.mutate(basis, 10, 0.3, 1, 1400, n_ins=2, n_del=2)
    head, s1, s2, tg = _sums(basis, 700, cases.SEED)
    pre = cases.splitmix64_bytes(11, 12345)
    fd = _file(tmp_path, "off", np.concatenate([pre, src, pre]))
    try:
        got, dig = eng.hash_search_fd(fd, src.size, head, s1, s2, tg, cases.SEED, offset=pre.size, file_sum=True)
    finally:
        os.close(fd)
    want, _, _ = orc.hash_search(src, head, s1, s2, tg, cases.SEED)
    assert got == want and dig == orc.file_sum(1, cases.SEED, src)


@pytest.mark.parametrize("sum_threads", ["1", "4"])
def test_fd_batch_many_files(eng, tmp_path, sum_threads):
    """rsg_hash_search_fd_batch (SendFiles' loop over open files): every job's
    matches equal the oracle's hashSearch and every whole-file sum its
    MD4(int32_LE(seed) || source), whatever the number of sum threads; jobs
    of several block lengths, a sendFile job (count == 0), an empty source, a
    source at an offset into its descriptor, a file shorter than its stated
    length (that job alone fails with "file has changed mid-transfer"), a job
    with bad arguments (that job alone RSG_ERR_INVALID)."""
    import rsync_amd
    rng = np.random.default_rng(77)
    jobs, want, fds = [], [], []
    try:
        for k, blen in enumerate([700, 1024, 4097, 32768, 700, 2048]):
            basis = cases.splitmix64_bytes(900 + k, int(rng.integers(1 << 20, 3 << 20)))
            src = cases.mutate(basis, blen, 0.5, 1, 2 * blen, n_ins=4, n_del=4)
            head, s1, s2, tg = _sums(basis, blen, cases.SEED)
            fd = _file(tmp_path, f"s{k}", src)
            fds.append(fd)
            jobs.append((fd, src.size, head, s1, s2, tg))
            want.append((orc.hash_search(src, head, s1, s2, tg, cases.SEED)[0], orc.file_sum(1, cases.SEED, src)))
        # sendFile (no sums) and an empty source
        src = cases.splitmix64_bytes(950, 300_001)
        fd = _file(tmp_path, "send", src)
        fds.append(fd)
        jobs.append((fd, src.size, (0, 0, 0, 0), np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8),
                     np.zeros(0, np.int32)))
        want.append(([], orc.file_sum(1, cases.SEED, src)))
        head, s1, s2, tg = _sums(cases.splitmix64_bytes(951, 5000), 700, cases.SEED)
        fd = _file(tmp_path, "empty", np.zeros(0, np.uint8))
        fds.append(fd)
        jobs.append((fd, 0, head, s1, s2, tg))
        want.append(([], orc.file_sum(1, cases.SEED, np.zeros(0, np.uint8))))
        # at an offset into its descriptor
        basis = cases.splitmix64_bytes(952, 2 << 20)
        src = cases.mutate(basis, 700, 0.3, 1, 1400)
        head, s1, s2, tg = _sums(basis, 700, cases.SEED)
        fd = _file(tmp_path, "off", np.concatenate([np.full(12345, 7, np.uint8), src]))
        fds.append(fd)
        jobs.append((fd, src.size, head, s1, s2, tg, 12345))
        want.append((orc.hash_search(src, head, s1, s2, tg, cases.SEED)[0], orc.file_sum(1, cases.SEED, src)))
        # short file: the job fails, the others do not
        basis = cases.splitmix64_bytes(953, 1 << 20)
        head, s1, s2, tg = _sums(basis, 1024, cases.SEED)
        fd = _file(tmp_path, "short", basis[:-1000])
        fds.append(fd)
        jobs.append((fd, basis.size, head, s1, s2, tg))
        want.append(None)
        # bad arguments: targets not a permutation
        head, s1, s2, tg = _sums(basis, 1024, cases.SEED)
        fd = _file(tmp_path, "bad", basis)
        fds.append(fd)
        jobs.append((fd, basis.size, head, s1, s2, np.zeros_like(tg)))
        want.append("invalid")
        old = os.environ.get("RSG_SUM_THREADS")
        os.environ["RSG_SUM_THREADS"] = sum_threads  # read per call
        try:
            got = eng.hash_search_fd_batch(jobs, cases.SEED, raise_on_error=False)
        finally:
            if old is None:
                del os.environ["RSG_SUM_THREADS"]
            else:
                os.environ["RSG_SUM_THREADS"] = old
        for k, ((st, m, dig), w) in enumerate(zip(got, want)):
            if w is None:
                assert st == -7, k
            elif w == "invalid":
                assert st == -1, k
            else:
                assert st == 0, (k, st)
                assert m == w[0], k
                assert dig == w[1], k
        with pytest.raises(rsync_amd.RsgError) as e:
            eng.hash_search_fd_batch(jobs[:-1], cases.SEED)
        assert "changed mid-transfer" in str(e.value)
    finally:
        for fd in fds:
            os.close(fd)
