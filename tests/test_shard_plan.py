"""Single-process multi-GPU entry points (include/rsg.h "one process, many
GPUs").

CPU: rsg_shard_plan (the C++ plan a Go host calls) equals the Python layout
the multi-process bench uses (rsync_amd.dist.shard_layout) piece for piece,
for world 1..40 and 1..5 batches.

GPU: the one-process calls over several contexts -- rsg_block_sums_host_multi,
rsg_generate_files_fd_multi, rsg_block_sums_d2h_multi and (one-rank RCCL
communicator from rsg_comm_init_all) rsg_block_sums_gather_multi -- give the
single-context output byte for byte, and the block sums equal the oracle.
The builder's box has one GPU, so the several contexts share device 0 (RCCL
needs distinct devices: the gather runs at N = 1 here; the driver's 8-GPU
node is its first multi-device run)."""
import os
import tempfile

import numpy as np
import pytest

import cases
from oracle import oracle as orc


def _lengths(seed, n):
    rng = np.random.default_rng(seed)
    kinds = rng.integers(0, 4, n)
    out = []
    for k in kinds:
        if k == 0:
            out.append(0)
        elif k == 1:
            out.append(int(rng.integers(1, 4000)))
        elif k == 2:
            out.append(int(rng.integers(4000, 300_000)))
        else:
            out.append(int(rng.integers(300_000, 3_000_000)))
    return out


def _py_pieces(lengths, world, nbatch, block_len):
    from rsync_amd.dist import shard_layout
    from rsync_amd.shard import file_heads
    lay = shard_layout(lengths, world, nbatch, block_len)
    heads = file_heads(lengths, block_len)
    first = np.concatenate([[0], np.cumsum([h.count for h in heads])]).astype(int)
    out = []
    for q in range(world):
        for b in range(nbatch):
            for p in lay.batches[q][b]:
                out.append((p.file, p.b0, p.b1, p.offset, p.length, int(first[p.file]) + p.b0, p.block_len, q, b))
    return out, lay.records


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8, 13, 16, 40])
@pytest.mark.parametrize("nbatch", [1, 2, 5])
@pytest.mark.parametrize("block_len", [0, 700, "per-file"])
def test_c_plan_equals_python_layout(world, nbatch, block_len):
    from rsync_amd.multi import shard_plan
    lengths = _lengths(world * 31 + nbatch, 40)
    if block_len == "per-file":
        rng = np.random.default_rng(world + nbatch)
        block_len = [int(x) for x in rng.choice([0, 700, 1024, 4097], len(lengths))]
    got, grecs = shard_plan(lengths, world, nbatch, block_len)
    want, wrecs = _py_pieces(lengths, world, nbatch, block_len)
    assert got == want
    assert grecs == wrecs


def test_c_plan_cfg4_shape():
    """cfg4's 100 000 files at 8 ranks, 4 batches: same as the Python plan,
    every block exactly once, ranks within one block of byte balance."""
    from rsync_amd.multi import shard_plan
    rng = np.random.default_rng(4)
    lengths = [int(x) for x in rng.integers(4096, 65537, 100_000)]
    got, recs = shard_plan(lengths, 8, 4, 700)
    want, wrecs = _py_pieces(lengths, 8, 4, 700)
    assert got == want and recs == wrecs
    per_rank = [0] * 8
    for p in got:
        per_rank[p[7]] += p[4]
    assert max(per_rank) - min(per_rank) <= 2 * 700
    assert sum(sum(r) for r in recs) == sum(-(-n // 700) for n in lengths)


def test_c_plan_rejects_bad_arguments():
    import rsync_amd
    from rsync_amd.multi import shard_plan
    with pytest.raises(rsync_amd.RsgError):
        shard_plan([10, 20], 0)
    with pytest.raises(rsync_amd.RsgError):
        shard_plan([10, 20], 2, 0)
    with pytest.raises(rsync_amd.RsgError):
        shard_plan([10], 2, 1, (1 << 29) + 1)


# ------------------------------------------------------------------ GPU
def _files():
    lens = [1 << 16, 0, 700 * 5 + 3, 12345, 1, 200_000, 64, 777_777, 0, 3 << 20]
    return [cases.splitmix64_bytes(7000 + i, n) for i, n in enumerate(lens)]


@pytest.mark.gpu
@pytest.mark.parametrize("nctx", [1, 2, 3])
@pytest.mark.parametrize("block_len", [700, 0])
def test_block_sums_host_multi(nctx, block_len):
    import rsync_amd
    from rsync_amd.multi import MultiEngine
    files = _files()
    me = MultiEngine([rsync_amd.Engine(0) for _ in range(nctx)])
    try:
        heads, rec = me.block_sums(files, cases.SEED, block_len)
        want = b"".join(orc.block_sums(f, block_len, cases.SEED) for f in files)
        assert rec == want
        assert [h.astuple() for h in heads] == [orc.sum_head(f.size, block_len) for f in files]
    finally:
        me.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nctx", [1, 2, 3])
@pytest.mark.parametrize("mux", [False, True])
def test_generate_files_fd_multi(nctx, mux):
    """The multi-context stream, demuxed, equals the single-context call's
    (idx, SumHead, records, phase markers); files split between ranks."""
    import rsync_amd
    from rsync_amd.multi import MultiEngine
    files = _files()
    tmp = tempfile.mkdtemp()
    fds = []
    try:
        for i, f in enumerate(files):
            p = os.path.join(tmp, f"f{i}")
            with open(p, "wb") as fh:
                fh.write(f.tobytes())
            fds.append(os.open(p, os.O_RDONLY))
        desc = [(fd, f.size) for fd, f in zip(fds, files)]
        idx = [3 * i + 1 for i in range(len(files))]
        one = rsync_amd.Engine(0)
        single = []
        one.generate_files_fd(desc, cases.SEED, single.append, block_len=700, idx=idx, mux=False)
        one.close()
        me = MultiEngine([rsync_amd.Engine(0) for _ in range(nctx)])
        out = []
        heads, nw = me.generate_files_fd(desc, cases.SEED, out.append, block_len=700, idx=idx, mux=mux)
        me.close()
        got = b"".join(out)
        assert nw == len(got)
        if mux:
            got = rsync_amd.mux_deframe(got)
        assert got == b"".join(single)
        assert [h.astuple() for h in heads] == [orc.sum_head(f.size, 700) for f in files]
    finally:
        for fd in fds:
            os.close(fd)
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.mark.gpu
def test_generate_files_fd_multi_bounded_queue():
    """Rank q's records wait in host memory until ranks < q are written; with
    the per-rank bound set to 64 KiB (far below one rank's records) the
    generators block instead of queueing everything, the stream is unchanged
    and no queue ever held more than the bound plus one generator chunk."""
    import ctypes
    import rsync_amd
    from rsync_amd import _lib
    from rsync_amd.multi import MultiEngine
    files = [cases.splitmix64_bytes(7100 + i, 8 << 20) for i in range(16)]  # 64 MiB per rank: >= 2 batches
    tmp = tempfile.mkdtemp()
    fds = []
    peak = ctypes.c_uint64(0)
    try:
        for i, f in enumerate(files):
            p = os.path.join(tmp, f"f{i}")
            with open(p, "wb") as fh:
                fh.write(f.tobytes())
            fds.append(os.open(p, os.O_RDONLY))
        desc = [(fd, f.size) for fd, f in zip(fds, files)]
        one = rsync_amd.Engine(0)
        single = []
        one.generate_files_fd(desc, cases.SEED, single.append, block_len=700)
        one.close()
        _lib.lib.rsg_testing_multi_queue(64 << 10, None)
        me = MultiEngine([rsync_amd.Engine(0) for _ in range(2)])
        out = []
        me.generate_files_fd(desc, cases.SEED, out.append, block_len=700)
        me.close()
        _lib.lib.rsg_testing_multi_queue(0, ctypes.byref(peak))
        assert b"".join(out) == b"".join(single)
        # one chunk is at most one generator batch's records (32 MiB of blocks)
        chunk = (32 << 20) // 700 * 20 + 20
        assert 0 < peak.value <= (64 << 10) + chunk, peak.value
    finally:
        _lib.lib.rsg_testing_multi_queue(256 << 20, None)
        for fd in fds:
            os.close(fd)
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.mark.gpu
def test_generate_files_fd_multi_short_file():
    """A file shorter than its stated length on a non-first rank: RSG_ERR_IO
    (io.ReadFull's unexpected EOF), the bytes written a prefix of the stream."""
    import rsync_amd
    from rsync_amd.multi import MultiEngine
    files = _files()
    tmp = tempfile.mkdtemp()
    fds = []
    try:
        for i, f in enumerate(files):
            p = os.path.join(tmp, f"f{i}")
            with open(p, "wb") as fh:
                fh.write(f.tobytes()[: max(0, f.size - 10)] if i == len(files) - 1 else f.tobytes())
            fds.append(os.open(p, os.O_RDONLY))
        desc = [(fd, f.size) for fd, f in zip(fds, files)]
        me = MultiEngine([rsync_amd.Engine(0) for _ in range(2)])
        out = []
        with pytest.raises(rsync_amd.RsgError) as e:
            me.generate_files_fd(desc, cases.SEED, out.append, block_len=700)
        assert e.value.status == -7
        me.close()
    finally:
        for fd in fds:
            os.close(fd)
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.mark.gpu
@pytest.mark.parametrize("nbatch", [1, 3])
def test_device_multi_d2h_and_gather(nbatch):
    """rsg_block_sums_d2h_multi over two contexts (both on device 0) and
    rsg_block_sums_gather_multi over a one-rank communicator from
    rsg_comm_init_all: both deliver the single-call record stream."""
    import rsync_amd
    from rsync_amd.dist import ShardedBlockSums, rank_arena, shard_layout
    from rsync_amd.multi import MultiEngine
    files = _files()
    lengths = [f.size for f in files]
    want = b"".join(orc.block_sums(f, 700, cases.SEED) for f in files)
    for world in (2, 1):
        lay = shard_layout(lengths, world, nbatch, 700)
        engines = [rsync_amd.Engine(0) for _ in range(world)]
        me = MultiEngine(engines)
        arenas, recs, sbs = [], [], []
        for q, eng in enumerate(engines):
            pos, arena_bytes = rank_arena(lengths, lay, q)
            arena = eng.alloc(arena_bytes)
            host = np.zeros(arena_bytes, np.uint8)
            for f, o in pos.items():
                host[o:o + lengths[f]] = files[f]
            arena.upload(host)
            arenas.append(arena)
            recs.append(eng.alloc(max(sum(lay.records[q]), 1) * 20))
            sbs.append(ShardedBlockSums.from_layout(eng, lay, q, pos, arena_bytes))
        h = np.zeros(lay.total_records * 20, np.uint8)
        me.d2h(sbs, arenas, cases.SEED, recs, lay.rank_offset[:-1], h)
        assert h.tobytes() == want
        if world == 1:
            me.comm_init_all()
            recv = engines[0].alloc(lay.total_records * 20)
            me.gather(sbs, arenas, cases.SEED, recs, recv, 0)
            assert recv.download(lay.total_records * 20).tobytes() == want
        for sb in sbs:
            sb.close()
        me.close()
