"""Multi-rank sharding of the generator step -- the host
logic of rsync_amd.shard / rsync_amd.dist on CPU (gloo, world_size 2 and 3),
and on the GPU box the same product path with the real engine.

Files are independent (generator.go:20-52 emits each file's sums in
file-list order), so each rank hashes a contiguous, byte-balanced block range,
cut again into batches so the records of batch b can travel while batch b+1
is hashed.  What must hold: every block exactly once, the ragged per-(rank,
batch) sizes, and landing offsets that rebuild the single-GPU stream byte for
byte.  On CPU the record bytes of a piece come from the oracle (the checker;
there is no device here); the GPU tests below run rsync_amd's own engine.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cases
from oracle import oracle as orc


def _files():
    lens = [1 << 16, 0, 700 * 5 + 3, 12345, 1, 200_000, 64, 777_777]
    return [cases.splitmix64_bytes(9000 + i, n).tobytes() for i, n in enumerate(lens)]


def _piece_records(files, p, seed):
    """Expected records of one piece (checker: the oracle)."""
    d = np.frombuffer(files[p.file], np.uint8)[p.offset:p.offset + p.length]
    return orc.block_sums(np.ascontiguousarray(d), p.block_len, seed)


def _single(files, block_len, seed):
    return b"".join(orc.block_sums(np.frombuffer(f, np.uint8), block_len, seed) for f in files)


@pytest.mark.parametrize("world,nbatch,block_len", [(1, 3, 700), (2, 4, 700), (3, 2, 0), (8, 5, 1773), (40, 3, 700)])
def test_layout_rebuilds_single_stream(world, nbatch, block_len):
    """Placing every (rank, batch) group's records at the layout's root
    offsets, with the layout's ragged sizes, rebuilds the single-GPU stream;
    the groups tile it without gaps or overlaps."""
    from rsync_amd.dist import shard_layout
    files = _files()
    lay = shard_layout([len(f) for f in files], world, nbatch, block_len)
    want = _single(files, block_len, cases.SEED)
    assert lay.total_records * 20 == len(want)
    out = bytearray(len(want))
    covered = np.zeros(len(want), np.int32)
    for b in range(nbatch):
        sizes, offs = lay.send_bytes(b), lay.recv_offsets(b)
        for q in range(world):
            rec = b"".join(_piece_records(files, p, cases.SEED) for p in lay.batches[q][b])
            assert len(rec) == sizes[q], (q, b)
            out[offs[q]:offs[q] + sizes[q]] = rec
            covered[offs[q]:offs[q] + sizes[q]] += 1
    assert (covered == 1).all()
    assert bytes(out) == want


@pytest.mark.parametrize("nbatch", [1, 2, 3, 7, 50])
def test_split_batches_cover_and_balance(nbatch):
    """A rank's pieces cut into batches: same blocks in the same order, pieces
    continue on block boundaries, byte shares within one block (+ one tail)."""
    from rsync_amd.dist import split_batches
    from rsync_amd.shard import plan_shards
    lens = [len(f) for f in _files()] + [5 << 20]
    pieces = plan_shards(lens, 2, 700)[1]
    groups = split_batches(pieces, nbatch)
    assert len(groups) == nbatch
    flat = [(p.file, b) for g in groups for p in g for b in range(p.b0, p.b1)]
    assert flat == [(p.file, b) for p in pieces for b in range(p.b0, p.b1)]
    for g in groups:
        for p in g:
            assert p.offset == p.b0 * p.block_len
    total = sum(p.length for p in pieces)
    for g in groups:
        assert sum(p.length for p in g) <= total / nbatch + 700 + 1


@pytest.mark.parametrize("world", [1, 2, 3, 8, 40])
def test_plan_shards_partition(world):
    from rsync_amd.shard import plan_shards, shard_record_counts
    lens = [len(f) for f in _files()] + [5 << 20]
    shards = plan_shards(lens, world, 700)
    seq = [(p.file, b) for s in shards for p in s for b in range(p.b0, p.b1)]
    want = [(f, b) for f, n in enumerate(lens) for b in range(orc.sum_head(n, 700)[0])]
    assert seq == want
    assert sum(shard_record_counts(shards)) == len(want)
    total = sum(lens)
    for s in shards:
        assert sum(p.length for p in s) <= total / world + 700


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cfg4_shard_plan(world):
    """bench.py --workload cfg4's plan: 100k files of 4-64 KiB at B = 700 cut
    into `world` contiguous ranges and 4 batches per rank that cover every
    block exactly once, in global order, each rank within one block (+ one
    file tail) of the byte share; the arena placement holds every piece."""
    from rsync_amd.dist import batch_descriptors, rank_arena, shard_layout
    from rsync_amd.shard import file_heads
    lengths = np.random.default_rng(4).integers(4096, 65537, 100_000).tolist()
    lay = shard_layout(lengths, world, 4, 700)
    heads = file_heads(lengths, 700)
    flat = [p for s in lay.batches for g in s for p in g]
    assert sum(p.b1 - p.b0 for p in flat) == sum(h.count for h in heads) == lay.total_records
    nxt = {}
    for p in flat:
        assert p.b0 == nxt.get(p.file, 0) and p.offset == p.b0 * 700
        nxt[p.file] = p.b1
    assert all(nxt[f] == h.count for f, h in enumerate(heads))
    share = sum(lengths) / world
    for s in lay.shards:
        assert abs(sum(p.length for p in s) - share) <= 2 * 700 + 65536
    pos, arena_bytes = rank_arena(lengths, lay, world - 1)
    for g in batch_descriptors(lay, world - 1, pos):
        for off, n, b in g:
            assert off % 4 == 0 and off + n <= arena_bytes and b == 700


# ---------------------------------------------------------------- gloo, multi-process
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nbatch, block_len, use_engine, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsync_amd.dist import gather_host, rank_records_host, shard_layout
    files = _files()
    lay = shard_layout([len(f) for f in files], world, nbatch, block_len)
    if use_engine:  # GPU box: every rank hashes with the real engine (ranks share the one GPU)
        import rsync_amd
        eng = rsync_amd.Engine(0)
        local = rank_records_host(eng, files, lay, rank, cases.SEED)
        eng.close()
    else:  # CPU: the rank's slice from the checker, in the layout's batch order
        local = b"".join(_piece_records(files, p, cases.SEED) for g in lay.batches[rank] for p in g)
    got = gather_host(local, lay, rank)
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(world, nbatch, block_len, use_engine):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nbatch, block_len, use_engine, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,nbatch,block_len", [(2, 3, 700), (3, 1, 0), (2, 2, 1773)])
def test_gather_host_ragged(world, nbatch, block_len):
    """rsync_amd.dist.gather_host over gloo: ragged per-rank sizes (rank 1's
    range ends mid-file), the root's assembly equals the single stream."""
    assert _run_ranks(world, nbatch, block_len, False) == _single(_files(), block_len, cases.SEED)


@pytest.mark.gpu
def test_sharded_generator_two_ranks_on_gpu():
    """The product path end to end on the GPU box: two processes, each
    hashing its shard's batches with rsync_amd's engine (both on GPU 0),
    host gather to rank 0 -- equal to the single-GPU stream."""
    assert _run_ranks(2, 3, 700, True) == _single(_files(), 700, cases.SEED)


@pytest.mark.gpu
@pytest.mark.parametrize("nbatch", [1, 3])
def test_pipelined_gather_and_d2h_one_rank(nbatch):
    """rsg_block_sums_gather (RCCL communicator of one rank: the root's own
    batches are written by its kernels straight to their recv offsets) and
    rsg_block_sums_d2h, each pipelined over `nbatch` batches: both deliver
    exactly the single-call records."""
    import rsync_amd
    from rsync_amd.dist import ShardedBlockSums, rank_arena, shard_layout
    files = [np.frombuffer(f, np.uint8) for f in _files()]
    lengths = [f.size for f in files]
    lay = shard_layout(lengths, 1, nbatch, 700)
    eng = rsync_amd.Engine(0)
    try:
        pos, arena_bytes = rank_arena(lengths, lay, 0)
        arena = eng.alloc(arena_bytes)
        host = np.zeros(arena_bytes, np.uint8)
        for f, o in pos.items():
            host[o:o + lengths[f]] = files[f]
        arena.upload(host)
        eng.comm_init(1, 0, rsync_amd.Engine.comm_unique_id())
        sb = ShardedBlockSums.from_layout(eng, lay, 0, pos, arena_bytes)
        recs = eng.alloc(lay.total_records * 20)
        recv = eng.alloc(lay.total_records * 20)
        sb.run_gather(arena, cases.SEED, recs, recv, 0)
        want = _single(_files(), 700, cases.SEED)
        assert recv.download(lay.total_records * 20).tobytes() == want
        h = eng.alloc_pinned(lay.total_records * 20)
        sb.run_d2h(arena, cases.SEED, recs, h)
        assert h.tobytes() == want
        eng.free_pinned(h)
        sb.close()
    finally:
        eng.close()


def _parity_worker(rank, world, port, corrupt, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsync_amd.dist import all_ranks, gather_host, gather_parity, records_digest, shard_layout
    files = _files()
    lay = shard_layout([len(f) for f in files], world, 2, 700)
    local = b"".join(_piece_records(files, p, cases.SEED) for g in lay.batches[rank] for p in g)
    info = all_ranks((records_digest(local), len(local) // 20), world)
    got = gather_host(local, lay, rank)  # the root's delivered buffer
    if rank == 0:
        buf = bytearray(got)
        if corrupt is not None:  # one byte of rank `corrupt`'s slice flipped on its way to the root
            buf[lay.rank_offset[corrupt] * 20 + 7] ^= 0x10
        out.put(gather_parity(bytes(buf), [d for d, _ in info], [n for _, n in info]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, None), (2, 1), (3, 0), (3, 2)])
def test_gather_parity_detects_a_bad_slice(world, corrupt):
    """The multi-GPU bench's self-check (bench.py measure_delivery ->
    delivery.gather_parity): every rank's SHA-256 of its own records goes to
    every rank over gloo, and the root compares each rank's slice of the
    delivered buffer (rank order = file-list order, generator.go:20-52) with
    it.  An intact gather passes on every rank; one flipped byte fails
    exactly the rank it belongs to."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res["ranks_equal"] == [corrupt is None or q != corrupt for q in range(world)]
    assert res["all_equal"] == (corrupt is None)
