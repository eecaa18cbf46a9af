"""Multi-rank sharding of the block-sum batch, exercised on CPU with the gloo
backend (world_size 2 and 3).  The per-rank hashing is stood in by the CPU
oracle (test infrastructure); what is under test is the host logic of
rsync_amd.shard: byte-balanced contiguous block ranges, pieces cut on block
boundaries, and a rank-ordered gather that reproduces the single-process
record stream exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import cases
from oracle import oracle as orc


class OracleEngine:
    """CPU stand-in with Engine.block_sums' signature (tests only)."""

    def block_sums(self, files, seed, block_len=0):
        bl = block_len if isinstance(block_len, list) else [block_len] * len(files)
        rec = b"".join(orc.block_sums(np.frombuffer(bytes(f), np.uint8), b, seed) for f, b in zip(files, bl))
        return None, rec, None


def _files():
    lens = [1 << 16, 0, 700 * 5 + 3, 12345, 1, 200_000, 64, 777_777]
    return [cases.splitmix64_bytes(9000 + i, n).tobytes() for i, n in enumerate(lens)]


def _gather_gloo(rank, world):
    def gather(local: bytes, nbytes):
        mx = max(max(nbytes), 1)
        t = torch.zeros(mx, dtype=torch.uint8)
        if local:
            t[: len(local)] = torch.frombuffer(bytearray(local), dtype=torch.uint8)
        bufs = [torch.zeros(mx, dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
        dist.gather(t, bufs, dst=0)
        if rank != 0:
            return None
        return b"".join(bytes(b[:n].numpy()) for b, n in zip(bufs, nbytes))
    return gather


def _worker(rank, world, port, block_len, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rsync_amd.shard import sharded_block_sums
    got = sharded_block_sums(OracleEngine(), _files(), cases.SEED, world, rank, _gather_gloo(rank, world),
                             block_len)
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,block_len", [(2, 700), (3, 0), (2, 1773)])
def test_sharded_gather_matches_single(world, block_len):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, block_len, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = b"".join(orc.block_sums(np.frombuffer(f, np.uint8), block_len, cases.SEED) for f in _files())
    assert got == want


@pytest.mark.parametrize("world", [1, 2, 3, 8, 40])
def test_plan_shards_partition(world):
    from rsync_amd.shard import plan_shards, shard_record_counts
    lens = [len(f) for f in _files()] + [5 << 20]
    shards = plan_shards(lens, world, 700)
    # every block exactly once, in global order
    seq = [(p.file, b) for s in shards for p in s for b in range(p.b0, p.b1)]
    want = [(f, b) for f, n in enumerate(lens) for b in range(orc.sum_head(n, 700)[0])]
    assert seq == want
    assert sum(shard_record_counts(shards)) == len(want)
    # byte balance: no rank exceeds its share by more than one block
    total = sum(lens)
    for s in shards:
        assert sum(p.length for p in s) <= total / world + 700


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cfg4_shard_plan(world):
    """bench.py --workload cfg4's plan: 100k files of 4-64 KiB at B = 700 cut
    into `world` contiguous ranges that cover every block exactly once, in
    global order, each within one block (+ one file tail) of the byte share."""
    from rsync_amd.shard import file_heads, plan_shards
    lengths = np.random.default_rng(4).integers(4096, 65537, 100_000).tolist()
    shards = plan_shards(lengths, world, 700)
    heads = file_heads(lengths, 700)
    flat = [p for s in shards for p in s]
    expect = [(f, b) for f, h in enumerate(heads) for b in [0]]  # every file starts once
    assert sum(p.b1 - p.b0 for p in flat) == sum(h.count for h in heads)
    nxt = {}
    for p in flat:  # contiguity: each piece continues where the last one of its file ended
        assert p.b0 == nxt.get(p.file, 0) and p.offset == p.b0 * 700
        nxt[p.file] = p.b1
    assert all(nxt[f] == h.count for f, h in enumerate(heads)) and len(nxt) == len(expect)
    share = sum(lengths) / world
    for s in shards:
        assert abs(sum(p.length for p in s) - share) <= 2 * 700 + 65536
