"""File-list sharding across the GPUs of one node.

Block sums of different blocks are independent (generator.go:332-348 hashes
each block on its own), so the batch's global block sequence -- the files in
file-list order, each cut into SumSizesSqroot blocks -- is split into one
contiguous range per rank, balanced by bytes.  A range may start or end inside
a file, always on a block boundary.  Each rank hashes only its range; the one
exchange step is the gather of the ranks' record ranges to the root, where
their concatenation in rank order IS the global record order, i.e. exactly the
bytes the single-GPU (and the reference's) loop would write.

Pure host arithmetic: no device code, no torch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Sequence

from .engine import RECORD_BYTES, sum_sizes_sqroot


@dataclass(frozen=True)
class Piece:
    file: int     # index in the file list
    b0: int       # first block (inclusive)
    b1: int       # last block (exclusive)
    offset: int   # byte offset of block b0 in the file
    length: int   # bytes covered: blocks b0..b1-1 (the last may be the short remainder)
    block_len: int


def file_heads(lengths: Sequence[int], block_len=0):
    bl = list(block_len) if isinstance(block_len, (list, tuple)) else [block_len] * len(lengths)
    return [sum_sizes_sqroot(n, b) for n, b in zip(lengths, bl)]


def plan_shards(lengths: Sequence[int], world: int, block_len=0) -> List[List[Piece]]:
    """Split the global block sequence into `world` contiguous, byte-balanced
    ranges.  Returns, per rank, its pieces in global order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heads = file_heads(lengths, block_len)
    total = sum(lengths)
    shards: List[List[Piece]] = [[] for _ in range(world)]
    done = 0  # bytes assigned so far
    r = 0
    for f, (n, h) in enumerate(zip(lengths, heads)):
        B = h.block_len
        b = 0
        while b < h.count:
            # byte target where rank r's range ends
            target = (total * (r + 1)) // world if r < world - 1 else total
            room = max(target - done, 0)
            nb = h.count - b
            if r < world - 1:
                nb = min(nb, max(room // B, 0))
                if nb == 0:
                    if room > 0 and not shards[r]:
                        nb = 1  # a rank takes at least one block when bytes remain
                    else:
                        r += 1
                        continue
            b1 = b + nb
            off = b * B
            ln = min(b1 * B, n) - off
            shards[r].append(Piece(f, b, b1, off, ln, B))
            done += ln
            b = b1
    return shards


def shard_record_counts(shards: Sequence[Sequence[Piece]]) -> List[int]:
    return [sum(p.b1 - p.b0 for p in s) for s in shards]


def piece_views(files: Sequence, pieces: Sequence[Piece]):
    """Host byte views of a rank's pieces, for Engine.block_sums(...,
    block_len=[p.block_len ...])."""
    out = []
    for p in pieces:
        out.append(memoryview(files[p.file])[p.offset:p.offset + p.length] if p.length else b"")
    return out


def sharded_block_sums(eng, files: Sequence, seed: int, world: int, rank: int,
                       gather: Callable[[bytes, List[int]], bytes], block_len=0):
    """Hash this rank's share of the batch on its GPU, then gather every
    rank's records to the root with `gather(local_bytes, bytes_per_rank)`
    (RCCL over xGMI in production: Engine.gather_bytes).  The root receives
    the full batch's records in file order."""
    lengths = [len(memoryview(f).cast("B")) for f in files]
    shards = plan_shards(lengths, world, block_len)
    mine = shards[rank]
    views = piece_views(files, mine)
    if mine:
        _, rec, _ = eng.block_sums(views, seed, [p.block_len for p in mine])
    else:
        rec = b""
    counts = shard_record_counts(shards)
    return gather(rec, [c * RECORD_BYTES for c in counts])
