"""Multi-GPU generator step: the file list sharded over the
ranks of one node, block sums on every rank, and the one exchange step --
the rank-ordered records delivered to the root -- overlapped with hashing.

Block sums of different blocks are independent (generator.go:332-348), so
rank r owns a contiguous, byte-balanced range of the batch's global block
sequence (shard.plan_shards).  Its range is cut again into `nbatch` batches
of about equal bytes (cut on block boundaries), so batch b's records can
travel while batch b+1 is hashed:

  rsg_block_sums_gather: batch b's records go to the root over RCCL (xGMI)
      on a second stream while the kernel of batch b+1 runs;
  rsg_block_sums_d2h:    every rank copies batch b's records to host memory
      (its own PCIe link) while batch b+1 is hashed -- the "N concurrent D2H"
      alternative to gather-then-one-D2H.

At the root the records of (rank q, batch b) land at
rank_offset[q] + batch_offset[q][b], so the concatenation is exactly the
single-GPU record stream in file order (generator.go:20-52 emits files in
file-list order).  Everything here is host arithmetic; the device work is the
C-ABI's (include/rsg.h).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .engine import RECORD_BYTES, Engine, Plan, _i32
from .shard import Piece, plan_shards


def split_batches(pieces: Sequence[Piece], nbatch: int) -> List[List[Piece]]:
    """Cut one rank's pieces (global order) into `nbatch` groups of about
    equal bytes, splitting a piece on a block boundary where a cut falls
    inside it.  Concatenated, the groups cover exactly the same blocks in the
    same order."""
    if nbatch < 1:
        raise ValueError("nbatch must be >= 1")
    total = sum(p.length for p in pieces)
    out: List[List[Piece]] = [[] for _ in range(nbatch)]
    done, b = 0, 0
    for p in pieces:
        b0 = p.b0
        while b0 < p.b1:
            target = (total * (b + 1)) // nbatch if b < nbatch - 1 else total
            room = target - done
            nb = p.b1 - b0
            if b < nbatch - 1:
                nb = min(nb, max(room // p.block_len, 0))
                if nb == 0:
                    if room > 0 and not out[b]:
                        nb = 1
                    else:
                        b += 1
                        continue
            off = b0 * p.block_len
            end = min((b0 + nb) * p.block_len, p.offset + p.length)
            out[b].append(Piece(p.file, b0, b0 + nb, off, end - off, p.block_len))
            done += end - off
            b0 += nb
    return out


@dataclass
class ShardLayout:
    """Where every (rank, batch) group of records lives.

    records[q][b]     record count of rank q's batch b
    rank_offset[q]    first global record of rank q
    batch_offset[q][b] first record of batch b inside rank q's range
    """
    world: int
    nbatch: int
    shards: List[List[Piece]]
    batches: List[List[List[Piece]]]
    records: List[List[int]]
    rank_offset: List[int]
    batch_offset: List[List[int]]

    @property
    def total_records(self) -> int:
        return self.rank_offset[-1]

    def send_bytes(self, b: int) -> List[int]:
        """Every rank's bytes of batch b (the gather's ragged sizes)."""
        return [self.records[q][b] * RECORD_BYTES for q in range(self.world)]

    def recv_offsets(self, b: int) -> List[int]:
        """Byte offsets on the root where every rank's batch b lands."""
        return [(self.rank_offset[q] + self.batch_offset[q][b]) * RECORD_BYTES for q in range(self.world)]


def shard_layout(lengths: Sequence[int], world: int, nbatch: int = 1, block_len=0) -> ShardLayout:
    shards = plan_shards(lengths, world, block_len)
    batches = [split_batches(s, nbatch) for s in shards]
    records = [[sum(p.b1 - p.b0 for p in g) for g in bs] for bs in batches]
    rank_offset = [0]
    for q in range(world):
        rank_offset.append(rank_offset[-1] + sum(records[q]))
    batch_offset = [list(np.cumsum([0] + r[:-1]).astype(int).tolist()) for r in records]
    return ShardLayout(world, nbatch, shards, batches, records, rank_offset, batch_offset)


def rank_arena(lengths: Sequence[int], layout: ShardLayout, rank: int) -> Tuple[dict, int]:
    """Arena placement of the files rank `rank` touches: whole files back to
    back at 128-byte aligned offsets (as the library packs its own arenas, so
    blocks whose length is a multiple of 128 start on 128-byte lines).
    -> ({file: offset}, arena bytes)."""
    files = sorted({p.file for g in layout.batches[rank] for p in g})
    at, pos = 0, {}
    for f in files:
        pos[f] = at
        at += (lengths[f] + 127) & ~127
    return pos, max(at, 16)


def batch_descriptors(layout: ShardLayout, rank: int, file_pos: dict) -> List[List[Tuple[int, int, int]]]:
    """Per batch, the (arena offset, length, B) triples of the rank's pieces:
    a piece starting inside a file starts on a block boundary, so planning it
    as a file of its own gives the reference's blocks."""
    return [[(file_pos[p.file] + p.offset, p.length, p.block_len) for p in g] for g in layout.batches[rank]]


class ShardedBlockSums:
    """One rank's side of the sharded generator step: `descs[b]` = the
    (arena offset, length, B) triples of batch b's pieces, whose records start
    at record `record_offset[b]` of this rank's records buffer;
    send_bytes[b] / recv_offsets[b] = every rank's bytes of batch b and where
    they land on the root.  run_gather() delivers every rank's records to the
    root's device buffer over RCCL, pipelined with the kernels; run_d2h()
    copies this rank's records to host memory, pipelined the same way;
    run_kernels() is the kernel-only step."""

    def __init__(self, eng: Engine, descs, arena_bytes: int, record_offset: Sequence[int],
                 send_bytes: Sequence[Sequence[int]], recv_offsets: Sequence[Sequence[int]]):
        self.eng = eng
        self.nbatch = len(descs)
        self.plans: List[Optional[Plan]] = [eng.plan(d, arena_bytes) if d else None for d in descs]
        self.record_offset = list(record_offset)
        self.my_records = sum(p.total_records for p in self.plans if p is not None)
        self._keep = []
        arr = (_lib.ShardBatch * max(self.nbatch, 1))()
        for b in range(self.nbatch):
            sb = (ctypes.c_uint64 * len(send_bytes[b]))(*send_bytes[b])
            ro = (ctypes.c_uint64 * len(recv_offsets[b]))(*recv_offsets[b])
            self._keep += [sb, ro]
            arr[b].plan = self.plans[b].handle if self.plans[b] else None
            arr[b].record_offset = self.record_offset[b]
            arr[b].send_bytes = sb
            arr[b].recv_offsets = ro
        self.batches = arr

    @classmethod
    def from_layout(cls, eng: Engine, layout: ShardLayout, rank: int, file_pos: dict, arena_bytes: int):
        return cls(eng, batch_descriptors(layout, rank, file_pos), arena_bytes, layout.batch_offset[rank],
                   [layout.send_bytes(b) for b in range(layout.nbatch)],
                   [layout.recv_offsets(b) for b in range(layout.nbatch)])

    def run_kernels(self, arena, seed: int, records, stream=None):
        """Kernel-only step: every batch's launch, asynchronous on `stream`."""
        for b, p in enumerate(self.plans):
            if p is not None:
                p.run(arena, seed, records.ptr + self.record_offset[b] * RECORD_BYTES, stream)

    def run_gather(self, arena, seed: int, records, recv, root: int = 0):
        _lib.check(_lib.lib.rsg_block_sums_gather(
            self.eng.ctx, self.batches, self.nbatch, ctypes.c_void_p(arena.ptr), _i32(seed),
            ctypes.c_void_p(records.ptr), ctypes.c_void_p(recv.ptr if recv is not None else 0), root), self.eng.ctx)

    def run_d2h(self, arena, seed: int, records, host: np.ndarray):
        _lib.check(_lib.lib.rsg_block_sums_d2h(
            self.eng.ctx, self.batches, self.nbatch, ctypes.c_void_p(arena.ptr), _i32(seed),
            ctypes.c_void_p(records.ptr), ctypes.c_void_p(host.ctypes.data)), self.eng.ctx)

    def close(self):
        for p in self.plans:
            if p is not None:
                p.close()


def gather_host(local: bytes, layout: ShardLayout, rank: int, root: int = 0):
    """Host-side assembly for the d2h mode when ranks are separate processes:
    every rank's records (already in its host memory, rank order = global
    order) go to the root over the torch.distributed control plane (gloo),
    padded to the largest rank's size; the root places them at their global
    offsets.  Returns the whole record stream on the root, None elsewhere."""
    import torch
    import torch.distributed as dist
    sizes = [sum(layout.records[q]) * RECORD_BYTES for q in range(layout.world)]
    if len(local) != sizes[rank]:
        raise ValueError(f"rank {rank}: {len(local)} record bytes, layout says {sizes[rank]}")
    mx = max(max(sizes), 1)
    t = torch.zeros(mx, dtype=torch.uint8)
    if local:
        t[: len(local)] = torch.frombuffer(bytearray(local), dtype=torch.uint8)
    bufs = [torch.zeros(mx, dtype=torch.uint8) for _ in range(layout.world)] if rank == root else None
    dist.gather(t, bufs, dst=root)
    if rank != root:
        return None
    out = bytearray(layout.total_records * RECORD_BYTES)
    for q in range(layout.world):
        o = layout.rank_offset[q] * RECORD_BYTES
        out[o:o + sizes[q]] = bytes(bufs[q][: sizes[q]].numpy())
    return bytes(out)


def rank_records_host(eng: Engine, files: Sequence, layout: ShardLayout, rank: int, seed: int) -> bytes:
    """This rank's records of a host-resident file list (the PCIe-inclusive
    path): every batch's pieces through Engine.block_sums, concatenated in
    batch order = the rank's slice of the global record stream."""
    out = []
    for g in layout.batches[rank]:
        if not g:
            continue
        views = [memoryview(files[p.file]).cast("B")[p.offset:p.offset + p.length] for p in g]
        _, rec, _ = eng.block_sums(views, seed, [p.block_len for p in g])
        out.append(rec)
    return b"".join(out)


def records_digest(records) -> str:
    """SHA-256 of one rank's record bytes (what it sent to the root)."""
    import hashlib
    return hashlib.sha256(memoryview(records).cast("B")).hexdigest()


def all_ranks(obj, world: int) -> list:
    """obj of every rank, in rank order, on every rank, over the control plane
    (gloo all_gather_object); world 1 needs no process group."""
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def gather_parity(recv, digests: Sequence[str], records: Sequence[int]) -> dict:
    """The root's check of a gather (GenerateFiles emits every file's sums in
    file-list order, generator.go:20-52; rank q's records are the global
    slice starting at the exclusive prefix of the ranks' counts): the
    gathered buffer `recv` (bytes on the root) holds, at each rank's slice,
    exactly the bytes that rank hashed -- their SHA-256 equals the digest
    the rank reported -- and nothing beyond the last slice is expected.
    -> {"ranks_equal": [bool per rank], "all_equal": bool}."""
    mv = memoryview(recv).cast("B")
    want = sum(records) * RECORD_BYTES
    ok, o = [], 0
    for d, n in zip(digests, records):
        seg = mv[o:o + n * RECORD_BYTES]
        ok.append(len(seg) == n * RECORD_BYTES and records_digest(seg) == d)
        o += n * RECORD_BYTES
    return {"ranks_equal": ok, "all_equal": all(ok) and len(mv) >= want}
