"""One process driving several GPUs (include/rsg.h
"one process, many GPUs"): the shape of gokr-rsync's receiver, one process
whose generator goroutine writes every file's sums in file-list order
(internal/receiver/do.go:96-98, generator.go:20-52).

    shard_plan      rsg_shard_plan: the global block sequence cut into
                    contiguous byte-balanced ranges (one per device) and
                    batches (C++ restatement of shard.plan_shards +
                    dist.split_batches; tests/test_shard_plan.py checks they
                    agree)
    MultiEngine     N contexts: rsg_comm_init_all, rsg_block_sums_host_multi,
                    rsg_generate_files_fd_multi, rsg_block_sums_{gather,d2h}_multi
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import numpy as np

from . import _lib
from ._lib import File, SumHead, check, lib
from .engine import RECORD_BYTES, Engine, _i32, _ptr, _u8


def shard_plan(lengths: Sequence[int], world: int, nbatch: int = 1, block_len=0):
    """-> (pieces, records) with pieces = [(file, b0, b1, offset, length,
    record, block_len, rank, batch)] in global order and records[q][b] the
    record count of rank q's batch b."""
    n = len(lengths)
    ln = np.ascontiguousarray(lengths, dtype=np.uint64)
    bl = None
    if isinstance(block_len, (list, tuple, np.ndarray)):
        bl = np.ascontiguousarray(block_len, dtype=np.int32)
    scalar = 0 if bl is not None else int(block_len)
    cnt = ctypes.c_uint64()
    recs = np.zeros(world * nbatch, np.uint64)
    st = lib.rsg_shard_plan(ln.ctypes.data if n else None, bl.ctypes.data if bl is not None else None, n, scalar,
                            world, nbatch, None, 0, ctypes.byref(cnt), recs.ctypes.data)
    if st not in (_lib.OK, _lib.ERR_TRUNCATED):
        check(st)
    arr = (_lib.Piece * max(cnt.value, 1))()
    check(lib.rsg_shard_plan(ln.ctypes.data if n else None, bl.ctypes.data if bl is not None else None, n, scalar,
                             world, nbatch, arr, cnt.value, ctypes.byref(cnt), recs.ctypes.data))
    pieces = [(p.file, p.b0, p.b1, p.offset, p.length, p.record, p.block_len, p.rank, p.batch)
              for p in arr[:cnt.value]]
    return pieces, recs.reshape(world, nbatch).astype(int).tolist()


class MultiEngine:
    """N device contexts driven from this thread (one rank per context)."""

    def __init__(self, engines: Sequence[Engine]):
        self.engines = list(engines)
        self.n = len(self.engines)
        self._ctxs = (ctypes.c_void_p * self.n)(*[e.ctx.value for e in self.engines])

    def comm_init_all(self):
        """RCCL communicator over the engines' devices (ncclCommInitAll): one
        rank per device, engine q = rank q."""
        check(lib.rsg_comm_init_all(self._ctxs, self.n), self.engines[0].ctx)

    def block_sums(self, files: Sequence, seed: int, block_len=0):
        """rsg_block_sums_host_multi: host buffers in, the whole record stream
        out, every device hashing its share.  -> (heads, records bytes)."""
        n = len(files)
        bl = list(block_len) if isinstance(block_len, (list, tuple)) else [block_len] * n
        arrs = [_u8(f) for f in files]
        desc = (File * max(n, 1))()
        for i, a in enumerate(arrs):
            desc[i].data = a.ctypes.data if a.size else None
            desc[i].len = a.size
            desc[i].block_len = bl[i]
        heads = (SumHead * max(n, 1))()
        total = ctypes.c_uint64()
        check(lib.rsg_plan_block_sums(desc, n, heads, None, ctypes.byref(total)))
        out = np.empty(max(total.value, 1) * RECORD_BYTES, dtype=np.uint8)
        check(lib.rsg_block_sums_host_multi(self._ctxs, self.n, desc, n, _i32(seed), _ptr(out), total.value),
              self.engines[0].ctx)
        return [heads[i] for i in range(n)], out[: total.value * RECORD_BYTES].tobytes()

    def generate_files_fd(self, files: Sequence, seed: int, write, block_len=0, idx=None,
                          terminate: bool = True, mux: bool = False):
        """rsg_generate_files_fd_multi: Engine.generate_files_fd's stream with
        the global block sequence sharded over the devices.
        -> (heads, bytes written)."""
        n = len(files)
        bl = list(block_len) if isinstance(block_len, (list, tuple)) else [block_len] * n
        desc = (_lib.FdFile * max(n, 1))()
        for i, f in enumerate(files):
            desc[i].fd = f[0]
            desc[i].len = f[1]
            desc[i].offset = f[2] if len(f) > 2 else 0
            desc[i].block_len = bl[i]
            desc[i].idx = idx[i] if idx is not None else 0
        flags = (_lib.GEN_IDX if idx is not None else 0) | (_lib.GEN_TERMINATE if terminate else 0) | \
                (_lib.GEN_MUX if mux else 0)
        err = []

        def _cb(_user, data, nbytes):
            try:
                write(ctypes.string_at(data, nbytes))
                return 0
            except Exception as e:  # surfaces as RSG_ERR_IO; re-raised below
                err.append(e)
                return -1

        cb = _lib.WRITE_FN(_cb)
        heads = (SumHead * max(n, 1))()
        written = ctypes.c_uint64()
        st = lib.rsg_generate_files_fd_multi(self._ctxs, self.n, desc, n, _i32(seed), flags, cb, None, heads,
                                             ctypes.byref(written))
        if err:
            raise err[0]
        check(st, self.engines[0].ctx)
        return [heads[i] for i in range(n)], written.value

    def _ranks(self, sharded: Sequence, arenas, records, rank_offsets):
        arr = (_lib.ShardRank * self.n)()
        for q in range(self.n):
            arr[q].ctx = self.engines[q].ctx.value
            arr[q].d_arena = arenas[q].ptr
            arr[q].d_records = records[q].ptr
            arr[q].batches = sharded[q].batches
            arr[q].nbatch = sharded[q].nbatch
            arr[q].rank_record_offset = rank_offsets[q] if rank_offsets is not None else 0
        return arr

    def gather(self, sharded: Sequence, arenas, seed: int, records, recv, root: int = 0):
        """rsg_block_sums_gather_multi over dist.ShardedBlockSums of every
        rank (plans of engine q): every rank's records to recv on `root`."""
        check(lib.rsg_block_sums_gather_multi(self._ranks(sharded, arenas, records, None), self.n, _i32(seed),
                                              ctypes.c_void_p(recv.ptr), root), self.engines[0].ctx)

    def d2h(self, sharded: Sequence, arenas, seed: int, records, rank_offsets: Sequence[int], host: np.ndarray):
        """rsg_block_sums_d2h_multi: every rank's records into host (global
        order: rank q's at rank_offsets[q])."""
        check(lib.rsg_block_sums_d2h_multi(self._ranks(sharded, arenas, records, rank_offsets), self.n,
                                           _i32(seed), ctypes.c_void_p(host.ctypes.data)), self.engines[0].ctx)

    def close(self):
        for e in self.engines:
            e.close()
