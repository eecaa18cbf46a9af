"""Host-side mirror of the reference's block-checksum surface over librsg.so.

The reference (Go) keeps these entry points, which this module mirrors name
for name so parity tests read like the reference's own code:

  rsyncchecksum.Checksum1 / Checksum2      rsyncchecksum.go:29-58   -> checksum1 / checksum2
  rsynccommon.SumSizesSqroot               rsynccommon.go:14-37     -> sum_sizes_sqroot
  (*receiver.Transfer).generateAndSendSums generator.go:325-350     -> Engine.generate_and_send_sums
  (*sender.Transfer).hashSearch            match.go:21-230          -> Engine.hash_search
  matched / simpleSendToken                match.go:233, token.go:4 -> encode_tokens
  (*receiver.Transfer).receiveData         receiver.go:98-188       -> Engine.receive_data / apply_tokens

Every checksum is computed by the HIP kernels; nothing here hashes bytes on
the CPU.  Errors surface as RsgError (the Go side maps them to `error`).
"""
from __future__ import annotations

import ctypes
import struct
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import File, Match, RsgError, SumHead, check, lib

RECORD_BYTES = _lib.RECORD_BYTES


def _u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    return np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def sum_sizes_sqroot(content_len: int, block_len: int = 0) -> SumHead:
    """rsynccommon.SumSizesSqroot (rsynccommon.go:14-37); block_len > 0 overrides B."""
    h = SumHead()
    check(lib.rsg_sum_head_for(content_len, block_len, ctypes.byref(h)))
    return h


def device_count() -> int:
    return int(lib.rsg_device_count())


_MATCH_DT = np.dtype([("offset", "<i8"), ("index", "<i4"), ("reserved", "<i4")])


def _matches_list(out, n: int):
    """(offset, block index) pairs from an rsg_match array, converted in C
    (a per-element ctypes loop costs ~1 ms per 10 000 matches)."""
    if n == 0:
        return []
    a = np.frombuffer(out, dtype=_MATCH_DT, count=n)
    return list(zip(a["offset"].tolist(), a["index"].tolist()))


class DeviceBuffer:
    """HBM allocation owned by an Engine (plain device pointer + size)."""

    def __init__(self, engine: "Engine", nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib.rsg_alloc_device(engine.ctx, max(self.nbytes, 1), ctypes.byref(p)), engine.ctx)
        self.ptr = p.value

    def upload(self, data, offset: int = 0):
        a = _u8(data)
        if offset + a.size > self.nbytes:
            raise ValueError("upload past the end of the buffer")
        if a.size:
            check(lib.rsg_memcpy_h2d(self.engine.ctx, ctypes.c_void_p(self.ptr + offset), _ptr(a), a.size),
                  self.engine.ctx)

    def download(self, nbytes: Optional[int] = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.uint8)
        if n:
            check(lib.rsg_memcpy_d2h(self.engine.ctx, _ptr(out), ctypes.c_void_p(self.ptr + offset), n),
                  self.engine.ctx)
        return out

    def free(self):
        if self.ptr is not None:
            lib.rsg_free_device(self.engine.ctx, ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr is not None and self.engine.ctx:
                self.free()
        except Exception:
            pass


class Plan:
    """Device-resident block-sum plan for a fixed file layout in an arena."""

    def __init__(self, engine: "Engine", files: Sequence[Tuple[int, int, int]], arena_bytes: int):
        self.engine = engine
        arr = (File * max(len(files), 1))()
        for i, (off, ln, bl) in enumerate(files):
            arr[i].offset, arr[i].len, arr[i].block_len = off, ln, bl
        p = ctypes.c_void_p()
        check(lib.rsg_plan_create(engine.ctx, arr, len(files), arena_bytes, ctypes.byref(p)), engine.ctx)
        self.handle = p.value
        self.total_records = int(lib.rsg_plan_total_records(ctypes.c_void_p(self.handle)))
        heads = (SumHead * max(len(files), 1))()
        first = (ctypes.c_uint64 * max(len(files), 1))()
        check(lib.rsg_plan_block_sums(arr, len(files), heads, first, None))
        self.heads = [heads[i] for i in range(len(files))]
        self.first_record = [int(first[i]) for i in range(len(files))]

    def run(self, arena: "DeviceBuffer | int", seed: int, records: "DeviceBuffer | int", stream=None):
        aptr = arena.ptr if isinstance(arena, DeviceBuffer) else int(arena)
        rptr = records.ptr if isinstance(records, DeviceBuffer) else int(records)
        check(lib.rsg_block_sums_planned(self.engine.ctx, ctypes.c_void_p(self.handle), ctypes.c_void_p(aptr),
                                         _i32(seed), ctypes.c_void_p(rptr), ctypes.c_void_p(stream or 0)),
              self.engine.ctx)

    def close(self):
        if self.handle:
            lib.rsg_plan_destroy(ctypes.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Conn:
    """Writer side of rsyncwire.Conn (wire.go:131-159): int32 LE + raw bytes."""

    def __init__(self, writer=None):
        self.buf = bytearray() if writer is None else None
        self.writer = writer

    def write(self, b: bytes):
        if self.buf is not None:
            self.buf += b
        else:
            self.writer.write(b)

    def write_int32(self, v: int):
        self.write(struct.pack("<i", _i32(v)))


class SearchBatch:
    """A prepared rsg_hash_search_batch_* call: the rsg_search_job array (with
    every job's match array) is built once, so repeated calls time only the
    C-ABI call itself (bench.py's cfg4-sender workload).  jobs as
    Engine.hash_search_batch."""

    def __init__(self, engine: "Engine", jobs, device: bool = True):
        self.engine, self.device, self.n = engine, device, len(jobs)
        self.arr = (_lib.SearchJob * max(self.n, 1))()
        self._keep, self.outs = [], []
        for k, (src, src_len, head, sum1, sum2, targets) in enumerate(jobs):
            j = self.arr[k]
            if device:
                j.src, j.src_len = src.ptr, src_len
            else:
                a = _u8(src)
                self._keep.append(a)
                j.src, j.src_len = _ptr(a).value, a.size if src_len is None else src_len
            j.head = head if isinstance(head, SumHead) else SumHead(*head)
            s1 = np.ascontiguousarray(sum1, dtype=np.uint32)
            s2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
            tg = np.ascontiguousarray(targets, dtype=np.int32)
            self._keep += [s1, s2, tg]
            j.sum1, j.sum2, j.targets = _ptr(s1).value, _ptr(s2).value, _ptr(tg).value
            cap = j.src_len // max(j.head.block_len, 1) + 2
            out = np.empty(cap, dtype=_MATCH_DT)
            self.outs.append(out)
            j.matches, j.match_cap = ctypes.cast(out.ctypes.data, ctypes.POINTER(Match)), cap
        self._fn = lib.rsg_hash_search_batch_device if device else lib.rsg_hash_search_batch_host

    def run(self, seed: int) -> int:
        """One rsg_hash_search_batch_* call; returns its status."""
        return self._fn(self.engine.ctx, self.arr, self.n, _i32(seed))

    def status(self, k: int) -> int:
        return self.arr[k].status

    def n_matches(self, k: int) -> int:
        return self.arr[k].n_matches

    def matches(self, k: int, as_arrays: bool = False):
        m = self.outs[k][: self.arr[k].n_matches]
        return m if as_arrays else _matches_list(m, len(m))


class Engine:
    """One device context (rsg_ctx): its own stream, scratch and RCCL comm."""

    def __init__(self, device: int = 0):
        p = ctypes.c_void_p()
        check(lib.rsg_ctx_create(device, ctypes.byref(p)))
        self.ctx = p
        self.device = device

    def close(self):
        if self.ctx:
            lib.rsg_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ memory
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def alloc_pinned(self, nbytes: int) -> np.ndarray:
        """Page-locked host memory (rsg_alloc_pinned) as a uint8 array.  Files
        read into it go to HBM by DMA with no staging copy.  Release with
        free_pinned(arr) before the engine closes."""
        p = ctypes.c_void_p()
        check(lib.rsg_alloc_pinned(self.ctx, max(nbytes, 1), ctypes.byref(p)), self.ctx)
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value)
        return np.frombuffer(buf, dtype=np.uint8)[:nbytes]

    def free_pinned(self, arr: np.ndarray):
        check(lib.rsg_free_pinned(self.ctx, ctypes.c_void_p(arr.ctypes.data)), self.ctx)

    def fill_splitmix64(self, buf: DeviceBuffer, nbytes: int, seed: int, offset: int = 0, stream=None):
        check(lib.rsg_fill_splitmix64(self.ctx, ctypes.c_void_p(buf.ptr + offset), nbytes, seed & (2**64 - 1),
                                      ctypes.c_void_p(stream or 0)), self.ctx)

    def synchronize(self, stream=None):
        check(lib.rsg_synchronize(self.ctx, ctypes.c_void_p(stream or 0)), self.ctx)

    def plan(self, files: Sequence[Tuple[int, int, int]], arena_bytes: int) -> Plan:
        return Plan(self, files, arena_bytes)

    def set_block_sums_kernel(self, variant: int):
        """rsg_set_block_sums_kernel: this context's block-sum kernel variant
        (-1 automatic; every variant gives identical records)."""
        check(lib.rsg_set_block_sums_kernel(self.ctx, variant), self.ctx)

    def block_sums_fallbacks(self, reset: bool = True) -> Tuple[int, int]:
        """Fallback census (rsg_block_sums_fallbacks): (staged waves, park
        tiles) of full 64-block groups hashed with per-lane loads instead of
        the LDS-DMA path since the last reset.  Waits for the device."""
        c = (ctypes.c_uint64 * 2)()
        check(lib.rsg_block_sums_fallbacks(self.ctx, c, int(reset)), self.ctx)
        return int(c[0]), int(c[1])

    # ------------------------------------------------------------ receiver
    def block_sums(self, files: Sequence, seed: int, block_len=0):
        """Block sums of host buffers (the PCIe-inclusive path).
        -> (heads, records bytes, first_record)."""
        n = len(files)
        bl = list(block_len) if isinstance(block_len, (list, tuple)) else [block_len] * n
        arrs = [_u8(f) for f in files]
        desc = (File * max(n, 1))()
        for i, a in enumerate(arrs):
            desc[i].data = a.ctypes.data if a.size else None
            desc[i].len = a.size
            desc[i].block_len = bl[i]
        heads = (SumHead * max(n, 1))()
        first = (ctypes.c_uint64 * max(n, 1))()
        total = ctypes.c_uint64()
        check(lib.rsg_plan_block_sums(desc, n, heads, first, ctypes.byref(total)))
        out = np.empty(max(total.value, 1) * RECORD_BYTES, dtype=np.uint8)
        check(lib.rsg_block_sums_host(self.ctx, desc, n, _i32(seed), _ptr(out), total.value), self.ctx)
        return ([heads[i] for i in range(n)], out[: total.value * RECORD_BYTES].tobytes(),
                [int(first[i]) for i in range(n)])

    def block_sums_device(self, arena: DeviceBuffer, files: Sequence[Tuple[int, int, int]], seed: int,
                          records: Optional[DeviceBuffer] = None):
        """One-shot device-resident call. files = [(offset, len, block_len)]."""
        n = len(files)
        desc = (File * max(n, 1))()
        for i, (off, ln, b) in enumerate(files):
            desc[i].offset, desc[i].len, desc[i].block_len = off, ln, b
        total = ctypes.c_uint64()
        check(lib.rsg_plan_block_sums(desc, n, None, None, ctypes.byref(total)))
        if records is None:
            records = self.alloc(max(total.value, 1) * RECORD_BYTES)
        check(lib.rsg_block_sums_device(self.ctx, ctypes.c_void_p(arena.ptr), arena.nbytes, desc, n, _i32(seed),
                                        ctypes.c_void_p(records.ptr), records.nbytes // RECORD_BYTES), self.ctx)
        return records, total.value

    def generate_and_send_sums(self, conn: Conn, data, file_len: int, seed: int, block_len: int = 0):
        """(*receiver.Transfer).generateAndSendSums (generator.go:325-350):
        SumHead then count x (int32 sum1, sum2[16]) on conn."""
        a = _u8(data)
        if a.size != file_len:
            raise RsgError(_lib.ERR_INVALID, f"short read: {a.size} of {file_len} bytes")
        heads, rec, _ = self.block_sums([a], seed, block_len)
        h = heads[0]
        conn.write(struct.pack("<4i", *h.astuple()))  # SumHead.WriteTo, types.go:79-86
        conn.write(rec)
        return h

    def generate_files(self, conn: Conn, files: Sequence, seed: int, block_len=0, s2len: int = 16,
                       mux: bool = False) -> List[SumHead]:
        """GenerateFiles (generator.go:20-41) for a file list whose every entry
        goes to generateAndSendSums (regular files with a basis, -I): one
        batched kernel call, then the whole sums stream -- idx, SumHead and
        records per file, the two -1 phase markers -- in one buffer, framed in
        <= 256 KiB MsgData messages when mux (the server side, wire.go:28-36)."""
        heads, rec, _ = self.block_sums(files, seed, block_len)
        if s2len != 16:
            heads = [SumHead(h.count, h.block_len, s2len, h.rem) for h in heads]
        stream = encode_sums(heads, rec, file_idx=range(len(heads)), terminate=True)
        conn.write(mux_frame(stream) if mux else stream)
        return heads

    def generate_files_fd(self, files: Sequence, seed: int, write, block_len=0, idx=None,
                          terminate: bool = True, mux: bool = False) -> Tuple[List[SumHead], int]:
        """GenerateFiles' host loop from open files (generator.go:143-350):
        files = [(fd, len)] or [(fd, len, offset)]; file bytes are read by the
        engine (pread, overlapped with the GPU), the sums stream goes to
        write(bytes) once per batch.  idx = file-list indices written before
        each SumHead (None: no idx words).  -> (heads, bytes written)."""
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
        st = lib.rsg_generate_files_fd(self.ctx, desc, n, _i32(seed), flags, cb, None, heads, ctypes.byref(written))
        if err:
            raise err[0]
        check(st, self.ctx)
        return [heads[i] for i in range(n)], written.value

    # ------------------------------------------------------------ whole-file sums
    def file_sums(self, files: Sequence, mode: int = _lib.FILESUM_PLAIN, seed: int = 0) -> List[bytes]:
        """Whole-file MD4 of each host buffer, one GPU lane per file:
        FILESUM_PLAIN = rsyncchecksum.ReaderChecksum (rsyncchecksum.go:60-66),
        FILESUM_SEEDED = the transfer's MD4(int32_LE(seed) || file)
        (match.go:52-53, receiver.go:117-120)."""
        n = len(files)
        if n == 0:
            return []
        arrs = [_u8(f) for f in files]
        desc = (File * n)()
        for i, a in enumerate(arrs):
            desc[i].data = a.ctypes.data if a.size else None
            desc[i].len = a.size
        out = np.empty(16 * n, dtype=np.uint8)
        check(lib.rsg_file_sums_host(self.ctx, desc, n, mode, _i32(seed), _ptr(out)), self.ctx)
        return [out[16 * i: 16 * i + 16].tobytes() for i in range(n)]

    def receive_data(self, stream, head, basis, seed: int) -> Tuple[bytes, int]:
        """(*receiver.Transfer).receiveData (receiver.go:98-188): rebuild the file
        from `stream` (tokens, int32 0, 16-byte whole-file sum) and the basis
        (None = no local file), then check MD4(int32_LE(seed) || file) on the
        GPU against the sender's sum.  -> (file bytes, stream bytes consumed).
        RsgError status ERR_CORRUPT = the reference's "file corruption"."""
        t = _u8(stream)
        b = _u8(basis) if basis is not None else None
        h = head if isinstance(head, SumHead) else SumHead(*head)
        n, used = ctypes.c_uint64(), ctypes.c_uint64()
        bp, bl = (_ptr(b), b.size) if b is not None else (ctypes.c_void_p(0), 0)
        st = lib.rsg_apply_tokens(_ptr(t), t.size, ctypes.byref(h), bp, bl, None, 0, ctypes.byref(n),
                                  ctypes.byref(used))
        if st != _lib.ERR_TRUNCATED:
            check(st)
        out = np.empty(max(n.value, 1), dtype=np.uint8)
        check(lib.rsg_receive_data(self.ctx, _ptr(t), t.size, ctypes.byref(h), bp, bl, _i32(seed), _ptr(out),
                                   n.value, ctypes.byref(n), ctypes.byref(used)), self.ctx)
        return out[: n.value].tobytes(), used.value

    def receive_data_batch(self, jobs, seed: int, raise_on_error: bool = True):
        """RecvFiles' per-file receiveData calls (receiver.go:18-188) in one
        batched call: jobs = [(stream, head, basis)] as receive_data takes
        them.  The whole-file sums of all files are checked together on the
        GPU (one lane per file).  Returns [(file bytes, consumed)], or with
        raise_on_error=False [(status, file bytes, consumed)]."""
        n = len(jobs)
        arr = (_lib.RecvJob * max(n, 1))()
        keep, outs = [], []
        for k, (stream, head, basis) in enumerate(jobs):
            t = _u8(stream)
            b = _u8(basis) if basis is not None else None
            h = head if isinstance(head, SumHead) else SumHead(*head)
            need, used = ctypes.c_uint64(), ctypes.c_uint64()
            bp, bl = (_ptr(b), b.size) if b is not None else (ctypes.c_void_p(0), 0)
            st = lib.rsg_apply_tokens(_ptr(t), t.size, ctypes.byref(h), bp, bl, None, 0, ctypes.byref(need),
                                      ctypes.byref(used))
            cap = need.value if st in (_lib.OK, _lib.ERR_TRUNCATED) else 0
            out = np.empty(max(cap, 1), dtype=np.uint8)
            keep += [t, b]
            outs.append(out)
            j = arr[k]
            j.tokens, j.tokens_len, j.head = _ptr(t).value, t.size, h
            j.basis, j.basis_len = bp.value, bl
            j.out, j.out_cap = out.ctypes.data, cap
        st = lib.rsg_receive_data_batch(self.ctx, arr, n, _i32(seed))
        if raise_on_error:
            check(st, self.ctx)
            return [(outs[k][: arr[k].out_len].tobytes(), arr[k].consumed) for k in range(n)]
        return [(arr[k].status, outs[k][: arr[k].out_len].tobytes() if arr[k].status == _lib.OK else b"",
                 arr[k].consumed) for k in range(n)]

    def file_sums_device(self, arena: DeviceBuffer, files: Sequence[Tuple[int, int]], mode: int = _lib.FILESUM_PLAIN,
                         seed: int = 0, out: Optional[DeviceBuffer] = None) -> DeviceBuffer:
        """Same for files already in device memory: files = [(offset, len)];
        returns a device buffer of len(files) * 16 digest bytes."""
        n = len(files)
        desc = (File * max(n, 1))()
        for i, (off, ln) in enumerate(files):
            desc[i].offset, desc[i].len = off, ln
        if out is None:
            out = self.alloc(max(n, 1) * 16)
        check(lib.rsg_file_sums_device(self.ctx, ctypes.c_void_p(arena.ptr), arena.nbytes, desc, n, mode, _i32(seed),
                                       ctypes.c_void_p(out.ptr)), self.ctx)
        return out

    # ------------------------------------------------------------ sender
    def hash_search(self, src, head, sum1, sum2, targets, seed: int) -> List[Tuple[int, int]]:
        """(*sender.Transfer).hashSearch (match.go:21-230): the greedy match
        list [(offset, block index)] in offset order."""
        a = _u8(src)
        h = head if isinstance(head, SumHead) else SumHead(*head)
        s1 = np.ascontiguousarray(sum1, dtype=np.uint32)
        s2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
        tg = np.ascontiguousarray(targets, dtype=np.int32)
        cap = a.size // max(h.block_len, 1) + 2
        out = (Match * cap)()
        nm = ctypes.c_uint64()
        check(lib.rsg_hash_search_host(self.ctx, _ptr(a), a.size, ctypes.byref(h), _ptr(s1), _ptr(s2), _ptr(tg),
                                       _i32(seed), out, cap, ctypes.byref(nm)), self.ctx)
        return _matches_list(out, nm.value)

    def hash_search_device(self, src: DeviceBuffer, src_len: int, head, sum1, sum2, targets, seed: int):
        h = head if isinstance(head, SumHead) else SumHead(*head)
        s1 = np.ascontiguousarray(sum1, dtype=np.uint32)
        s2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
        tg = np.ascontiguousarray(targets, dtype=np.int32)
        cap = src_len // max(h.block_len, 1) + 2
        out = (Match * cap)()
        nm = ctypes.c_uint64()
        check(lib.rsg_hash_search_device(self.ctx, ctypes.c_void_p(src.ptr), src_len, ctypes.byref(h), _ptr(s1),
                                         _ptr(s2), _ptr(tg), _i32(seed), out, cap, ctypes.byref(nm)), self.ctx)
        return _matches_list(out, nm.value)

    def hash_search_fd(self, fd: int, src_len: int, head, sum1, sum2, targets, seed: int, offset: int = 0,
                       file_sum: bool = False):
        """hashSearch over a source the engine reads from `fd` in windows
        (rsg_hash_search_fd; sendFile's mapFile/ptr, fileio.go:31-112).
        -> matches, or (matches, MD4(int32_LE(seed) || source)) with file_sum."""
        h = head if isinstance(head, SumHead) else SumHead(*head)
        s1 = np.ascontiguousarray(sum1, dtype=np.uint32)
        s2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
        tg = np.ascontiguousarray(targets, dtype=np.int32)
        cap = src_len // max(h.block_len, 1) + 2
        out = (Match * cap)()
        nm = ctypes.c_uint64()
        dig = np.zeros(16, np.uint8)
        check(lib.rsg_hash_search_fd(self.ctx, fd, offset, src_len, ctypes.byref(h), _ptr(s1), _ptr(s2), _ptr(tg),
                                     _i32(seed), out, cap, ctypes.byref(nm),
                                     _ptr(dig) if file_sum else None), self.ctx)
        m = _matches_list(out, nm.value)
        return (m, dig.tobytes()) if file_sum else m

    def hash_search_fd_batch(self, jobs, seed: int, file_sums: bool = True, raise_on_error: bool = True):
        """SendFiles' loop over sources that are open files
        (rsg_hash_search_fd_batch): jobs = [(fd, src_len, head, sum1, sum2,
        targets)] or with a 7th item, the offset in fd.  Each source is
        searched as hash_search_fd would, in job order, while the whole-file
        sums MD4(int32_LE(seed) || source) of several files run on host
        threads side by side.  -> [(matches, file_sum or None)], or with
        raise_on_error=False [(status, matches, file_sum)]."""
        n = len(jobs)
        arr = (_lib.FdSearchJob * max(n, 1))()
        keep, outs, sums = [], [], []
        for k, job in enumerate(jobs):
            fd, src_len, head, sum1, sum2, targets = job[:6]
            j = arr[k]
            j.fd, j.src_len, j.offset = fd, src_len, (job[6] if len(job) > 6 else 0)
            j.head = head if isinstance(head, SumHead) else SumHead(*head)
            s1 = np.ascontiguousarray(sum1, dtype=np.uint32)
            s2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
            tg = np.ascontiguousarray(targets, dtype=np.int32)
            keep += [s1, s2, tg]
            j.sum1, j.sum2, j.targets = _ptr(s1).value, _ptr(s2).value, _ptr(tg).value
            cap = src_len // max(j.head.block_len, 1) + 2
            out = np.empty(cap, dtype=_MATCH_DT)
            outs.append(out)
            j.matches, j.match_cap = ctypes.cast(out.ctypes.data, ctypes.POINTER(Match)), cap
            dig = np.zeros(16, np.uint8)
            sums.append(dig)
            j.file_sum = _ptr(dig).value if file_sums else None
        st = lib.rsg_hash_search_fd_batch(self.ctx, arr, n, _i32(seed))

        def res(k):
            m = outs[k][: arr[k].n_matches]
            return _matches_list(m, len(m))
        if raise_on_error:
            check(st, self.ctx)
            return [(res(k), sums[k].tobytes() if file_sums else None) for k in range(n)]
        return [(arr[k].status, res(k) if arr[k].status == _lib.OK else [],
                 sums[k].tobytes() if file_sums and arr[k].status == _lib.OK else None) for k in range(n)]

    def hash_search_batch(self, jobs, seed: int, device: bool = True, raise_on_error: bool = True,
                          as_arrays: bool = False):
        """SendFiles' per-file hashSearch loop (sender.go:19-115) in one
        pipelined call.  jobs = [(src, src_len, head, sum1, sum2, targets)]:
        src is a DeviceBuffer (or any object with a device address in .ptr)
        when device, else host bytes / a uint8 array (src_len None = its
        length).  Returns one match list per job, or with raise_on_error=False
        a list of (status, matches) pairs.  as_arrays: matches stay the
        C-ABI's rsg_match records (numpy structured arrays with fields offset /
        index), as a Go caller would read them."""
        b = SearchBatch(self, jobs, device)
        st = b.run(seed)
        if raise_on_error:
            check(st, self.ctx)
            return [b.matches(k, as_arrays) for k in range(b.n)]
        return [(b.status(k), b.matches(k, as_arrays) if b.status(k) == _lib.OK else []) for k in range(b.n)]

    SEARCH_OPTIONS = {"path": 0, "host_tables": 1, "force_table_ovf": 2, "spec": 3, "confirm_cus": 4, "recv_md4": 5,
                      "fs_key_shift": 6}

    def set_option(self, name: str, value: int):
        """rsg_testing_search_option: one of SEARCH_OPTIONS on this context
        (include/rsg_testing.h; results are identical under every value)."""
        check(lib.rsg_testing_search_option(self.ctx, self.SEARCH_OPTIONS[name], int(value)), self.ctx)

    def set_search_path(self, mode: int):
        """0 = small sources through the one-wave-per-file kernel (default),
        1 = every source through the large-file pipeline."""
        self.set_option("path", mode)

    def set_kernel_timing(self, on: bool = True):
        """rsg_set_kernel_timing: bracket the sender's kernels with HIP events."""
        check(lib.rsg_set_kernel_timing(self.ctx, int(on)), self.ctx)

    def kernel_times(self, reset: bool = True) -> dict:
        """Totals since the last reset: roll_ms, roll_launches, confirm_ms,
        confirm_batches, candidates (offsets the rolls returned), windows
        (confirmed by the strong-sum kernel), filesums_ms, filesums_launches."""
        o = (ctypes.c_double * 8)()
        check(lib.rsg_kernel_times(self.ctx, o, int(reset)), self.ctx)
        return {"roll_ms": o[0], "roll_launches": int(o[1]), "confirm_ms": o[2], "confirm_batches": int(o[3]),
                "candidates": int(o[4]), "windows": int(o[5]), "filesums_ms": o[6], "filesums_launches": int(o[7])}

    # ------------------------------------------------------------ multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        check(lib.rsg_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        check(lib.rsg_comm_init(self.ctx, nranks, rank, buf), self.ctx)

    def gather_bytes(self, send: DeviceBuffer, send_bytes: Sequence[int], recv: Optional[DeviceBuffer], root: int = 0,
                     stream=None):
        sb = (ctypes.c_uint64 * len(send_bytes))(*send_bytes)
        check(lib.rsg_gather_bytes(self.ctx, ctypes.c_void_p(send.ptr), sb,
                                   ctypes.c_void_p(recv.ptr if recv is not None else 0), root,
                                   ctypes.c_void_p(stream or 0)), self.ctx)


def encode_tokens(src, head, matches: Iterable[Tuple[int, int]]) -> bytes:
    """Token bytes of matched()/simpleSendToken (match.go:233-282, token.go:4-31)."""
    a = _u8(src)
    h = head if isinstance(head, SumHead) else SumHead(*head)
    ms = list(matches)
    arr = (Match * max(len(ms), 1))()
    for i, (o, ix) in enumerate(ms):
        arr[i].offset, arr[i].index = o, ix
    n = ctypes.c_uint64()
    check(lib.rsg_encode_tokens(_ptr(a), a.size, ctypes.byref(h), arr, len(ms), None, 0, ctypes.byref(n)))
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    check(lib.rsg_encode_tokens(_ptr(a), a.size, ctypes.byref(h), arr, len(ms), _ptr(out), n.value,
                                ctypes.byref(n)))
    return out[: n.value].tobytes()


def apply_tokens(stream, head, basis) -> Tuple[bytes, int]:
    """The token loop of receiveData (receiver.go:122-163) without the sum
    check: -> (file bytes, offset of the whole-file sum in `stream`)."""
    t = _u8(stream)
    b = _u8(basis) if basis is not None else None
    h = head if isinstance(head, SumHead) else SumHead(*head)
    n, used = ctypes.c_uint64(), ctypes.c_uint64()
    bp, bl = (_ptr(b), b.size) if b is not None else (ctypes.c_void_p(0), 0)
    st = lib.rsg_apply_tokens(_ptr(t), t.size, ctypes.byref(h), bp, bl, None, 0, ctypes.byref(n), ctypes.byref(used))
    if st != _lib.ERR_TRUNCATED:
        check(st)
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    check(lib.rsg_apply_tokens(_ptr(t), t.size, ctypes.byref(h), bp, bl, _ptr(out), n.value, ctypes.byref(n),
                               ctypes.byref(used)))
    return out[: n.value].tobytes(), used.value


# ------------------------------------------------------------------ wire formats
MSG_DATA, MSG_ERROR, MSG_INFO = 0, 1, 2  # wire.go:12-14


def _sized(call) -> bytes:
    """Runs a size-query/fill pair of an rsg_* formatter (out == NULL first)."""
    n = ctypes.c_uint64()
    check(call(None, 0, ctypes.byref(n)))
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    check(call(_ptr(out), n.value, ctypes.byref(n)))
    return out[: n.value].tobytes()


def encode_sums(heads, records, file_idx: Optional[Sequence[int]] = None, terminate: bool = False) -> bytes:
    """The generator's sums stream for a batch (generator.go:317,325-350 and the
    phase markers at :31,40): [int32 idx] SumHead records per file."""
    hs = [h if isinstance(h, SumHead) else SumHead(*h) for h in heads]
    ha = (SumHead * max(len(hs), 1))(*hs)
    r = _u8(records)
    ix = None
    if file_idx is not None:
        ix = np.ascontiguousarray(np.asarray(file_idx, dtype=np.int64).astype(np.int32))
    return _sized(lambda o, cap, n: lib.rsg_encode_sums(_ptr(ix) if ix is not None else None, ha, len(hs),
                                                        _ptr(r), int(terminate), o, cap, n))


def decode_sums(wire) -> Tuple[SumHead, np.ndarray, np.ndarray, int]:
    """SumHead.ReadFrom + receiveSums (types.go:38-77, sender.go:118-151)
    -> (head, sum1[count] u32, sum2[count,16] u8, bytes consumed)."""
    w = _u8(wire)
    h, used = SumHead(), ctypes.c_uint64()
    st = lib.rsg_decode_sums(_ptr(w), w.size, ctypes.byref(h), None, None, 0, ctypes.byref(used))
    if st != _lib.ERR_TRUNCATED:
        check(st)
    s1 = np.empty(max(h.count, 1), dtype=np.uint32)
    s2 = np.empty((max(h.count, 1), 16), dtype=np.uint8)
    check(lib.rsg_decode_sums(_ptr(w), w.size, ctypes.byref(h), _ptr(s1), _ptr(s2), h.count, ctypes.byref(used)))
    return h, s1[: h.count], s2[: h.count], used.value


def mux_frame(data, tag: int = MSG_DATA, max_message: int = _lib.CHUNK_SIZE) -> bytes:
    """MultiplexWriter.WriteMsg (wire.go:28-36) in <= max_message pieces."""
    d = _u8(data)
    return _sized(lambda o, cap, n: lib.rsg_mux_frame(_ptr(d), d.size, tag, max_message, o, cap, n))


def mux_deframe(wire) -> bytes:
    """MultiplexReader (wire.go:49-95): the MsgData payloads, MsgInfo skipped."""
    w = _u8(wire)
    return _sized(lambda o, cap, n: lib.rsg_mux_deframe(_ptr(w), w.size, o, cap, n))


def put_int64(v: int) -> bytes:
    """Conn.WriteInt64 (wire.go:108-117)."""
    out = np.empty(12, dtype=np.uint8)
    n = ctypes.c_uint64()
    check(lib.rsg_put_int64(v, _ptr(out), ctypes.byref(n)))
    return out[: n.value].tobytes()


def get_int64(b) -> Tuple[int, int]:
    """Conn.ReadInt64 (wire.go:177-195) -> (value, bytes consumed)."""
    a = _u8(b)
    v, n = ctypes.c_int64(), ctypes.c_uint64()
    check(lib.rsg_get_int64(_ptr(a), a.size, ctypes.byref(v), ctypes.byref(n)))
    return v.value, n.value


_default: Optional[Engine] = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine(0)
    return _default


def checksum1(buf) -> int:
    """rsyncchecksum.Checksum1 of one buffer, computed on the GPU (one block of len(buf))."""
    a = _u8(buf)
    if a.size == 0:
        return 0
    _, rec, _ = default_engine().block_sums([a], 0, a.size)
    return struct.unpack_from("<I", rec, 0)[0]


def checksum2(seed: int, buf) -> bytes:
    """rsyncchecksum.Checksum2 = MD4(buf || int32_LE(seed)), computed on the GPU."""
    a = _u8(buf)
    if a.size == 0:  # MD4(seed_LE): the whole-file kernel's seeded form of an empty file
        return default_engine().file_sums([a], _lib.FILESUM_SEEDED, seed)[0]
    _, rec, _ = default_engine().block_sums([a], seed, a.size)
    return rec[4:20]


def reader_checksum(buf) -> bytes:
    """rsyncchecksum.ReaderChecksum (rsyncchecksum.go:60-66): MD4 of the whole
    buffer, on the GPU."""
    return default_engine().file_sums([_u8(buf)], _lib.FILESUM_PLAIN)[0]
