"""ctypes front end of the CPU parity oracle (oracle/rsg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package ``rsync_amd``.

Also holds ``py_hash_search``: an independent pure-Python transcription of the
reference's sender search (internal/sender/match.go:21-282, token.go:4-31),
used on small inputs to cross-check the C restatement.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
CHUNK_SIZE = 256 * 1024  # internal/sender/flist.go:52

_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_fill_splitmix64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_checksum1.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.orc_checksum1.restype = ctypes.c_uint32
        L.orc_tag.argtypes = [ctypes.c_uint32]
        L.orc_tag.restype = ctypes.c_uint16
        L.orc_md4.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_checksum2.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_file_sum.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p]
        L.orc_sum_sizes_sqroot.argtypes = [ctypes.c_int64, ctypes.c_void_p]
        L.orc_block_sums.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_void_p]
        L.orc_block_sums.restype = ctypes.c_int64
        L.orc_hash_search.argtypes = [
            ctypes.c_void_p, ctypes.c_int64,
            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int32,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
            ctypes.c_void_p,
        ]
        L.orc_hash_search.restype = ctypes.c_int64
        L.orc_receive_data.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.orc_receive_data.restype = ctypes.c_int64
        del u8p
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf.view(np.uint8).reshape(-1))
    return np.frombuffer(bytes(buf), dtype=np.uint8)


# ---------------------------------------------------------------------------
def splitmix64_bytes(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().orc_fill_splitmix64(seed & (2**64 - 1), _ptr(out), n)
    return out


def checksum1(buf) -> int:
    """rsyncchecksum.Checksum1 (rsyncchecksum.go:29-51)."""
    a = _as_u8(buf)
    return int(lib().orc_checksum1(_ptr(a), a.size))


def tag(sum1: int) -> int:
    """rsyncchecksum.Tag (rsyncchecksum.go:15-17)."""
    return int(lib().orc_tag(sum1 & 0xFFFFFFFF))


def md4(buf) -> bytes:
    a = _as_u8(buf)
    out = np.zeros(16, dtype=np.uint8)
    lib().orc_md4(_ptr(a), a.size, _ptr(out))
    return out.tobytes()


def checksum2(seed: int, buf) -> bytes:
    """rsyncchecksum.Checksum2 = MD4(buf || int32_LE(seed)) (rsyncchecksum.go:53-58)."""
    a = _as_u8(buf)
    out = np.zeros(16, dtype=np.uint8)
    lib().orc_checksum2(ctypes.c_int32(_i32(seed)), _ptr(a), a.size, _ptr(out))
    return out.tobytes()


def file_sum(mode: int, seed: int, buf) -> bytes:
    """Whole-file MD4: mode 0 = MD4(file) (rsyncchecksum.go:60-66), mode 1 =
    MD4(int32_LE(seed) || file) (match.go:52-53, receiver.go:117-120)."""
    a = _as_u8(buf)
    out = np.zeros(16, dtype=np.uint8)
    lib().orc_file_sum(ctypes.c_int32(mode), ctypes.c_int32(_i32(seed)), _ptr(a), a.size, _ptr(out))
    return out.tobytes()


def sum_sizes_sqroot(n: int):
    """rsynccommon.SumSizesSqroot (rsynccommon.go:14-37) -> (count, blen, s2len, rem)."""
    out = np.zeros(4, dtype=np.int32)
    lib().orc_sum_sizes_sqroot(n, _ptr(out))
    return tuple(int(x) for x in out)


def sum_head(n: int, block_len: int = 0):
    if block_len <= 0:
        return sum_sizes_sqroot(n)
    return ((n + block_len - 1) // block_len, block_len, 16, n % block_len)


def block_sums(data, block_len: int, seed: int) -> bytes:
    """generateAndSendSums (generator.go:325-350): count x 20-byte records."""
    a = _as_u8(data)
    count = sum_head(a.size, block_len)[0]
    out = np.zeros(max(count, 1) * 20, dtype=np.uint8)
    got = lib().orc_block_sums(_ptr(a), a.size, block_len, _i32(seed), _ptr(out))
    assert got == count
    return out[: count * 20].tobytes()


def head_bytes(head) -> bytes:
    """SumHead.WriteTo (types.go:79-86): 4 x int32 LE."""
    return struct.pack("<4i", *head)


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def parse_records(rec: bytes):
    """-> (sum1 u32 array, sum2 (count,16) u8 array)."""
    a = np.frombuffer(rec, dtype=np.uint8).reshape(-1, 20)
    sum1 = a[:, :4].copy().view("<u4").reshape(-1)
    sum2 = a[:, 4:].copy()
    return sum1, sum2


def stable_targets(sum1: np.ndarray) -> np.ndarray:
    """targets order of sender.go:60-75 with a STABLE tie-break (Go's sort.Slice
    is unstable; only duplicate-tag order differs)."""
    s = sum1.astype(np.uint32)
    tags = ((s & 0xFFFF) + (s >> 16)) & 0xFFFF
    return np.argsort(tags, kind="stable").astype(np.int32)


def hash_search(src, head, sum1, sum2, targets, seed: int):
    """C restatement of hashSearch.  -> (matches [(offset, idx)], token_bytes, file_sum)."""
    a = _as_u8(src)
    count, blen, s2len, rem = head
    sum1 = np.ascontiguousarray(sum1, dtype=np.uint32)
    sum2 = np.ascontiguousarray(sum2, dtype=np.uint8).reshape(-1)
    targets = np.ascontiguousarray(targets, dtype=np.int32)
    mcap = a.size // max(blen, 1) + 2
    moff = np.zeros(mcap, dtype=np.int64)
    midx = np.zeros(mcap, dtype=np.int32)
    tcap = a.size + 16 * (a.size // CHUNK_SIZE + 2) + 4 * mcap + 16
    tok = np.zeros(tcap, dtype=np.uint8)
    tlen = ctypes.c_int64(0)
    fsum = np.zeros(16, dtype=np.uint8)
    L = lib()
    nm = L.orc_hash_search(_ptr(a), a.size, count, blen, s2len, rem,
                           _ptr(sum1), _ptr(sum2), _ptr(targets), _i32(seed),
                           _ptr(moff), _ptr(midx), mcap,
                           _ptr(tok), tcap, ctypes.byref(tlen), _ptr(fsum))
    if nm < 0:
        raise ValueError("invalid sum head")
    assert nm <= mcap and tlen.value <= tcap
    matches = [(int(moff[i]), int(midx[i])) for i in range(nm)]
    return matches, tok[: tlen.value].tobytes(), fsum.tobytes()


# ---------------------------------------------------------------------------
# Independent pure-Python transcription of match.go (small inputs only).
def _sx(b: int) -> int:
    return b - 256 if b >= 128 else b


def py_checksum1(buf: bytes) -> int:
    s1 = s2 = 0
    for b in buf:
        s1 = (s1 + _sx(b)) & 0xFFFFFFFF
        s2 = (s2 + s1) & 0xFFFFFFFF
    return ((s1 & 0xFFFF) + (s2 << 16)) & 0xFFFFFFFF


def py_hash_search(src: bytes, head, sum1, sum2, targets, seed: int, c2=None):
    """Literal transcription of hashSearch/matched/simpleSendToken with Python
    ints; the whole-file sum is left out (the C oracle covers it).
    -> (matches, token_bytes)."""
    count, blen, s2len, rem = head
    size = len(src)
    lens = [rem if (i == count - 1 and rem != 0) else blen for i in range(count)]
    out = bytearray()
    matches = []
    state = {"last": 0}

    def send_token(token, offset, n):
        l = 0
        while l < n:
            n1 = min(CHUNK_SIZE, n - l)
            out.extend(struct.pack("<i", n1))
            out.extend(src[offset + l: offset + l + n1])
            l += n1
        if token != -2:
            out.extend(struct.pack("<i", -(token + 1)))

    def matched(offset, i):
        n = offset - state["last"]
        send_token(i, state["last"], n)
        if i >= 0:
            matches.append((offset, i))
            state["last"] = offset + lens[i]
        else:
            state["last"] = offset

    if count > 0 and size > 0:
        tags = [((int(sum1[t]) & 0xFFFF) + (int(sum1[t]) >> 16)) & 0xFFFF for t in targets]
        table = {}
        for idx in range(count - 1, -1, -1):
            table[tags[idx]] = idx
        end = size + 1 - lens[count - 1]
        offset = 0
        k = min(blen, size - offset)
        s = py_checksum1(src[offset: offset + k])
        s1, s2 = s & 0xFFFF, s >> 16
        while True:
            tg = (s1 + s2) & 0xFFFF
            brk = False
            if tg in table:
                j = table[tg]
                sm = (s1 & 0xFFFF) | (s2 << 16)
                local2 = None
                while j < count and tags[j] == tg:
                    i = int(targets[j])
                    j += 1
                    if sm != int(sum1[i]):
                        continue
                    l = min(blen, size - offset)
                    if l != lens[i]:
                        continue
                    if local2 is None:
                        local2 = (c2 or checksum2)(seed, src[offset: offset + l])
                    if local2[:s2len] != bytes(sum2[i][:s2len]):
                        continue
                    matched(offset, i)
                    offset += lens[i] - 1
                    k = min(blen, size - offset)
                    s = py_checksum1(src[offset: offset + k])
                    s1, s2 = s & 0xFFFF, s >> 16
                    if offset >= end:
                        brk = True
                    break
            if brk:
                break
            backup = max(offset - state["last"], 0)
            more = offset + k < size
            x0 = _sx(src[offset])
            s1 = (s1 - x0) & 0xFFFFFFFF
            s2 = (s2 - k * x0) & 0xFFFFFFFF
            if more:
                s1 = (s1 + _sx(src[offset + k])) & 0xFFFFFFFF
                s2 = (s2 + s1) & 0xFFFFFFFF
            else:
                k -= 1
            s1 &= 0xFFFF
            s2 &= 0xFFFF
            if backup >= blen + CHUNK_SIZE and end - offset > CHUNK_SIZE:
                matched(offset - blen, -2)
            offset += 1
            if offset >= end:
                break
    matched(size, -1)
    return matches, bytes(out)


def receive_data(stream: bytes, head, basis, seed: int):
    """receiveData (receiver.go:98-188): rebuild the file from `stream` (tokens,
    int32 0, 16-byte whole-file sum) and the basis; checks the seeded whole-file
    MD4.  -> (rebuilt bytes, bytes consumed).  Raises ValueError with the
    oracle's code (-1 short stream, -2 basis read out of range, -3 corruption)."""
    t = _as_u8(stream)
    b = _as_u8(basis) if basis is not None else None
    count, blen, _, rem = head
    used = ctypes.c_int64(0)
    L = lib()
    bp = _ptr(b) if b is not None else None
    blen_b = b.size if b is not None else 0
    n = L.orc_receive_data(_ptr(t), t.size, count, blen, rem, bp, blen_b, _i32(seed), None, 0, ctypes.byref(used))
    if n < 0:
        raise ValueError(int(n))
    out = np.zeros(max(n, 1), dtype=np.uint8)
    L.orc_receive_data(_ptr(t), t.size, count, blen, rem, bp, blen_b, _i32(seed), _ptr(out), n, ctypes.byref(used))
    return out[:n].tobytes(), int(used.value)


# ---------------------------------------------------------------- wire formats
# Pure-Python restatements of the Go wire code around the checksum path
# (SURVEY.md §8f row 4); small inputs only.

def py_generate_files_stream(files, seed: int, block_lens, s2len: int = 16) -> bytes:
    """GenerateFiles' bytes for files that all go through generateAndSendSums
    (generator.go:20-41,317-321,325-350): per file int32 idx, SumHead, per block
    int32 sum1 + Checksum2[:s2len]; then int32 -1 twice (phase markers)."""
    out = bytearray()
    for idx, (data, bl) in enumerate(zip(files, block_lens)):
        h = sum_head(len(data), bl)
        h = (h[0], h[1], s2len, h[3])
        out += struct.pack("<i", idx) + head_bytes(h)
        for i in range(h[0]):
            blk = bytes(data[i * h[1]:(i + 1) * h[1]])
            out += struct.pack("<I", checksum1(blk)) + checksum2(seed, blk)[:s2len]
    out += struct.pack("<ii", -1, -1)
    return bytes(out)


def py_receive_sums(wire: bytes):
    """SumHead.ReadFrom + receiveSums (types.go:38-77, sender.go:118-151)
    -> (head tuple, [(sum1, sum2 bytes padded to 16)], consumed); raises
    ValueError with the reference's message on an invalid head."""
    if len(wire) < 16:
        raise ValueError("unexpected EOF")
    count, blen, s2len, rem = struct.unpack_from("<4i", wire)
    if count < 0:
        raise ValueError(f"invalid checksum count {count}")
    if blen < 0 or blen > 1 << 29:
        raise ValueError(f"invalid block length {blen}")
    if s2len < 0 or s2len > 16:
        raise ValueError(f"invalid checksum length {s2len}")
    if rem < 0 or rem > blen:
        raise ValueError(f"invalid remainder length {rem}")
    pos, sums = 16, []
    for _ in range(count):
        if pos + 4 + s2len > len(wire):
            raise ValueError("unexpected EOF")
        s1 = struct.unpack_from("<I", wire, pos)[0]
        sums.append((s1, wire[pos + 4:pos + 4 + s2len] + bytes(16 - s2len)))
        pos += 4 + s2len
    return (count, blen, s2len, rem), sums, pos


def py_mux_write(data: bytes, tag: int = 0, max_message: int = CHUNK_SIZE) -> bytes:
    """MultiplexWriter.WriteMsg (wire.go:28-36), one message per <= max_message piece."""
    out = bytearray()
    for at in range(0, len(data), max_message):
        p = data[at:at + max_message]
        out += struct.pack("<I", ((7 + tag) << 24) | len(p)) + p
    return bytes(out)


def py_mux_read(wire: bytes) -> bytes:
    """MultiplexReader.ReadMsg/Read (wire.go:49-95) over a whole stream."""
    out, at = bytearray(), 0
    while at < len(wire):
        (hdr,) = struct.unpack_from("<I", wire, at)
        tag, n = ((hdr >> 24) - 7) & 0xFF, hdr & 0xFFFFFF
        if n > CHUNK_SIZE:
            raise ValueError(f"length {n} exceeds max message size ({CHUNK_SIZE})")
        p = wire[at + 4:at + 4 + n]
        if len(p) != n:
            raise ValueError("unexpected EOF")
        at += 4 + n
        if tag == 0:
            out += p
        elif tag == 1:
            raise ValueError(p.decode(errors="replace"))
        elif tag != 2:
            raise ValueError(f"unexpected tag: got {tag}, want 0")
    return bytes(out)


def py_write_int64(v: int) -> bytes:
    """Buffer.WriteInt64 / Conn.WriteInt64 (wire.go:108-117)."""
    return struct.pack("<i", v) if 0 <= v <= 0x7FFFFFFF else struct.pack("<iq", -1, v)
