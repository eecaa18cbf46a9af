"""Wire formats around the checksum path: the
generator's sums stream (generator.go:20-41,317-350, types.go:79-86), its
parser on the sender (types.go:38-77, sender.go:118-151), mux framing
(wire.go:28-95) and the int64 escape (wire.go:108-117,177-195).

The CPU tests compare librsg's host formatting with the oracle's pure-Python
restatements, feeding oracle-computed records (no kernel runs); the GPU test
formats records the block-sum kernel produced and checks the whole stream
byte for byte."""
import struct

import numpy as np
import pytest

from oracle import oracle as orc

SEED = 0x1BADB002


def _files(seed=7):
    rng = np.random.default_rng(seed)
    lens = [0, 1, 699, 700, 701, 1400, 5000, 70000]
    return [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]


def _oracle_records(files, block_lens, seed):
    heads, rec = [], b""
    for f, bl in zip(files, block_lens):
        heads.append(orc.sum_head(len(f), bl))
        rec += orc.block_sums(f, heads[-1][1], seed)
    return heads, rec


@pytest.mark.parametrize("block_len", [700, 0, 1024])
def test_encode_sums_matches_generator(block_len):
    import rsync_amd
    files = _files()
    bls = [block_len] * len(files)
    heads, rec = _oracle_records(files, bls, SEED)
    got = rsync_amd.encode_sums(heads, rec, file_idx=range(len(files)), terminate=True)
    assert got == orc.py_generate_files_stream(files, SEED, bls)


def test_encode_sums_short_s2len_and_no_index():
    import rsync_amd
    files = _files(3)
    heads, rec = _oracle_records(files, [700] * len(files), SEED)
    short = [(h[0], h[1], 2, h[3]) for h in heads]
    got = rsync_amd.encode_sums(short, rec)
    exp = orc.py_generate_files_stream(files, SEED, [700] * len(files), s2len=2)
    # same stream without the idx words and the phase markers
    out, at = bytearray(), 0
    for h in short:
        at += 4
        n = 16 + h[0] * 6
        out += exp[at:at + n]
        at += n
    assert got == bytes(out)


def test_encode_sums_rejects_bad_head():
    import rsync_amd
    with pytest.raises(rsync_amd.RsgError):
        rsync_amd.encode_sums([(1, 700, 17, 0)], bytes(20))
    with pytest.raises(rsync_amd.RsgError):
        rsync_amd.encode_sums([(1, 700, 16, 701)], bytes(20))


@pytest.mark.parametrize("s2len", [16, 8, 2, 0])
def test_decode_sums_matches_receive_sums(s2len):
    import rsync_amd
    f = _files(11)[-1]
    h = orc.sum_head(len(f), 700)
    rec = orc.block_sums(f, 700, SEED)
    wire = rsync_amd.encode_sums([(h[0], h[1], s2len, h[3])], rec) + b"tail"
    head, s1, s2, used = rsync_amd.decode_sums(wire)
    eh, esums, eused = orc.py_receive_sums(wire)
    assert head.astuple() == eh and used == eused == len(wire) - 4
    assert [int(x) for x in s1] == [s for s, _ in esums]
    assert [bytes(r) for r in s2] == [b for _, b in esums]
    # round trip back to the records' sum1 and sum2 prefix
    ref1, ref2 = orc.parse_records(rec)
    assert (s1 == ref1).all() and (s2[:, :s2len] == ref2[:, :s2len]).all()


@pytest.mark.parametrize("head,msg", [((-1, 700, 16, 0), "invalid checksum count"),
                                      ((1, (1 << 29) + 1, 16, 0), "invalid block length"),
                                      ((1, 700, 17, 0), "invalid checksum length"),
                                      ((1, 700, 16, 701), "invalid remainder length")])
def test_decode_sums_validation(head, msg):
    import rsync_amd
    wire = struct.pack("<4i", *head) + bytes(20)
    with pytest.raises(ValueError, match=msg):
        orc.py_receive_sums(wire)
    with pytest.raises(rsync_amd.RsgError, match=msg):
        rsync_amd.decode_sums(wire)


def test_decode_sums_short_stream():
    import rsync_amd
    wire = struct.pack("<4i", 3, 700, 16, 0) + bytes(40)
    with pytest.raises(rsync_amd.RsgError, match="EOF"):
        rsync_amd.decode_sums(wire)
    with pytest.raises(rsync_amd.RsgError, match="EOF"):
        rsync_amd.decode_sums(bytes(12))
    h, s1, s2, used = rsync_amd.decode_sums(struct.pack("<4i", 0, 0, 16, 0))
    assert h.count == 0 and used == 16 and s1.size == 0


@pytest.mark.parametrize("n,max_message", [(0, 1 << 18), (5, 1 << 18), ((1 << 18) * 3 + 17, 1 << 18),
                                           (100000, 4096)])
def test_mux_round_trip(n, max_message):
    import rsync_amd
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    framed = rsync_amd.mux_frame(data, 0, max_message)
    assert framed == orc.py_mux_write(data, 0, max_message)
    assert rsync_amd.mux_deframe(framed) == data == orc.py_mux_read(framed)


def test_mux_reader_tags_and_limits():
    import rsync_amd
    info = orc.py_mux_write(b"hello", tag=2)
    data = orc.py_mux_write(b"payload")
    assert rsync_amd.mux_deframe(info + data) == b"payload"
    with pytest.raises(rsync_amd.RsgError, match="boom"):
        rsync_amd.mux_deframe(data + orc.py_mux_write(b"boom", tag=1))
    with pytest.raises(rsync_amd.RsgError, match="unexpected tag"):
        rsync_amd.mux_deframe(orc.py_mux_write(b"x", tag=5))
    big = struct.pack("<I", (7 << 24) | ((1 << 18) + 1))
    with pytest.raises(rsync_amd.RsgError, match="exceeds max message size"):
        rsync_amd.mux_deframe(big + bytes((1 << 18) + 1))
    with pytest.raises(rsync_amd.RsgError, match="EOF"):
        rsync_amd.mux_deframe(data[:-1])
    with pytest.raises(rsync_amd.RsgError):
        rsync_amd.mux_frame(b"x", 0, (1 << 18) + 1)


@pytest.mark.parametrize("v", [0, 1, 0x7FFFFFFF, 0x80000000, -1, -(1 << 40), 1 << 62, 34359738368])
def test_int64_escape(v):
    import rsync_amd
    b = rsync_amd.put_int64(v)
    assert b == orc.py_write_int64(v)
    assert rsync_amd.get_int64(b + b"zz") == (v, len(b))


@pytest.mark.gpu
def test_gpu_records_to_wire_and_back():
    """GPU block sums -> generator stream -> mux framing -> demux -> receiveSums,
    byte-identical to the oracle's restatement of the whole path."""
    import rsync_amd
    files = _files(5)
    bls = [700] * len(files)
    with rsync_amd.Engine(0) as eng:
        heads, rec, _ = eng.block_sums(files, SEED, 700)
    stream = rsync_amd.encode_sums(heads, rec, file_idx=range(len(files)), terminate=True)
    assert stream == orc.py_generate_files_stream(files, SEED, bls)
    framed = rsync_amd.mux_frame(stream)
    assert rsync_amd.mux_deframe(framed) == stream
    at = 0
    for i, f in enumerate(files):
        assert struct.unpack_from("<i", stream, at)[0] == i
        head, s1, s2, used = rsync_amd.decode_sums(stream[at + 4:])
        r1, r2 = orc.parse_records(orc.block_sums(f, 700, SEED))
        assert (s1 == r1).all() and (s2 == r2).all()
        at += 4 + used
    assert stream[at:] == struct.pack("<ii", -1, -1)


@pytest.mark.gpu
@pytest.mark.parametrize("mux,s2len", [(False, 16), (True, 16), (True, 4)])
def test_gpu_generate_files(mux, s2len):
    """Engine.generate_files = the generator's whole output for a batch,
    byte-identical to the oracle's GenerateFiles restatement (after demux)."""
    import rsync_amd
    files = _files(9)
    conn = rsync_amd.Conn()
    with rsync_amd.Engine(0) as eng:
        eng.generate_files(conn, files, SEED, 700, s2len=s2len, mux=mux)
    got = bytes(conn.buf)
    if mux:
        hdr = struct.unpack_from("<I", got)[0]
        assert hdr >> 24 == 7 and (hdr & 0xFFFFFF) <= 1 << 18  # MsgData, <= 256 KiB
        got = rsync_amd.mux_deframe(got)
    assert got == orc.py_generate_files_stream(files, SEED, [700] * len(files), s2len=s2len)
