"""GPU parity of the generator's host loop, rsg_generate_files_fd (SURVEY.md
§8f row 1): files read from descriptors, block sums on the GPU, the sums
stream of GenerateFiles (generator.go:20-41,317-350) handed to a writer.
The expected stream is built from the oracle's block sums
(orc_block_sums, generator.go:325-350) and SumHead bytes (types.go:79-86);
mux framing is undone with the oracle's MultiplexReader restatement."""
import os
import struct

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
SEED = 0x1BADB002


@pytest.fixture(scope="module")
def eng():
    import rsync_amd
    e = rsync_amd.Engine(0)
    yield e
    e.close()


def expected_stream(datas, block_lens, idx=None, terminate=True):
    out = bytearray()
    for k, (d, bl) in enumerate(zip(datas, block_lens)):
        h = orc.sum_head(len(d), bl)
        if idx is not None:
            out += struct.pack("<i", idx[k])
        out += orc.head_bytes(h)
        if h[0]:
            out += orc.block_sums(d, h[1], SEED)
    if terminate:
        out += struct.pack("<ii", -1, -1)
    return bytes(out)


def write_files(tmp_path, datas):
    fds = []
    for k, d in enumerate(datas):
        p = tmp_path / f"basis{k}"
        p.write_bytes(d)
        fds.append(os.open(p, os.O_RDONLY))
    return fds


def test_generate_files_fd_stream(eng, tmp_path):
    """Ragged lengths (empty files between others, a tail block, a file that
    spans batches), mixed explicit and SumSizesSqroot block lengths: the
    stream equals GenerateFiles' bytes exactly."""
    rng = np.random.default_rng(11)
    lens = [0, 1, 699, 700, 701, 5000, 0, 70000, 3 << 20, (65 << 20) + 123, 0]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    bls = [700, 0, 700, 700, 0, 1024, 700, 0, 700, 700, 0]
    fds = write_files(tmp_path, datas)
    try:
        chunks = []
        idx = [3 * k + 1 for k in range(len(datas))]
        heads, n = eng.generate_files_fd([(fd, len(d)) for fd, d in zip(fds, datas)], SEED, chunks.append,
                                         block_len=bls, idx=idx)
        got = b"".join(chunks)
        assert n == len(got)
        assert [h.astuple() for h in heads] == [orc.sum_head(len(d), b) for d, b in zip(datas, bls)]
        assert got == expected_stream(datas, bls, idx=idx)
        assert len(chunks) >= 2  # the 65 MiB file spans two batches
        # server side: <= 256 KiB MsgData messages, same bytes once demuxed
        chunks = []
        eng.generate_files_fd([(fd, len(d)) for fd, d in zip(fds, datas)], SEED, chunks.append, block_len=bls,
                              idx=idx, mux=True)
        assert orc.py_mux_read(b"".join(chunks)) == got
    finally:
        for fd in fds:
            os.close(fd)


def test_generate_files_fd_offsets_no_idx(eng, tmp_path):
    """Files at offsets of one descriptor, no idx words, no phase markers:
    generateAndSendSums' own output per file (generator.go:325-350)."""
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (1400, 333, 1 << 20, 4096)]
    blob = b"".join(datas)
    p = tmp_path / "blob"
    p.write_bytes(blob)
    fd = os.open(p, os.O_RDONLY)
    try:
        offs = np.cumsum([0] + [len(d) for d in datas])[:-1].tolist()
        chunks = []
        eng.generate_files_fd([(fd, len(d), o) for d, o in zip(datas, offs)], SEED, chunks.append, block_len=700,
                              terminate=False)
        assert b"".join(chunks) == expected_stream(datas, [700] * 4, terminate=False)
    finally:
        os.close(fd)


def test_generate_files_fd_errors(eng, tmp_path):
    import rsync_amd
    data = np.arange(5000, dtype=np.uint8).tobytes()
    fds = write_files(tmp_path, [data])
    try:
        # the file is shorter than the length the generator stat'ed: io.ReadFull fails
        with pytest.raises(rsync_amd.RsgError) as e:
            eng.generate_files_fd([(fds[0], 6000)], SEED, lambda b: None, block_len=700)
        assert e.value.status == rsync_amd._lib.ERR_IO and "unexpected EOF" in str(e.value)

        class Boom(Exception):
            pass

        def bad_writer(b):
            raise Boom()
        with pytest.raises(Boom):
            eng.generate_files_fd([(fds[0], 5000)], SEED, bad_writer, block_len=700)
        # the context still works afterwards
        chunks = []
        eng.generate_files_fd([(fds[0], 5000)], SEED, chunks.append, block_len=700, terminate=False)
        assert b"".join(chunks) == expected_stream([data], [700], terminate=False)
    finally:
        os.close(fds[0])


def test_generate_files_fd_writer_fails_mid_stream(eng, tmp_path):
    """A writer that fails on the second batch leaves nothing queued: the next
    call (with larger batches, so the staging buffers grow) is exact."""
    import rsync_amd
    rng = np.random.default_rng(21)
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in ((40 << 20) + 7, 3 << 20)]
    fds = write_files(tmp_path, datas)
    try:
        calls = []

        def flaky(b):
            calls.append(len(b))
            if len(calls) == 2:
                raise IOError("peer went away")
        with pytest.raises(IOError):
            eng.generate_files_fd([(fd, len(d)) for fd, d in zip(fds, datas)], SEED, flaky, block_len=700)
        os.environ["RSG_GEN_BATCH_MB"] = "128"
        try:
            chunks = []
            eng.generate_files_fd([(fd, len(d)) for fd, d in zip(fds, datas)], SEED, chunks.append, block_len=700)
        finally:
            del os.environ["RSG_GEN_BATCH_MB"]
        assert b"".join(chunks) == expected_stream(datas, [700, 700])
    finally:
        for fd in fds:
            os.close(fd)
