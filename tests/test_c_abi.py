"""C-language conformance of include/rsg.h (tests/c/abi_conformance.c).

The reference has no FFI of its own (release builds are CGO_ENABLED=0,
Makefile:4); its cgo binding (go/rsyncgpu) sees rsg.h's
structs with the C compiler's layout.  The C program pins that layout at
compile time; here it is compared with the ctypes mirror the Python tests go
through, so a header/binding mismatch in rsg_search_job or rsg_fd_file
cannot hide behind ctypes.  The GPU case runs one block-sum -> encode ->
decode round trip from C (entry points replacing rsyncchecksum.go:29,53 via
generator.go:325-350, and sender.go:118-151).
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

import cases
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c")
BIN = os.path.join(CDIR, "abi_conformance")


def _binary():
    """The program built by __graft_entry__.build(); rebuilt here when gcc is
    available and the binary is missing or stale (CPU box only)."""
    srcs = [os.path.join(CDIR, "abi_conformance.c"), os.path.join(CDIR, "..", "..", "include", "rsg.h")]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", CDIR], check=True)
    return BIN


def _ctypes_layout(cls):
    return {"size": ctypes.sizeof(cls),
            **{name: [getattr(cls, name).offset, getattr(cls, name).size] for name, _ in cls._fields_}}


def test_layout_matches_ctypes_mirror():
    from rsync_amd import _lib
    out = subprocess.run([_binary(), "layout"], check=True, capture_output=True, text=True).stdout
    c = json.loads(out)
    assert c["abi_version"] == _lib.ABI_VERSION == int(_lib.lib.rsg_abi_version())
    assert c["record_bytes"] == _lib.RECORD_BYTES
    assert c["chunk_size"] == _lib.CHUNK_SIZE
    for name, cls in (("rsg_sum_head", _lib.SumHead), ("rsg_file", _lib.File), ("rsg_match", _lib.Match),
                      ("rsg_search_job", _lib.SearchJob), ("rsg_fd_search_job", _lib.FdSearchJob),
                      ("rsg_fd_file", _lib.FdFile),
                      ("rsg_shard_batch", _lib.ShardBatch), ("rsg_recv_job", _lib.RecvJob),
                      ("rsg_piece", _lib.Piece), ("rsg_shard_rank", _lib.ShardRank)):
        assert c[name] == _ctypes_layout(cls), name


def test_no_device_contract_from_c():
    """Without a gfx950 device (this container) rsg_ctx_create returns
    RSG_ERR_NODEV with a message and never aborts; host-only arithmetic
    (SumSizesSqroot, rsynccommon.go:14-37) still works."""
    import rsync_amd
    if rsync_amd.device_count() > 0:
        pytest.skip("a gfx950 device is visible")
    r = subprocess.run([_binary(), "nodev"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout)
    assert res["status"] == -4 and res["ctx_null"] == 1 and res["message"]


@pytest.mark.gpu
def test_round_trip_from_c(tmp_path):
    """Block sums of a 1 MiB (B=700), a 1000-byte (SumSizesSqroot) and an
    empty file from C, the generator stream encoded and file 0 decoded back;
    the records equal the oracle's."""
    out = tmp_path / "records.bin"
    r = subprocess.run([BIN, "gpu", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout)
    assert res["round_trip_ok"] == 1
    files = [cases.splitmix64_bytes(1, 1 << 20), cases.splitmix64_bytes(2, 1000), np.zeros(0, np.uint8)]
    want = b"".join(orc.block_sums(f, b, 0x1BADB002) for f, b in zip(files, (700, 0, 700)))
    assert out.read_bytes() == want
