"""CPU-side checks of the C-ABI library: it loads, exports every symbol
include/*.h declare, and its host-only arithmetic (sizing, token encoding)
matches the oracle.  No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

import cases
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    syms = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            txt = open(os.path.join(ROOT, "include", h)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            syms |= set(re.findall(r"\b(rsg_[a-z0-9_]+)\s*\(", txt))
    return sorted(syms)


def test_library_exports_every_header_symbol():
    from rsync_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert set(syms) == set(_lib.EXPORTED)
    assert _lib.lib.rsg_abi_version() == _lib.ABI_VERSION == 5


def test_no_device_fails_loudly():
    import rsync_amd
    if rsync_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(rsync_amd.RsgError) as e:
        rsync_amd.Engine(0)
    assert e.value.status == -4


def test_product_does_not_import_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "rsync_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.replace("oracle_", ""), f
    from rsync_amd import _lib
    out = os.popen(f"ldd {_lib.LIB_PATH}").read()
    assert "liboracle" not in out


@pytest.mark.parametrize("n,bl", [(0, 0), (1, 0), (490000, 0), (490001, 0), (1 << 20, 0), (1 << 30, 0),
                                  (32 << 30, 0), (5, 700), (1 << 20, 700), (12345, 1773), (7, 1)])
def test_sum_sizes(n, bl):
    import rsync_amd
    assert rsync_amd.sum_sizes_sqroot(n, bl).astuple() == orc.sum_head(n, bl)


def test_sum_sizes_rejects_bad():
    import rsync_amd
    with pytest.raises(rsync_amd.RsgError):
        rsync_amd.sum_sizes_sqroot(-1)
    with pytest.raises(rsync_amd.RsgError):
        rsync_amd.sum_sizes_sqroot(10, (1 << 29) + 1)


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
def test_encode_tokens_matches_oracle(name):
    """rsg_encode_tokens (host formatting) == the oracle's token stream given the
    oracle's match list (match.go:233-282, token.go:4-31)."""
    import rsync_amd
    src, basis, blen, seed = cases.match_cases()[name]
    head = orc.sum_head(basis.size, blen)
    rec = orc.block_sums(basis, blen, seed)
    s1, s2 = orc.parse_records(rec) if head[0] else (np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8))
    matches, tokens, _ = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    assert rsync_amd.encode_tokens(src, head, matches) == tokens


def test_plan_block_sums_layout():
    from rsync_amd import _lib
    lens = cases.ragged_lengths()
    arr = (_lib.File * len(lens))()
    for i, n in enumerate(lens):
        arr[i].len, arr[i].block_len = n, 700
    heads = (_lib.SumHead * len(lens))()
    first = (ctypes.c_uint64 * len(lens))()
    total = ctypes.c_uint64()
    _lib.check(_lib.lib.rsg_plan_block_sums(arr, len(lens), heads, first, ctypes.byref(total)))
    acc = 0
    for i, n in enumerate(lens):
        assert heads[i].astuple() == orc.sum_head(n, 700)
        assert first[i] == acc
        acc += heads[i].count
    assert total.value == acc


def _token_stream(name):
    src, basis, blen, seed = cases.match_cases()[name]
    head = orc.sum_head(basis.size, blen)
    rec = orc.block_sums(basis, blen, seed)
    s1, s2 = orc.parse_records(rec) if head[0] else (np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8))
    _, tokens, fsum = orc.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
    return src, basis, head, seed, tokens, fsum


@pytest.mark.parametrize("name", sorted(cases.match_cases()))
def test_apply_tokens_matches_oracle(name):
    """rsg_apply_tokens (host byte copying of receiveData's token loop,
    receiver.go:122-163) rebuilds what the oracle's receive_data rebuilds."""
    import rsync_amd
    src, basis, head, seed, tokens, fsum = _token_stream(name)
    want, used = orc.receive_data(tokens + fsum, head, basis, seed)
    got, sum_at = rsync_amd.apply_tokens(tokens + fsum, head, basis)
    assert got == want == src.tobytes()
    assert sum_at == len(tokens) and used == sum_at + 16


def test_apply_tokens_errors():
    import rsync_amd
    src, basis, head, seed, tokens, fsum = _token_stream("shifted_700")
    for stream, b in [(tokens[:-4], basis), (tokens[:10], basis), (tokens, basis[:1000]), (tokens, None)]:
        with pytest.raises(rsync_amd.RsgError) as e:
            rsync_amd.apply_tokens(stream, head, b)
        assert e.value.status == -1
    # literal-only stream needs no basis
    lit = rsync_amd.encode_tokens(src, head, [])
    got, _ = rsync_amd.apply_tokens(lit, head, None)
    assert got == src.tobytes()


def test_block_sums_rule_boundaries():
    """The block-sum kernel choice (rsg_set_block_sums_kernel's automatic
    rule, rsg.h), pinned at every boundary on the host: unaligned blocks, or
    blocks of >= 704 bytes off the 128-byte lines -> line windows (7); aligned
    512..703 -> park (2); on the lines up to 32 KiB -> 4; else 1.  Forced
    variants the batch cannot take fall back (arena_align: 0 / 1 / 2 = the
    arena base not 4-byte / 4-byte / 128-byte aligned)."""
    from rsync_amd import _lib
    ch = _lib.lib.rsg_testing_block_sums_choice
    for B in (64, 700, 4096, 8191, 8192, 131072):
        assert ch(-1, 0, 0, 2, B) == 7
        assert ch(-1, 0, 0, 1, B) == 6                          # line windows need a 128-byte aligned arena
        assert ch(-1, 0, 0, 0, B) == (3 if B >= 8192 else 0)
    want = {64: 1, 511: 1, 512: 2, 703: 2, 704: 7, 1024: 7, 1448: 7, 4096: 7, 24577: 7, 32768: 7, 131072: 7}
    for B, v in want.items():
        assert ch(-1, 1, 0, 2, B) == v, B                       # aligned, off the lines
        assert ch(-1, 1, 0, 1, B) == (1 if v == 7 else v), B     # ... in an arena off the lines
    for B, v in {511: 1, 512: 2, 703: 2, 704: 4, 2176: 4, 16384: 4, 32768: 4, 32769: 1}.items():
        assert ch(-1, 1, 1, 2, B) == v, B
    assert ch(2, 1, 0, 2, 704) == 1          # park holds blocks <= 703 bytes
    for v in (1, 2, 4):
        assert ch(v, 0, 0, 2, 700) == 0      # LDS-DMA kernels need 4-byte aligned blocks
    assert ch(6, 0, 0, 0, 32768) == 3 and ch(6, 0, 0, 0, 700) == 0
    assert ch(7, 0, 0, 0, 32768) == 3 and ch(7, 0, 0, 0, 700) == 0
    assert ch(7, 0, 0, 1, 700) == 6 and ch(7, 1, 0, 1, 700) == 1
    for v in (0, 1, 3, 4, 6, 7):
        assert ch(v, 1, 1, 2, 4096) == v
    for bad in (5, 8, 9, 10, 11, 12, 13, 14, 15, 16, -2):
        assert ch(bad, 1, 0, 2, 700) == -2
