"""CPU emulation of the data movement of the line-ring block-sum kernel
(rsync_amd/csrc/rsg_blocksums.hip, block_sums_lring<MODE, SHARE>).

The kernel moves each lane's block through aligned 128-byte lines: coalesced
loads of whole lines -> a 2-slot LDS ring -> per-lane realigned 32-word reads.
With SHARE, a lane copies its last line out of its right neighbour's slot
instead of loading it again.  This test replays exactly that index arithmetic
(line numbers, load masks, slot rotation, tail copies, realignment) in numpy for
one wave of 64 blocks and checks that the words each step hands to the hash
are the block's bytes, for layouts that stress the edge cases: blocks of any
4-aligned offset, one-line blocks, chains of tiny files sharing lines, blocks
ending at the arena's end.  It needs no GPU; the GPU parity tests check the
compiled kernel itself against the oracle."""
import numpy as np
import pytest

LINE = 128


def emulate_wave(arena: np.ndarray, arena_addr: int, offs, lens, share_on: bool):
    """Returns, per lane, the bytes the hash consumes (steps x 128 bytes)."""
    assert len(offs) == len(lens) == 64
    abs_ = [arena_addr + o for o in offs]
    base = min(abs_) & ~(LINE - 1)
    end_abs = arena_addr + arena.size
    rel = [a - base for a in abs_]
    d = [r & 127 for r in rel]
    n = list(lens)
    nl = [(d[j] + n[j] + 127) >> 7 for j in range(64)]
    l0 = [r >> 7 for r in rel]
    share0 = [share_on and j < 63 and l0[j + 1] == l0[j] + nl[j] - 1 for j in range(64)]
    next_self = [(not share0[(j + 1) % 64]) or nl[(j + 1) % 64] > 1 for j in range(64)]
    share = [share0[j] and next_self[j] for j in range(64)]
    nl_load = [nl[j] - (1 if share[j] else 0) for j in range(64)]
    steps = [((nn >> 6) + 2) >> 1 for nn in n]
    T = max(steps)

    def mem(addr, k):  # k bytes at absolute addr, zero past the arena (buffer range check)
        out = np.zeros(k, np.uint8)
        for i in range(k):
            a = addr + i
            if arena_addr <= a < end_abs:
                out[i] = arena[a - arena_addr]
            elif a >= end_abs:
                out[i] = 0
            else:  # bytes before the arena in the same line: real memory, value irrelevant
                out[i] = 0xEE
        return out

    def load_line(t):
        return [mem(base + (l0[j] + t) * LINE, LINE) if t < nl_load[j] else np.zeros(LINE, np.uint8)
                for j in range(64)]

    slots = [[np.full(LINE, 0xCD, np.uint8) for _ in range(64)] for _ in range(2)]
    tail = [None] * 64

    def store(t, slot, data):
        for j in range(64):
            slots[slot][j] = data[j].copy()

    def put_tail(t, slot):
        for j in range(64):
            if share[j] and t == nl[j] - 1:
                slots[slot][j] = tail[j].copy()

    consumed = [bytearray() for _ in range(64)]

    def step(sa):
        for j in range(64):
            split = (128 - d[j]) >> 2
            X = bytearray()
            for k in range(32):
                if k < split:
                    X += bytes(slots[sa][j][d[j] + 4 * k: d[j] + 4 * k + 4])
                else:
                    q = d[j] + 4 * k - 128
                    X += bytes(slots[sa ^ 1][j][q: q + 4])
            consumed[j] += X

    bufA, bufB = load_line(0), load_line(1)
    store(0, 0, bufA)
    for j in range(64):
        tail[j] = slots[0][(j + 1) % 64].copy()
    put_tail(0, 0)
    store(1, 1, bufB)
    put_tail(1, 1)
    bufA, bufB = load_line(2), load_line(3)
    i = 0
    while i < T:
        step(0)
        store(i + 2, 0, bufA)
        put_tail(i + 2, 0)
        bufA = load_line(i + 4)
        step(1)
        store(i + 3, 1, bufB)
        put_tail(i + 3, 1)
        bufB = load_line(i + 5)
        i += 2
    loaded_lines = sum(nl_load)
    return consumed, steps, loaded_lines


def check(arena, arena_addr, offs, lens, share_on):
    got, steps, loaded = emulate_wave(arena, arena_addr, offs, lens, share_on)
    for j in range(64):
        want = arena[offs[j]: offs[j] + lens[j]].tobytes()
        assert len(got[j]) >= steps[j] * 128 >= lens[j]
        assert bytes(got[j][:lens[j]]) == want, (j, offs[j], lens[j])
    return loaded


def contiguous_layout(rng, B, lead, nfiles=1):
    offs, lens = [], []
    o = lead
    while len(offs) < 64:
        flen = B * rng.integers(1, 9) + int(rng.integers(0, B))
        fo = o
        while fo < o + flen and len(offs) < 64:
            offs.append(fo)
            lens.append(min(B, o + flen - fo))
            fo += B
        o += flen
        o = (o + 3) & ~3  # files 4-byte aligned
    return offs, lens, o


@pytest.mark.parametrize("share_on", [False, True])
@pytest.mark.parametrize("B", [700, 64, 128, 1024, 1773 & ~3, 4])
@pytest.mark.parametrize("lead", [0, 4, 60, 124])
def test_lring_dataflow(share_on, B, lead):
    rng = np.random.default_rng(B * 131 + lead)
    offs, lens, end = contiguous_layout(rng, B, lead)
    arena = rng.integers(0, 256, end + int(rng.integers(0, 40)), dtype=np.uint8)
    check(arena, 1 << 20, offs, lens, share_on)


@pytest.mark.parametrize("share_on", [False, True])
def test_lring_tiny_file_chains(share_on):
    """One-line blocks in a row (64-, 1-, 5-, 0-byte files packed 16-byte
    aligned, the host path's layout): the neighbour-line copies must not
    chain through a block that never loads its own line."""
    rng = np.random.default_rng(7)
    sizes = [64, 1, 5, 12, 3, 700, 700, 40, 8, 1] * 7
    offs, lens, o = [], [], 0
    for sz in sizes:
        if len(offs) == 64:
            break
        offs.append(o)
        lens.append(sz)
        o += (sz + 15) & ~15
    arena = rng.integers(0, 256, o, dtype=np.uint8)
    check(arena, 1 << 20, offs, lens, share_on)


def test_lring_arena_end_and_unaligned_base():
    """Last block ends exactly at the arena end; arena base not line aligned."""
    rng = np.random.default_rng(3)
    offs = [j * 700 for j in range(64)]
    lens = [700] * 64
    arena = rng.integers(0, 256, 64 * 700, dtype=np.uint8)
    for addr in (1 << 20, (1 << 20) + 16, (1 << 20) + 100):
        check(arena, addr, offs, lens, True)


def test_lring_share_saves_lines():
    """For contiguous 700-byte blocks every line is loaded once with SHARE
    (lane 63's last line aside), ~1 line per block more without."""
    rng = np.random.default_rng(5)
    offs = [j * 700 for j in range(64)]
    lens = [700] * 64
    arena = rng.integers(0, 256, 64 * 700, dtype=np.uint8)
    with_share = check(arena, 1 << 20, offs, lens, True)
    without = check(arena, 1 << 20, offs, lens, False)
    lines_touched = (64 * 700 + 127) // 128
    assert with_share <= lines_touched + 1
    assert without >= lines_touched + 50
