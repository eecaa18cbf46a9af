"""Used by tests/test_gpu_match.py::test_search_modes_vs_oracle on a context
whose search options (rsg_testing_search_option) were changed: the golden
match cases, seeded random searches and a multi-job batch through the C-ABI
against the C oracle.  Returns the number of searches checked; raises on the
first mismatch."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import cases  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def check_all(eng):
    gold = json.load(open(os.path.join(HERE, "golden", "match_cases.json")))
    n = 0
    for name, (src, basis, blen, seed) in sorted(cases.match_cases().items()):
        head = orc.sum_head(basis.size, blen)
        if head[0]:
            s1, s2 = orc.parse_records(orc.block_sums(basis, blen, seed))
        else:
            s1, s2 = np.zeros(0, np.uint32), np.zeros((0, 16), np.uint8)
        got = eng.hash_search(src, head, s1, s2, orc.stable_targets(s1), seed)
        assert [list(m) for m in got] == gold[name]["matches"], name
        n += 1
    for k in range(6):
        rng = np.random.default_rng(300 + k)
        size = int(rng.integers(1, 3_000_000))
        basis = cases.splitmix64_bytes(900 + k, size)
        src = cases.mutate(basis, 950 + k, float(rng.uniform(0, 0.6)), 1, 70000,
                           n_ins=int(rng.integers(0, 5)), n_del=int(rng.integers(0, 5)))
        blen = int(rng.choice([0, 700, 4096, 32768]))
        seed = int(rng.integers(-2**31, 2**31))
        head = orc.sum_head(basis.size, blen)
        s1, s2 = orc.parse_records(orc.block_sums(basis, blen, seed))
        tg = orc.stable_targets(s1)
        want, _, _ = orc.hash_search(src, head, s1, s2, tg, seed)
        assert eng.hash_search(src, head, s1, s2, tg, seed) == want, k
        n += 1
    # a multi-job batch: walks (tails) on worker threads beside the next
    # jobs' confirmations, with their extra round trips in this mode
    jobs, want = [], []
    for k in range(5):
        rng = np.random.default_rng(400 + k)
        size = int(rng.integers(200_000, 6_000_000)) if k != 4 else 40_000
        basis = cases.splitmix64_bytes(1900 + k, size)
        src = cases.mutate(basis, 1950 + k, 0.5, 1, 70000, n_ins=3, n_del=3)
        seed = 0x1BADB002
        head = orc.sum_head(basis.size, 0)
        s1, s2 = orc.parse_records(orc.block_sums(basis, head[1], seed))
        tg = orc.stable_targets(s1)
        jobs.append((src, None, head, s1, s2, tg))
        want.append(orc.hash_search(src, head, s1, s2, tg, seed)[0])
    assert eng.hash_search_batch(jobs, 0x1BADB002, device=False) == want
    n += len(jobs)
    return n
