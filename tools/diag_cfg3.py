"""Diagnostic: the cfg3 sender workload step by step with progress prints
(single-file call, then the batched call), under a traceback watchdog."""
import faulthandler
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
faulthandler.dump_traceback_later(60, repeat=True)
import bench  # noqa: E402
import rsync_amd  # noqa: E402

nfiles = int(sys.argv[1]) if len(sys.argv) > 1 else 2
eng = rsync_amd.Engine(0)
size = 1 << 30
rng = np.random.default_rng(3)
basis = eng.alloc(size)
jobs = []
for f in range(nfiles):
    src = eng.alloc(size + 4096)
    n = bench.make_cfg3_file(eng, basis, src, size, f + 3, 32768, rng)
    recs, total = eng.block_sums_device(basis, [(0, size, 0)], bench.SEED)
    rec = recs.download(total * 20).reshape(-1, 20)
    recs.free()
    s1 = rec[:, :4].copy().view("<u4").reshape(-1)
    s2 = rec[:, 4:].copy()
    tags = ((s1 & 0xFFFF) + (s1 >> 16)) & 0xFFFF
    tg = np.argsort(tags, kind="stable").astype(np.int32)
    head = rsync_amd.sum_sizes_sqroot(size)
    jobs.append((src, n, head, s1, s2, tg))
eng.synchronize()
print("data ready", flush=True)
for i, (src, n, head, s1, s2, tg) in enumerate(jobs):
    t = time.perf_counter()
    m = eng.hash_search_device(src, n, head, s1, s2, tg, bench.SEED)
    print(f"single {i}: {len(m)} matches {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
for k in range(int(os.environ.get("DIAG_BATCHES", "3"))):
    t = time.perf_counter()
    res = eng.hash_search_batch(jobs, bench.SEED, as_arrays=True)
    print(f"batch {k}: {sum(len(r) for r in res)} matches {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
print("done", flush=True)
