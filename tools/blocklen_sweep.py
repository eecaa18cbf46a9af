#!/usr/bin/env python3
"""Kernel-variant timing for other block-sum shapes than bench.py's cfg2.

    python tools/blocklen_sweep.py

For each shape (files x file bytes, block length) and each variant, the
block-sum launch is timed with HIP events over rotating input arenas (inputs
resident in HBM).  Prints one JSON line per shape.  Diagnostic only: bench.py
is the metric.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 0x1BADB002
SHAPES_UNALIGNED = [  # files at odd offsets (every block unaligned): direct / long / unaligned staged
    (1024, 1 << 20, 700, 2),
    (1024, 1 << 20, 1024, 2),
    (256, 4 << 20, 4096, 2),
]
VARIANTS_UNALIGNED = {0: "direct", 3: "long_deep_prefetch", 6: "staged_unaligned", 7: "lines"}
SHAPES = [  # (files, file bytes, block length, arenas)
    (1, 1 << 30, 131072, 2),      # one 1 GiB file, cfg5's block length
    (1024, 1 << 20, 1024, 2),     # 1 MiB files at the reference's own sizing (B = 1024)
    (256, 4 << 20, 4096, 2),      # 4 KiB blocks
    (1, 32 << 30, 131072, 1),     # cfg5's per-GPU share: one 32 GiB file
    (512, 2 << 20, 2048, 2),      # 2 MiB files (B = 2048)
    (256, 4 << 20, 4160, 2),      # 5-7: B = 4096 +- 64 (is the 4 KiB stride itself the cost?)
    (256, 4 << 20, 4032, 2),
    (256, 4 << 20, 4112, 2),
    (1, 1 << 30, 32768, 2),       # 8: one 1 GiB file at the reference's sizing (B = sqrt(len) = 32768)
]
VARIANTS = {-1: "automatic", 1: "staged", 4: "staged_seg128", 2: "park",
            3: "long_deep_prefetch", 7: "lines", 6: "staged_unaligned"}
# SWEEP_SQRT=1 (or a list of MiB, "2,3"): the reference's own block length B = int(sqrt(len)) (rsynccommon.go:22) for files of
# len = 1, 2, 3, 5, 9, 17, 33, 64 MiB, ~1 GiB of them per shape, at the library's 128-byte packing
SQRT_LENS_MIB = [1, 2, 3, 5, 9, 17, 33, 64]


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--unaligned":
        return unaligned()
    import torch
    import rsync_amd
    from rsync_amd import _lib
    eng = rsync_amd.Engine(0)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    # SWEEP_SHAPES="1,2": only those entries of SHAPES; SWEEP_ROUNDS: interleaved rounds
    pick = os.environ.get("SWEEP_SHAPES")
    shapes = [SHAPES[int(k)] for k in pick.split(",")] if pick else SHAPES
    # SWEEP_BLENS="1000,4000": 256 x 4 MiB files at each of those block lengths instead
    if os.environ.get("SWEEP_BLENS"):
        shapes = [(256, 4 << 20, int(b), 2) for b in os.environ["SWEEP_BLENS"].split(",")]
    if os.environ.get("SWEEP_SQRT"):
        import math
        mibs = SQRT_LENS_MIB if os.environ["SWEEP_SQRT"] == "1" else [int(x) for x in os.environ["SWEEP_SQRT"].split(",")]
        shapes = [(max(1, (1 << 30) // (m << 20)), m << 20, int(math.isqrt(m << 20)), 2) for m in mibs]
    rounds = int(os.environ.get("SWEEP_ROUNDS", "1"))
    only = os.environ.get("SWEEP_ONLY")  # comma-separated variant names
    for nf, fb, blen, narena in shapes:
        total = nf * fb
        arenas = [eng.alloc(total) for _ in range(narena)]
        for k, a in enumerate(arenas):
            for f in range(nf):
                eng.fill_splitmix64(a, fb, 1 + f + 7919 * k, offset=f * fb, stream=sp)
        plan = eng.plan([(f * fb, fb, blen) for f in range(nf)], total)
        recs = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
        eng.synchronize(sp)
        res = {}
        runs = [(v, name) for v, name in VARIANTS.items()]
        if only:
            runs = [r for r in runs if r[1] in only.split(",")]
        # the memory clock ramps up over the first ~15 ms of launches: warm up
        # before the first variant so it is not timed on a cold card
        eng.set_block_sums_kernel(-1)
        import time
        w0 = time.perf_counter()
        while time.perf_counter() - w0 < 0.3:
            plan.run(arenas[0], SEED, recs, stream=sp)
            eng.synchronize(sp)
        for v, name in [r for _ in range(rounds) for r in runs]:
            eng.set_block_sums_kernel(v)
            steps = 5 if total > (4 << 30) else 30
            print(f"shape {nf}x{fb} B={blen}: {name}", file=sys.stderr, flush=True)
            for i in range(10):
                plan.run(arenas[i % narena], SEED, recs, stream=sp)
            eng.synchronize(sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(steps):
                plan.run(arenas[i % narena], SEED, recs, stream=sp)
            e1.record(stream)
            eng.synchronize(sp)
            ms = e0.elapsed_time(e1) / steps
            r = {"kernel_ms": round(ms, 4), "gib_s": round(total / 2**30 / (ms / 1e3), 1),
                 "hbm_frac_8tbs": round((total + plan.total_records * 20) / (ms / 1e3) / 8e12, 4)}
            if name in res:  # interleaved rounds: keep every round's time
                prev = res[name]
                r["rounds_ms"] = prev.get("rounds_ms", [prev["kernel_ms"]]) + [r["kernel_ms"]]
            res[name] = r
        eng.set_block_sums_kernel(-1)
        print(json.dumps({"files": nf, "file_bytes": fb, "block_len": blen, "records": plan.total_records,
                          "variants": res}), flush=True)
        plan.close()
        for a in arenas:
            a.free()
        recs.free()


def unaligned():
    """Files placed at offsets f * (file bytes + 1): no block is 4-byte aligned
    after the first file, so the batch takes the unaligned kernels."""
    import time
    import torch
    import rsync_amd
    from rsync_amd import _lib
    eng = rsync_amd.Engine(0)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    for nf, fb, blen, narena in SHAPES_UNALIGNED:
        stride = fb + 1
        total = nf * stride
        arenas = [eng.alloc(total) for _ in range(narena)]
        for k, a in enumerate(arenas):
            for f in range(nf):
                eng.fill_splitmix64(a, fb, 1 + f + 7919 * k, offset=f * stride, stream=sp)
        plan = eng.plan([(f * stride, fb, blen) for f in range(nf)], total)
        recs = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
        eng.synchronize(sp)
        w0 = time.perf_counter()
        while time.perf_counter() - w0 < 0.3:
            plan.run(arenas[0], SEED, recs, stream=sp)
            eng.synchronize(sp)
        res = {}
        for v, name in VARIANTS_UNALIGNED.items():
            eng.set_block_sums_kernel(v)
            for i in range(10):
                plan.run(arenas[i % narena], SEED, recs, stream=sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(30):
                plan.run(arenas[i % narena], SEED, recs, stream=sp)
            e1.record(stream)
            eng.synchronize(sp)
            ms = e0.elapsed_time(e1) / 30
            res[name] = {"kernel_ms": round(ms, 4), "hbm_frac_8tbs": round((nf * fb + plan.total_records * 20) / (ms / 1e3) / 8e12, 4)}
        eng.set_block_sums_kernel(-1)
        print(json.dumps({"files": nf, "file_bytes": fb, "block_len": blen, "unaligned": True, "variants": res}), flush=True)
        plan.close()
        for a in arenas:
            a.free()
        recs.free()


if __name__ == "__main__":
    main()
