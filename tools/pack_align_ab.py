#!/usr/bin/env python3
"""A/B of the arena packing alignment for block sums (diagnostic).

    python tools/pack_align_ab.py

1 GiB of files with lengths drawn around 1 MiB / 4 MiB, packed back to back
at 16- or 128-byte aligned offsets (the library packs at 128 since late
round 5), block lengths 1024 / 2048 / 4096 (multiples of 128).  With 16-byte
packing most blocks start off the 128-byte lines, so the plan's lines128
flag is false and the automatic choice leaves 128-byte segments.  Prints one
JSON line per (B, alignment): the automatic kernel's time per launch."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import rsync_amd
    eng = rsync_amd.Engine(0)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    rng = np.random.default_rng(5)
    for B, mean in ((1024, 1 << 20), (2048, 4 << 20), (4096, 16 << 20)):
        lens = []
        while sum(lens) < (1 << 30) - 2 * mean:
            lens.append(int(rng.integers(mean // 2, mean * 3 // 2)))
        for align in (16, 128):
            offs, at = [], 0
            for n in lens:
                offs.append(at)
                at += (n + align - 1) & ~(align - 1)
            arena = eng.alloc(at)
            eng.fill_splitmix64(arena, at, 7, stream=sp)
            plan = eng.plan([(o, n, B) for o, n in zip(offs, lens)], at)
            recs = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
            for variant in (-1, 4):
                eng.set_block_sums_kernel(variant)
                for _ in range(10):
                    plan.run(arena, 1, recs, stream=sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(30):
                    plan.run(arena, 1, recs, stream=sp)
                e1.record(stream)
                eng.synchronize(sp)
                ms = e0.elapsed_time(e1) / 30
                print(json.dumps({"block_len": B, "pack_align": align, "files": len(lens), "bytes": sum(lens),
                                  "variant": "automatic" if variant == -1 else "staged_seg128",
                                  "kernel_ms_per_gib": round(ms * (1 << 30) / sum(lens), 4)}), flush=True)
            eng.set_block_sums_kernel(-1)
            plan.close()
            arena.free()
            recs.free()


if __name__ == "__main__":
    main()
