#!/usr/bin/env python3
"""Timing probe for the sender's confirmation shape: N windows of B bytes at
odd offsets of a 1 GiB device source (the unaligned block-sum kernel,
variant 6), hashed by one plan launch, HIP events over 20 launches.
Diagnostic only.   python tools/confirm_probe.py [B] [N ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import rsync_amd
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    counts = [int(x) for x in sys.argv[2:]] or [37 * 64, 2350, 4700, 23515]
    eng = rsync_amd.Engine(0)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    size = 1 << 30
    src = eng.alloc(size + 4096)
    eng.fill_splitmix64(src, size + 4096, 7, stream=sp)
    rng = np.random.default_rng(5)
    for n in counts:
        offs = np.sort(rng.choice((size - B) // 2, n, replace=False)) * 2 + 1  # odd offsets
        plan = eng.plan([(int(o), B, B) for o in offs], size + 4096)
        recs = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
        for _ in range(5):
            plan.run(src, 1, recs, stream=sp)
        eng.synchronize(sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            plan.run(src, 1, recs, stream=sp)
        e1.record(stream)
        eng.synchronize(sp)
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"B": B, "windows": n, "waves": (n + 63) // 64, "ms": round(ms, 4),
                          "us_per_compression_per_wave": round(ms * 1e3 / (B // 64 + 1), 3)}), flush=True)
        plan.close()
        recs.free()


if __name__ == "__main__":
    main()
