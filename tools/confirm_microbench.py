"""Time the block-sum kernel on the sender's confirmation shape: N unaligned
32 KiB windows (one per lane) of a 1 GiB device arena, N = 3K .. 48K.  A time
that stays flat as N doubles means the kernel is bound by one window's serial
MD4 chain, not by issue slots or bandwidth.  Prints one JSON line per N."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import rsync_amd  # noqa: E402
from rsync_amd import _lib  # noqa: E402


def main():
    eng = rsync_amd.Engine(0)
    size = 1 << 30
    arena = eng.alloc(size)
    eng.fill_splitmix64(arena, size, 5)
    rng = np.random.default_rng(1)
    B = 32768
    variant = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    eng.set_block_sums_kernel(variant)
    for n in (3072, 6144, 12288, 24576, 49152):
        offs = np.sort(rng.choice(size - 2 * B, n, replace=False)) | 1  # odd: unaligned windows
        files = [(int(o), B, B) for o in offs]
        plan = eng.plan(files, size)
        out = eng.alloc(n * 20)
        for _ in range(3):
            plan.run(arena, 7, out)
        eng.synchronize()
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run(arena, 7, out)
        eng.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"windows": n, "ms": round(dt * 1e3, 4), "variant": variant}), flush=True)
        out.free()
    eng.set_block_sums_kernel(-1)
    eng.close()


if __name__ == "__main__":
    main()
