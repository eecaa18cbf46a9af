#!/usr/bin/env python3
"""Host-loop rate of rsg_generate_files_fd for a few batch
sizes and reader-thread counts: 256 x 1 MiB files written to /dev/shm (page
cache), B = 700, mux-framed sums stream to a counting writer.  Each setting
runs in a child process (the knobs are environment variables read per call,
but a fresh process keeps the settings' pinned buffers apart).

    python tools/host_loop_sweep.py
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS = [(64, 8), (32, 8), (16, 8), (32, 16), (16, 16), (8, 16)]


def child(tmp):
    sys.path.insert(0, ROOT)
    import numpy as np
    import rsync_amd
    eng = rsync_amd.Engine(0)
    fds = [os.open(os.path.join(tmp, f"f{i}"), os.O_RDONLY) for i in range(256)]
    sink = [0]

    def count(b):
        sink[0] += len(b)
    gen = [(fd, 1 << 20) for fd in fds]
    eng.generate_files_fd(gen, 0x1BADB002, count, block_len=700, idx=list(range(256)), mux=True)
    best = []
    for _ in range(5):
        t0 = time.perf_counter()
        eng.generate_files_fd(gen, 0x1BADB002, count, block_len=700, idx=list(range(256)), mux=True)
        best.append(time.perf_counter() - t0)
    print(json.dumps({"gib_s_best": round(256 / 1024 / min(best), 3),
                      "gib_s_median": round(256 / 1024 / sorted(best)[2], 3)}))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    import numpy as np
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    rng = np.random.default_rng(1)
    for i in range(256):
        with open(os.path.join(tmp, f"f{i}"), "wb") as fh:
            fh.write(rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes())
    try:
        for mb, th in SETTINGS:
            env = dict(os.environ, RSG_GEN_BATCH_MB=str(mb), RSG_COPY_THREADS=str(th))
            out = subprocess.run([sys.executable, __file__, "--child", tmp], env=env, capture_output=True,
                                 text=True, timeout=120)
            line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-300:]
            print(json.dumps({"batch_mb": mb, "threads": th, "result": line}), flush=True)
    finally:
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
