#!/usr/bin/env python3
"""bench.py -- device-resident block-checksum throughput on MI355X.

Metric (BASELINE.json): GiB/s block-checksummed (weak + MD4), device-resident.
Workload: BASELINE.json configs[1] -- 1024 x 1 MiB random files, 700-byte
blocks, receiver block-sum generation -- per GPU (weak scaling: rank r owns
its own 1024 files).  One step = one launch of the block-sum kernel over the
rank's 1 GiB batch, inputs already resident in HBM; two input arenas are
alternated so the 256 MiB Infinity Cache cannot serve repeats.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.  Extra objects: roofline (HIP-event kernel
time vs the HBM roofline), cpu_baseline (the scalar C restatement on host
cores, bounded sample), host_path (PCIe-inclusive rate), and for N > 1 the
RCCL sums gather.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FILES_PER_GPU = 1024
FILE_BYTES = 1 << 20
BLOCK_LEN = 700
SEED = 0x1BADB002


def cpu_model() -> str:
    """The host CPU the CPU baseline ran on (state the model)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--windows", type=int, default=5,
                    help="timed windows of exactly --steps steps; the line reports the median window")
    ap.add_argument("--warmup-ms", type=float, default=200.0,
                    help="keep warming up (beyond --warmup steps) until this much time has passed: the "
                         "GPU takes ~15 ms of back-to-back launches to reach its steady memory clock")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bound of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-delivery", action="store_true", help="skip the pipelined gather / D2H delivery modes")
    ap.add_argument("--ab", action="store_true", help="A/B the block-sum kernel variants (interleaved rounds)")
    ap.add_argument("--workload", default="cfg2",
                    choices=["cfg2", "cfg3", "cfg4", "cfg4-sender", "cfg5", "filesums", "receive"],
                    help="cfg2 = receiver block sums (the metric); cfg3 = sender match, reported separately")
    ap.add_argument("--cfg3-files", type=int, default=10)
    ap.add_argument("--search-option", action="append", default=[], metavar="NAME=VALUE",
                    help="cfg3 A/B only: a per-context sender option (engine.SEARCH_OPTIONS, e.g. confirm_cus=24)")
    ap.add_argument("--batches", type=int, default=None,
                    help="batches per rank for the pipelined delivery modes (records of batch b move while "
                         "batch b+1 is hashed); default 4, or 1 at N = 1, where the root's records are "
                         "written in place and nothing moves for the gather")
    ap.add_argument("--delivery-steps", type=int, default=20, help="timed steps of each delivery mode")
    return ap.parse_args()


def keep_stdout_for_the_line():
    """The bench line is the only thing on stdout: native libraries that print
    there (RCCL's version banner at communicator init) write to stderr
    instead.  fd 1 becomes a copy of fd 2; Python's sys.stdout keeps the
    original stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(real, "w", buffering=1)


def main():
    args = parse()
    keep_stdout_for_the_line()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; data moves over RCCL
    # one rank per GPU: RCCL refuses two ranks on one device, so a launch with
    # more ranks than visible GPUs stops here with a clear message
    ndev = torch.cuda.device_count()
    if world > ndev or local >= ndev:
        if rank == 0:
            print(json.dumps({"metric": "GiB/s block-checksummed (weak+MD4), device-resident, at 1/2/4/8 MI355X",
                              "value": None, "n_gpus": world,
                              "error": f"{world} ranks but {ndev} visible GPU(s): one rank per GPU is required "
                                       f"(RCCL cannot put two ranks on one device)"}), flush=True)
        sys.exit(2)
    torch.cuda.set_device(local)
    import rsync_amd
    if args.workload == "cfg3":
        return bench_sender(args, rank, world, local)
    if args.workload == "cfg4":
        return bench_mixed(args, rank, world, local)
    if args.workload == "cfg4-sender":
        return bench_sender_small(args, rank, world, local)
    if args.workload == "cfg5":
        return bench_long(args, rank, world, local)
    if args.workload == "filesums":
        return bench_filesums(args, rank, world, local)
    if args.workload == "receive":
        return bench_receive(args, rank, world, local)

    eng = rsync_amd.Engine(local)
    stream = torch.cuda.Stream(device=local)
    sptr = stream.cuda_stream

    # ---- workload: this rank's 1024 files, global file ids rank*1024 + f
    n = FILES_PER_GPU
    arena_bytes = n * FILE_BYTES
    arenas = [eng.alloc(arena_bytes) for _ in range(2)]
    for a in arenas:
        for f in range(n):
            eng.fill_splitmix64(a, FILE_BYTES, rank * n + f + 1, offset=f * FILE_BYTES, stream=sptr)
    plan = eng.plan([(f * FILE_BYTES, FILE_BYTES, BLOCK_LEN) for f in range(n)], arena_bytes)
    recs = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
    eng.synchronize(sptr)

    def step(i):
        plan.run(arenas[i & 1], SEED, recs, stream=sptr)

    w0 = time.perf_counter()
    warm = 0
    while warm < args.warmup or (time.perf_counter() - w0) * 1e3 < args.warmup_ms:
        step(warm)
        warm += 1
        if warm % 20 == 0:
            eng.synchronize(sptr)
    eng.synchronize(sptr)

    def window():
        """EXACTLY args.steps steps, bracketed by a barrier + synchronize on
        both sides; -> (wall s, HIP-event kernel ms per step), max over ranks."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(args.steps):
            step(i)
        ev1.record(stream)
        eng.synchronize(sptr)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        w, k = time.perf_counter() - t0, ev0.elapsed_time(ev1) / args.steps
        return max_over_ranks(world, w, k)

    # The headline is the median of --windows timed windows (each exactly K
    # steps), so one optimistic window cannot set it.
    wins = sorted(window() for _ in range(max(1, args.windows)))
    wall, kernel_ms = wins[len(wins) // 2]
    extra = {}
    if args.ab:
        from rsync_amd import _lib
        # the shipped block-sum variants on the same plan (identical records)
        names = {2: "park", 1: "staged_seg256", 4: "staged_seg128", 7: "lines", 0: "direct"}
        only = os.environ.get("AB_ONLY")  # comma-separated substrings: A/B only the matching entries
        if only:
            names = {v: n for v, n in names.items() if any(o in n for o in only.split(","))}
        res = {v: [] for v in names}
        for _ in range(int(os.environ.get("AB_ROUNDS", "5"))):
            for v in names:
                print(f"ab: {names[v]}", file=sys.stderr, flush=True)
                eng.set_block_sums_kernel(v)
                for i in range(3):
                    step(i)
                a0 = torch.cuda.Event(enable_timing=True)
                a1 = torch.cuda.Event(enable_timing=True)
                a0.record(stream)
                for i in range(args.steps):
                    step(i)
                a1.record(stream)
                eng.synchronize(sptr)
                res[v].append(a0.elapsed_time(a1) / args.steps)
        eng.set_block_sums_kernel(-1)
        step(0)
        eng.synchronize(sptr)
        extra["ab_kernel_ms"] = {names[v]: [round(x, 4) for x in sorted(res[v])] for v in names}
        # consecutive batches on two streams (the generator's two-slot
        # pipeline): batch i+1's workgroups take the CUs batch i's leave
        s2 = torch.cuda.Stream(device=local)
        recs2 = eng.alloc(plan.total_records * rsync_amd.RECORD_BYTES)
        two = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                if i & 1:
                    plan.run(arenas[1], SEED, recs2, stream=s2.cuda_stream)
                else:
                    plan.run(arenas[0], SEED, recs, stream=sptr)
            torch.cuda.synchronize()
            two.append((time.perf_counter() - t0) * 1e3 / args.steps)
            one0 = time.perf_counter()
            for i in range(args.steps):
                step(i)
            eng.synchronize(sptr)
            two.append(-(time.perf_counter() - one0) * 1e3 / args.steps)
        extra["ab_wall_ms_per_step"] = {"two_streams": sorted(round(x, 4) for x in two if x > 0),
                                        "one_stream": sorted(round(-x, 4) for x in two if x < 0)}
        recs2.free()

    in_bytes = float(arena_bytes)
    out_bytes = float(plan.total_records * rsync_amd.RECORD_BYTES)
    value = world * in_bytes * args.steps / wall / GIB
    achieved = (in_bytes + out_bytes) / (kernel_ms * 1e-3) / 1e9

    cpu = None  # filled in below on rank 0 at N = 1

    def bench_line(more):
        traffic = None
        tp = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tp):
            try:
                traffic = json.load(open(tp)).get("block_sums_kernel_cfg2_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "GiB/s block-checksummed (weak+MD4), device-resident, at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_effective": warm,
            "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "windows_ms_per_step": [round(w * 1e3 / args.steps, 4) for w, _ in wins],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {"workload": "cfg2: receiver block sums, 1024 x 1 MiB files per GPU, B=700, weak+MD4",
                       "files_per_gpu": n, "file_bytes": FILE_BYTES, "block_len": BLOCK_LEN,
                       "records_per_gpu": plan.total_records, "parallelism": f"files sharded, {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": "profiles/traffic.json: rocprofv3 PMC passes of this bench command "
                                           "(FETCH_SIZE x2 + WRITE_SIZE per launch), not measured in this run",
                         "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": int(in_bytes + out_bytes)},
            "cpu_baseline": cpu,
        }
        line.update(more)
        return line

    # ---- delivery of the records (the one exchange step), pipelined with the
    # hashing: RCCL gather to rank 0, and every rank's own D2H
    if not args.no_delivery:
        from rsync_amd.dist import ShardedBlockSums
        nb = max(1, args.batches if args.batches is not None else (1 if world == 1 else 4))
        per = -(-n // nb)
        groups = [list(range(g * per, min(n, (g + 1) * per))) for g in range(nb)]
        groups = [g for g in groups if g]
        recs_per_file = plan.total_records // n
        descs = [[(f * FILE_BYTES, FILE_BYTES, BLOCK_LEN) for f in g] for g in groups]
        rec_off = [g[0] * recs_per_file for g in groups]
        send = [[len(g) * recs_per_file * rsync_amd.RECORD_BYTES] * world for g in groups]
        recv_off = [[(q * plan.total_records + g[0] * recs_per_file) * rsync_amd.RECORD_BYTES for q in range(world)]
                    for g in groups]
        sb = ShardedBlockSums(eng, descs, arena_bytes, rec_off, send, recv_off)
        def oracle_check(got):
            """orc_block_sums of files 0, n/2 and n-1 of every rank (rank q's
            file f is splitmix64(q n + f + 1)) against their gathered records."""
            from oracle import oracle as orc
            ok, k = True, 0
            for q in range(world):
                for f in (0, n // 2, n - 1):
                    want = orc.block_sums(orc.splitmix64_bytes(q * n + f + 1, FILE_BYTES), BLOCK_LEN, SEED)
                    o = (q * plan.total_records + plan.first_record[f]) * rsync_amd.RECORD_BYTES
                    ok &= bytes(got[o:o + len(want)]) == want
                    k += 1
            return {"oracle_files_checked": k, "oracle_equal": bool(ok)}
        extra["delivery"] = guarded_delivery(args, eng, sb, arenas, recs, world, rank, world * in_bytes,
                                             world * plan.total_records,
                                             lambda d: print(json.dumps(bench_line(dict(extra, delivery=d))),
                                                             flush=True), oracle_check)
        sb.close()

    # ---- PCIe-inclusive host path (rank 0, N = 1): host buffers in, records out
    if rank == 0 and world == 1 and not args.no_host_path:
        import cases
        files = [cases.splitmix64_bytes(f + 1, FILE_BYTES) for f in range(256)]
        eng.block_sums(files[:8], SEED, BLOCK_LEN)  # warm the staging buffers
        h0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            _, host_rec, _ = eng.block_sums(files, SEED, BLOCK_LEN)
        hdt = (time.perf_counter() - h0) / reps
        extra["host_path"] = {"gib_s": round(256 * FILE_BYTES / hdt / GIB, 3),
                              "sample": "256 x 1 MiB host buffers, H2D + kernel + D2H, pinned staging"}
        # the same files read straight into engine-pinned memory: DMA from the
        # caller's buffers, no staging copy
        pin = eng.alloc_pinned(256 * FILE_BYTES)
        views = [pin[f * FILE_BYTES:(f + 1) * FILE_BYTES] for f in range(256)]
        for v, f in zip(views, files):
            v[:] = f
        eng.block_sums(views[:8], SEED, BLOCK_LEN)
        h0 = time.perf_counter()
        for _ in range(reps):
            _, pin_rec, _ = eng.block_sums(views, SEED, BLOCK_LEN)
        pdt = (time.perf_counter() - h0) / reps
        extra["host_path"]["pinned_sources_gib_s"] = round(256 * FILE_BYTES / pdt / GIB, 3)
        extra["host_path"]["pinned_sources_parity"] = pin_rec == host_rec
        del views
        eng.free_pinned(pin)
        # the generator's whole host loop (rsg_generate_files_fd): the files
        # on a filesystem (page cache), read by the engine, sums stream (idx,
        # SumHead, records, phase markers) handed to a writer that counts it
        import tempfile
        tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        fds = []
        try:
            for f, d in enumerate(files):
                p = os.path.join(tmp, f"f{f}")
                with open(p, "wb") as fh:
                    fh.write(d.tobytes())
                fds.append(os.open(p, os.O_RDONLY))
            sink = [0]

            def count(b):
                sink[0] += len(b)
            gen = [(fd, FILE_BYTES) for fd in fds]
            eng.generate_files_fd(gen, SEED, count, block_len=BLOCK_LEN, idx=list(range(256)), mux=True)
            gts = []
            for _ in range(5):  # median of 5 full calls after a full warm-up call
                h0 = time.perf_counter()
                _, nw = eng.generate_files_fd(gen, SEED, count, block_len=BLOCK_LEN, idx=list(range(256)), mux=True)
                gts.append(time.perf_counter() - h0)
            gdt = sorted(gts)[2]
            extra["host_path"]["generate_files_fd_gib_s"] = round(256 * FILE_BYTES / gdt / GIB, 3)
            extra["host_path"]["generate_files_fd_sample"] = (
                f"256 x 1 MiB files in {tmp.rsplit('/', 1)[0]} (page cache), pread by the engine, mux-framed sums "
                f"stream of {nw} bytes to a counting writer, median of 5 calls")
        finally:
            for fd in fds:
                os.close(fd)
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)

    # ---- CPU baseline: the scalar C restatement (oracle) on 1 host core
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import cases
        from oracle import oracle as orc
        lib = orc.lib()
        sample_files = [cases.splitmix64_bytes(f + 1, FILE_BYTES) for f in range(min(n, 64))]
        done_bytes, t_cpu, f = 0, 0.0, 0
        sample_parity = True
        out = np.empty(1498 * 20, np.uint8)
        while t_cpu < args.cpu_seconds:
            data = sample_files[f % len(sample_files)]
            c0 = time.perf_counter()
            lib.orc_block_sums(orc._ptr(data), data.size, BLOCK_LEN, orc._i32(SEED), orc._ptr(out))
            t_cpu += time.perf_counter() - c0
            done_bytes += data.size
            if f < 4:  # spot parity of the benchmarked GPU output
                got = recs.download(1498 * 20, offset=plan.first_record[f] * 20)
                sample_parity &= bool((got == out).all())
            f += 1
        cpu = {"value": round(done_bytes / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"{f} x 1 MiB files (cycling the first 64 of the workload's files) at B=700, "
                         f"oracle/rsg_oracle.c orc_block_sums (scalar C restatement of generator.go:325-350), "
                         f"1 thread, {t_cpu:.1f} s",
               "gpu_parity_on_sample": sample_parity}
        # the same restatement on T host threads, files partitioned;
        # ctypes drops the GIL for the foreign call, so the threads run in parallel
        import threading
        T = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16
        wall_s = max(2.0, args.cpu_seconds / 2)
        counts = [0] * T

        def cpu_worker(k):
            o = np.empty(1498 * 20, np.uint8)
            t_end = time.perf_counter() + wall_s
            j = k
            while time.perf_counter() < t_end:
                d = sample_files[j % len(sample_files)]
                lib.orc_block_sums(orc._ptr(d), d.size, BLOCK_LEN, orc._i32(SEED), orc._ptr(o))
                counts[k] += d.size
                j += T

        w0 = time.perf_counter()
        ths = [threading.Thread(target=cpu_worker, args=(k,)) for k in range(T)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wdt = time.perf_counter() - w0
        extra["cpu_baseline_all_cores"] = {
            "value": round(sum(counts) / wdt / GIB, 4), "unit": "GiB/s", "cores": T, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{sum(counts) // FILE_BYTES} x 1 MiB files on {T} threads (files partitioned), "
                      f"same orc_block_sums, {wdt:.1f} s wall"}

    if rank == 0:
        print(json.dumps(bench_line(extra)), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def max_over_ranks(world, *vals):
    if world == 1:
        return vals
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(vals), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return tuple(float(x) for x in t)


def measure_delivery(args, eng, sb, arenas, recs, world, rank, bytes_all, records_all, oracle_check=None):
    """The generator step with its records delivered, pipelined per batch
    (rsg_block_sums_gather / rsg_block_sums_d2h): kernel of batch b+1 while
    batch b's records move.  Each timed step hashes the rank's whole share
    and delivers it; rates are all ranks' input bytes / the max-over-ranks
    wall time.  -> dict for the bench line, with "gather_parity": the root's
    gathered buffer against every rank's SHA-256 of its own records, every
    rank's D2H copy against the same, and oracle_check(gathered bytes) (the
    C oracle on sampled files of every rank).
    The communicator is set up before any leg is timed, ~0.1 s of steps run
    after its init, and every leg runs 8 untimed steps first (see below).
    BENCH_DELIVERY_DIAG=2 (one rank): per-chunk kernel times before and
    after the init, and the gather again after the d2h leg."""
    import rsync_amd
    out = {"batches": sb.nbatch}
    steps = max(2, args.delivery_steps)
    diag = os.environ.get("BENCH_DELIVERY_DIAG") == "2" and world == 1
    if diag:  # per-chunk times of the kernel synchronised per step, before and after the communicator's init
        import torch
        ts = torch.cuda.Stream()

        def chunk():
            t0 = time.perf_counter()
            for i in range(20):
                sb.run_kernels(arenas[i & 1], SEED, recs)
                eng.synchronize()
            wall = (time.perf_counter() - t0) / 20
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ts)
            for i in range(20):
                sb.run_kernels(arenas[i & 1], SEED, recs, stream=ts.cuda_stream)
            e1.record(ts)
            e1.synchronize()
            return [round(wall * 1e3, 4), round(e0.elapsed_time(e1) / 20, 4)]
        out["diag_before_comm"] = [chunk() for _ in range(5)]
    if world > 1:
        import torch.distributed as dist
        uid = [rsync_amd.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        uid = uid[0]
    else:
        uid = rsync_amd.Engine.comm_unique_id()
    eng.comm_init(world, rank, uid)
    if diag:
        t_init = time.perf_counter()
        out["diag_after_comm"] = [chunk() + [round((time.perf_counter() - t_init) * 1e3, 1)] for _ in range(12)]
    recv = eng.alloc(max(records_all, 1) * rsync_amd.RECORD_BYTES) if rank == 0 else None

    def synced(i):
        sb.run_kernels(arenas[i & 1], SEED, recs)
        eng.synchronize()
    # ~0.1 s of steps before any leg is timed: the kernel ran up to 25 % slower
    # in the first ~25 ms after ncclCommInitRank (r05q: HIP-event kernel time
    # 0.231, 0.211, 0.198 ms in the first three 20-step chunks, 0.186-0.191
    # after), a start-up transient of the communicator, not a cost of the step
    t_w = time.perf_counter()
    i = 0
    while time.perf_counter() - t_w < 0.1:
        synced(i)
        i += 1

    def timed(fn):
        for i in range(8):
            fn(i)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        (dt,) = max_over_ranks(world, time.perf_counter() - t0)
        return {"ms_per_step": round(dt * 1e3 / steps, 4), "gib_s": round(bytes_all * steps / dt / GIB, 2)}

    # floor of any synchronous delivery call: the same kernels, one host
    # synchronisation per step, nothing moved
    out["kernel_synced"] = timed(synced)
    # RCCL gather of every rank's records to rank 0 (one rank: its kernels
    # write the records where they land, nothing moves)
    out["kernel_plus_gather_pipelined"] = timed(lambda i: sb.run_gather(arenas[i & 1], SEED, recs, recv, 0))
    out["kernel_plus_gather_pipelined"]["bytes_to_root"] = (records_all - sb.my_records) * rsync_amd.RECORD_BYTES
    # every rank copies its own records to pinned host memory over its own PCIe link
    host = eng.alloc_pinned(max(sb.my_records, 1) * rsync_amd.RECORD_BYTES)
    out["d2h_parallel_pipelined"] = timed(lambda i: sb.run_d2h(arenas[i & 1], SEED, recs, host))
    out["d2h_parallel_pipelined"]["bytes_to_host_per_rank"] = sb.my_records * rsync_amd.RECORD_BYTES
    # ---- self-check, after the timed legs: every rank's own records (its
    # d_records, written by the d2h leg's kernels) against what the gather put
    # on the root and what its D2H put in host memory (generator.go:20-52:
    # every file's sums, in file-list order)
    from rsync_amd.dist import all_ranks, gather_parity, records_digest
    nbytes = sb.my_records * rsync_amd.RECORD_BYTES
    mine = recs.download(nbytes) if nbytes else np.zeros(0, np.uint8)
    dg = records_digest(mine)
    info = all_ranks((dg, sb.my_records, records_digest(host[:nbytes]) == dg), world)
    eng.free_pinned(host)
    if rank == 0:
        got = recv.download(sum(n for _, n, _ in info) * rsync_amd.RECORD_BYTES)
        par = gather_parity(got, [d for d, _, _ in info], [n for _, n, _ in info])
        par["d2h_ranks_equal"] = [ok for _, _, ok in info]
        if oracle_check is not None:
            par.update(oracle_check(got))
        par["all_equal"] = bool(par["all_equal"] and all(par["d2h_ranks_equal"]) and par.get("oracle_equal", True))
        out["gather_parity"] = par
    if diag:
        out["diag_gather_after_d2h"] = timed(lambda i: sb.run_gather(arenas[i & 1], SEED, recs, recv, 0))
        out["diag_synced_after_d2h"] = timed(synced)
    out["recv"] = recv
    return out


def guarded_delivery(args, eng, sb, arenas, recs, world, rank, bytes_all, records_all, print_line,
                     oracle_check=None):
    """measure_delivery under a watchdog: a collective that stalls for 120 s
    makes rank 0 print the bench line with the error and every rank exit 3
    (a failed collective must not look like success); an exception is
    reported in the line."""
    import threading
    done = threading.Event()

    def watchdog():
        if not done.wait(120.0):
            if rank == 0:
                print_line({"error": "delivery timed out after 120 s (stalled collective)"})
            os._exit(3)
    if world > 1:
        threading.Thread(target=watchdog, daemon=True).start()
    try:
        d = measure_delivery(args, eng, sb, arenas, recs, world, rank, bytes_all, records_all, oracle_check)
        d.pop("recv", None)
    except Exception as e:  # reported, never fatal to the bench line
        d = {"error": str(e)[:300]}
    done.set()
    return d



def bench_sender(args, rank, world, local):
    """cfg3: sender byte-rolling match, 10 x 1 GiB sources vs 50%-modified bases
    on one GPU (the files shard across GPUs with no exchange).  Metric: source
    GiB scanned per second, device-resident, end to end through the C-ABI."""
    import torch
    import rsync_amd
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cases
    eng = rsync_amd.Engine(local)
    for opt in args.search_option:
        name, value = opt.split("=")
        eng.set_option(name, int(value))
    size = 1 << 30
    rng = np.random.default_rng(3 + rank)
    basis = eng.alloc(size)
    srcs, metas = [], []
    for f in range(args.cfg3_files):
        src = eng.alloc(size + 4096)
        seed = 1000 * rank + f + 3
        n = cases.make_cfg3_file(eng, basis, src, size, seed, 32768, rng)
        recs, total = eng.block_sums_device(basis, [(0, size, 0)], SEED)
        rec = recs.download(total * 20).reshape(-1, 20)
        recs.free()
        s1 = rec[:, :4].copy().view("<u4").reshape(-1)
        s2 = rec[:, 4:].copy()
        tags = ((s1 & 0xFFFF) + (s1 >> 16)) & 0xFFFF
        tg = np.argsort(tags, kind="stable").astype(np.int32)
        head = rsync_amd.sum_sizes_sqroot(size)
        srcs.append(src)
        metas.append((n, head, s1, s2, tg))
    eng.synchronize()
    jobs = [(src, n, head, s1, s2, tg) for (n, head, s1, s2, tg), src in zip(metas, srcs)]
    # warm up (with the kernel-timing events on: their first use costs a few
    # ms once, which otherwise landed in the first timed call), then time K
    # passes over the file set: one batched call per pass (SendFiles' loop
    # over the files, pipelined across files)
    eng.set_kernel_timing(True)
    for _ in range(max(1, min(args.warmup, 2))):
        eng.hash_search_batch(jobs, SEED, as_arrays=True)
    steps = max(1, min(args.steps, 5))
    import torch.distributed as dist
    if world > 1:  # files shard across ranks with no exchange: max-over-ranks wall time
        dist.barrier()
    eng.kernel_times(reset=True)
    t0 = time.perf_counter()
    nm = 0
    call_ms = []
    for _ in range(steps):
        c0 = time.perf_counter()
        res = eng.hash_search_batch(jobs, SEED, as_arrays=True)
        call_ms.append(round((time.perf_counter() - c0) * 1e3, 3))
        nm += sum(len(m) for m in res)
    dt = time.perf_counter() - t0
    kt = eng.kernel_times(reset=True)  # HIP events around every roll / confirmation on their own streams
    eng.set_kernel_timing(False)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    # the same files through one single-file call each (no cross-file overlap)
    t1 = time.perf_counter()
    for j in jobs:
        eng.hash_search_device(*j, SEED)
    dt1 = time.perf_counter() - t1
    scanned = sum(m[0] for m in metas) * steps
    single_gib_s = round(scanned / steps / dt1 / GIB, 2)  # this rank's files, one call each
    if world > 1:  # every rank's files (all ranks scan the same number of bytes)
        st = torch.tensor([float(scanned)], dtype=torch.float64)
        dist.all_reduce(st)
        scanned = float(st[0])
    roll_ms = kt["roll_ms"] / max(kt["roll_launches"], 1)
    confirm_ms = kt["confirm_ms"] / max(kt["confirm_batches"], 1)
    src_bytes = sum(m[0] for m in metas) / len(metas)  # algorithmic bytes of one roll launch: its source, read once
    cpu, parity = None, None
    if rank == 0 and not args.no_cpu:
        # cpu_baseline leg: the C restatement of hashSearch (match.go:21-230)
        # on the first 256 MiB of file 0 against file 0's basis sums, 1 core;
        # its matches also check the benchmarked match list of file 0 (the
        # greedy walk is left to right, so every match whose window ends
        # before the sample's last block is the same in both)
        from oracle import oracle as orc
        n0, head0, s1_0, s2_0, tg0 = metas[0]
        P = min(256 << 20, n0)
        sample = srcs[0].download(P)
        c0 = time.perf_counter()
        om, _, _ = orc.hash_search(sample, head0.astuple(), s1_0, s2_0, tg0, SEED)
        t_cpu = time.perf_counter() - c0
        B0 = head0.block_len
        cut = P - B0
        gm = [(int(o), int(i)) for o, i in zip(res[0]["offset"], res[0]["index"])]
        want = [m for m in om if m[0] + B0 <= cut]
        parity = {"matches_compared": len(want), "equal": want == [m for m in gm if m[0] + B0 <= cut]}
        cpu = {"value": round(P / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"first {P >> 20} MiB of file 0 vs its basis sums, oracle/rsg_oracle.c orc_hash_search "
                         f"(scalar C restatement of match.go:21-282), 1 thread, {t_cpu:.1f} s"}
    host_path = None
    if rank == 0 and world == 1 and not args.no_host_path:
        host_path = sender_host_path(eng, srcs, metas, res)
    if rank == 0:
        print(json.dumps({"metric": "GiB/s source scanned (sender rolling match), device-resident",
                          "value": round(scanned / dt / GIB, 2), "unit": "GiB/s", "n_gpus": world,
                          "steps": steps, "higher_is_better": True, "dtype": "u32",
                          "data": "synthetic (splitmix64 bases; sources 50% overwritten + shifts)",
                          "config": {"workload": "cfg3: 10 x 1 GiB sources vs 50%-modified bases, B=32768",
                                     "files": args.cfg3_files, "matches_per_pass": nm // steps,
                                     **({"search_options": args.search_option} if args.search_option else {}),
                                     "call": "rsg_hash_search_batch_device, one call per pass"},
                          "ms_per_file": round(dt * 1e3 / (steps * len(metas)), 3), "call_ms": call_ms,
                          "single_file_calls_gib_s": single_gib_s,
                          "roofline": {"bound": "hbm", "kernel": "roll_packed_kernel (edge tiles included)",
                                       "note": "the roll is VALU-issue-bound (integer ops at 4 cycles per wave64, "
                                               "DESIGN.md section 4.2); frac is its HBM fraction, as the metric's unit",
                                       "achieved": round(src_bytes / (roll_ms * 1e-3) / 1e9, 1),
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": round(src_bytes / (roll_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       "traffic": cfg3_traffic(), "kernel_ms": round(roll_ms, 4),
                                       "launches": kt["roll_launches"],
                                       "algorithmic_bytes_per_launch": int(src_bytes),
                                       "valu_issue": roll_valu_issue(roll_ms, world),
                                       "confirm_ms_per_batch": round(confirm_ms, 4),
                                       "confirm_batches": kt["confirm_batches"],
                                       "candidates_per_launch": kt["candidates"] // max(kt["roll_launches"], 1),
                                       "windows_confirmed_per_launch": kt["windows"] // max(kt["roll_launches"], 1)},
                          "oracle_parity_file0": parity,
                          "host_path": host_path,
                          "cpu_baseline": cpu}), flush=True)
    eng.close()


def sender_host_path(eng, srcs, metas, dev_res):
    """The sender from files (rows a13 + f2): the sources written to /dev/shm
    (page cache) and read by the engine in 256 MiB windows (pread -> pinned
    -> H2D, overlapped with the search).
    * file 0 alone through rsg_hash_search_fd, with and without the
      whole-file sum MD4(seed || source) (match.go:52-53) on a host thread;
    * all files through rsg_hash_search_fd_batch (SendFiles' loop), the
      files' sums on RSG_SUM_THREADS host threads side by side.
    PCIe-inclusive; never the line's value."""
    import tempfile
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    out = {}
    fds = []
    try:
        for k, (src, meta) in enumerate(zip(srcs, metas)):
            data = src.download(meta[0])
            p = os.path.join(tmp, f"src{k}")
            with open(p, "wb") as fh:
                fh.write(data.tobytes())
            del data
            fds.append(os.open(p, os.O_RDONLY))
        n, head, s1, s2, tg = metas[0]
        fd = fds[0]
        want0 = [(int(o), int(i)) for o, i in zip(dev_res[0]["offset"], dev_res[0]["index"])]
        eng.hash_search_fd(fd, n, head, s1, s2, tg, SEED)  # warm the staging buffers
        for tag, fs in (("search_only", False), ("with_file_sum", True)):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = eng.hash_search_fd(fd, n, head, s1, s2, tg, SEED, file_sum=fs)
                ts.append(time.perf_counter() - t0)
            m = r[0] if fs else r
            dt = sorted(ts)[1]
            out[tag] = {"gib_s": round(n / dt / GIB, 3), "s": round(dt, 4), "matches_equal_device_path": m == want0}
        jobs = [(fd_k, m[0], m[1], m[2], m[3], m[4]) for fd_k, m in zip(fds, metas)]
        total = sum(m[0] for m in metas)
        for tag, fs in (("batch_search_only", False), ("batch_with_file_sums", True)):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = eng.hash_search_fd_batch(jobs, SEED, file_sums=fs)
                ts.append(time.perf_counter() - t0)
            dt = sorted(ts)[1]
            eq = all([(int(o), int(i)) for o, i in zip(d["offset"], d["index"])] == m for d, (m, _) in zip(dev_res, r))
            out[tag] = {"gib_s": round(total / dt / GIB, 3), "s": round(dt, 4), "files": len(jobs),
                        "matches_equal_device_path": eq}
            if fs:
                out[tag]["sum_threads"] = int(os.environ.get("RSG_SUM_THREADS", "10"))
                # file 0's sum against the single-file call's (itself checked against the oracle in the tests)
                out[tag]["file0_sum_equal_single_call"] = r[0][1] == eng.hash_search_fd(
                    fds[0], n, head, s1, s2, tg, SEED, file_sum=True)[1]
    finally:
        for f in fds:
            os.close(f)
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    out["sample"] = ("sources in /dev/shm read by the engine in 256 MiB windows; median of 3. search_only / "
                     "with_file_sum: file 0 through rsg_hash_search_fd (its MD4(seed || source) on one host "
                     "thread); batch_*: all files through rsg_hash_search_fd_batch, the files' sums on host "
                     "threads side by side")
    return out


class _DevView:
    """A device address (and size) inside a torch-allocated arena, in the
    shape the engine's calls take (.ptr, .nbytes)."""

    def __init__(self, ptr, nbytes=0):
        self.ptr, self.nbytes = int(ptr), int(nbytes)


def bench_sender_small(args, rank, world, local):
    """cfg4-sender: the sender over a file tree of small sources -- SendFiles'
    per-file hashSearch (sender.go:19-115, match.go:21-230) for 100 000
    sources of 4-64 KiB (cfg4's lengths, PRNG seed 4), each its basis with one
    deletion of 1-63 bytes (so matches also fall off block boundaries) and
    random runs of 1-1400 bytes overwritten over ~50 % of it; B =
    SumSizesSqroot (700 at these sizes).  Sources device-resident, sums and
    targets in host memory as receiveSums leaves them, match lists written to
    host arrays: one rsg_hash_search_batch_device call per pass (the
    small-file kernel, one wave per file, a few launches per call).  Ranks
    take every world-th file (strong scaling)."""
    import torch
    import torch.distributed as dist
    import rsync_amd
    from rsync_amd.engine import SearchBatch
    from rsync_amd._lib import check as _check
    NF = 100_000
    lengths = np.random.default_rng(4).integers(4096, 65537, NF)
    mine = np.arange(rank, NF, world)
    L = lengths[mine]
    eng = rsync_amd.Engine(local)
    dev = torch.device("cuda", local)
    a16 = lambda x: (x + 15) // 16 * 16  # noqa: E731
    bofs = np.concatenate([[0], np.cumsum(a16(L))[:-1]])
    tb = int(a16(L).sum())
    bt = torch.empty(tb, dtype=torch.uint8, device=dev)
    for k, f in enumerate(mine.tolist()):
        eng.fill_splitmix64(_DevView(bt.data_ptr()), int(L[k]), f + 1, offset=int(bofs[k]))
    eng.synchronize()
    # basis sums (reference sizing: B = 700 for every file here) and targets
    recs, total = eng.block_sums_device(_DevView(bt.data_ptr(), tb), [(int(o), int(n), 0) for o, n in zip(bofs, L)],
                                       SEED)
    rec = recs.download(total * 20).reshape(-1, 20)
    recs.free()
    heads = [rsync_amd.sum_sizes_sqroot(int(n)) for n in L]
    counts = np.array([h.count for h in heads], np.int64)
    first = np.concatenate([[0], np.cumsum(counts)[:-1]])
    s1 = rec[:, :4].copy().view("<u4").reshape(-1)
    s2 = rec[:, 4:].copy()
    tags = ((s1 & 0xFFFF) + (s1 >> 16)) & 0xFFFF
    fob = np.repeat(np.arange(len(L)), counts)
    order = np.lexsort((tags, fob))  # per file, stable by tag (sender.go:60-83)
    targets = (order - first[fob[order]]).astype(np.int32)
    # sources: one deletion, then ~50 % of the bytes overwritten in runs
    rng = np.random.default_rng(40 + rank)
    d = rng.integers(1, 64, len(L))
    p = (rng.random(len(L)) * (L - d)).astype(np.int64)
    Ls = L - d
    sofs = np.concatenate([[0], np.cumsum(a16(Ls))[:-1]])
    ts = int(a16(Ls).sum())
    st = torch.empty(ts, dtype=torch.uint8, device=dev)
    for k in range(len(L)):
        so, bo, pk, dk, lk = int(sofs[k]), int(bofs[k]), int(p[k]), int(d[k]), int(L[k])
        st[so:so + pk] = bt[bo:bo + pk]
        st[so + pk:so + lk - dk] = bt[bo + pk + dk:bo + lk]
    nr = np.maximum(1, np.round(0.5 * Ls / 700).astype(np.int64))
    rf = np.repeat(np.arange(len(L)), nr)
    rl = rng.integers(1, 1401, rf.size)
    rl = np.minimum(rl, Ls[rf])
    rs = sofs[rf] + (rng.random(rf.size) * (Ls[rf] - rl + 1)).astype(np.int64)
    diff = torch.zeros(ts + 1, dtype=torch.int32, device=dev)
    diff.index_add_(0, torch.from_numpy(rs).to(dev), torch.ones(rf.size, dtype=torch.int32, device=dev))
    diff.index_add_(0, torch.from_numpy(rs + rl).to(dev), torch.full((rf.size,), -1, dtype=torch.int32, device=dev))
    cov = diff.cumsum(0, dtype=torch.int32)[:-1] > 0
    del diff
    rnd = torch.empty_like(st)
    torch.cuda.synchronize()
    eng.fill_splitmix64(_DevView(rnd.data_ptr()), ts, 0xC0FFEE + rank)
    eng.synchronize()
    st = torch.where(cov, rnd, st)
    touched = float(cov.sum()) / float(Ls.sum())
    del rnd, cov, bt
    torch.cuda.synchronize()
    jobs = []
    for k in range(len(L)):
        c0, c = int(first[k]), int(counts[k])
        jobs.append((_DevView(st.data_ptr() + int(sofs[k])), int(Ls[k]), heads[k], s1[c0:c0 + c], s2[c0:c0 + c],
                     targets[c0:c0 + c]))
    batch = SearchBatch(eng, jobs, device=True)
    eng.set_kernel_timing(True)
    for _ in range(2):
        _check(batch.run(SEED), eng.ctx)
    steps = max(1, min(args.steps, 20))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.kernel_times(reset=True)
    call_ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        c0 = time.perf_counter()
        _check(batch.run(SEED), eng.ctx)
        call_ms.append(round((time.perf_counter() - c0) * 1e3, 3))
    dt = time.perf_counter() - t0
    kt = eng.kernel_times(reset=True)
    eng.set_kernel_timing(False)
    nmatch = sum(batch.n_matches(k) for k in range(batch.n))
    scanned = float(Ls.sum())
    if world > 1:
        tt = torch.tensor([dt, scanned], dtype=torch.float64)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:])
        dt, scanned = float(tt[0]), float(tt[1])
    kernel_ms = kt["roll_ms"] / steps  # every small-file launch of one call
    src_bytes = float(Ls.sum())
    cpu, parity, pipeline = None, None, None
    if rank == 0:
        # the same files' first 2000 through the large-file pipeline, for
        # comparison (rsg_testing_set_search_path 1: one roll, confirmation
        # and walk per file)
        sub = SearchBatch(eng, jobs[:2000], device=True)
        eng.set_search_path(1)
        t1 = time.perf_counter()
        _check(sub.run(SEED), eng.ctx)
        t_pipe = time.perf_counter() - t1
        eng.set_search_path(0)
        pipeline = {"files": 2000, "gib_s": round(float(Ls[:2000].sum()) / t_pipe / GIB, 3),
                    "matches_equal": all(sub.matches(k) == batch.matches(k) for k in range(2000))}
    if rank == 0 and not args.no_cpu:
        # cpu_baseline leg: the C restatement of hashSearch on a bounded sample
        # of the files, which also checks the benchmarked match lists
        from oracle import oracle as orc
        t_cpu, done, k, eq, checked = 0.0, 0, 0, True, 0
        while k < len(L) and (t_cpu < args.cpu_seconds or k < 512):
            src = st[int(sofs[k]):int(sofs[k]) + int(Ls[k])].cpu().numpy()
            h, (c0, c) = heads[k], (int(first[k]), int(counts[k]))
            c_0 = time.perf_counter()
            om, _, _ = orc.hash_search(src, h.astuple(), s1[c0:c0 + c], s2[c0:c0 + c], targets[c0:c0 + c], SEED)
            t_cpu += time.perf_counter() - c_0
            done += src.size
            eq &= om == batch.matches(k)
            checked += 1
            k += 1
        parity = {"files_compared": checked, "equal": bool(eq)}
        cpu = {"value": round(done / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
               "cpu_model": cpu_model(),
               "sample": f"first {checked} files of the set vs their basis sums, oracle/rsg_oracle.c orc_hash_search "
                         f"(scalar C restatement of match.go:21-282), 1 thread, {t_cpu:.1f} s"}
    if rank == 0:
        print(json.dumps({"metric": "GiB/s source scanned (sender rolling match), device-resident",
                          "value": round(scanned * steps / dt / GIB, 2), "unit": "GiB/s", "n_gpus": world,
                          "steps": steps, "higher_is_better": True, "scaling": "strong", "dtype": "u32",
                          "ms_per_step": round(dt * 1e3 / steps, 3), "call_ms": call_ms,
                          "data": f"synthetic (splitmix64 bases; sources: one 1-63 byte deletion, "
                                  f"{touched:.0%} of bytes overwritten in 1-1400 byte runs)",
                          "config": {"workload": "cfg4-sender: 100k sources of 4-64 KiB vs 50%-modified bases, "
                                                 "B = SumSizesSqroot (700)", "files": NF,
                                     "rank0_files": int(len(L)), "rank0_bytes": int(src_bytes),
                                     "matches_per_pass": nmatch,
                                     "call": "rsg_hash_search_batch_device, one call per pass (sums and targets "
                                             "in host memory, match lists to host arrays)"},
                          "roofline": {"bound": "hbm", "kernel": "search_small_kernel (roll + confirmation + walk, "
                                                                 "one wave per file)",
                                       "note": "per call: every launch of the small-file kernel; the kernel is "
                                               "VALU-bound, frac is its HBM fraction as the metric's unit",
                                       "achieved": round(src_bytes / (kernel_ms * 1e-3) / 1e9, 1),
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": round(src_bytes / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       "traffic": committed_traffic("search_small_kernel_cfg4s_bytes_per_call"),
                                       "kernel_ms_per_call": round(kernel_ms, 4),
                                       "launches_per_call": kt["roll_launches"] // steps,
                                       "algorithmic_bytes_per_call": int(src_bytes)},
                          "pipeline_first_2000_files": pipeline,
                          "oracle_parity": parity,
                          "cpu_baseline": cpu}), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


ROLL_ISSUE_NS = 1.91  # measured, see roll_valu_issue


def roll_valu_issue(roll_ms, world):
    """The roll's VALU-issue bound (it is VALU-issue-bound, not HBM-bound,
    DESIGN.md §4.2): SQ_INSTS_VALU per launch from the committed PMC pass of
    the cfg3 bench (profiles/counters.json; not measured in this run) x 2
    cycles per wave64 instruction (two waves interleaving,
    MI355X_MICROARCH.md) / the SIMDs of the roll's CUs / the clock -> the
    floor; frac = floor / the measured roll time."""
    try:
        c = json.load(open(os.path.join(ROOT, "profiles", "counters.json")))["roll_packed_kernel_cfg3"]
    except Exception:
        return None
    simds = 4 * int(c["roll_cus"])
    floor_ms = float(c["valu_wave_insts_per_launch"]) * 2 / simds / (float(c["clock_ghz"]) * 1e9) * 1e3
    # The same count at the issue interval measured for the roll's own
    # instructions (tools/valu_issue.hip, profiles/r04za_valu_issue.txt: 8
    # waves per SIMD, 16 independent chains each): v_perm / v_pk_* / SDWA /
    # v_add3 / v_dot4 alone 1.97 ns per wave-instruction per SIMD, v_xor /
    # v_and / v_add alone 1.17 ns, an alternating mix of the two kinds 1.91 ns
    # (the cheap kind gains nothing beside the other).  1.91 ns is the floor of
    # this mix, whatever the clock did.
    floor_meas_ms = float(c["valu_wave_insts_per_launch"]) * ROLL_ISSUE_NS * 1e-9 / simds * 1e3
    return {"valu_wave_insts_per_launch": c["valu_wave_insts_per_launch"], "simds": simds,
            "clock_ghz": c["clock_ghz"], "floor_ms": round(floor_ms, 4), "frac": round(floor_ms / roll_ms, 4),
            "measured_issue_ns": ROLL_ISSUE_NS, "floor_ms_measured_issue": round(floor_meas_ms, 4),
            "frac_measured_issue": round(floor_meas_ms / roll_ms, 4),
            "issue_source": "profiles/r04za_valu_issue.txt (tools/valu_issue.hip)",
            "source": c.get("source")}


def cfg3_traffic():
    """HBM bytes per roll launch from the committed PMC pass of the cfg3 bench
    (FETCH_SIZE x 2, profiles/traffic.json; not measured in this run)."""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
        return int(t["roll_packed_kernel_cfg3_bytes_per_launch"])
    except Exception:
        return None


def committed_traffic(key):
    """HBM bytes per launch of a workload's kernel from the committed rocprofv3
    PMC passes (FETCH_SIZE x 2 + WRITE_SIZE, profiles/traffic.json, written by
    tools/summarize_profile.py --traffic-key); not measured in this run."""
    try:
        return int(json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))[key])
    except Exception:
        return None


def cfg4_traffic(world, records):
    """Rank 0's HBM bytes per launch (1 GPU only: the profile is of one rank's
    whole set)."""
    return committed_traffic("block_sums_kernel_cfg4_bytes_per_launch") if world == 1 else None


def bench_mixed(args, rank, world, local):
    """cfg4: 100 000 files of uniform length in [4096, 65536] (PRNG seed 4),
    B = 700, block sums with the file list sharded by bytes over the ranks
    (rsync_amd.dist.shard_layout: contiguous block ranges, so rank order of
    the records is the global order; strong scaling, total work fixed), each
    rank's range cut into --batches batches.  Each rank's files sit back to
    back at 16-byte aligned offsets of one arena; a piece that starts inside a
    file starts on a block boundary, so it is planned as a file of its own
    with the same blocks.  Reported beside cfg2, never as the headline.
    Three numbers: kernel-only (the value), and the records delivered while
    the next batch hashes -- gathered to rank 0 over RCCL, or copied to host
    by every rank in parallel."""
    import torch
    import torch.distributed as dist
    import rsync_amd
    from rsync_amd.dist import ShardedBlockSums, rank_arena, shard_layout
    NF = 100_000
    lengths = np.random.default_rng(4).integers(4096, 65537, NF).tolist()
    lay = shard_layout(lengths, world, max(1, args.batches if args.batches is not None else (1 if world == 1 else 4)),
                       BLOCK_LEN)
    eng = rsync_amd.Engine(local)
    stream = torch.cuda.Stream(device=local)
    sptr = stream.cuda_stream
    pos, arena_bytes = rank_arena(lengths, lay, rank)
    arenas = [eng.alloc(arena_bytes) for _ in range(2)]
    for a in arenas:
        for f, o in pos.items():
            eng.fill_splitmix64(a, lengths[f], f + 1, offset=o, stream=sptr)
    sb = ShardedBlockSums.from_layout(eng, lay, rank, pos, arena_bytes)
    recs = eng.alloc(max(sb.my_records, 1) * rsync_amd.RECORD_BYTES)
    mine = [p for g in lay.batches[rank] for p in g]
    my_bytes = sum(p.length for p in mine)
    # kernel-only step: the rank's whole share as ONE launch (the batches
    # exist for the delivery modes below)
    whole = eng.plan([(pos[p.file] + p.offset, p.length, p.block_len) for p in mine], arena_bytes) if mine else None
    eng.synchronize(sptr)

    def kernel_step(i):
        if whole is not None:
            whole.run(arenas[i & 1], SEED, recs, stream=sptr)
    for i in range(max(args.warmup, 20)):
        kernel_step(i)
    eng.synchronize(sptr)
    eng.block_sums_fallbacks(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        kernel_step(i)
    ev1.record(stream)
    eng.synchronize(sptr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    fallbacks = eng.block_sums_fallbacks(reset=True)
    wall, kernel_ms = max_over_ranks(world, wall, kernel_ms)
    total = sum(lengths)
    cpu = None
    if rank == 0 and not args.no_cpu:
        # cpu_baseline leg: the oracle on a bounded sample of this rank's
        # pieces, which also spot-checks the benchmarked records
        from oracle import oracle as orc
        lib = orc.lib()
        t_cpu, done, k, parity = 0.0, 0, 0, True
        first = np.cumsum([0] + [p.b1 - p.b0 for p in mine]).tolist()
        while t_cpu < args.cpu_seconds / 2 and k < 4 * len(mine):
            j = k % len(mine)
            p = mine[j]
            data = orc.splitmix64_bytes(p.file + 1, lengths[p.file])[p.offset:p.offset + p.length]
            data = np.ascontiguousarray(data)
            cnt = p.b1 - p.b0
            out = np.empty(cnt * 20, np.uint8)
            c0 = time.perf_counter()
            lib.orc_block_sums(orc._ptr(data), data.size, BLOCK_LEN, orc._i32(SEED), orc._ptr(out))
            t_cpu += time.perf_counter() - c0
            done += data.size
            if k < 64:
                parity &= bool((recs.download(cnt * 20, offset=first[j] * 20) == out).all())
            k += 1
        cpu = {"value": round(done / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"{k} pieces of rank 0's cfg4 shard at B=700, oracle/rsg_oracle.c orc_block_sums, "
                         f"1 thread, {t_cpu:.1f} s", "gpu_parity_on_sample": parity}
    algo = my_bytes + sb.my_records * rsync_amd.RECORD_BYTES

    def line(more):
        d = {
            "metric": "GiB/s block-checksummed (weak+MD4), device-resident, at 1/2/4/8 MI355X",
            "value": round(total * args.steps / wall / GIB, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {"workload": "cfg4: 100k files, lengths uniform in [4096, 65536], B=700, block sums, "
                                   "file list sharded by bytes", "files": NF, "total_bytes": total,
                       "rank0_pieces": len(mine), "rank0_records": sb.my_records, "batches_per_rank": lay.nbatch,
                       "parallelism": f"file list sharded, {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(algo / (kernel_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": cfg4_traffic(world, sb.my_records),
                         "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": int(algo)},
            "fallback_census_rank0": {"staged_waves": fallbacks[0], "park_tiles": fallbacks[1]},
            "cpu_baseline": cpu}
        d.update(more)
        return d

    more = {}
    if not args.no_delivery:
        gfirst = np.concatenate([[0], np.cumsum([-(-ln // BLOCK_LEN) for ln in lengths])])

        def oracle_check(got):
            """orc_block_sums of 16 files spread over the list (every rank's
            share) against their gathered records at their global offsets."""
            from oracle import oracle as orc
            ok, picks = True, np.linspace(0, NF - 1, 16).astype(int).tolist()
            for f in picks:
                want = orc.block_sums(orc.splitmix64_bytes(f + 1, lengths[f]), BLOCK_LEN, SEED)
                o = int(gfirst[f]) * rsync_amd.RECORD_BYTES
                ok &= bytes(got[o:o + len(want)]) == want
            return {"oracle_files_checked": len(picks), "oracle_equal": bool(ok)}
        more["delivery"] = guarded_delivery(args, eng, sb, arenas, recs, world, rank, float(total),
                                            lay.total_records, lambda d: print(json.dumps(line({"delivery": d})),
                                                                               flush=True), oracle_check)
    if rank == 0:
        print(json.dumps(line(more)), flush=True)
    sb.close()
    if whole is not None:
        whole.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def bench_long(args, rank, world, local):
    """cfg5: 8 x 32 GiB files at B = 128 KiB, one file per GPU (weak scaling:
    rank r hashes its own 32 GiB file, generated on the device).  One step =
    one launch over the whole file (262 144 blocks of 2049 MD4 compressions).
    Parity by sampled blocks (1024 random + the last) against the oracle, which
    also times the CPU baseline on them.  Reported beside cfg2."""
    import torch
    import torch.distributed as dist
    import rsync_amd
    size, B = 32 << 30, 131072
    eng = rsync_amd.Engine(local)
    stream = torch.cuda.Stream(device=local)
    sptr = stream.cuda_stream
    arena = eng.alloc(size)
    eng.fill_splitmix64(arena, size, 5000 + rank, stream=sptr)
    plan = eng.plan([(0, size, B)], size)
    nrec = plan.total_records
    recs = eng.alloc(nrec * rsync_amd.RECORD_BYTES)
    eng.synchronize(sptr)
    steps = max(1, args.steps)
    for _ in range(max(3, min(args.warmup, 40))):
        plan.run(arena, SEED, recs, stream=sptr)
    eng.synchronize(sptr)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        plan.run(arena, SEED, recs, stream=sptr)
    ev1.record(stream)
    eng.synchronize(sptr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / steps
    if world > 1:
        tt = torch.tensor([wall, kernel_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kernel_ms = float(tt[0]), float(tt[1])
    cpu, parity = None, None
    if rank == 0:
        from oracle import oracle as orc
        lib = orc.lib()
        rng = np.random.default_rng(55)
        sample = sorted(set(rng.integers(0, nrec, 1024).tolist()) | {nrec - 1})
        got_all = recs.download(nrec * 20).reshape(-1, 20)
        out = np.empty(20, np.uint8)
        t_cpu, parity = 0.0, True
        for b in sample:
            blk = arena.download(B, offset=b * B)
            c0 = time.perf_counter()
            lib.orc_block_sums(orc._ptr(blk), blk.size, B, orc._i32(SEED), orc._ptr(out))
            t_cpu += time.perf_counter() - c0
            parity &= bool((got_all[b] == out).all())
        if not args.no_cpu:
            cpu = {"value": round(len(sample) * B / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                   "sample": f"{len(sample)} sampled 128 KiB blocks of rank 0's file (1024 random + the last), "
                             f"oracle/rsg_oracle.c orc_block_sums, 1 thread, {t_cpu:.1f} s"}
        algo = size + nrec * rsync_amd.RECORD_BYTES
        print(json.dumps({
            "metric": "GiB/s block-checksummed (weak+MD4), device-resident, at 1/2/4/8 MI355X",
            "value": round(world * size * steps / wall / GIB, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {"workload": "cfg5: one 32 GiB file per GPU (8 x 32 GiB at 8 GPUs), B=131072, weak+MD4",
                       "file_bytes": size, "block_len": B, "records_per_gpu": nrec,
                       "parallelism": f"one file per GPU, {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(algo / (kernel_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": committed_traffic("block_sums_kernel_cfg5_bytes_per_launch") if world == 1 else None,
                         "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": int(algo)},
            "sampled_block_parity": {"blocks": len(sample), "equal": parity},
            "cpu_baseline": cpu}), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def bench_filesums(args, rank, world, local):
    """Whole-file MD4 over cfg4's file set: 100 000
    files of uniform length in [4096, 65536] (PRNG seed 4), one lane per file,
    both modes -- seeded MD4(int32_LE(seed) || file), the transfer's file sum
    (match.go:52-53, receiver.go:117-120), and plain MD4(file), the
    --checksum file list (rsyncchecksum.go:60-66).  One step = one
    rsg_file_sums_device call (descriptor upload + launch + wait) over the
    whole set, resident in HBM.  Spot parity and the CPU baseline use the
    oracle's orc_file_sum."""
    import ctypes
    import rsync_amd
    from rsync_amd import _lib
    NF = 100_000
    lengths = np.random.default_rng(4).integers(4096, 65537, NF).tolist()
    eng = rsync_amd.Engine(local)
    for opt in args.search_option:
        name, value = opt.split("=")
        eng.set_option(name, int(value))
    offs, at = [], 0
    for n in lengths:
        offs.append(at)
        at += (n + 15) & ~15
    arenas = [eng.alloc(at) for _ in range(2)]
    for k, a in enumerate(arenas):
        for f in range(0, NF, 1):
            eng.fill_splitmix64(a, lengths[f], f + 1, offset=offs[f])
    eng.synchronize()
    desc = (_lib.File * NF)()
    for i, (o, n) in enumerate(zip(offs, lengths)):
        desc[i].offset, desc[i].len = o, n
    out = eng.alloc(NF * 16)
    total = sum(lengths)
    res = {}
    for mode, name in ((_lib.FILESUM_SEEDED, "seeded"), (_lib.FILESUM_PLAIN, "plain")):
        def call(i):
            _lib.check(_lib.lib.rsg_file_sums_device(eng.ctx, ctypes.c_void_p(arenas[i & 1].ptr), at, desc, NF,
                                                     mode, ctypes.c_int32(SEED),
                                                     ctypes.c_void_p(out.ptr)), eng.ctx)
        for i in range(5):
            call(i)
        steps = max(4, min(args.steps, 40))
        t0 = time.perf_counter()
        for i in range(steps):
            call(i)
        dt = (time.perf_counter() - t0) / steps
        # the kernel alone: HIP events around each launch on its stream (a
        # separate pass, so the per-call time above carries no event cost)
        eng.set_kernel_timing(True)
        eng.kernel_times(reset=True)
        for i in range(steps):
            call(i)
        kt = eng.kernel_times(reset=True)
        eng.set_kernel_timing(False)
        kms = kt["filesums_ms"] / max(kt["filesums_launches"], 1)
        res[name] = {"ms_per_call": round(dt * 1e3, 4), "gib_s": round(total / dt / GIB, 2),
                     "hbm_frac_8tbs": round(total / dt / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel_ms": round(kms, 4),
                     "kernel_hbm_frac_8tbs": round(total / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    # parity (plain mode is the last one run, on arena (steps - 1) & 1) and the CPU baseline
    from oracle import oracle as orc
    last = arenas[(steps - 1) & 1]
    dig = out.download(NF * 16).reshape(NF, 16)
    parity, t_cpu, done, k = True, 0.0, 0, 0
    rng = np.random.default_rng(9)
    while t_cpu < args.cpu_seconds / 2 and k < 4096:
        f = int(rng.integers(0, NF))
        data = last.download(lengths[f], offset=offs[f])
        c0 = time.perf_counter()
        want = orc.file_sum(_lib.FILESUM_PLAIN, 0, data)
        t_cpu += time.perf_counter() - c0
        done += lengths[f]
        if k < 256:
            parity &= bytes(dig[f]) == want
        k += 1
    print(json.dumps({
        "metric": "GiB/s whole-file MD4 (lane per file), device-resident", "value": res["seeded"]["gib_s"],
        "unit": "GiB/s", "n_gpus": 1, "steps": steps, "higher_is_better": True, "dtype": "u32",
        "data": "synthetic (splitmix64 bytes generated on device)",
        "config": {"workload": "whole-file MD4 over cfg4's 100k files (4-64 KiB)", "files": NF, "total_bytes": total,
                   "call": "rsg_file_sums_device, descriptors uploaded and waited on per call",
                   **({"search_options": args.search_option} if args.search_option else {})},
        "modes": res, "spot_parity": {"files": min(k, 256), "equal": parity},
        "roofline": {"bound": "hbm", "kernel": "file_sums_staged<seeded>",
                     "achieved": round(total / (res["seeded"]["kernel_ms"] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": res["seeded"]["kernel_hbm_frac_8tbs"],
                     "traffic": committed_traffic("file_sums_kernel_cfg4set_bytes_per_launch"),
                     "kernel_ms": res["seeded"]["kernel_ms"], "algorithmic_bytes_per_launch": int(total),
                     "note": "value = per call (descriptor staging + lane order + upload + launch + wait); "
                             "roofline = the kernel alone (HIP events)"},
        "cpu_baseline": {"value": round(done / t_cpu / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                         "sample": f"{k} random files of the set, oracle/rsg_oracle.c orc_file_sum (plain), "
                                   f"1 thread, {t_cpu:.1f} s"}}), flush=True)
    eng.close()


def bench_receive(args, rank, world, local):
    """receiveData (receiver.go:98-188) latency and batch
    rate: token application on the host plus the seeded whole-file MD4 check
    (receiver.go:117-120).  MD4 is one serial chain per file: a single file
    (rsg_receive_data) is hashed on the host as its tokens are applied (on the
    GPU it would get one lane, ~10x slower than a core: measured here too with
    recv_md4 = GPU (rsg_testing_search_option 5) on the 1 MiB file); the batched call
    (rsg_receive_data_batch) hashes many files at once on the GPU, one lane
    per file, and sends a batch's few large files to host threads when that
    is faster (its cost split).  Streams: every block of an identical basis
    matched, i.e. the whole file is rebuilt from the basis."""
    import rsync_amd
    import cases
    from oracle import oracle as orc
    eng = rsync_amd.Engine(local)
    seed = SEED
    res = {}

    def stream_for(data):
        head = rsync_amd.sum_sizes_sqroot(data.size)
        B = head.block_len
        matches = [(i * B, i) for i in range(head.count)]
        c0 = time.perf_counter()
        fsum = orc.file_sum(1, seed, data)  # the sender's whole-file sum; also the CPU MD4 baseline
        t_cpu = time.perf_counter() - c0
        return rsync_amd.encode_tokens(data, head, matches) + fsum, head, t_cpu

    def timed(fn, reps=1):
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        return r, best

    for name, size in (("1MiB", 1 << 20), ("1GiB", 1 << 30)):
        data = cases.splitmix64_bytes(77, size)
        stream, head, t_cpu = stream_for(data)
        eng.receive_data(stream, head, data, seed)  # warm-up
        (out, used), dt = timed(lambda: eng.receive_data(stream, head, data, seed), 5 if size <= (1 << 20) else 2)
        r = {"s": round(dt, 4), "gib_s": round(size / dt / GIB, 4),
             "equal": out == data.tobytes() and used == len(stream),
             "md4_on": "host (fused with token application)",
             "cpu_md4_1core_s": round(t_cpu, 4), "cpu_md4_1core_gib_s": round(size / t_cpu / GIB, 4)}
        if size <= (1 << 20):
            eng.set_option("recv_md4", 1)
            try:
                (out, used), dg = timed(lambda: eng.receive_data(stream, head, data, seed), 5)
            finally:
                eng.set_option("recv_md4", 0)
            r["gpu_one_lane_s"] = round(dg, 4)
        res[f"single_{name}"] = r
        del data, stream, out

    def batch(tag, n, size):
        files = [cases.splitmix64_bytes(1000 + f, size) for f in range(n)]
        jobs, t_cpu = [], 0.0
        for d in files:
            st, head, tc = stream_for(d)
            jobs.append((st, head, d))
            t_cpu += tc
        # one whole call first: the staging buffers are allocated and the
        # callers' output pages (np.empty per call) come back from the heap
        # warm, as for every later call, whichever mode runs first
        eng.receive_data_batch(jobs, seed)
        got, dt = timed(lambda: eng.receive_data_batch(jobs, seed), 3)
        res[tag] = {"s": round(dt, 4), "gib_s": round(n * size / dt / GIB, 3),
                    "equal": all(g[0] == d.tobytes() for g, d in zip(got, files)),
                    "cpu_md4_1core_gib_s": round(n * size / t_cpu / GIB, 4)}
        if n >= 64:
            for mode in ("host", "gpu"):
                eng.set_option("recv_md4", 2 if mode == "host" else 1)
                try:
                    _, dh = timed(lambda: eng.receive_data_batch(jobs, seed), 3)
                finally:
                    eng.set_option("recv_md4", 0)
                res[tag]["all_host_threads_gib_s" if mode == "host" else "all_gpu_lanes_gib_s"] = \
                    round(n * size / dh / GIB, 3)

    batch("batch_1024x1MiB", 1024, 1 << 20)
    batch("batch_4x256MiB", 4, 256 << 20)
    print(json.dumps({"metric": "receiveData (token application + seeded whole-file MD4 check)",
                      "value": res["batch_1024x1MiB"]["gib_s"], "unit": "GiB/s", "n_gpus": 1,
                      "higher_is_better": True, "dtype": "u32",
                      "data": "synthetic (splitmix64 files, identical basis: every block a match token)",
                      "config": {"workload": "receive: single 1 MiB / 1 GiB files (latency), 1024 x 1 MiB and "
                                             "4 x 256 MiB batches"},
                      "results": res}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
