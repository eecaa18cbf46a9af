// rsg_match.cpp -- sender hash search (internal/sender/match.go:21-230) on the GPU.
//
// Division of labour:
//   GPU  weak sum at every offset + exact-equivalent filter against the basis
//        sums (rsg_match_kernels.hip), and the strong sum (MD4 || seed) plus
//        Checksum1 of every window the greedy walk needs to confirm
//        (rsg_blocksums.hip, the same kernel the receiver uses).
//   host the greedy walk of match.go over the (sorted, sparse) candidate
//        offsets: O(candidates), no hashing.
// The result is exactly the (offset, block index) sequence hashSearch passes
// to matched(): a visited offset q (q = 0, or q < end = size + 1 - lastLen,
// match.go:70) matches the FIRST block i in `targets` order with
// Sum1_i == weak(q), Len_i == min(B, size - q) and MD4(window || seed)[:s2len]
// == Sum2_i[:s2len] (match.go:108-136); after a match the next visited offset
// is q + Len_i (match.go:158), otherwise q + 1.
#include <errno.h>
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <functional>
#include <future>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rsg_testing.h"
#include "rsg_host.h"

using namespace rsgh;
using rsg::DevFile;
using rsg::kRecordBytes;
using rsg::kScanTile;
using rsg::TileAgg;
using rsg::TilePrefix;

namespace rsgh {

hipEvent_t timed_begin(rsg_ctx *ctx, hipStream_t stream) {
    if (!ctx->timing) return nullptr;
    hipEvent_t a = nullptr;
    if (hipEventCreate(&a) != hipSuccess) return nullptr;
    if (hipEventRecord(a, stream) != hipSuccess) {
        hipEventDestroy(a);
        return nullptr;
    }
    return a;
}

void timed_end(rsg_ctx *ctx, hipEvent_t a, hipStream_t stream, int kind) {
    if (!a) return;
    hipEvent_t b = nullptr;
    if (hipEventCreate(&b) != hipSuccess || hipEventRecord(b, stream) != hipSuccess) {
        if (b) hipEventDestroy(b);
        hipEventDestroy(a);
        return;
    }
    std::lock_guard<std::mutex> g(ctx->spans_mu);
    ctx->spans.push_back({a, b, kind});
}

}  // namespace rsgh

namespace {

constexpr uint32_t kCandCap = 1u << 22;      // candidates per roll launch (32 MiB)
constexpr uint64_t kSparseBatch = 1u << 16;  // windows per verification batch
constexpr uint64_t kDenseBatch = 1u << 14;   // reach-set windows per dense round trip (Walker)

// RSG_TIMING=1 prints the host-side phase times of each search to stderr.
struct PhaseTimer {
    bool on;
    std::chrono::steady_clock::time_point t0, t;
    PhaseTimer() : on(getenv("RSG_TIMING") != nullptr), t0(std::chrono::steady_clock::now()), t(t0) {}
    void mark(const char *what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[rsg] %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};


struct Search {
    PhaseTimer pt;
    rsg_ctx *ctx;
    SearchSlot *sl;
    hipStream_t st;
    const uint8_t *d_src;
    uint64_t size;
    rsg_sum_head head;
    int32_t seed;
    int64_t end;  // visited offsets are q < end (end >= 1: offset 0 is always visited)
    std::vector<rsg_match> out;
    hipStream_t side = nullptr;  // prefix pass (beside the previous file's roll)
    hipStream_t copy = nullptr;  // candidate read-back
    hipStream_t cst = nullptr;   // confirmation batches (the compute stream)
    // Called once, right after the first confirmation batch is issued (or at
    // the end of finish() if none is): the batch issues a later job there.
    std::function<rsg_status()> hook;        // issues the next job's stage 1 (may wait for its tables)
    std::function<bool()> hook_ready;        // hook() would not wait
    std::function<rsg_status()> tail;        // set by finish(): the rest of the job (wait + walk), any thread
    // device tables inside the slot's blob
    uint64_t off_filter = 0, off_filter16 = 0, off_table = 0, off_keys = 0, blob_a_bytes = 0;  // part A
    bool gpu_tab = false;   // part A built on the GPU from the Sum1 copy at off_sum1 (tables_roll)
    uint64_t off_sum1 = 0;
    uint64_t off_groups = 0, off_hi16 = 0, off_sum2 = 0, blob_bytes = 0;                       // part B
    std::future<rsg_status> part_b;  // part B's build (a worker's), if not done inline
    bool part_b_up = false;          // part B's upload is queued
    const uint2 *d_groups = nullptr;
    const uint32_t *d_hi16 = nullptr, *d_filter = nullptr;
    const uint16_t *d_filter16 = nullptr;  // packed roll (nullptr: not built)
    const uint8_t *d_sum2 = nullptr;
    const uint64_t *d_table = nullptr;
    const uint32_t *d_table_keys = nullptr;
    uint32_t ntiles = 0, tile_end = 0, bmask = 0, cus = 256;
    uint32_t roll_grid = 0;    // roll workgroups (0 = one per CU)
    uint32_t confirm_lds = 0;  // dynamic LDS of the confirmation kernel's workgroups
    bool fused = false;  // roll derives its window sums itself (B <= kFusedMaxB)
    bool pending = false;  // prepare() launched the roll of [0, tile_end) and its count read-back
    uint64_t pos0 = 0;     // the walk's first position (a window of rsg_hash_search_fd: carried over)
    uint64_t pos_end = 0;  // its position when finish() (or the tail) is done

    int64_t len_of(int32_t i) const {
        return (i == head.count - 1 && head.rem != 0) ? head.rem : head.block_len;  // sender.go:135-139
    }
    uint32_t window(uint64_t q) const {
        return (uint32_t)std::min<uint64_t>((uint64_t)head.block_len, size - q);  // match.go:114-117
    }
};

// Candidate offsets arrive in atomic-append order: LSD radix sort on 16-bit
// digits (as many passes as the largest offset needs), std::sort for few.
// Bits below `lowbit` are a payload the order need not respect.
void sort_offsets(std::vector<uint64_t> &C, int lowbit = 0) {
    if (C.size() < 4096) {
        std::sort(C.begin(), C.end());
        return;
    }
    uint64_t mx = 0;
    for (uint64_t c : C) mx = std::max(mx, c);
    std::vector<uint64_t> tmp(C.size());
    std::vector<uint32_t> cnt(65537);
    for (int shift = lowbit; shift < 64 && (mx >> shift) != 0; shift += 16) {
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (uint64_t c : C) cnt[((c >> shift) & 0xffffu) + 1]++;
        for (size_t h = 1; h < cnt.size(); h++) cnt[h] += cnt[h - 1];
        for (uint64_t c : C) tmp[cnt[(c >> shift) & 0xffffu]++] = c;
        C.swap(tmp);
    }
}

// Flags of the events the host waits on (spin-waits: a blocking-sync
// event measured no better beside the table builders and walks).
unsigned sync_event_flags() { return hipEventDisableTiming; }

// Issue the next job's stage 1 (its roll queues behind this job's on the
// compute stream) once its tables, built on a worker thread, are ready;
// block = wait for them.  Called at several points of a job's finish so the
// compute stream never runs dry and this thread never idles on the worker.
rsg_status run_hook(Search &S, bool block) {
    if (!S.hook) return RSG_OK;
    if (!block && S.hook_ready && !S.hook_ready()) return RSG_OK;
    const std::function<rsg_status()> h = std::move(S.hook);
    S.hook = nullptr;
    return h();
}

// Part B on the device before the first resolve of this search: waits for its
// build (a worker's) and queues its upload on the confirmation stream.
rsg_status need_resolve_tables(Search &S) {
    if (S.part_b_up) return RSG_OK;
    if (S.part_b.valid()) {
        const rsg_status s = S.part_b.get();
        if (s != RSG_OK) return s;
    }
    // on the side stream, where part A went (an H2D queued on the
    // confirmation stream measured up to 6.5 ms of host blocking), ordered
    // before the confirmation by an event
    SearchSlot &sl = *S.sl;
    if (!sl.tables_b) RSG_HIP(S.ctx, hipEventCreateWithFlags(&sl.tables_b, hipEventDisableTiming));
    RSG_HIP(S.ctx, hipMemcpyAsync((uint8_t *)sl.blob.p + S.off_groups, (uint8_t *)sl.stage.p + S.off_groups,
                                  S.blob_bytes - S.off_groups, hipMemcpyHostToDevice, S.side));
    RSG_HIP(S.ctx, hipEventRecord(sl.tables_b, S.side));
    RSG_HIP(S.ctx, hipStreamWaitEvent(S.cst, sl.tables_b, 0));
    S.part_b_up = true;
    return RSG_OK;
}

// Confirm a batch of candidates (indices into C): Checksum1 + MD4(window ||
// seed) on the GPU, then the first block in targets order whose sums and
// length agree.  res[i]: -2 unknown, -1 no match, else the block index.
rsg_status verify(Search &S, const std::vector<uint64_t> &C, std::vector<int32_t> &res,
                  const std::vector<uint32_t> &idx) {
    if (idx.empty()) return RSG_OK;
    rsg_ctx *ctx = S.ctx;
    // One block per window: the plan is direct (record i = window i).
    HostPlan plan;
    plan.files.resize(idx.size());
    plan.total_blocks = idx.size();
    plan.aligned = false;
    plan.arena_bytes = S.size;
    plan.max_blen = 0;
    plan.lds_reserve = S.confirm_lds;
    std::vector<uint32_t> wlen(idx.size());
    for (size_t i = 0; i < idx.size(); i++) {
        const uint64_t q = C[idx[i]];
        const uint32_t k = S.window(q);
        wlen[i] = k;
        plan.files[i] = DevFile{q, k, i, k, 1};
        plan.max_blen = std::max(plan.max_blen, k);
    }
    plan.nwg = (uint32_t)((idx.size() + rsg::kBlockSumThreads - 1) / rsg::kBlockSumThreads);
    plan.wg_file.resize(plan.nwg + 1);
    for (uint32_t w = 0; w <= plan.nwg; w++)
        plan.wg_file[w] = (uint32_t)std::min<uint64_t>((uint64_t)w * rsg::kBlockSumThreads, idx.size() - 1);
    rsg_status s;
    if ((s = need_resolve_tables(S)) != RSG_OK) return s;
    S.pt.mark("v.plan");
    // the slot's own confirmation scratch: this may run on a worker thread
    // (a job's tail) while the calling thread queues another slot's
    // confirmation; the slot's results buffers were consumed before the walk
    SearchSlot &sl = *S.sl;
    if ((s = ensure_dev(ctx, sl.cfiles, plan.files.size() * sizeof(DevFile) + 32)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, sl.cwg, plan.wg_file.size() * sizeof(uint32_t) + 4)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, sl.cout, plan.total_blocks * kRecordBytes)) != RSG_OK) return s;
    RSG_HIP(ctx, hipMemcpyAsync(sl.cfiles.p, plan.files.data(), plan.files.size() * sizeof(DevFile),
                                hipMemcpyHostToDevice, S.cst));
    RSG_HIP(ctx, hipMemcpyAsync(sl.cwg.p, plan.wg_file.data(), plan.wg_file.size() * sizeof(uint32_t),
                                hipMemcpyHostToDevice, S.cst));
    if ((s = ensure_dev(ctx, sl.cfb, rsg::block_sums_scratch_bytes(plan.total_blocks))) != RSG_OK) return s;
    hipEvent_t t0 = timed_begin(ctx, S.cst);
    if (ctx->timing) {
        std::lock_guard<std::mutex> g(ctx->spans_mu);
        ctx->stat_windows += idx.size();
    }
    if ((s = launch_plan(ctx, plan, sl.cfiles.p, sl.cwg.p, S.d_src, S.seed, sl.cout.p, sl.cfb.p, S.cst)) != RSG_OK)
        return s;
    // Each window resolves on the GPU to the first block in targets order with
    // equal Sum1, length and sum2[:s2len] (match.go:108-136); only the block
    // indices come back.
    if ((s = ensure_dev(ctx, sl.res, plan.total_blocks * 4)) != RSG_OK) return s;
    RSG_HIP(ctx, rsg::launch_resolve((const uint8_t *)sl.cout.p, (const DevFile *)sl.cfiles.p,
                                     plan.total_blocks, S.d_groups, S.d_hi16, S.d_sum2,
                                     S.head.count, S.head.block_len, S.head.rem, S.head.s2len,
                                     (int32_t *)sl.res.p, S.cst));
    timed_end(ctx, t0, S.cst, 1);
    if ((s = ensure_pin(ctx, sl.hres, plan.total_blocks * 4)) != RSG_OK) return s;
    const int32_t *found = (const int32_t *)sl.hres.p;
    RSG_HIP(ctx, hipMemcpyAsync(sl.hres.p, sl.res.p, plan.total_blocks * 4, hipMemcpyDeviceToHost, S.cst));
    if (!S.sl->confirmed) RSG_HIP(ctx, hipEventCreateWithFlags(&S.sl->confirmed, sync_event_flags()));
    RSG_HIP(ctx, hipEventRecord(S.sl->confirmed, S.cst));
    if ((s = run_hook(S, false)) != RSG_OK) return s;  // the next job's roll, if its tables are built
    RSG_HIP(ctx, hipEventSynchronize(S.sl->confirmed));
    S.pt.mark("v.kernel");
    for (size_t i = 0; i < idx.size(); i++) res[idx[i]] = found[i];
    S.pt.mark("v.resolve");
    return RSG_OK;
}

// Greedy walk over one range's sorted candidates (match.go:93-210 reduced to
// the offsets where the weak sum can hit): visit offset C[i]; a match of
// block b moves the walk to C[i] + Len_b (match.go:158 + the roll), a miss to
// the next candidate.  Results come from `verify` (GPU confirmation) in
// batches; res[i] = -2 until known.
//
// Batching (bounded GPU round trips):
//  * sparse stretches (hashing every pending candidate costs at most twice
//    the span they cover): the next kSparseBatch pending candidates at once;
//  * dense stretches (repetitive data, where a match skips B candidates):
//    (a) the chain of offsets the walk visits if every confirmation
//    succeeds, plus one successor per step (exact on periodic data: 4096
//    matches per round trip), and (b) the reach set: from the interval of
//    positions the walk can be at, the candidates in it plus `width` more,
//    step after step, up to kDenseBatch windows (robust when some of the
//    chain's confirmations fail).  A round trip after which the walk
//    visits no more than `width` candidates before needing another one
//    means a run of failures longer than `width` (dense FALSE candidates:
//    equal weak sums, different MD4): width grows x4 up to kSparseBatch, so
//    such a stretch costs O(log) round trips to reach full batches instead
//    of one round trip per ~2 candidates (round 3's d1 stall: ~240 000
//    round trips of one 32 KiB MD4 chain each).
//  * the sparse test scans up to kSparseBatch pending candidates; a dense
//    verdict is remembered up to the last candidate it scanned, so a dense
//    stretch does not rescan them every round trip.
struct Walker {
    int64_t end = 0;   // visited offsets are < end (match.go:70)
    uint64_t size = 0;
    rsg_sum_head head{};
    std::function<rsg_status(const std::vector<uint32_t> &idx, std::vector<int32_t> &res)> verify;
    std::vector<rsg_match> *out = nullptr;
    uint64_t batches = 0, windows = 0;  // round trips, windows confirmed
    uint64_t dense_until = 0;           // candidates below this offset were judged dense
    uint32_t width = 2;                 // successors per chain step in a dense stretch

    bool spec = false;                  // speculative selection of sparse batches (rsg_ctx::Options::spec)

    uint32_t window(uint64_t q) const { return (uint32_t)std::min<uint64_t>((uint64_t)head.block_len, size - q); }
    int64_t len_of(int32_t i) const { return (i == head.count - 1 && head.rem != 0) ? head.rem : head.block_len; }

    // Speculative selection of sparse batches (rsg_ctx::Options::spec): off
    // by default -- it confirms 15 % fewer windows on cfg3 (19 957 against
    // 23 515 per GiB) but must sort the roll's list before queueing them and
    // costs a round trip where a guess fails, while without it the
    // confirmation is queued straight from the list; cfg3 1014-1038 against
    // 1002-1058 GiB/s, two interleaved rounds (profiles/r05q_cfg3_confirm_ab.txt).
    // Candidate j sits in a chain: another candidate exactly B before or after
    // it, as consecutive matched blocks give (match.go:158 moves the walk
    // from a match at q to q + B).  A random false weak hit almost never does.
    // f / b: monotone cursors (the callers visit j in increasing order), so a
    // selection over n candidates costs O(n), not 2 n binary searches.
    bool chained(const std::vector<uint64_t> &C, size_t j, size_t &f, size_t &b) const {
        const uint64_t B = (uint64_t)head.block_len, c = C[j];
        if (f <= j) f = j + 1;
        while (f < C.size() && C[f] < c + B) f++;
        if (f < C.size() && C[f] == c + B) return true;
        if (c < B) return false;
        while (b < j && C[b] < c - B) b++;
        return b < j && C[b] == c - B;
    }
    // The pending candidates the walk visits from C[i] (visited) on if every
    // chained pending candidate matches a block of length window() and every
    // other one fails; known results are taken as they are.  Confirming only
    // these skips the false weak hits inside matched spans, which the greedy
    // walk jumps over (match.go:158-167); a wrong guess only uncovers
    // candidates the next round trip confirms.
    void spec_batch(const std::vector<uint64_t> &C, const std::vector<int32_t> &res, size_t i,
                    std::vector<uint32_t> &batch) const {
        uint64_t x = C[i];
        size_t f = i + 1, b = 0;
        for (size_t j = i; j < C.size() && batch.size() < kSparseBatch && (int64_t)C[j] < end; j++) {
            const uint64_t c = C[j];
            if (c < x) continue;
            if (res[j] == -2) {
                batch.push_back((uint32_t)j);
                x = chained(C, j, f, b) ? c + window(c) : c + 1;
            } else {
                x = res[j] >= 0 ? c + (uint64_t)len_of(res[j]) : c + 1;
            }
        }
    }

    rsg_status run(const std::vector<uint64_t> &C, uint64_t &pos, std::vector<int32_t> *known) {
        std::vector<int32_t> res = known ? std::move(*known) : std::vector<int32_t>(C.size(), -2);
        size_t i = std::lower_bound(C.begin(), C.end(), pos) - C.begin();
        std::vector<uint32_t> batch;
        uint64_t consumed = 0;     // candidates visited since the last dense round trip
        bool last_dense = false;   // the last round trip was a dense chain
        while (i < C.size()) {
            const uint64_t c = C[i];
            if ((int64_t)c >= end) break;
            if (res[i] == -2) {
                batch.clear();
                bool dense = c < dense_until;
                if (!dense) {
                    uint64_t hashed = 0;
                    size_t j = i;
                    for (; j < C.size() && batch.size() < kSparseBatch && (int64_t)C[j] < end; j++) {
                        if (res[j] == -2) {
                            batch.push_back((uint32_t)j);
                            hashed += window(C[j]);
                        }
                    }
                    const uint64_t span = (j > i ? C[j - 1] - c : 0) + (uint64_t)head.block_len;
                    if (hashed > 2 * span + (1u << 20)) {
                        dense = true;
                        dense_until = C[j - 1];
                    } else {
                        width = 2;  // a sparse stretch: the next dense one starts narrow again
                        if (spec) {
                            batch.clear();
                            spec_batch(C, res, i, batch);
                        }
                    }
                }
                if (dense) {
                    // a pure failure run longer than the successors pushed
                    if (last_dense && consumed <= width)
                        width = (uint32_t)std::min<uint64_t>(4ull * width, kSparseBatch);
                    batch.clear();
                    // (a) the chain of offsets visited if every confirmation
                    // succeeds, plus one successor per step
                    uint64_t x = c;
                    for (int n = 0; n < 4096; n++) {
                        size_t a = std::lower_bound(C.begin() + i, C.end(), x) - C.begin();
                        if (a >= C.size() || (int64_t)C[a] >= end) break;
                        if (res[a] == -2) batch.push_back((uint32_t)a);
                        if (a + 1 < C.size() && (int64_t)C[a + 1] < end && res[a + 1] == -2)
                            batch.push_back((uint32_t)(a + 1));
                        x = C[a] + window(C[a]);
                    }
                    // (b) every offset the walk can reach: from the interval
                    // of possible positions [lo, hi], the candidates in it plus
                    // `width` after it; a success at any of them lands in the
                    // next interval [C[a] + len, C[e - 1] + len]
                    const size_t cap_b = batch.size() + std::max<uint64_t>(kDenseBatch, width);
                    uint64_t lo = c, hi = c;
                    for (int n = 0; n < 4096 && batch.size() < cap_b; n++) {
                        const size_t a = std::lower_bound(C.begin() + i, C.end(), lo) - C.begin();
                        if (a >= C.size() || (int64_t)C[a] >= end) break;
                        size_t e = std::upper_bound(C.begin() + a, C.end(), hi) - C.begin();
                        e = std::min<size_t>(std::max(e, a + 1) + (width - 1), C.size());
                        e = std::min<size_t>(e, a + (cap_b - batch.size()));
                        while (e > a + 1 && (int64_t)C[e - 1] >= end) e--;
                        for (size_t b = a; b < e; b++)
                            if (res[b] == -2) batch.push_back((uint32_t)b);
                        lo = C[a] + window(C[a]);
                        hi = C[e - 1] + window(C[e - 1]);
                    }
                    std::sort(batch.begin(), batch.end());
                    batch.erase(std::unique(batch.begin(), batch.end()), batch.end());
                }
                last_dense = dense;
                consumed = 0;
                batches++;
                windows += batch.size();
                rsg_status s = verify(batch, res);
                if (s != RSG_OK) return s;
            }
            consumed++;
            const int32_t b = res[i];
            if (b >= 0) {
                out->push_back(rsg_match{(int64_t)c, b, 0});
                pos = c + (uint64_t)len_of(b);  // match.go:158 + the roll
                while (i < C.size() && C[i] < pos) i++;  // each candidate is stepped over once
            } else {
                pos = c + 1;
                i++;
            }
        }
        return RSG_OK;
    }
};

rsg_status walk(Search &S, const std::vector<uint64_t> &C, uint64_t &pos, std::vector<int32_t> *known = nullptr) {
    Walker w;
    w.end = S.end;
    w.size = S.size;
    w.head = S.head;
    w.spec = S.ctx->opts.spec;
    w.out = &S.out;
    w.verify = [&S, &C](const std::vector<uint32_t> &idx, std::vector<int32_t> &res) { return verify(S, C, res, idx); };
    return w.run(C, pos, known);
}

rsg_status launch_range(Search &S, uint32_t lo, uint32_t hi);
rsg_status queue_confirm(Search &S, const uint64_t *off, uint32_t m);

// A sparse range's candidates confirmed in one batch with the plan built on
// the GPU (confirm_plan_kernel) from the windows' offsets (the roll's list,
// pinned host memory the roll wrote).  Speculative selection (RSG_CONFIRM_SPEC=1):
// the host sorts the list first and picks the windows the walk will visit
// (Walker::spec_batch: chained candidates assumed to match, the false weak
// hits inside their spans skipped).  C = the sorted distinct offsets, sel[k] =
// the index in C of the k-th confirmed window (results in that order).
rsg_status confirm_all(Search &S, uint32_t n, uint64_t pos, std::vector<uint64_t> &C, std::vector<uint32_t> &sel) {
    SearchSlot &sl = *S.sl;
    rsg_status s;
    Walker w;
    w.end = S.end;
    w.size = S.size;
    w.head = S.head;
    w.spec = S.ctx->opts.spec;
    // Without the speculative selection every candidate is confirmed, so the
    // confirmation is queued straight from the roll's list in its append
    // order, and the host sorts while the GPU hashes (sorting first kept the
    // confirmation waiting 0.25-0.3 ms per 1 GiB file, r05n).
    const bool raw = !w.spec;
    if (raw) {
        sel.clear();
        S.pt.mark("c.select");
        if ((s = queue_confirm(S, (const uint64_t *)sl.list.p, n)) != RSG_OK) return s;
        // (offset << 22 | list index) sorted by offset; sel[k] = the sorted
        // index of list entry k (found[] is in list order)
        static_assert(kCandCap <= (1u << 22), "list index in 22 bits");
        std::vector<uint64_t> key(n);
        const uint64_t *list = (const uint64_t *)sl.list.p;
        for (uint32_t k = 0; k < n; k++) key[k] = (list[k] << 22) | k;
        sort_offsets(key, 22);
        C.clear();
        C.reserve(n);
        sel.assign(n, 0);
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t c = key[i] >> 22;
            if (C.empty() || C.back() != c) C.push_back(c);
            sel[key[i] & ((1u << 22) - 1)] = (uint32_t)(C.size() - 1);
        }
        S.pt.mark("c.sort");
        return run_hook(S, false);  // the next job's roll, if its tables are built
    }
    C.resize(n);
    memcpy(C.data(), sl.list.p, (size_t)n * 8);
    sort_offsets(C);
    C.erase(std::unique(C.begin(), C.end()), C.end());
    sel.clear();
    const size_t i0 = std::lower_bound(C.begin(), C.end(), pos) - C.begin();
    if (i0 < C.size() && (int64_t)C[i0] < S.end) w.spec_batch(C, std::vector<int32_t>(C.size(), -2), i0, sel);
    S.pt.mark("c.select");
    std::vector<uint64_t> so(sel.size());
    for (size_t k = 0; k < sel.size(); k++) so[k] = C[sel[k]];
    if ((s = queue_confirm(S, so.data(), (uint32_t)so.size())) != RSG_OK) return s;
    return run_hook(S, false);  // the next job's roll, if its tables are built
}

// Queue the confirmation of the m windows at offsets off[0..m) (host memory,
// copied to the slot's pinned buffer unless it is that buffer or the roll's
// list): plan built on the GPU, block sums, resolve, results to pinned
// memory in off[] order; event `confirmed` behind them.
rsg_status queue_confirm(Search &S, const uint64_t *off, uint32_t m) {
    rsg_ctx *ctx = S.ctx;
    SearchSlot &sl = *S.sl;
    rsg_status s;
    if (ctx->timing) {
        std::lock_guard<std::mutex> g(ctx->spans_mu);
        ctx->stat_windows += m;
    }
    if (m) {
        HostPlan plan;
        plan.total_blocks = m;
        plan.nwg = (m + rsg::kBlockSumThreads - 1) / rsg::kBlockSumThreads;
        plan.aligned = false;
        plan.arena_bytes = S.size;
        plan.max_blen = (uint32_t)S.head.block_len;  // windows are at most B long
        plan.lds_reserve = S.confirm_lds;
        if ((s = need_resolve_tables(S)) != RSG_OK) return s;
        S.pt.mark("c.partb");
        const uint64_t *so = off;
        if (off != (const uint64_t *)sl.list.p) {  // the GPU reads the offsets from pinned memory
            if ((s = ensure_pin(ctx, sl.sel, (uint64_t)m * 8)) != RSG_OK) return s;
            memcpy(sl.sel.p, off, (size_t)m * 8);
            so = (const uint64_t *)sl.sel.p;
        }
        // the slot's own scratch: the last job's confirmation runs on the roll
        // stream beside job n-2's on the confirmation stream (search_batch)
        if ((s = ensure_dev(ctx, sl.cfiles, (uint64_t)m * sizeof(DevFile) + 32)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, sl.cwg, ((uint64_t)plan.nwg + 1) * sizeof(uint32_t) + 4)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, sl.cout, (uint64_t)m * kRecordBytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, sl.cfb, rsg::block_sums_scratch_bytes(m))) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, sl.res, (uint64_t)m * 4)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, sl.hres, (uint64_t)m * 4)) != RSG_OK) return s;
        RSG_HIP(ctx, rsg::launch_confirm_plan(so, m, S.size, (uint32_t)S.head.block_len, (DevFile *)sl.cfiles.p,
                                              (uint32_t *)sl.cwg.p, plan.nwg, S.cst));
        hipEvent_t t0 = timed_begin(ctx, S.cst);
        if ((s = launch_plan(ctx, plan, sl.cfiles.p, sl.cwg.p, S.d_src, S.seed, sl.cout.p, sl.cfb.p, S.cst)) != RSG_OK)
            return s;
        RSG_HIP(ctx, rsg::launch_resolve((const uint8_t *)sl.cout.p, (const DevFile *)sl.cfiles.p, m,
                                         S.d_groups, S.d_hi16, S.d_sum2, S.head.count, S.head.block_len, S.head.rem,
                                         S.head.s2len, (int32_t *)sl.res.p, S.cst));
        timed_end(ctx, t0, S.cst, 1);
        RSG_HIP(ctx, hipMemcpyAsync(sl.hres.p, sl.res.p, (uint64_t)m * 4, hipMemcpyDeviceToHost, S.cst));
    }
    if (!sl.confirmed) RSG_HIP(ctx, hipEventCreateWithFlags(&sl.confirmed, sync_event_flags()));
    RSG_HIP(ctx, hipEventRecord(sl.confirmed, S.cst));
    S.pt.mark("c.launch");
    return RSG_OK;
}

// The rest of a confirm_all job, after its confirmation was queued: wait for
// the results, walk (confirming, in further round trips, any window the
// selection did not foresee).  Touches only S and its slot's pinned results
// (no HIP call but an event wait) until the walk needs another round trip, so
// it can run on a worker thread while the next jobs are confirmed and rolled.
rsg_status confirm_all_tail(Search &S, const std::vector<uint64_t> &C, const std::vector<uint32_t> &sel,
                            uint64_t &pos) {
    if (hipEventSynchronize(S.sl->confirmed) != hipSuccess) return RSG_ERR_HIP;
    S.pt.mark("c.kernel");
    const int32_t *found = (const int32_t *)S.sl->hres.p;
    std::vector<int32_t> res(C.size(), -2);
    for (size_t k = 0; k < sel.size(); k++) res[sel[k]] = found[k];
    rsg_status s = walk(S, C, pos, &res);
    S.pt.mark("walk");
    return s;
}

// Stage 1 of a search, host part: the basis tables, packed into the slot's
// pinned staging blob in two parts.  Part A is what the roll reads: Bloom
// filter of every Sum1 + the packed roll's 16-bit filter + a 2-choice bucketed
// table {Sum1, flags: bit1 = a block of length B, bit2 = the remainder block}
// (and its key-only copy), built straight from the sums (no sort), so the
// roll can start before part B exists.  Part B is what the confirmation's
// resolve reads: basis sums grouped by Sum1 in targets order, their sum2s.
// Blob layout: filter | filter16 | table | keys | groups | hi16 | sum2.
// Options::host_tables (tests, A/B): part A built on the host (the first job
// of a batch waited ~0.5 ms for it with the GPU idle, r05t)
rsg_status tables_roll(Search &S, const uint32_t *sum1, const int32_t *targets) {
    (void)targets;
    rsg_ctx *ctx = S.ctx;
    SearchSlot &sl = *S.sl;
    TableScratch &T = sl.hs;
    const int64_t B = S.head.block_len;
    const int32_t count = S.head.count;
    const int64_t last_len = (S.head.rem != 0) ? S.head.rem : B;
    S.end = std::max<int64_t>((int64_t)S.size + 1 - last_len, 1);  // match.go:70 (offset 0 always visited)
    const uint64_t ntiles64 = (S.size + kScanTile - 1) / kScanTile;
    if (ntiles64 >= 0xFFFFFFF0ull) return fail(ctx, RSG_ERR_INVALID, "source too large");
    S.ntiles = (uint32_t)ntiles64;
    auto up = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    const bool packed = (uint32_t)B <= rsg::kFusedMaxB;
    if (!ctx->opts.host_tables && count > 0) {
        // the same blob layout, filled by build_tables_kernel (enqueue_scan)
        // from a copy of the Sum1 array; at least two buckets per key
        uint32_t nb = 16;
        while (nb < 2u * (uint32_t)count) nb <<= 1;
        S.bmask = nb - 1;
        S.gpu_tab = true;
        const uint64_t n_filter = rsg::kFilterBits / 8, n_filter16 = packed ? rsg::kFilter16Words * 2ull : 0;
        const uint64_t n_table = (uint64_t)nb * rsg::kBucketWays * 8, n_keys = (uint64_t)nb * rsg::kBucketWays * 4;
        S.off_filter = 0;
        S.off_filter16 = up(n_filter);
        S.off_table = S.off_filter16 + up(n_filter16);
        S.off_keys = S.off_table + up(n_table);
        S.off_sum1 = S.off_keys + up(n_keys);
        S.blob_a_bytes = S.off_sum1 + up((uint64_t)count * 4);
        S.off_groups = S.blob_a_bytes;
        S.off_hi16 = S.off_groups + up((uint64_t)count * 8);
        S.off_sum2 = S.off_hi16 + up(65537ull * 4);
        S.blob_bytes = S.off_sum2 + up((uint64_t)count * 16);
        rsg_status s;
        if ((s = ensure_pin(ctx, sl.stage, S.blob_bytes)) != RSG_OK) return s;
        memcpy((uint8_t *)sl.stage.p + S.off_sum1, sum1, (size_t)count * 4);
        S.pt.mark("tables");
        return RSG_OK;
    }
    S.gpu_tab = false;
    // the filters on a second thread (they need only the sums; bits set per
    // block, a repeated Sum1 sets the same bits)
    auto &bitmap = T.bitmap;
    auto &filter16 = T.filter16;  // the packed roll's filter (interior tiles of the fused mode)
    std::thread filters([&] {
        bitmap.assign(rsg::kFilterBits / 32, 0);
        filter16.clear();
        if (packed) filter16.assign(rsg::kFilter16Words, 0);
        for (int32_t k = 0; k < count; k++) {
            const uint32_t key = sum1[k];
            bitmap[rsg::sel_word(key)] |= rsg::sel_mask(key);
            if (packed) filter16[rsg::f16_word(key, (uint32_t)B)] |= (uint16_t)rsg::f16_mask(key);
        }
    });
    // Sum1 -> flags into the 2-choice bucket table, straight from the sums.
    // First without looking for an equal key (a repeated Sum1 then sits in
    // the table twice: the probes OR the flags of every equal entry, and the
    // packed roll's key test only asks for presence); only if a bucket pair
    // fills up -- many equal sums, e.g. periodic data -- again with equal
    // keys merged (match.go:108's candidates are every block with that Sum1).
    uint32_t nb = 16;
    while (nb < (uint32_t)count / 2) nb <<= 1;
    auto &table = T.table;
    auto &fill = T.fill;
    constexpr uint32_t W = rsg::kBucketWays;
    const uint32_t first_key = count ? sum1[0] : 0u;
    auto build = [&](bool merge) -> bool {
        table.assign((size_t)nb * W, 0);
        fill.assign(nb, 0);
        for (int32_t k = 0; k < count; k++) {
            const uint32_t v = sum1[k];
            const uint32_t f = 1u | ((S.len_of(k) == B) ? 2u : 4u);
            const uint32_t h1 = rsg::bucket_hash1(v) & (nb - 1), h2 = rsg::bucket_hash2(v) & (nb - 1);
            if (merge) {
                bool found = false;
                for (uint32_t hh : {h1, h2}) {
                    for (uint32_t w = 0; w < fill[hh] && !found; w++) {
                        uint64_t &e = table[(size_t)hh * W + w];
                        if ((uint32_t)(e >> 32) == v) {
                            e |= f;
                            found = true;
                        }
                    }
                    if (found || h2 == h1) break;
                }
                if (found) continue;
            }
            const uint32_t h = fill[h2] < fill[h1] ? h2 : h1;
            if (fill[h] == W) return false;
            table[(size_t)h * W + fill[h]++] = ((uint64_t)v << 32) | f;
        }
        return true;
    };
    while (!build(false) && !build(true)) nb <<= 1;
    S.bmask = nb - 1;
    auto &tkeys = T.table_keys;  // the packed roll's key-only copy
    tkeys.resize(table.size());
    for (size_t i = 0; i < table.size(); i++) {
        const uint64_t e = table[i];
        tkeys[i] = (uint32_t)e != 0 ? (uint32_t)(e >> 32) : first_key;  // empty slots: a key that exists
    }
    S.pt.mark("t.table");
    filters.join();
    S.pt.mark("t.filt");
    // blob layout, 256-byte aligned parts; the whole blob is sized here so
    // part B never regrows the stage under part A's upload
    const uint64_t n_filter = bitmap.size() * 4, n_table = table.size() * 8, n_filter16 = filter16.size() * 2;
    const uint64_t n_groups = (uint64_t)count * 8, n_hi16 = 65537ull * 4, n_sum2 = (uint64_t)count * 16;
    S.off_filter = 0;
    S.off_filter16 = up(n_filter);
    S.off_table = S.off_filter16 + up(n_filter16);
    S.off_keys = S.off_table + up(n_table);
    S.blob_a_bytes = S.off_keys + up(tkeys.size() * 4);
    S.off_groups = S.blob_a_bytes;
    S.off_hi16 = S.off_groups + up(n_groups);
    S.off_sum2 = S.off_hi16 + up(n_hi16);
    S.blob_bytes = S.off_sum2 + up(n_sum2);
    rsg_status s;
    if ((s = ensure_pin(ctx, sl.stage, S.blob_bytes)) != RSG_OK) return s;
    uint8_t *st = (uint8_t *)sl.stage.p;
    memcpy(st + S.off_filter, bitmap.data(), n_filter);
    if (n_filter16) memcpy(st + S.off_filter16, filter16.data(), n_filter16);
    memcpy(st + S.off_table, table.data(), n_table);
    memcpy(st + S.off_keys, tkeys.data(), tkeys.size() * 4);
    S.pt.mark("tables");
    return RSG_OK;
}

// Part B (after tables_roll, which sized the blob).
rsg_status tables_resolve(Search &S, const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets) {
    TableScratch &T = S.sl->hs;
    const int32_t count = S.head.count;
    // (sum1, block) in targets order, stably sorted by sum1: each sum's blocks
    // are one run, in targets order (match.go:108 walks targets in that
    // order); hi16[h] = index of the first sum with high half h.
    auto &groups = T.groups;
    auto &hi16 = T.hi16;
    {
        // Stable LSD radix sort (two 16-bit passes) of the targets-ordered list.
        auto &tmp = T.pairs;
        tmp.resize((size_t)count);
        groups.resize((size_t)count);
        for (int32_t k = 0; k < count; k++) tmp[(size_t)k] = {sum1[targets[k]], targets[k]};
        T.cnt.resize(65537);
        for (int pass = 0; pass < 2; pass++) {
            auto &from = pass == 0 ? tmp : groups;
            auto &to = pass == 0 ? groups : tmp;
            const int shift = 16 * pass;
            std::fill(T.cnt.begin(), T.cnt.end(), 0u);
            for (auto &e : from) T.cnt[((e.first >> shift) & 0xffffu) + 1]++;
            for (size_t h = 1; h < T.cnt.size(); h++) T.cnt[h] += T.cnt[h - 1];
            for (auto &e : from) to[T.cnt[(e.first >> shift) & 0xffffu]++] = e;
        }
        groups.swap(tmp);
        hi16.assign(65537, 0);
        for (auto &e : groups) hi16[(e.first >> 16) + 1]++;
        for (size_t h = 1; h < hi16.size(); h++) hi16[h] += hi16[h - 1];
    }
    static_assert(sizeof(groups[0]) == 8, "(sum1, block) pair must be 8 bytes");
    uint8_t *st = (uint8_t *)S.sl->stage.p;
    if (count) memcpy(st + S.off_groups, groups.data(), (size_t)count * 8);
    memcpy(st + S.off_hi16, hi16.data(), hi16.size() * 4);
    if (count) memcpy(st + S.off_sum2, sum2, (size_t)count * 16);
    return RSG_OK;  // (no S.pt mark: this may run on a worker beside the job's own thread)
}

// Both parts, in order (callers that need the whole blob at once).
rsg_status tables(Search &S, const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets) {
    rsg_status s = tables_roll(S, sum1, targets);
    return s != RSG_OK ? s : tables_resolve(S, sum1, sum2, targets);
}

// Stage 1, GPU part.  Side stream: (realigning copy,) prefix pass, blob
// upload; compute stream: after those the roll over the whole
// scan range and its candidate count read-back (event `rolled`).  The roll
// queues behind whatever the compute stream holds (the previous file's roll),
// never beside it.
rsg_status enqueue_scan(Search &S, const uint8_t *src, bool host_src) {
    rsg_ctx *ctx = S.ctx;
    SearchSlot &sl = *S.sl;
    rsg_status s;
    if (!sl.scanned) RSG_HIP(ctx, hipEventCreateWithFlags(&sl.scanned, hipEventDisableTiming));
    if (!sl.rolled) RSG_HIP(ctx, hipEventCreateWithFlags(&sl.rolled, sync_event_flags()));
    if ((s = ensure_dev(ctx, sl.agg, (uint64_t)S.ntiles * sizeof(TileAgg) + 64)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, sl.prefix, ((uint64_t)S.ntiles + 1) * sizeof(TilePrefix) + 64)) != RSG_OK) return s;
    if ((s = ensure_pin(ctx, sl.list, (uint64_t)kCandCap * 8)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, sl.counts, 64)) != RSG_OK) return s;
    if ((s = ensure_pin(ctx, sl.count, 64)) != RSG_OK) return s;
    if (sl.counts_zeroed != sl.counts.p) {  // a new counter: zero once (each roll's count_out re-zeroes it)
        // (word 1: the GPU table build's overflow flag)
        RSG_HIP(ctx, hipMemsetAsync(sl.counts.p, 0, 8, S.side));
        sl.counts_zeroed = sl.counts.p;
    }
    if ((s = ensure_dev(ctx, sl.blob, S.blob_bytes)) != RSG_OK) return s;
    if (host_src || ((uintptr_t)src & 15u)) {  // the scan kernels read 16-byte vectors at 16-byte strides
        if ((s = ensure_dev(ctx, sl.src, S.size + 64)) != RSG_OK) return s;
        RSG_HIP(ctx, hipMemcpyAsync(sl.src.p, src, S.size, host_src ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                                    S.side));
        src = (const uint8_t *)sl.src.p;
    }
    S.d_src = src;
    S.fused = (uint32_t)S.head.block_len <= rsg::kFusedMaxB;
    if (!S.fused) {  // long blocks: global prefix sums of the source first
        const uint32_t r = (uint32_t)(S.head.block_len % kScanTile);
        RSG_HIP(ctx, rsg::launch_tile_agg(S.d_src, S.size, r, (TileAgg *)sl.agg.p, S.ntiles, S.side));
        RSG_HIP(ctx, rsg::launch_tile_scan((const TileAgg *)sl.agg.p, S.ntiles, (TilePrefix *)sl.prefix.p, S.side));
    }
    // The tables' upload (~1.7 MB for a 32 768-block basis) goes on the side
    // stream too: on the compute stream it sat between two files' rolls
    // (≈ 50 µs of PCIe per file in the batch timeline).
    if (S.gpu_tab) {
        // the Sum1 copy up, the filters and table zeroed, then built in place
        uint8_t *b = (uint8_t *)sl.blob.p;
        RSG_HIP(ctx, hipMemcpyAsync(b + S.off_sum1, (const uint8_t *)sl.stage.p + S.off_sum1,
                                    (uint64_t)S.head.count * 4, hipMemcpyHostToDevice, S.side));
        RSG_HIP(ctx, hipMemsetAsync(b, 0, S.off_keys, S.side));
        RSG_HIP(ctx, hipMemsetAsync((uint32_t *)sl.counts.p + 1, 0, 4, S.side));
        RSG_HIP(ctx, rsg::launch_build_tables(
                         (const uint32_t *)(b + S.off_sum1), S.head.count, (uint32_t)S.head.block_len,
                         (uint32_t)S.head.rem, S.off_table > S.off_filter16, (uint32_t *)(b + S.off_filter),
                         (uint16_t *)(b + S.off_filter16), (uint64_t *)(b + S.off_table), (uint32_t *)(b + S.off_keys),
                         S.bmask + 1, (uint32_t *)sl.counts.p + 1, ctx->opts.force_table_ovf, S.side));
    } else {
        RSG_HIP(ctx, hipMemcpyAsync(sl.blob.p, sl.stage.p, S.blob_a_bytes, hipMemcpyHostToDevice, S.side));
    }
    RSG_HIP(ctx, hipEventRecord(sl.scanned, S.side));  // also orders the realigning copy and the upload
    const uint8_t *blob = (const uint8_t *)sl.blob.p;
    S.d_groups = (const uint2 *)(blob + S.off_groups);
    S.d_hi16 = (const uint32_t *)(blob + S.off_hi16);
    S.d_sum2 = blob + S.off_sum2;
    S.d_filter = (const uint32_t *)(blob + S.off_filter);
    S.d_filter16 = S.off_table > S.off_filter16 ? (const uint16_t *)(blob + S.off_filter16) : nullptr;
    S.d_table = (const uint64_t *)(blob + S.off_table);
    S.d_table_keys = (const uint32_t *)(blob + S.off_keys);
    RSG_HIP(ctx, hipStreamWaitEvent(S.st, sl.scanned, 0));

    int dev_cus = 256;
    hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
    S.cus = S.roll_grid ? std::min<uint32_t>(S.roll_grid, (uint32_t)dev_cus) : (uint32_t)dev_cus;
    const uint64_t scan_end = std::min<uint64_t>((uint64_t)S.end, S.size);
    S.tile_end = (uint32_t)((scan_end + kScanTile - 1) / kScanTile);
    if ((s = launch_range(S, 0, S.tile_end)) != RSG_OK) return s;
    S.pending = true;
    return RSG_OK;
}

// Roll kernel over tiles [lo, hi) + its candidate count to the pinned host
// word (and the counter re-zeroed), on the compute stream; event `rolled`
// marks both done.
rsg_status launch_range(Search &S, uint32_t lo, uint32_t hi) {
    rsg_ctx *ctx = S.ctx;
    SearchSlot &sl = *S.sl;
    hipEvent_t t0 = timed_begin(ctx, S.st);
    RSG_HIP(ctx, rsg::launch_roll(S.d_src, S.size, (uint32_t)S.head.block_len, (uint32_t)S.head.rem, (uint64_t)S.end,
                                  lo, hi, (const TileAgg *)sl.agg.p, (const TilePrefix *)sl.prefix.p, S.ntiles,
                                  S.d_filter, S.d_filter16, S.d_table, S.d_table_keys, S.bmask, (uint64_t *)sl.list.p, kCandCap,
                                  (uint32_t *)sl.counts.p, (const uint32_t *)sl.counts.p + 1, S.cus, S.fused, S.st));
    timed_end(ctx, t0, S.st, 0);
    RSG_HIP(ctx, rsg::launch_roll_count_out((uint32_t *)sl.counts.p, (uint32_t *)sl.count.p, S.st));
    RSG_HIP(ctx, hipEventRecord(sl.rolled, S.st));
    return RSG_OK;
}

// Stage 2: candidates of each scan range back to the host (copy stream),
// sorted, walked in match.go's greedy order with GPU confirmation on the
// compute stream.  Synchronous.
rsg_status finish(Search &S) {
    rsg_ctx *ctx = S.ctx;
    SearchSlot &sl = *S.sl;
    uint32_t lo = 0, span = S.tile_end;
    uint64_t pos = S.pos0;
    std::vector<uint64_t> C;
    rsg_status s;
    while (lo < S.tile_end) {
        const uint32_t hi = std::min(S.tile_end, lo + span);
        if ((uint64_t)hi * kScanTile <= pos) {  // the walk already jumped past this range
            if (S.pending) {  // its roll was launched: nothing may outlive the search
                RSG_HIP(ctx, hipEventSynchronize(sl.rolled));
                S.pending = false;
            }
            lo = hi;
            continue;
        }
        if (!S.pending && (s = launch_range(S, lo, hi)) != RSG_OK) return s;
        S.pending = false;
        RSG_HIP(ctx, hipEventSynchronize(sl.rolled));
        const uint32_t n = *(const volatile uint32_t *)sl.count.p;
        if (n > kCandCap) {  // dense range (repetitive data): halve it and retry
            if (hi - lo == 1) return fail(ctx, RSG_ERR_INVALID, "internal: candidate overflow in one tile");
            span = std::max<uint32_t>(1, (hi - lo) / 2);
            continue;
        }
        if (ctx->timing) ctx->stat_candidates += n;
        S.pt.mark("roll");
        if ((s = run_hook(S, false)) != RSG_OK) return s;
        // sparse range (the hashing of every candidate stays below twice the
        // range, walk()'s own batching rule): confirm them all at once
        const uint64_t range = std::min<uint64_t>((uint64_t)hi * kScanTile, S.size) - (uint64_t)lo * kScanTile;
        if (n > 0 && n <= kSparseBatch && S.size < (1ull << 42) &&
            (uint64_t)n * (uint64_t)S.head.block_len <= 2 * range + (1u << 20)) {
            auto Cs = std::make_shared<std::vector<uint64_t>>();
            auto sel = std::make_shared<std::vector<uint32_t>>();
            if ((s = confirm_all(S, n, pos, *Cs, *sel)) != RSG_OK) return s;
            if (hi == S.tile_end) {
                // the job's last range: the caller may run the rest anywhere
                Search *Sp = &S;
                const uint64_t p0 = pos;
                S.tail = [Sp, Cs, sel, p0]() {
                    uint64_t p = p0;
                    const rsg_status st = confirm_all_tail(*Sp, *Cs, *sel, p);
                    Sp->pos_end = p;
                    return st;
                };
                break;
            }
            if ((s = confirm_all_tail(S, *Cs, *sel, pos)) != RSG_OK) return s;
            lo = hi;
            continue;
        }
        C.resize(n);
        if (n) memcpy(C.data(), sl.list.p, (size_t)n * 8);  // pinned host memory the roll wrote
        sort_offsets(C);
        C.erase(std::unique(C.begin(), C.end()), C.end());
        if ((s = walk(S, C, pos)) != RSG_OK) return s;
        S.pt.mark("walk");
        lo = hi;
    }
    S.pos_end = pos;
    if ((s = run_hook(S, true)) != RSG_OK) return s;
    return RSG_OK;
}

// SumHead.ReadFrom validation (types.go:38-77) plus the arrays' consistency.
rsg_status check_args(rsg_ctx *ctx, const rsg_sum_head *head, const uint32_t *sum1, const uint8_t *sum2,
                      const int32_t *targets, rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    if (!head || !n_matches) return fail(ctx, RSG_ERR_INVALID, "NULL head or n_matches");
    if (head->count < 0) return fail(ctx, RSG_ERR_INVALID, "invalid checksum count %d", head->count);
    if (head->block_len < 0 || head->block_len > RSG_MAX_BLOCK_LEN)
        return fail(ctx, RSG_ERR_INVALID, "invalid block length %d", head->block_len);
    if (head->s2len < 0 || head->s2len > 16) return fail(ctx, RSG_ERR_INVALID, "invalid checksum length %d", head->s2len);
    if (head->rem < 0 || head->rem > head->block_len)
        return fail(ctx, RSG_ERR_INVALID, "invalid remainder length %d", head->rem);
    if (head->count > 0 && head->block_len == 0) return fail(ctx, RSG_ERR_INVALID, "zero block length");
    if (head->count > 0 && (!sum1 || !sum2 || !targets)) return fail(ctx, RSG_ERR_INVALID, "NULL sums or targets");
    if (match_cap && !matches) return fail(ctx, RSG_ERR_INVALID, "NULL matches");
    std::vector<uint8_t> seen((size_t)head->count, 0);
    for (int32_t k = 0; k < head->count; k++) {
        const int32_t i = targets[k];
        if (i < 0 || i >= head->count || seen[(size_t)i]) return fail(ctx, RSG_ERR_INVALID, "targets is not a permutation");
        seen[(size_t)i] = 1;
    }
    return RSG_OK;
}

// Bad arguments and truncation belong to one job; anything else (HIP,
// allocation) stops the batch.
bool job_local(rsg_status s) { return s == RSG_ERR_INVALID || s == RSG_ERR_TRUNCATED; }

// The jobs in order, three in flight (scratch slot i % 3).  Job i+1 is issued
// before job i is finished, and job i+2 is issued from inside job i's
// finish() as soon as its confirmation batch is queued, so on the GPU
//   compute stream (side[0]):  roll(i+1) | confirm(i) | roll(i+2) | confirm(i+1) ...
//   side stream (side[1]):     prefix pass(i+2) beside roll(i+1) / confirm(i)
//   copy stream (ctx->stream): candidate read-back
// while the host sorts and walks job i's candidates during roll(i+1) and
// builds job i+2's tables during confirm(i).  Two files' kernels never share
// the CUs except the memory-bound prefix pass: a confirmation kernel (few
// lanes, serial MD4 chains) beside a roll kernel ran 3x slower.
rsg_status search_batch(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed, bool host_src) {
    if (njobs && !jobs) return fail(ctx, RSG_ERR_INVALID, "NULL jobs");
    PhaseTimer bt;  // RSG_TIMING: the call's start-up and drain
    for (uint64_t i = 0; i < njobs; i++) {
        jobs[i].n_matches = 0;
        jobs[i].status = RSG_OK;
    }
    rsg_status first = RSG_OK;
    std::string first_err;
    auto note = [&](uint64_t i, rsg_status st) {
        jobs[i].status = st;
        if (st != RSG_OK && first == RSG_OK) {
            first = st;
            first_err = ctx->err;
        }
    };
    // Sources written on the context's stream (fills, copies) come first.
    RSG_HIP(ctx, hipEventRecord(ctx->side_done[0], ctx->stream));
    for (int k = 0; k < 2; k++) RSG_HIP(ctx, hipStreamWaitEvent(ctx->side[k], ctx->side_done[0], 0));

    // RSG_CONFIRM_CUS: CUs the roll leaves to the confirmation of the
    // previous job (0 = the confirmation queues behind the next roll on one
    // stream, as before)
    int dev_cus = 256;
    RSG_HIP(ctx, hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const int spare = std::max(0, std::min(ctx->opts.confirm_cus, dev_cus - 1));
    const bool split = spare > 0 && njobs > 1;  // one job: nothing to overlap its confirmation with
    std::unique_ptr<Search> live[kSearchSlots];
    // Job i's stage 1 in two steps.  prepare(i): validate the job and start
    // building its basis tables (host sorting and hashing, ~0.3-0.8 ms for a
    // 32 768-block basis) on a worker thread.  issue(): wait for those tables
    // and queue the job's GPU work.  Job i+2 is prepared while job i is
    // finished on this thread, and issued once job i's confirmation is queued.
    // Both return only fatal statuses; a job-local failure is recorded on
    // the job, which then holds no search.
    std::future<rsg_status> tails[kSearchSlots];  // job i's walk (confirm_all_tail) on a worker
    bool tail_live[kSearchSlots] = {};
    // Job i's results into the caller's job record once its search is done
    // (finish() and, if it handed one back, its tail).
    auto complete = [&](uint64_t i, rsg_status s) -> rsg_status {
        Search *S = live[i % kSearchSlots].get();
        if (s == RSG_OK) {
            rsg_search_job &j = jobs[i];
            j.n_matches = S->out.size();
            const uint64_t ncopy = std::min<uint64_t>(S->out.size(), j.match_cap);
            if (ncopy) memcpy(j.matches, S->out.data(), ncopy * sizeof(rsg_match));
            if (S->out.size() > j.match_cap)
                note(i, fail(ctx, RSG_ERR_TRUNCATED, "%llu matches, capacity %llu",
                             (unsigned long long)S->out.size(), (unsigned long long)j.match_cap));
            return RSG_OK;
        }
        if (job_local(s)) return note(i, s), RSG_OK;
        if (s == RSG_ERR_HIP) return fail(ctx, RSG_ERR_HIP, "confirmation wait failed");
        return s;
    };
    // join job i's tail (if any) and finish its record; its slot is free after
    auto join = [&](uint64_t i) -> rsg_status {
        const int slot = (int)(i % kSearchSlots);
        rsg_status f = RSG_OK;
        if (tail_live[slot]) {
            tail_live[slot] = false;
            f = complete(i, tails[slot].get());
        }
        live[slot].reset();
        return f;
    };
    struct Pending {
        bool valid = false;
        uint64_t i = 0;
        std::unique_ptr<Search> S;
        std::future<rsg_status> tab;
    } pends[2];  // job i is prepared into pends[i & 1]
    // inline_a: part A on this thread (job 0 of a serial start: the caller
    // waits for it next anyway, and a fresh worker thread built it ~2x slower)
    auto prepare = [&](uint64_t i, bool inline_a = false) -> rsg_status {
        rsg_search_job &j = jobs[i];
        const int slot = (int)(i % kSearchSlots);
        live[slot].reset();  // job i - 3 of this slot was finished, its GPU work waited for
        rsg_status s = check_args(ctx, &j.head, j.sum1, j.sum2, j.targets, j.matches, j.match_cap, &j.n_matches);
        if (s != RSG_OK) return note(i, s), RSG_OK;
        if (j.head.count == 0 || j.src_len == 0) return RSG_OK;  // sendFile path / empty source: no matches
        if (!j.src) return note(i, fail(ctx, RSG_ERR_INVALID, "NULL source")), RSG_OK;
        std::unique_ptr<Search> S(new Search());
        S->ctx = ctx;
        S->sl = &ctx->search[slot];
        S->st = ctx->side[0];
        S->cst = ctx->side[0];
        if (split) {
            // Confirmation of job i on its own stream, beside the roll of job
            // i+1: the roll leaves `spare` CUs free (one persistent workgroup
            // per CU on the others), and the confirmation workgroups reserve
            // 8 KiB of LDS they do not use, which cannot fit beside a roll
            // workgroup's 156 KiB, so they land on the free CUs (or on CUs the
            // roll has finished with) instead of slowing the roll's SIMDs.
            S->cst = ctx->confirm;
            S->roll_grid = (uint32_t)std::max(1, dev_cus - spare);
            S->confirm_lds = 8192;
            if (i + 1 == njobs) {
                // the last job's confirmation has no roll to share the chip
                // with: it queues behind its own roll on the roll stream and
                // runs beside job i-1's, instead of after it (the drain was
                // confirm(n-2)'s rest + confirm(n-1), r05q trace)
                S->cst = ctx->side[0];
                S->confirm_lds = 0;
            }
        }
        S->side = ctx->side[1];
        S->copy = ctx->stream;
        S->size = j.src_len;
        S->head = j.head;
        S->seed = seed;
        Search *raw = S.get();
        Pending &pend = pends[i & 1];
        // part A (the roll's tables) is what issue() waits for; part B (the
        // resolve's) follows on the same worker and is waited for at the
        // job's first confirmation
        auto part_a = std::make_shared<std::promise<rsg_status>>();
        pend.tab = part_a->get_future();
        if (inline_a) {
            const rsg_status sa = tables_roll(*raw, j.sum1, j.targets);
            part_a->set_value(sa);
            raw->part_b = std::async(std::launch::async, [raw, &j, sa] {
                return sa != RSG_OK ? sa : tables_resolve(*raw, j.sum1, j.sum2, j.targets);
            });
        } else {
            raw->part_b = std::async(std::launch::async, [raw, &j, part_a] {
                const rsg_status sa = tables_roll(*raw, j.sum1, j.targets);
                part_a->set_value(sa);
                return sa != RSG_OK ? sa : tables_resolve(*raw, j.sum1, j.sum2, j.targets);
            });
        }
        pend.S = std::move(S);
        pend.i = i;
        pend.valid = true;
        return RSG_OK;
    };
    auto issue = [&](uint64_t i) -> rsg_status {
        Pending &pend = pends[i & 1];
        if (!pend.valid || pend.i != i) return RSG_OK;  // job i holds no search
        pend.valid = false;
        rsg_status s = pend.tab.get();
        std::unique_ptr<Search> S = std::move(pend.S);
        if (s == RSG_OK) s = enqueue_scan(*S, (const uint8_t *)jobs[i].src, host_src);
        if (s != RSG_OK) {
            if (!job_local(s)) return s;
            note(i, s);
            return RSG_OK;
        }
        live[i % kSearchSlots] = std::move(S);
        return RSG_OK;
    };
    rsg_status fatal = RSG_OK;
    uint64_t i = 0;
    // job 0 alone first: its roll queues as soon as its own tables are built
    // on this thread (built beside job 1's they took twice as long, and the
    // GPU idles until then: +1.5 %, r05); job 1's tables build while roll 0 runs
    if (njobs) fatal = prepare(0, true);
    if (fatal == RSG_OK && njobs) fatal = issue(0);
    if (fatal == RSG_OK && njobs > 1) fatal = prepare(1);
    if (fatal == RSG_OK && njobs > 1) fatal = issue(1);
    bt.mark("b.issued");
    for (; fatal == RSG_OK && i < njobs; i++) {
        const uint64_t ahead = i + 2;
        // job i+2 takes job i-2's slot: that job's walk (a worker) is done by
        // now; then job i+2's tables build on a worker while job i finishes
        // here
        if (i >= 2 && (fatal = join(i - 2)) != RSG_OK) break;
        if (ahead < njobs && (fatal = prepare(ahead)) != RSG_OK) break;
        auto next = [&, ahead]() -> rsg_status { return ahead < njobs ? issue(ahead) : RSG_OK; };
        const int slot = (int)(i % kSearchSlots);
        Search *S = live[slot].get();
        if (!S) {
            if ((fatal = next()) != RSG_OK) break;
            continue;
        }
        S->hook = next;
        S->hook_ready = [&, ahead]() {
            const Pending &pend = pends[ahead & 1];
            return ahead >= njobs || !pend.valid || pend.i != ahead ||
                   pend.tab.wait_for(std::chrono::seconds(0)) == std::future_status::ready;
        };
        rsg_status s = finish(*S);
        // the next job's issue stays on this thread: a tail on a worker must
        // not find it (its walk's round trips call run_hook)
        std::function<rsg_status()> hook = std::move(S->hook);
        S->hook = nullptr;
        S->hook_ready = nullptr;
        if (s == RSG_OK && S->tail) {  // the walk runs beside the next jobs' confirmations and rolls
            tails[slot] = std::async(std::launch::async, S->tail);
            tail_live[slot] = true;
        }
        if (!tail_live[slot] && (fatal = complete(i, s)) != RSG_OK) break;
        if (hook && (fatal = hook()) != RSG_OK) {  // not run by finish() (tables not ready, or a job-local error)
            i++;
            break;
        }
    }
    bt.mark("b.loop");
    // the last jobs' walks (and, after a fatal error, any still running)
    for (uint64_t k = i >= kSearchSlots ? i - kSearchSlots : 0; k < i; k++) {
        const rsg_status f = join(k);
        if (fatal == RSG_OK) fatal = f;
    }
    if (fatal != RSG_OK) {
        const std::string msg = ctx->err;
        for (uint64_t k = i; k < njobs; k++) jobs[k].status = fatal;
        if (first == RSG_OK) {
            first = fatal;
            first_err = msg;
        }
    }
    // nothing outlives the call: a fatal error inside a hook can return
    // before a job's confirmation (ctx->confirm, then its D2H into
    // ctx->h_out[0]) has been waited for
    for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(ctx->side[k]);
    (void)hipStreamSynchronize(ctx->confirm);
    (void)hipStreamSynchronize(ctx->stream);
    if (first != RSG_OK) ctx->err = first_err;
    bt.mark("b.drain");
    return first;
}

// A search batch: small sources through the one-wave-per-file kernel
// (rsg_sender_small.cpp), the rest -- and any small source whose candidates
// overflowed that kernel's lists -- through the pipeline above.  Each job's
// result is the same either way.  Returns RSG_OK or the first failing job's
// status (job order) with its message.
rsg_status search_jobs(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed, bool host_src) {
    if (njobs && !jobs) return fail(ctx, RSG_ERR_INVALID, "NULL jobs");
    std::vector<uint64_t> rest;
    std::vector<std::string> msg;
    rsg_status fatal = search_small_batch(ctx, jobs, njobs, seed, host_src, rest, msg);
    struct Drain {  // the small path's kernels write pinned host memory: nothing outlives the call
        rsg_ctx *c;
        ~Drain() {
            for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(c->side[k]);
        }
    } drain{ctx};
    if (fatal != RSG_OK) {
        const std::string m = ctx->err;
        for (uint64_t i = 0; i < njobs; i++)
            if (jobs[i].status == RSG_OK) jobs[i].status = fatal;
        ctx->err = m;
        return fatal;
    }
    std::string rest_err;
    if (!rest.empty()) {
        std::vector<rsg_search_job> sub(rest.size());
        for (size_t k = 0; k < rest.size(); k++) sub[k] = jobs[rest[k]];
        if (search_batch(ctx, sub.data(), sub.size(), seed, host_src) != RSG_OK) rest_err = ctx->err;
        for (size_t k = 0; k < rest.size(); k++) {
            jobs[rest[k]].n_matches = sub[k].n_matches;
            jobs[rest[k]].status = sub[k].status;
        }
    }
    for (uint64_t i = 0; i < njobs; i++)
        if (jobs[i].status != RSG_OK) {
            ctx->err = msg[i].empty() ? rest_err : msg[i];
            return jobs[i].status;
        }
    return RSG_OK;
}

// ---------------------------------------------------------------- streaming sender (§8 a13)
// io.ReadFull-style pread of [off, off + n) on a few threads; -1 = EOF
// before n bytes, else 0 or an errno.
int pread_full(int fd, int64_t off, uint8_t *dst, uint64_t n) {
    const uint64_t piece = 4ull << 20;
    const uint64_t npieces = (n + piece - 1) / piece;
    const int nt = (int)std::min<uint64_t>(8, std::max<uint64_t>(1, npieces));
    std::atomic<uint64_t> next{0};
    std::atomic<int> bad{0};
    auto worker = [&] {
        for (uint64_t k; (k = next.fetch_add(1)) < npieces && bad.load() == 0;) {
            uint64_t o = k * piece, m = std::min(piece, n - o);
            while (m) {
                const ssize_t r = pread(fd, dst + o, (size_t)m, (off_t)(off + (int64_t)o));
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {
                    int expected = 0;
                    bad.compare_exchange_strong(expected, r < 0 ? errno : -1);
                    return;
                }
                o += (uint64_t)r;
                m -= (uint64_t)r;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
    return bad.load();
}

// Window of the streamed source: RSG_SEARCH_WINDOW_KB (default 256 MiB),
// whole scan tiles, at least 2 B.
uint64_t search_window_bytes(uint32_t B) {
    const char *e = getenv("RSG_SEARCH_WINDOW_KB");
    uint64_t w = (e ? (uint64_t)std::max(1L, atol(e)) : 256ull * 1024) << 10;
    w = std::max<uint64_t>(w, 2ull * B);
    return (w + kScanTile - 1) / kScanTile * kScanTile;
}

// hashSearch over a file read in windows (fileio.go:31-112 mapFile/ptr; the
// reference's window is max(3B, 256 KiB), match.go:34-35): window k holds
// bytes [kW, (k+1)W + B - 1) of the source in HBM and yields the walk over
// the offsets [kW, (k+1)W); the walk's position carries from window to
// window.  Two pinned staging slots and two device windows: window k+1 is
// read while window k is uploaded and searched.  With file_sum, h =
// MD4(int32_LE(seed) || source) (match.go:52-53) is computed on a host
// thread over the same staging bytes, in order.
rsg_status search_fd(rsg_ctx *ctx, int32_t fd, int64_t off0, uint64_t size, const rsg_sum_head *head,
                     const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                     std::vector<rsg_match> &out, uint8_t *file_sum) {
    rsg_status s;
    const bool search = head->count > 0 && size > 0;  // count == 0: sendFile (sender.go:86-88)
    const uint32_t B = search ? (uint32_t)head->block_len : 0;
    const uint64_t W = search_window_bytes(B);
    const uint64_t halo = B ? B - 1 : 0;
    const uint64_t cap = W + halo + 64;
    if (size && fd < 0) return fail(ctx, RSG_ERR_INVALID, "bad descriptor");
    const uint64_t nwin = (size + W - 1) / W;
    for (int k = 0; k < 2 && nwin; k++) {
        if ((s = ensure_pin(ctx, ctx->h_in[k], cap)) != RSG_OK) return s;
        if (search && (s = ensure_dev(ctx, ctx->d_in[k], cap)) != RSG_OK) return s;
    }
    struct Drain {
        rsg_ctx *c;
        ~Drain() {
            for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(c->side[k]);
            (void)hipStreamSynchronize(c->stream);
        }
    } drain_guard{ctx};
    Md4 h;
    h.init();
    if (file_sum) {
        const uint8_t sb[4] = {(uint8_t)seed, (uint8_t)(seed >> 8), (uint8_t)(seed >> 16), (uint8_t)(seed >> 24)};
        h.update(sb, 4);  // binary.Write(h, LittleEndian, st.Seed), match.go:52-53
    }
    std::future<void> md4_prev;  // the previous window's MD4 (windows hash in order)
    auto read_win = [&](uint64_t k) -> int {
        const uint64_t a = k * W, n = std::min(W + halo, size - a);
        return pread_full(fd, off0 + (int64_t)a, (uint8_t *)ctx->h_in[k & 1].p, n);
    };
    auto read_err = [&](int code) {
        if (code == -1) return fail(ctx, RSG_ERR_IO, "file has changed mid-transfer");  // fileio.go:99-104
        return fail(ctx, RSG_ERR_IO, "file has changed mid-transfer: %s", strerror(code));
    };
    // the basis tables, once (slot 0's pinned stage keeps them for every window)
    std::unique_ptr<Search> T;
    SearchSlot &sl = ctx->search[0];
    if (search) {
        T.reset(new Search());
        T->ctx = ctx;
        T->sl = &sl;
        T->size = size;
        T->head = *head;
        if ((s = tables(*T, sum1, sum2, targets)) != RSG_OK) return s;
    }
    const int64_t end_global = search ? T->end : 0;
    hipEvent_t up[2] = {nullptr, nullptr};
    struct Ev {
        hipEvent_t *e;
        ~Ev() {
            for (int k = 0; k < 2; k++)
                if (e[k]) hipEventDestroy(e[k]);
        }
    } ev_guard{up};
    for (int k = 0; k < 2; k++) RSG_HIP(ctx, hipEventCreateWithFlags(&up[k], hipEventDisableTiming));
    int code = nwin ? read_win(0) : 0;
    if (code) return read_err(code);
    uint64_t pos = 0;
    for (uint64_t k = 0; k < nwin; k++) {
        const int slot = (int)(k & 1);
        const uint64_t a = k * W, nnew = std::min(W, size - a), nread = std::min(W + halo, size - a);
        const uint8_t *hp = (const uint8_t *)ctx->h_in[slot].p;
        const bool visit = search && (int64_t)a < end_global && pos < a + W;
        if (visit)
            RSG_HIP(ctx, hipMemcpyAsync(ctx->d_in[slot].p, hp, nread, hipMemcpyHostToDevice, ctx->side[1]));
        RSG_HIP(ctx, hipEventRecord(up[slot], ctx->side[1]));
        if (file_sum) {
            std::future<void> prev = std::move(md4_prev);
            md4_prev = std::async(std::launch::async, [&h, hp, nnew, p = std::move(prev)]() mutable {
                if (p.valid()) p.wait();
                h.update(hp, nnew);
            });
        }
        // window k+1 into the other slot once window k-1's upload and MD4 left it
        std::future<int> next;
        if (k + 1 < nwin) {
            RSG_HIP(ctx, hipEventSynchronize(up[slot ^ 1]));
            next = std::async(std::launch::async, [&, k, slot]() {
                (void)slot;
                return read_win(k + 1);
            });
        }
        if (visit) {
            Search S;
            S.ctx = ctx;
            S.sl = &sl;
            S.st = S.cst = ctx->side[0];
            S.side = ctx->side[1];
            S.copy = ctx->stream;
            S.head = *head;
            S.seed = seed;
            S.size = nread;
            S.ntiles = (uint32_t)((nread + kScanTile - 1) / kScanTile);
            S.end = std::min<int64_t>((int64_t)W, end_global - (int64_t)a);
            S.off_filter = T->off_filter;
            S.off_filter16 = T->off_filter16;
            S.off_table = T->off_table;
            S.off_keys = T->off_keys;
            S.blob_a_bytes = T->blob_a_bytes;
            S.gpu_tab = T->gpu_tab;
            S.off_sum1 = T->off_sum1;
            S.off_groups = T->off_groups;
            S.off_hi16 = T->off_hi16;
            S.off_sum2 = T->off_sum2;
            S.blob_bytes = T->blob_bytes;  // part B is uploaded again per window (need_resolve_tables)
            S.bmask = T->bmask;
            S.pos0 = pos > a ? pos - a : 0;
            if ((s = enqueue_scan(S, (const uint8_t *)ctx->d_in[slot].p, false)) != RSG_OK) return s;
            if ((s = finish(S)) != RSG_OK) return s;
            if (S.tail && (s = S.tail()) != RSG_OK) return s == RSG_ERR_HIP ? fail(ctx, s, "confirmation wait failed") : s;
            for (const rsg_match &m : S.out) out.push_back(rsg_match{m.offset + (int64_t)a, m.index, 0});
            pos = a + S.pos_end;
        }
        if (next.valid() && (code = next.get()) != 0) {
            if (md4_prev.valid()) md4_prev.wait();
            return read_err(code);
        }
        // window k+2 reuses this slot: its MD4 must be done before that read
        if (file_sum && k + 1 < nwin) md4_prev.wait();
    }
    if (md4_prev.valid()) md4_prev.wait();
    if (file_sum) h.final(file_sum);
    return RSG_OK;
}

// MD4(int32_LE(seed) || bytes [off, off + n) of fd) (match.go:52-53), the
// bytes read with pread in 1 MiB pieces (hashed while cache-hot).  0, an
// errno, or -1 for EOF before n bytes.  A second read of the file, apart from
// the search's (the reference hashes the bytes it matches and sends): a file
// rewritten in place mid-transfer can give a sum of other contents
// (documented in rsg.h / DESIGN.md 4.2.1).
int file_sum_fd(int fd, int64_t off, uint64_t n, int32_t seed, uint8_t out[16], std::vector<uint8_t> &buf) {
    constexpr uint64_t kPiece = 1ull << 20;
    buf.resize(kPiece);
    Md4 h;
    h.init();
    const uint8_t sb[4] = {(uint8_t)seed, (uint8_t)(seed >> 8), (uint8_t)(seed >> 16), (uint8_t)(seed >> 24)};
    h.update(sb, 4);
    for (uint64_t o = 0; o < n;) {
        const uint64_t m = std::min(kPiece, n - o);
        uint64_t got = 0;
        while (got < m) {
            const ssize_t r = pread(fd, buf.data() + got, (size_t)(m - got), (off_t)(off + (int64_t)(o + got)));
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) return r < 0 ? errno : -1;
            got += (uint64_t)r;
        }
        h.update(buf.data(), m);
        o += m;
    }
    h.final(out);
    return 0;
}

// Host threads for the whole-file sums of a batch (RSG_SUM_THREADS, default
// 10): one serial MD4 chain per file, so files hash side by side.
int sum_threads() {  // read per call (one getenv per batch)
    const char *e = getenv("RSG_SUM_THREADS");
    const int v = e ? atoi(e) : 10;
    return std::max(1, std::min(v, 64));
}

}  // namespace

extern "C" {

rsg_status rsg_hash_search_fd_batch(rsg_ctx *ctx, rsg_fd_search_job *jobs, uint64_t njobs, int32_t seed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (njobs && !jobs) return fail(ctx, RSG_ERR_INVALID, "NULL jobs");
    std::vector<std::string> msg(njobs);
    for (uint64_t i = 0; i < njobs; i++) {
        rsg_fd_search_job &j = jobs[i];
        j.n_matches = 0;
        j.status = check_args(ctx, &j.head, j.sum1, j.sum2, j.targets, j.matches, j.match_cap, &j.n_matches);
        if (j.status == RSG_OK && (j.offset < 0 || j.src_len > (uint64_t)INT64_MAX))
            j.status = fail(ctx, RSG_ERR_INVALID, "bad offset / length");
        if (j.status == RSG_OK && j.src_len && j.fd < 0) j.status = fail(ctx, RSG_ERR_INVALID, "bad descriptor");
        if (j.status != RSG_OK) msg[i] = ctx->err;
    }
    // the whole-file sums, longest file first, on their own threads for the
    // whole call (sendFile hashes beside its reads too, sender.go:184-206)
    std::vector<uint64_t> order;
    for (uint64_t i = 0; i < njobs; i++)
        if (jobs[i].status == RSG_OK && jobs[i].file_sum) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return jobs[a].src_len > jobs[b].src_len; });
    std::vector<int> sum_code(njobs, 0);
    std::atomic<uint64_t> next{0};
    std::vector<std::thread> pool;
    const int nt = (int)std::min<uint64_t>(order.size(), (uint64_t)sum_threads());
    for (int t = 0; t < nt; t++)
        pool.emplace_back([&] {
            std::vector<uint8_t> buf;
            for (uint64_t k; (k = next.fetch_add(1)) < order.size();) {
                rsg_fd_search_job &j = jobs[order[k]];
                sum_code[order[k]] = file_sum_fd(j.fd, j.offset, j.src_len, seed, j.file_sum, buf);
            }
        });
    struct Join {
        std::vector<std::thread> &p;
        ~Join() {
            for (auto &t : p)
                if (t.joinable()) t.join();
        }
    } join_guard{pool};
    // the searches, in job order, on this thread (each as rsg_hash_search_fd)
    rsg_status fatal = RSG_OK;
    std::string fatal_msg;
    for (uint64_t i = 0; i < njobs && fatal == RSG_OK; i++) {
        rsg_fd_search_job &j = jobs[i];
        if (j.status != RSG_OK || j.head.count == 0 || j.src_len == 0) continue;  // sendFile path: the sum only
        std::vector<rsg_match> out;
        rsg_status st = search_fd(ctx, j.fd, j.offset, j.src_len, &j.head, j.sum1, j.sum2, j.targets, seed, out, nullptr);
        if (st == RSG_OK) {
            j.n_matches = out.size();
            if (out.size() > j.match_cap)
                st = fail(ctx, RSG_ERR_TRUNCATED, "%llu matches, capacity %llu", (unsigned long long)out.size(),
                          (unsigned long long)j.match_cap);
            else if (!out.empty())
                memcpy(j.matches, out.data(), out.size() * sizeof(rsg_match));
        }
        if (st != RSG_OK) {
            if (job_local(st) || st == RSG_ERR_IO) {
                j.status = st;
                msg[i] = ctx->err;
            } else {
                fatal = st;
                fatal_msg = ctx->err;
            }
        }
    }
    for (auto &t : pool) t.join();
    if (fatal != RSG_OK) {
        for (uint64_t i = 0; i < njobs; i++)
            if (jobs[i].status == RSG_OK) jobs[i].status = fatal, msg[i] = fatal_msg;
    }
    for (uint64_t i = 0; i < njobs; i++) {
        if (jobs[i].status != RSG_OK || sum_code[i] == 0) continue;
        jobs[i].status = RSG_ERR_IO;  // fileio.go:99-104
        msg[i] = sum_code[i] == -1 ? std::string("file has changed mid-transfer")
                                   : std::string("file has changed mid-transfer: ") + strerror(sum_code[i]);
    }
    for (uint64_t i = 0; i < njobs; i++)
        if (jobs[i].status != RSG_OK) {
            ctx->err = msg[i];
            return jobs[i].status;
        }
    return RSG_OK;
}

rsg_status rsg_set_kernel_timing(rsg_ctx *ctx, int32_t on) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    ctx->timing = on != 0;
    return RSG_OK;
}

rsg_status rsg_kernel_times(rsg_ctx *ctx, double out[8], int32_t reset) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (!out) return fail(ctx, RSG_ERR_INVALID, "out is NULL");
    for (int k = 0; k < 8; k++) out[k] = 0;
    out[4] = (double)ctx->stat_candidates;
    out[5] = (double)ctx->stat_windows;
    for (const rsg_ctx::TimedSpan &t : ctx->spans) {
        RSG_HIP(ctx, hipEventSynchronize(t.b));
        float ms = 0;
        RSG_HIP(ctx, hipEventElapsedTime(&ms, t.a, t.b));
        const int slot = t.kind == 2 ? 6 : 2 * t.kind;  // out[4..5] are the sender's counts
        out[slot] += ms;
        out[slot + 1] += 1;
    }
    if (reset) {
        for (const rsg_ctx::TimedSpan &t : ctx->spans) {
            hipEventDestroy(t.a);
            hipEventDestroy(t.b);
        }
        ctx->spans.clear();
        ctx->stat_candidates = ctx->stat_windows = 0;
    }
    return RSG_OK;
}

rsg_status rsg_hash_search_batch_device(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    return search_jobs(ctx, jobs, njobs, seed, false);
}

rsg_status rsg_hash_search_batch_host(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    return search_jobs(ctx, jobs, njobs, seed, true);
}

rsg_status rsg_testing_search_option(rsg_ctx *ctx, int32_t option, int32_t value) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    rsg_ctx::Options &o = ctx->opts;
    const bool b01 = value == 0 || value == 1;
    switch (option) {
        case 0: if (!b01) break; o.path = value; return RSG_OK;
        case 1: if (!b01) break; o.host_tables = value; return RSG_OK;
        case 2: if (!b01) break; o.force_table_ovf = value; return RSG_OK;
        case 3: if (!b01) break; o.spec = value; return RSG_OK;
        case 4: if (value < 0 || value > 1024) break; o.confirm_cus = value; return RSG_OK;
        case 5: if (value < 0 || value > 2) break; o.recv_md4 = value; return RSG_OK;
        case 6: if (value < 0 || value > 40) break; o.fs_key_shift = value; return RSG_OK;
        default: return fail(ctx, RSG_ERR_INVALID, "unknown option %d", option);
    }
    return fail(ctx, RSG_ERR_INVALID, "option %d: bad value %d", option, value);
}

// The single-file calls are batches of one.
static rsg_status search_one(rsg_ctx *ctx, const void *src, uint64_t src_len, const rsg_sum_head *head,
                             const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                             rsg_match *matches, uint64_t match_cap, uint64_t *n_matches, bool host_src) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (!head || !n_matches) return fail(ctx, RSG_ERR_INVALID, "NULL head or n_matches");
    rsg_search_job j{};
    j.src = src;
    j.src_len = src_len;
    j.head = *head;
    j.sum1 = sum1;
    j.sum2 = sum2;
    j.targets = targets;
    j.matches = matches;
    j.match_cap = match_cap;
    const rsg_status s = search_jobs(ctx, &j, 1, seed, host_src);
    *n_matches = j.n_matches;
    return s;
}

rsg_status rsg_hash_search_fd(rsg_ctx *ctx, int32_t fd, int64_t offset, uint64_t src_len, const rsg_sum_head *head,
                              const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                              rsg_match *matches, uint64_t match_cap, uint64_t *n_matches, uint8_t file_sum[16]) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    rsg_status s = check_args(ctx, head, sum1, sum2, targets, matches, match_cap, n_matches);
    if (s != RSG_OK) return s;
    *n_matches = 0;
    if (offset < 0 || src_len > (uint64_t)INT64_MAX) return fail(ctx, RSG_ERR_INVALID, "bad offset / length");
    std::vector<rsg_match> out;
    if ((s = search_fd(ctx, fd, offset, src_len, head, sum1, sum2, targets, seed, out, file_sum)) != RSG_OK) return s;
    *n_matches = out.size();
    if (out.size() > match_cap)
        return fail(ctx, RSG_ERR_TRUNCATED, "%llu matches, capacity %llu", (unsigned long long)out.size(),
                    (unsigned long long)match_cap);
    if (!out.empty()) memcpy(matches, out.data(), out.size() * sizeof(rsg_match));
    return RSG_OK;
}

// Test hook (include/rsg_testing.h): the sender's greedy walk with the GPU
// confirmation replaced by a table of answers, so its batching can be
// checked on a machine without a GPU.
rsg_status rsg_testing_walk(const uint64_t *cand, uint64_t n, const int32_t *truth, uint64_t size,
                            const rsg_sum_head *head, rsg_match *out, uint64_t cap, uint64_t *n_out,
                            uint64_t stats[2]) {
    if (!head || !n_out || !stats || (n && (!cand || !truth))) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    std::vector<uint64_t> C(cand, cand + n);
    for (uint64_t k = 1; k < n; k++)
        if (C[k] <= C[k - 1]) return fail(nullptr, RSG_ERR_INVALID, "candidates must be strictly increasing");
    std::vector<rsg_match> found;
    Walker w;
    const int64_t last_len = head->rem != 0 ? head->rem : head->block_len;
    w.end = std::max<int64_t>((int64_t)size + 1 - last_len, 1);
    w.size = size;
    w.head = *head;
    w.out = &found;
    w.spec = stats[0] == 1;  // on input: the selection mode (1 = speculative; 0 / 2 = every pending candidate)
    w.verify = [truth](const std::vector<uint32_t> &idx, std::vector<int32_t> &res) {
        for (uint32_t k : idx) res[k] = truth[k];
        return RSG_OK;
    };
    uint64_t pos = 0;
    const rsg_status s = w.run(C, pos, nullptr);
    if (s != RSG_OK) return s;
    *n_out = found.size();
    stats[0] = w.batches;
    stats[1] = w.windows;
    if (found.size() > cap) return fail(nullptr, RSG_ERR_TRUNCATED, "%llu matches", (unsigned long long)found.size());
    if (!found.empty()) memcpy(out, found.data(), found.size() * sizeof(rsg_match));
    return RSG_OK;
}

rsg_status rsg_hash_search_device(rsg_ctx *ctx, const void *d_src, uint64_t src_len, const rsg_sum_head *head,
                                  const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                  rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    return search_one(ctx, d_src, src_len, head, sum1, sum2, targets, seed, matches, match_cap, n_matches, false);
}

rsg_status rsg_hash_search_host(rsg_ctx *ctx, const uint8_t *src, uint64_t src_len, const rsg_sum_head *head,
                                const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    return search_one(ctx, src, src_len, head, sum1, sum2, targets, seed, matches, match_cap, n_matches, true);
}

}  // extern "C"
