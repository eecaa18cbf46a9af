// rsg_sender_small.cpp -- host side of the small-file sender
// (rsg_search_small.hip): SendFiles' per-file hashSearch loop
// (internal/sender/sender.go:19-115, match.go:21-230) for the many small
// sources of a file tree, a few thousand files per launch.
//
// Per launch ("chunk", files whose basis counts share one power-of-two class
// so they share one LDS layout): worker threads validate each job as
// SumHead.ReadFrom + build_hash_table would (types.go:38-77, sender.go:60-83)
// and copy its sums -- sum1[count] | targets[count] | sum2[16 count], and
// for host sources the source bytes -- into a pinned staging slot; one H2D
// (copy stream), one kernel (compute stream) whose per-file match lists and
// statuses land straight in pinned host memory.  Two slots: chunk c+1 is
// packed and uploaded while chunk c runs, chunk c-1's results are scattered
// into the callers' match arrays meanwhile.  (Scattering chunk c-2 instead,
// so that packing never waits for the kernel it feeds, measured slower:
// 12.4-13.1 against 11.1-11.4 ms per cfg4-sender call, round 6.)  Files whose candidates overflow
// the kernel's LDS list go back to the caller for the large-file pipeline.
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "rsg_host.h"

using rsg::SmallJob;
using rsg::SmallOut;

namespace rsgh {

namespace {

// the first launch is small, so the GPU starts after packing a few thousand
// files instead of 16 384 (the rest of the call's packing hides under it)
constexpr uint64_t kFirstChunkJobs = 2048;
constexpr uint64_t kChunkJobs = 16384;  // 8192 / 4096: 248-264 / 255-272 GiB/s against 280-285 (cfg4-sender, round 6)
constexpr uint64_t kChunkBlob = 128ull << 20;   // sums bytes per launch
constexpr uint64_t kChunkSrc = 256ull << 20;    // host-source bytes per launch
constexpr uint64_t kChunkMatches = 4ull << 20;  // match slots per launch (16 B each)

uint64_t a16(uint64_t x) { return (x + 15) & ~15ull; }
uint64_t a256(uint64_t x) { return (x + 255) & ~255ull; }
uint64_t blob_bytes(int32_t count) { return 2 * a16(4ull * (uint64_t)count) + 16ull * (uint64_t)count; }

uint32_t count_class(int32_t count) {
    uint32_t kc = 64;
    while ((int32_t)kc < count) kc <<= 1;
    return kc;
}

// match slots a job can need: a match consumes at least the shortest block
uint64_t match_slots(const rsg_search_job &j, uint32_t kc) {
    const uint32_t minlen = (j.head.rem != 0) ? (uint32_t)std::min(j.head.rem, j.head.block_len)
                                              : (uint32_t)j.head.block_len;
    return std::min<uint64_t>(rsg::small_ccap(kc), j.src_len / std::max(1u, minlen) + 1);
}

// Seven workers kept for the process (a call runs ~30 parallel loops; a
// thread per loop and worker cost ~3 ms of the 17 ms cfg4-sender call,
// round 6) plus the calling thread.  One loop at a time (calls into the
// small-file path hold their context's lock; a second context's loop waits
// for the pool).  A forked child has none of the parent's workers: there
// the calling thread runs the loop alone.
class Pool {
public:
    static Pool &get() {
        static Pool *p = new Pool;  // never destroyed: the workers idle in their wait until the process ends
        return *p;
    }
    void run(const std::function<void()> &work) {
        if (getpid() != pid_) {
            work();
            return;
        }
        std::unique_lock<std::mutex> one(busy_);
        {
            std::lock_guard<std::mutex> g(mu_);
            work_ = &work;
            pending_ = kWorkers;
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return pending_ == 0; });
        work_ = nullptr;
    }
private:
    static constexpr int kWorkers = 7;
    Pool() : pid_(getpid()) {
        for (int i = 0; i < kWorkers; i++) std::thread([this] { loop(); }).detach();
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void()> *w;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                w = work_;
            }
            (*w)();
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    const pid_t pid_;
    std::mutex busy_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void()> *work_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
};

template <class F>
void parallel_for(uint64_t n, F f) {
    std::atomic<uint64_t> next{0};
    const std::function<void()> work = [&] {
        for (uint64_t i; (i = next.fetch_add(64)) < n;)
            for (uint64_t k = i; k < std::min(n, i + 64); k++) f(k);
    };
    if (n < 512) work();
    else Pool::get().run(work);
}

// check_args of rsg_match.cpp without touching the context (worker threads):
// "" = valid.  SumHead.ReadFrom (types.go:38-77) and a permutation `targets`.
std::string validate(const rsg_search_job &j, std::vector<uint8_t> &seen) {
    char b[96];
    const rsg_sum_head &h = j.head;
    if (h.count < 0) return snprintf(b, sizeof b, "invalid checksum count %d", h.count), b;
    if (h.block_len < 0 || h.block_len > RSG_MAX_BLOCK_LEN)
        return snprintf(b, sizeof b, "invalid block length %d", h.block_len), b;
    if (h.s2len < 0 || h.s2len > 16) return snprintf(b, sizeof b, "invalid checksum length %d", h.s2len), b;
    if (h.rem < 0 || h.rem > h.block_len) return snprintf(b, sizeof b, "invalid remainder length %d", h.rem), b;
    if (h.count > 0 && h.block_len == 0) return "zero block length";
    if (h.count > 0 && (!j.sum1 || !j.sum2 || !j.targets)) return "NULL sums or targets";
    if (j.match_cap && !j.matches) return "NULL matches";
    if (h.count > 0 && j.src_len > 0 && !j.src) return "NULL source";
    seen.assign((size_t)h.count, 0);
    for (int32_t k = 0; k < h.count; k++) {
        const int32_t i = j.targets[k];
        if (i < 0 || i >= h.count || seen[(size_t)i]) return "targets is not a permutation";
        seen[(size_t)i] = 1;
    }
    return "";
}

// RSG_TIMING: the call's host phases, summed over its chunks, to stderr
struct SmallTimes {
    bool on = getenv("RSG_TIMING") != nullptr;
    double ms[6] = {};  // validate, chunk, pack, issue, wait, scatter
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(int k) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        ms[k] += std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    }
    ~SmallTimes() {
        if (on)
            fprintf(stderr, "[rsg] small: validate %.3f chunk %.3f pack %.3f issue %.3f wait %.3f scatter %.3f ms\n",
                    ms[0], ms[1], ms[2], ms[3], ms[4], ms[5]);
    }
};

struct Chunk {
    uint32_t kc = 64;
    std::vector<uint64_t> jobs;  // indices into the caller's jobs
    uint64_t blob = 0, src = 0, slots = 0;
};

}  // namespace

bool search_small_eligible(const rsg_ctx *ctx, const rsg_search_job &j) {
    return ctx->opts.path != 1 && j.src_len >= 1 && j.src_len <= rsg::kSmallMaxSrc && j.head.count >= 1 &&
           j.head.count <= rsg::kSmallMaxCount && j.head.block_len >= 1 &&
           (uint32_t)j.head.block_len <= rsg::kSmallMaxBlock;
}

rsg_status search_small_batch(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed, bool host_src,
                              std::vector<uint64_t> &rest, std::vector<std::string> &msg) {
    rest.clear();
    msg.assign(njobs, std::string());
    SmallTimes tm;
    // 1. validate every job (job-local errors settle it), settle the empty
    // ones (count 0: sendFile, sender.go:86-88; empty source), classify
    std::vector<uint8_t> kind(njobs, 0);  // 0 settled, 1 small, 2 rest
    parallel_for(njobs, [&](uint64_t i) {
        thread_local std::vector<uint8_t> seen;
        rsg_search_job &j = jobs[i];
        j.n_matches = 0;
        j.status = RSG_OK;
        std::string e = validate(j, seen);
        if (!e.empty()) {
            j.status = RSG_ERR_INVALID;
            msg[i] = std::move(e);
            return;
        }
        if (j.head.count == 0 || j.src_len == 0) return;
        kind[i] = search_small_eligible(ctx, j) ? 1 : 2;
    });
    tm.lap(0);
    // 2. chunks: per count class, in job order
    std::vector<Chunk> chunks;
    {
        Chunk open[5];
        for (int c = 0; c < 5; c++) open[c].kc = 64u << c;
        for (uint64_t i = 0; i < njobs; i++) {
            if (kind[i] == 2) rest.push_back(i);
            if (kind[i] != 1) continue;
            const rsg_search_job &j = jobs[i];
            const uint32_t kc = count_class(j.head.count);
            Chunk &ch = open[__builtin_ctz(kc) - 6];
            const uint64_t b = blob_bytes(j.head.count), s = host_src ? a16(j.src_len) : 0, m = match_slots(j, kc);
            const uint64_t cap_jobs = chunks.empty() ? kFirstChunkJobs : kChunkJobs;
            if (!ch.jobs.empty() && (ch.jobs.size() >= cap_jobs || ch.blob + b > kChunkBlob ||
                                     ch.src + s > kChunkSrc || ch.slots + m > kChunkMatches)) {
                chunks.push_back(std::move(ch));
                ch = Chunk();
                ch.kc = kc;
            }
            ch.jobs.push_back(i);
            ch.blob += b;
            ch.src += s;
            ch.slots += m;
        }
        for (Chunk &ch : open)
            if (!ch.jobs.empty()) chunks.push_back(std::move(ch));
    }
    tm.lap(1);
    if (chunks.empty()) return RSG_OK;
    // sources written on the context's stream (fills, copies) come first
    RSG_HIP(ctx, hipEventRecord(ctx->side_done[0], ctx->stream));
    for (int k = 0; k < 2; k++) RSG_HIP(ctx, hipStreamWaitEvent(ctx->side[k], ctx->side_done[0], 0));
    for (int s = 0; s < 2; s++) {
        SmallSlot &sl = ctx->small[s];
        if (!sl.up) RSG_HIP(ctx, hipEventCreateWithFlags(&sl.up, hipEventDisableTiming));
        if (!sl.done) RSG_HIP(ctx, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
    hipStream_t copy = ctx->side[1], comp = ctx->side[0];
    rsg_status s;
    // 3. results of chunk c (its kernel done): matches into the callers' arrays
    auto scatter = [&](const Chunk &ch, SmallSlot &sl) -> rsg_status {
        tm.lap(3);
        RSG_HIP(ctx, hipEventSynchronize(sl.done));
        tm.lap(4);
        const SmallOut *outs = (const SmallOut *)sl.outs.p;
        const rsg_match *ms = (const rsg_match *)sl.matches.p;
        std::atomic<bool> any_rest{false};
        std::vector<uint8_t> back(ch.jobs.size(), 0);
        parallel_for(ch.jobs.size(), [&](uint64_t k) {
            rsg_search_job &j = jobs[ch.jobs[k]];
            const SmallOut o = outs[k];
            if (o.status != 0) {
                back[k] = 1;
                any_rest = true;
                return;
            }
            j.n_matches = o.n;
            if (o.n > j.match_cap) {
                j.status = RSG_ERR_TRUNCATED;
                char b[96];
                snprintf(b, sizeof b, "%u matches, capacity %llu", o.n, (unsigned long long)j.match_cap);
                msg[ch.jobs[k]] = b;
            } else if (o.n) {
                memcpy(j.matches, ms + o.base, (size_t)o.n * sizeof(rsg_match));
            }
        });
        if (any_rest)
            for (uint64_t k = 0; k < ch.jobs.size(); k++)
                if (back[k]) rest.push_back(ch.jobs[k]);
        tm.lap(5);
        return RSG_OK;
    };
    for (size_t c = 0; c <= chunks.size(); c++) {
        if (c < chunks.size()) {
            const Chunk &ch = chunks[c];
            SmallSlot &sl = ctx->small[c & 1];
            const uint64_t J = ch.jobs.size();
            const uint64_t off_order = a256(J * sizeof(SmallJob)), off_blob = off_order + a256(J * 4);
            const uint64_t off_src = off_blob + a256(ch.blob), total = off_src + ch.src;
            // slot c & 1 was last used by chunk c - 2, scattered below in round c - 1
            if ((s = ensure_pin(ctx, sl.stage, total)) != RSG_OK) return s;
            if ((s = ensure_dev(ctx, sl.dev, total)) != RSG_OK) return s;
            if ((s = ensure_pin(ctx, sl.outs, J * sizeof(SmallOut))) != RSG_OK) return s;
            if ((s = ensure_pin(ctx, sl.matches, ch.slots * sizeof(rsg_match))) != RSG_OK) return s;
            if ((s = ensure_dev(ctx, sl.count, 64)) != RSG_OK) return s;
            uint8_t *st = (uint8_t *)sl.stage.p;
            const uint64_t dev = (uint64_t)(uintptr_t)sl.dev.p;
            // offsets (prefix over the chunk's jobs), then the copies in parallel
            std::vector<uint64_t> bo(J + 1, 0), so(J + 1, 0);
            for (uint64_t k = 0; k < J; k++) {
                const rsg_search_job &j = jobs[ch.jobs[k]];
                bo[k + 1] = bo[k] + blob_bytes(j.head.count);
                so[k + 1] = so[k] + (host_src ? a16(j.src_len) : 0);
            }
            SmallJob *desc = (SmallJob *)st;
            parallel_for(J, [&](uint64_t k) {
                const rsg_search_job &j = jobs[ch.jobs[k]];
                const uint64_t c4 = 4ull * (uint64_t)j.head.count;
                uint8_t *b = st + off_blob + bo[k];
                memcpy(b, j.sum1, c4);
                memcpy(b + a16(c4), j.targets, c4);
                memcpy(b + 2 * a16(c4), j.sum2, 4 * c4);
                uint64_t src = (uint64_t)(uintptr_t)j.src;
                if (host_src) {
                    memcpy(st + off_src + so[k], j.src, j.src_len);
                    src = dev + off_src + so[k];
                }
                desc[k] = SmallJob{src, bo[k], (uint32_t)j.src_len, j.head.count, (uint32_t)j.head.block_len,
                                   (uint32_t)j.head.rem, (uint32_t)j.head.s2len, 0};
            });
            // longest files first: the launch's last waves are its shortest
            // (a counting sort on the length in 4 KiB steps, kSmallMaxSrc = 1 MiB)
            uint32_t *order = (uint32_t *)(st + off_order);
            {
                constexpr uint32_t kBins = (uint32_t)(rsg::kSmallMaxSrc >> 12) + 1;
                uint32_t cnt[kBins + 1] = {};
                auto bin = [&](uint64_t k) { return kBins - 1 - (desc[k].size >> 12); };  // longest first
                for (uint64_t k = 0; k < J; k++) cnt[bin(k) + 1]++;
                for (uint32_t b = 0; b < kBins; b++) cnt[b + 1] += cnt[b];
                for (uint64_t k = 0; k < J; k++) order[cnt[bin(k)]++] = (uint32_t)k;
            }
            tm.lap(2);
            RSG_HIP(ctx, hipMemcpyAsync(sl.dev.p, st, total, hipMemcpyHostToDevice, copy));
            RSG_HIP(ctx, hipEventRecord(sl.up, copy));
            RSG_HIP(ctx, hipStreamWaitEvent(comp, sl.up, 0));
            RSG_HIP(ctx, hipMemsetAsync(sl.count.p, 0, 4, comp));
            hipEvent_t t0 = timed_begin(ctx, comp);  // counted with the rolls (rsg_kernel_times out[0..1])
            RSG_HIP(ctx, rsg::launch_search_small((const SmallJob *)sl.dev.p, (const uint32_t *)((uint8_t *)sl.dev.p + off_order),
                                                  (uint32_t)J, (const uint8_t *)sl.dev.p + off_blob, (uint32_t)seed,
                                                  ch.kc, sl.matches.p, (uint32_t)ch.slots, (uint32_t *)sl.count.p,
                                                  (SmallOut *)sl.outs.p, comp));
            timed_end(ctx, t0, comp, 0);
            RSG_HIP(ctx, hipEventRecord(sl.done, comp));
        }
        if (c >= 1 && (s = scatter(chunks[c - 1], ctx->small[(c - 1) & 1])) != RSG_OK) return s;
    }
    std::sort(rest.begin(), rest.end());
    return RSG_OK;
}

}  // namespace rsgh
