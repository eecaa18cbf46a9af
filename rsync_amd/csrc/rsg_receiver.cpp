// rsg_receiver.cpp -- the receiver's token application:
// receiveData + recvToken, internal/receiver/receiver.go:98-188 and
// internal/receiver/token.go:6-20.
//
// The token stream (after the SumHead) is: literal runs (int32 LE n > 0, then
// n bytes), block matches (int32 -(i+1): block i of the basis, BlockLength
// bytes at i*BlockLength, RemainderLength for the last block), the int32 0
// terminator, then the sender's 16-byte whole-file sum MD4(int32_LE(seed) ||
// file).  Rebuilding is byte copying (the reference does one ReadAt per
// matched block).  The whole-file sum h = MD4(int32_LE(seed) || file)
// (receiver.go:117-120,166) is one serial chain per file: the GPU's seeded
// file-sum kernel (rsg_filesums.hip) hashes many files at once, one lane per
// file, but a lane is ~10x slower than a host core, so a
// single file (rsg_receive_data) is hashed on the host while its tokens are
// applied, as the reference writes h as it goes (receiver.go:159-164), and
// a batch (rsg_receive_data_batch) hashes its small files on the GPU and its
// large ones (on_host below) on a host pool beside the GPU pipeline.
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "rsg_host.h"

using namespace rsgh;

namespace {

int32_t rd_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// Walks the stream; copies into out while it fits.  Sets *out_len (the
// rebuilt length) and *sum_at (offset of the 16-byte whole-file sum).
// With h, the rebuilt bytes are also fed to h as they are written (the
// reference's h.Write of every token's data, receiver.go:159-164).
rsg_status apply(rsg_ctx *ctx, const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                 const uint8_t *basis, uint64_t basis_len, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                 uint64_t *sum_at, Md4 *h = nullptr, std::atomic<uint64_t> *progress = nullptr) {
    if (!head || !out_len || (tokens_len && !tokens))
        return fail(ctx, RSG_ERR_INVALID, "NULL argument");
    uint64_t pos = 0, off = 0;
    bool fits = true;
    for (;;) {
        if (pos + 4 > tokens_len) return fail(ctx, RSG_ERR_INVALID, "token stream ends before its terminator");
        const int32_t token = rd_i32(tokens + pos);  // recvToken, token.go:8
        pos += 4;
        if (token == 0) break;  // receiver.go:128-130
        const uint8_t *data;
        uint64_t n;
        if (token > 0) {  // literal: io.ReadFull of token bytes, token.go:15-18
            n = (uint64_t)token;
            if (pos + n > tokens_len)
                return fail(ctx, RSG_ERR_INVALID, "literal of %llu bytes runs past the stream", (unsigned long long)n);
            data = tokens + pos;
            pos += n;
        } else {
            if (!basis)  // receiver.go:143-145 (no local file open)
                return fail(ctx, RSG_ERR_INVALID, "match token without a basis file");
            const int64_t idx = -((int64_t)token + 1);  // receiver.go:146
            const int64_t off2 = idx * (int64_t)head->block_len;
            n = (uint64_t)head->block_len;
            if (idx == head->count - 1 && head->rem != 0) n = (uint64_t)head->rem;  // :148-151
            if ((uint64_t)off2 + n > basis_len)  // ReadAt short read, :155-157
                return fail(ctx, RSG_ERR_INVALID, "block %lld reads past the basis (%llu bytes)", (long long)idx,
                            (unsigned long long)basis_len);
            data = basis + off2;
        }
        if (out && off + n <= out_cap) {
            memcpy(out + off, data, n);
            if (h) h->update(out + off, n);
            if (progress) progress->store(off + n, std::memory_order_release);
        } else if (out) {
            fits = false;
        }
        off += n;
    }
    *out_len = off;
    if (sum_at) *sum_at = pos;
    if (!fits) return fail(ctx, RSG_ERR_TRUNCATED, "rebuilt file needs %llu bytes", (unsigned long long)off);
    return RSG_OK;
}

// The whole-file sum's seed prefix, binary.Write(h, LittleEndian, seed)
// (receiver.go:117-120).
void md4_seeded(Md4 &h, int32_t seed) {
    h.init();
    const uint8_t sb[4] = {(uint8_t)seed, (uint8_t)(seed >> 8), (uint8_t)(seed >> 16), (uint8_t)(seed >> 24)};
    h.update(sb, 4);
}

// Which jobs hash on the host.  One GPU lane hashes ~0.09 GiB/s (one serial
// MD4 chain); the GPU path as a whole -- token application,
// staging, upload, many lanes at once -- moves a transfer's small files at
// ~5.5 GiB/s.  A file whose lane would take longer than the GPU path needs
// for a whole 256 MiB batch (> ~4 MiB) is hashed on host threads instead,
// beside the GPU pipeline: a host core does one chain at ~1 GiB/s.
// rsg_ctx::Options::recv_md4 = 1 (GPU) / 2 (host) forces one side (tests, A/B;
// rsg_testing_search_option 5).
constexpr uint64_t kHostMd4MinBytes = 4ull << 20;
// rsg_receive_data: files at least this large apply their tokens on a second
// thread while the caller's thread hashes behind it (one thread below: the
// thread start costs more than it saves).
constexpr uint64_t kPipelineMinBytes = 8ull << 20;
bool on_host(const rsg_recv_job &j, int mode) {
    if (mode) return mode == 2;
    return j.out_cap >= kHostMd4MinBytes;
}

int copy_threads() {
    const char *e = getenv("RSG_COPY_THREADS");
    const int t = e ? atoi(e) : 8;
    return std::max(1, std::min(t, 64));
}

// Token application of many jobs on a few host threads (byte copying; each
// job writes only its own output).  Sets every job's out_len / consumed /
// status; returns nothing (failures are per job).
// One job entirely on this thread: tokens applied with the seeded MD4 fed as
// the bytes are written (receiver.go:117-120,159-164), then the sum check.
void run_host_job(rsg_recv_job &j, int32_t seed) {
    j.out_len = 0;
    j.consumed = 0;
    uint64_t at = 0;
    Md4 h;
    md4_seeded(h, seed);
    rsg_status st = apply(nullptr, j.tokens, j.tokens_len, &j.head, j.basis, j.basis_len, j.out, j.out_cap,
                          &j.out_len, &at, &h);
    if (st == RSG_OK && at + 16 > j.tokens_len) st = RSG_ERR_INVALID;  // receiver.go:167-170
    if (st == RSG_OK && j.out_len && !j.out) st = RSG_ERR_INVALID;
    if (st == RSG_OK) {
        uint8_t local[16];
        h.final(local);
        j.consumed = at + 16;
        if (memcmp(local, j.tokens + at, 16) != 0) st = RSG_ERR_CORRUPT;  // receiver.go:171-173
    }
    j.status = st;
}

// host[k - i0] != 0: job k belongs to the host pool (run_host_job), skip it.
void apply_jobs(rsg_recv_job *jobs, uint64_t i0, uint64_t i1, std::vector<uint64_t> &sum_at,
                const std::vector<uint8_t> &host) {
    const int threads = copy_threads();
    std::atomic<uint64_t> next{i0};
    auto worker = [&] {
        for (uint64_t k; (k = next.fetch_add(1)) < i1;) {
            if (host[k - i0]) continue;
            rsg_recv_job &j = jobs[k];
            j.out_len = 0;
            j.consumed = 0;
            uint64_t at = 0;
            rsg_status st = apply(nullptr, j.tokens, j.tokens_len, &j.head, j.basis, j.basis_len, j.out, j.out_cap,
                                  &j.out_len, &at);
            if (st == RSG_OK && at + 16 > j.tokens_len) st = RSG_ERR_INVALID;  // receiver.go:167-170
            if (st == RSG_OK && j.out_len && !j.out) st = RSG_ERR_INVALID;
            sum_at[k - i0] = at;
            j.status = st;
        }
    };
    uint64_t bytes = 0;
    for (uint64_t k = i0; k < i1; k++) bytes += host[k - i0] ? 0 : jobs[k].tokens_len;
    const int nt = (int)std::min<uint64_t>((uint64_t)threads, std::min<uint64_t>(i1 - i0, 1 + bytes / (1ull << 20)));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
}

}  // namespace

extern "C" {

rsg_status rsg_apply_tokens(const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed) {
    uint64_t sum_at = 0;
    rsg_status s = apply(nullptr, tokens, tokens_len, head, basis, basis_len, out, out_cap, out_len, &sum_at);
    if (consumed) *consumed = sum_at;
    return s;
}

rsg_status rsg_receive_data(rsg_ctx *ctx, const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, int32_t seed, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    // One file: h = MD4(seed_LE || rebuilt file) (receiver.go:117-120,166) is
    // one serial chain, hashed here as the tokens are applied -- on a GPU it
    // would get one lane, ~10x slower than this core.
    // Options::recv_md4 = 1 checks it with the GPU's seeded file-sum kernel instead.
    const bool gpu = ctx->opts.recv_md4 == 1;
    Md4 h;
    md4_seeded(h, seed);
    uint64_t sum_at = 0;
    rsg_status s;
    if (!gpu && out && out_cap >= kPipelineMinBytes) {
        // A large file: the tokens are applied (byte copies, first touches
        // of out) on a worker thread while this thread hashes the rebuilt
        // prefix behind it, so the call takes about the MD4 chain alone.
        std::atomic<uint64_t> done{0};
        std::atomic<bool> finished{false};
        std::thread copier([&] {
            s = apply(ctx, tokens, tokens_len, head, basis, basis_len, out, out_cap, out_len, &sum_at, nullptr,
                      &done);
            finished.store(true, std::memory_order_release);
        });
        uint64_t hashed = 0;
        for (;;) {
            const bool fin = finished.load(std::memory_order_acquire);
            const uint64_t d = done.load(std::memory_order_acquire);
            if (d > hashed) {
                h.update(out + hashed, d - hashed);
                hashed = d;
            } else if (fin) {
                break;
            } else {
                std::this_thread::yield();
            }
        }
        copier.join();
        if (s == RSG_OK && hashed != *out_len) s = fail(ctx, RSG_ERR_INVALID, "internal: hashed %llu of %llu bytes",
                                                        (unsigned long long)hashed, (unsigned long long)*out_len);
    } else {
        s = apply(ctx, tokens, tokens_len, head, basis, basis_len, out, out_cap, out_len, &sum_at, gpu ? nullptr : &h);
    }
    if (s != RSG_OK) return s;
    if (sum_at + 16 > tokens_len)  // io.ReadFull(remoteSum), receiver.go:167-170
        return fail(ctx, RSG_ERR_INVALID, "token stream ends before the whole-file sum");
    if (*out_len && !out) return fail(ctx, RSG_ERR_INVALID, "NULL output");
    uint8_t local[16];
    if (gpu) {
        rsg_file f;
        memset(&f, 0, sizeof f);
        f.data = out;
        f.len = *out_len;
        if ((s = rsg_file_sums_host(ctx, &f, 1, RSG_FILESUM_SEEDED, seed, local)) != RSG_OK) return s;
    } else {
        h.final(local);
    }
    if (consumed) *consumed = sum_at + 16;
    if (memcmp(local, tokens + sum_at, 16) != 0)  // receiver.go:171-173
        return fail(ctx, RSG_ERR_CORRUPT, "file corruption: whole-file sum mismatch");
    return RSG_OK;
}

// Batched receiveData (receiver.go:98-188 for every file of a transfer):
// batches of jobs (<= 256 MiB of rebuilt bytes) alternate between two slots.
// For batch k: tokens applied on host threads into the callers' out buffers,
// the rebuilt files staged into pinned memory (or DMA'd straight from out
// when it is page-locked), H2D, the seeded whole-file sum of every file (one
// lane per file), digests back -- all on the slot's stream, while the host
// applies batch k+1.  Each job's status: RSG_OK, RSG_ERR_INVALID /
// RSG_ERR_TRUNCATED from its token stream, RSG_ERR_CORRUPT on a sum mismatch
// (receiver.go:171-173).
rsg_status rsg_receive_data_batch(rsg_ctx *ctx, rsg_recv_job *jobs, uint64_t njobs, int32_t seed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (njobs && !jobs) return fail(ctx, RSG_ERR_INVALID, "jobs is NULL");
    for (uint64_t q = 0; q < njobs; q++) jobs[q].status = RSG_OK;  // jobs a fatal error stops get its status
    struct Drain {  // nothing outlives the call
        rsg_ctx *c;
        ~Drain() {
            for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(c->side[k]);
        }
    } drain{ctx};
    const uint64_t kBatchBytes = 256ull << 20;
    struct Slot {
        uint64_t i0 = 0, i1 = 0;
        std::vector<uint64_t> sum_at;
        std::vector<uint64_t> lane;  // job of digest d, ~0 for jobs that failed before hashing
        bool busy = false;
    } slots[2];
    auto finish = [&](Slot &sl, int k) -> rsg_status {
        if (!sl.busy) return RSG_OK;
        RSG_HIP(ctx, hipStreamSynchronize(ctx->side[k]));
        const uint8_t *dig = (const uint8_t *)ctx->h_out[k].p;
        for (uint64_t d = 0; d < sl.lane.size(); d++) {
            rsg_recv_job &j = jobs[sl.lane[d]];
            j.consumed = sl.sum_at[sl.lane[d] - sl.i0] + 16;
            if (memcmp(dig + 16 * d, j.tokens + sl.sum_at[sl.lane[d] - sl.i0], 16) != 0) j.status = RSG_ERR_CORRUPT;
        }
        sl.busy = false;
        return RSG_OK;
    };
    // large files: a host pool beside the GPU pipeline (on_host)
    std::vector<uint8_t> is_host(njobs, 0);
    std::vector<uint64_t> host_jobs;
    const int md4_mode = ctx->opts.recv_md4;
    for (uint64_t q = 0; q < njobs; q++)
        if (on_host(jobs[q], md4_mode)) {
            is_host[q] = 1;
            host_jobs.push_back(q);
        }
    std::atomic<uint64_t> next_host{0};
    std::vector<std::thread> pool;
    const int npool = (int)std::min<uint64_t>((uint64_t)copy_threads(), host_jobs.size());
    for (int t = 0; t < npool; t++)
        pool.emplace_back([&] {
            for (uint64_t x; (x = next_host.fetch_add(1)) < host_jobs.size();) run_host_job(jobs[host_jobs[x]], seed);
        });
    struct Join {
        std::vector<std::thread> &p;
        ~Join() {
            for (auto &t : p)
                if (t.joinable()) t.join();
        }
    } join_pool{pool};
    rsg_status fatal = RSG_OK;
    uint64_t i = 0;
    for (int k = 0; i < njobs; k ^= 1) {
        Slot &sl = slots[k];
        if ((fatal = finish(sl, k)) != RSG_OK) break;
        // the batch: GPU jobs until ~kBatchBytes of rebuilt bytes (bounded
        // by out_cap, known before applying)
        uint64_t i1 = i, est = 0;
        while (i1 < njobs && (i1 == i || est + (is_host[i1] ? 0 : jobs[i1].out_cap) <= kBatchBytes))
            est += is_host[i1] ? 0 : jobs[i1].out_cap, i1++;
        sl.i0 = i;
        sl.i1 = i1;
        sl.sum_at.assign(i1 - i, 0);
        const std::vector<uint8_t> host(is_host.begin() + (int64_t)i, is_host.begin() + (int64_t)i1);
        apply_jobs(jobs, i, i1, sl.sum_at, host);
        sl.lane.clear();
        std::vector<rsg::FileSpan> spans;
        std::vector<CopyJob> copies;
        uint64_t off = 0;
        for (uint64_t q = i; q < i1; q++) {
            // host jobs first: a host-pool thread may be writing that job's
            // fields right now, so its status is not read here
            if (host[q - i] || jobs[q].status != RSG_OK) continue;  // checked on the host, or failed
            sl.lane.push_back(q);
            spans.push_back({off, jobs[q].out_len});
            if (jobs[q].out_len) copies.push_back({nullptr, jobs[q].out, jobs[q].out_len});
            off += (jobs[q].out_len + 15) & ~15ull;
        }
        i = i1;
        if (sl.lane.empty()) continue;
        if ((fatal = ensure_dev(ctx, ctx->d_in[k], off + 16)) != RSG_OK) break;
        if ((fatal = ensure_pin(ctx, ctx->h_in[k], off + 16)) != RSG_OK) break;
        if ((fatal = ensure_dev(ctx, ctx->d_out[k], sl.lane.size() * 16)) != RSG_OK) break;
        if ((fatal = ensure_pin(ctx, ctx->h_out[k], sl.lane.size() * 16)) != RSG_OK) break;
        uint8_t *stage = (uint8_t *)ctx->h_in[k].p;
        uint64_t at = 0;
        for (size_t c = 0, d = 0; d < sl.lane.size(); d++) {
            const uint64_t n = jobs[sl.lane[d]].out_len;
            if (n) copies[c++].dst = stage + at;
            at += (n + 15) & ~15ull;
        }
        parallel_copy(copies);
        hipStream_t st = ctx->side[k];
        hipError_t e = hipMemcpyAsync(ctx->d_in[k].p, stage, off, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) {
            fatal = hip_fail(ctx, e, "receive batch H2D");
            break;
        }
        if ((fatal = launch_file_sums_async(ctx, ctx->d_in[k].p, off, spans, RSG_FILESUM_SEEDED, seed,
                                            ctx->d_out[k].p, k, st)) != RSG_OK)
            break;
        e = hipMemcpyAsync(ctx->h_out[k].p, ctx->d_out[k].p, sl.lane.size() * 16, hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) {
            fatal = hip_fail(ctx, e, "receive batch D2H");
            break;
        }
        sl.busy = true;
    }
    for (int k = 0; k < 2 && fatal == RSG_OK; k++) fatal = finish(slots[k], k);
    for (auto &t : pool) t.join();  // the host pool's jobs are done (and keep their own statuses)
    if (fatal != RSG_OK) {
        for (uint64_t q = 0; q < njobs; q++)
            if (jobs[q].status == RSG_OK && !is_host[q]) jobs[q].status = fatal;
        return fatal;
    }
    for (uint64_t q = 0; q < njobs; q++) {
        if (jobs[q].status != RSG_OK) {
            const int32_t st = jobs[q].status;
            return fail(ctx, st, "job %llu: %s", (unsigned long long)q,
                        st == RSG_ERR_CORRUPT ? "file corruption: whole-file sum mismatch"
                                              : (st == RSG_ERR_TRUNCATED ? "output capacity too small"
                                                                         : "bad token stream"));
        }
    }
    return RSG_OK;
}

}  // extern "C"
