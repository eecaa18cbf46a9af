// rsg_shard.cpp -- one process driving the GPUs of a node.
//
// gokr-rsync's receiver is one process whose generator is one goroutine
// (internal/receiver/do.go:96-98) emitting every file's sums in file-list
// order (internal/receiver/generator.go:20-52).  Block sums of different
// blocks are independent (generator.go:332-348), so the file list's global
// block sequence is cut into one contiguous, byte-balanced range per device
// (plan_shards, cut on block boundaries) and each range into batches
// (split_batches); the concatenation of the ranks' records in rank order is
// exactly the single-device record stream.  rsync_amd/shard.py / dist.py
// restate the same arithmetic for the multi-process bench and the tests
// (tests/test_shard_plan.py checks the two agree byte for byte).
//
// Entry points (include/rsg.h): the plan, a single-process communicator
// (ncclCommInitAll), the device-resident gather / D2H step over N contexts
// from one thread, and the host-buffer and file-descriptor generator calls
// over N contexts.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rsg_host.h"

using namespace rsgh;
using rsg::kRecordBytes;

namespace {

struct Pc {
    uint64_t file, b0, b1, offset, length;
    uint32_t B;
};

// shard.plan_shards: rank r's range ends at byte total * (r + 1) / world of
// the global sequence, cut down to a block boundary; a rank takes at least one
// block while bytes remain; the last rank takes the rest.
bool plan_shards(const uint64_t *lengths, const int32_t *bls, uint64_t nfiles, int32_t bl, int world,
                 std::vector<std::vector<Pc>> &shards, std::vector<rsg_sum_head> &heads, std::string &err) {
    shards.assign((size_t)world, {});
    heads.resize(nfiles);
    unsigned __int128 total = 0;
    for (uint64_t f = 0; f < nfiles; f++) {
        if (lengths[f] > (uint64_t)INT64_MAX || !head_for((int64_t)lengths[f], bls ? bls[f] : bl, &heads[f])) {
            err = "file " + std::to_string(f) + ": bad length / block_len";
            return false;
        }
        total += lengths[f];
    }
    uint64_t done = 0;
    int r = 0;
    for (uint64_t f = 0; f < nfiles; f++) {
        const uint64_t B = (uint64_t)heads[f].block_len, cnt = (uint64_t)heads[f].count;
        uint64_t b = 0;
        while (b < cnt) {
            const uint64_t target = r < world - 1 ? (uint64_t)(total * (unsigned)(r + 1) / (unsigned)world) : (uint64_t)total;
            const uint64_t room = target > done ? target - done : 0;
            uint64_t nb = cnt - b;
            if (r < world - 1) {
                nb = std::min(nb, room / B);
                if (nb == 0) {
                    if (room > 0 && shards[(size_t)r].empty()) {
                        nb = 1;
                    } else {
                        r++;
                        continue;
                    }
                }
            }
            const uint64_t b1 = b + nb, off = b * B, ln = std::min(b1 * B, lengths[f]) - off;
            shards[(size_t)r].push_back({f, b, b1, off, ln, (uint32_t)B});
            done += ln;
            b = b1;
        }
    }
    return true;
}

// dist.split_batches: one rank's pieces cut into nbatch groups of about equal
// bytes, on block boundaries.
std::vector<std::vector<Pc>> split_batches(const std::vector<Pc> &pieces, int nbatch) {
    std::vector<std::vector<Pc>> out((size_t)nbatch);
    unsigned __int128 total = 0;
    for (const Pc &p : pieces) total += p.length;
    int64_t done = 0;
    int b = 0;
    for (const Pc &p : pieces) {
        uint64_t b0 = p.b0;
        while (b0 < p.b1) {
            const int64_t target = b < nbatch - 1 ? (int64_t)(total * (unsigned)(b + 1) / (unsigned)nbatch) : (int64_t)total;
            const int64_t room = target - done;
            uint64_t nb = p.b1 - b0;
            if (b < nbatch - 1) {
                nb = std::min<uint64_t>(nb, room > 0 ? (uint64_t)room / p.B : 0);
                if (nb == 0) {
                    if (room > 0 && out[(size_t)b].empty()) {
                        nb = 1;
                    } else {
                        b++;
                        continue;
                    }
                }
            }
            const uint64_t off = b0 * p.B, end = std::min<uint64_t>((b0 + nb) * p.B, p.offset + p.length);
            out[(size_t)b].push_back({p.file, b0, b0 + nb, off, end - off, p.B});
            done += (int64_t)(end - off);
            b0 += nb;
        }
    }
    return out;
}

// Locks every context of a multi-context call, in one canonical order (by
// address) whatever the caller's array order, so two threads calling with
// {a, b} and {b, a} cannot deadlock (callers pass distinct contexts; every
// entry point takes at most its own lock otherwise).
struct MultiLock {
    std::vector<rsg_ctx *> c;
    explicit MultiLock(const std::vector<rsg_ctx *> &v) : c(v) {
        std::sort(c.begin(), c.end(), std::less<rsg_ctx *>());
        for (rsg_ctx *x : c) x->mu.lock();
    }
    ~MultiLock() {
        for (auto it = c.rbegin(); it != c.rend(); ++it) (*it)->mu.unlock();
    }
};

rsg_status check_ctxs(rsg_ctx *const *ctxs, int32_t n, std::vector<rsg_ctx *> &out) {
    if (!ctxs || n < 1) return fail(nullptr, RSG_ERR_INVALID, "need n >= 1 contexts");
    out.assign(ctxs, ctxs + n);
    for (int q = 0; q < n; q++) {
        if (!out[(size_t)q]) return fail(nullptr, RSG_ERR_INVALID, "context %d is NULL", q);
        for (int k = 0; k < q; k++)
            if (out[(size_t)k] == out[(size_t)q]) return fail(out[0], RSG_ERR_INVALID, "context %d repeats context %d", q, k);
    }
    return RSG_OK;
}

// The device-resident step over many contexts: batch b's kernel on every
// rank's stream, then `move(q, b)` queued on the rank's side[0] stream behind
// an event of that kernel (every rank's move of batch b issued together).
// out(q, sb): where rank q writes batch sb's records.
template <class Out, class Move>
rsg_status multi_pipeline(const rsg_shard_rank *ranks, int32_t n, int32_t seed, Out out, Move move) {
    std::vector<rsg_ctx *> given((size_t)n), cs;
    for (int q = 0; q < n; q++) given[(size_t)q] = ranks[q].ctx;
    rsg_status s = check_ctxs(given.data(), n, cs);
    if (s != RSG_OK) return s;
    rsg_ctx *c0 = cs[0];
    const uint64_t nbatch = ranks[0].nbatch;
    for (int q = 0; q < n; q++) {
        if (ranks[q].nbatch != nbatch) return fail(c0, RSG_ERR_INVALID, "rank %d: %llu batches, rank 0 has %llu", q,
                                                   (unsigned long long)ranks[q].nbatch, (unsigned long long)nbatch);
        if (nbatch && !ranks[q].batches) return fail(c0, RSG_ERR_INVALID, "rank %d: NULL batches", q);
        for (uint64_t b = 0; b < nbatch; b++)
            if (ranks[q].batches[b].plan && ranks[q].batches[b].plan->ctx != cs[(size_t)q])
                return fail(c0, RSG_ERR_INVALID, "rank %d batch %llu: plan of another context", q, (unsigned long long)b);
    }
    MultiLock lock(cs);
    struct Drain {  // nothing outlives the call, whatever path leaves
        std::vector<rsg_ctx *> &c;
        ~Drain() {
            for (rsg_ctx *x : c) {
                (void)hipSetDevice(x->device);
                (void)hipStreamSynchronize(x->stream);
                (void)hipStreamSynchronize(x->side[0]);
            }
        }
    } drain{cs};
    struct Events {
        std::vector<std::pair<int, hipEvent_t>> ev;
        ~Events() {
            for (auto &e : ev) {
                (void)hipSetDevice(e.first);
                hipEventDestroy(e.second);
            }
        }
    } evs;
    for (uint64_t b = 0; b < nbatch; b++) {
        for (int q = 0; q < n; q++) {
            rsg_ctx *ctx = cs[(size_t)q];
            RSG_HIP(c0, hipSetDevice(ctx->device));
            const rsg_shard_batch &sb = ranks[q].batches[b];
            if (sb.plan) {
                s = launch_plan(ctx, sb.plan->host, sb.plan->d_files, sb.plan->d_wg, ranks[q].d_arena, seed,
                                out(q, sb), sb.plan->d_scratch, ctx->stream);
                if (s != RSG_OK) return fail(c0, s, "rank %d: %s", q, ctx->err.c_str());
            }
            hipEvent_t e = nullptr;
            RSG_HIP(c0, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            evs.ev.push_back({ctx->device, e});
            RSG_HIP(c0, hipEventRecord(e, ctx->stream));
            RSG_HIP(c0, hipStreamWaitEvent(ctx->side[0], e, 0));
        }
        if ((s = move(cs, b)) != RSG_OK) return s;
    }
    for (rsg_ctx *ctx : cs) {
        RSG_HIP(c0, hipSetDevice(ctx->device));
        RSG_HIP(c0, hipStreamSynchronize(ctx->stream));
        RSG_HIP(c0, hipStreamSynchronize(ctx->side[0]));
    }
    return RSG_OK;
}

uint64_t batch_records(const rsg_shard_batch &sb) { return sb.plan ? sb.plan->host.total_blocks : 0; }

// One rank's records as they come from its generator thread.  The records
// of ranks > the one being written wait here, so the queue is bounded: a
// rank's generator blocks once `cap` bytes of its records are queued (the
// reference generator streams its sums with bounded memory,
// generator.go:20-52); the host memory of one call is then at most
// (n - 1) * (cap + one chunk) beyond the generators' own staging.
std::atomic<uint64_t> g_queue_cap{256ull << 20};  // rsg_testing_set_multi_queue_cap
std::atomic<uint64_t> g_queue_peak{0};      // largest queue of the last call (process-wide: valid for single-threaded tests only)
struct RankQueue {
    std::mutex mu;
    std::condition_variable cv;     // consumer: a chunk arrived or the rank is done
    std::condition_variable space;  // producer: the consumer took a chunk, or abort
    std::deque<std::vector<uint8_t>> chunks;
    uint64_t bytes = 0, cap = 0;
    bool done = false;
    rsg_status status = RSG_OK;
    std::string err;
    std::atomic<bool> *abort = nullptr;
};

int32_t push_chunk(void *user, const uint8_t *data, uint64_t len) {
    RankQueue *rq = (RankQueue *)user;
    if (rq->abort->load()) return 1;
    std::vector<uint8_t> v(data, data + len);
    {
        std::unique_lock<std::mutex> lk(rq->mu);
        // an empty queue always takes the chunk, whatever its size
        rq->space.wait(lk, [&] { return rq->bytes == 0 || rq->bytes + len <= rq->cap || rq->abort->load(); });
        if (rq->abort->load()) return 1;
        rq->bytes += len;
        uint64_t pk = g_queue_peak.load();
        while (rq->bytes > pk && !g_queue_peak.compare_exchange_weak(pk, rq->bytes)) {
        }
        rq->chunks.push_back(std::move(v));
    }
    rq->cv.notify_one();
    return 0;
}

}  // namespace

extern "C" {

rsg_status rsg_shard_plan(const uint64_t *lengths, const int32_t *block_lens, uint64_t nfiles, int32_t block_len,
                          int32_t world, int32_t nbatch, rsg_piece *pieces, uint64_t cap, uint64_t *n_pieces,
                          uint64_t *records) {
    if (!n_pieces || (nfiles && !lengths)) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    if (world < 1 || nbatch < 1) return fail(nullptr, RSG_ERR_INVALID, "world and nbatch must be >= 1");
    std::vector<std::vector<Pc>> shards;
    std::vector<rsg_sum_head> heads;
    std::string err;
    if (!plan_shards(lengths, block_lens, nfiles, block_len, world, shards, heads, err))
        return fail(nullptr, RSG_ERR_INVALID, "%s", err.c_str());
    std::vector<uint64_t> first(nfiles + 1, 0);
    for (uint64_t f = 0; f < nfiles; f++) first[f + 1] = first[f] + (uint64_t)heads[f].count;
    uint64_t k = 0;
    for (int q = 0; q < world; q++) {
        const auto groups = split_batches(shards[(size_t)q], nbatch);
        for (int b = 0; b < nbatch; b++) {
            uint64_t recs = 0;
            for (const Pc &p : groups[(size_t)b]) {
                if (pieces && k < cap)
                    pieces[k] = rsg_piece{p.file, p.b0, p.b1, p.offset, p.length, first[p.file] + p.b0,
                                          (int32_t)p.B, q, b, 0};
                k++;
                recs += p.b1 - p.b0;
            }
            if (records) records[(size_t)q * (size_t)nbatch + (size_t)b] = recs;
        }
    }
    *n_pieces = k;
    if (!pieces || k > cap)
        return fail(nullptr, RSG_ERR_TRUNCATED, "%llu pieces, capacity %llu", (unsigned long long)k,
                    (unsigned long long)(pieces ? cap : 0));
    return RSG_OK;
}

rsg_status rsg_comm_init_all(rsg_ctx *const *ctxs, int32_t n) {
    std::vector<rsg_ctx *> cs;
    rsg_status s = check_ctxs(ctxs, n, cs);
    if (s != RSG_OK) return s;
    std::vector<int> devs((size_t)n);
    for (int q = 0; q < n; q++) {
        devs[(size_t)q] = cs[(size_t)q]->device;
        for (int k = 0; k < q; k++)
            if (devs[(size_t)k] == devs[(size_t)q])
                return fail(cs[0], RSG_ERR_INVALID, "contexts %d and %d share device %d: one rank per device", k, q,
                            devs[(size_t)q]);
    }
    MultiLock lock(cs);
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
    if (r != ncclSuccess) return fail(cs[0], RSG_ERR_HIP, "ncclCommInitAll: %s", ncclGetErrorString(r));
    for (int q = 0; q < n; q++) {
        rsg_ctx *ctx = cs[(size_t)q];
        if (ctx->comm) ncclCommDestroy(ctx->comm);
        ctx->comm = comms[(size_t)q];
        ctx->nranks = n;
        ctx->rank = q;
    }
    return RSG_OK;
}

rsg_status rsg_block_sums_gather_multi(const rsg_shard_rank *ranks, int32_t n, int32_t seed, void *d_recv,
                                       int32_t root) {
    if (!ranks || n < 1) return fail(nullptr, RSG_ERR_INVALID, "need n >= 1 ranks");
    if (root < 0 || root >= n || !d_recv) return fail(ranks[0].ctx, RSG_ERR_INVALID, "bad root / d_recv");
    for (int q = 0; q < n; q++) {
        rsg_ctx *ctx = ranks[q].ctx;
        if (!ctx || !ctx->comm || ctx->nranks != n || ctx->rank != q)
            return fail(ranks[0].ctx, RSG_ERR_INVALID, "rank %d: not rank %d of an %d-rank rsg_comm_init_all", q, q, n);
        for (uint64_t b = 0; b < ranks[q].nbatch; b++) {
            const rsg_shard_batch &sb = ranks[q].batches[b];
            if (!sb.send_bytes || !sb.recv_offsets || sb.send_bytes[q] != batch_records(sb) * kRecordBytes)
                return fail(ranks[0].ctx, RSG_ERR_INVALID, "rank %d batch %llu: send_bytes / recv_offsets", q,
                            (unsigned long long)b);
        }
    }
    // the root's kernels write its records straight to their landing offsets
    auto out = [&](int q, const rsg_shard_batch &sb) -> uint8_t * {
        return q == root ? (uint8_t *)d_recv + sb.recv_offsets[q]
                         : (uint8_t *)ranks[q].d_records + sb.record_offset * kRecordBytes;
    };
    return multi_pipeline(ranks, n, seed, out, [&](std::vector<rsg_ctx *> &cs, uint64_t b) -> rsg_status {
        // one thread drives every communicator: their sends and receives go
        // in one group
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) return fail(cs[0], RSG_ERR_HIP, "ncclGroupStart: %s", ncclGetErrorString(r));
        rsg_status s = RSG_OK;
        for (int q = 0; q < n && s == RSG_OK; q++) {
            rsg_ctx *ctx = cs[(size_t)q];
            const rsg_shard_batch &sb = ranks[q].batches[b];
            if (hipSetDevice(ctx->device) != hipSuccess) s = fail(cs[0], RSG_ERR_HIP, "hipSetDevice");
            else
                s = gatherv(ctx, (const uint8_t *)ranks[q].d_records + sb.record_offset * kRecordBytes, sb.send_bytes,
                            q == root ? d_recv : nullptr, sb.recv_offsets, root, ctx->side[0], true);
            if (s != RSG_OK && ctx != cs[0]) s = fail(cs[0], s, "rank %d: %s", q, ctx->err.c_str());
        }
        r = ncclGroupEnd();
        if (s == RSG_OK && r != ncclSuccess) s = fail(cs[0], RSG_ERR_HIP, "ncclGroupEnd: %s", ncclGetErrorString(r));
        return s;
    });
}

rsg_status rsg_block_sums_d2h_multi(const rsg_shard_rank *ranks, int32_t n, int32_t seed, uint8_t *h_records) {
    if (!ranks || n < 1) return fail(nullptr, RSG_ERR_INVALID, "need n >= 1 ranks");
    if (!h_records) return fail(ranks[0].ctx, RSG_ERR_INVALID, "h_records is NULL");
    auto out = [&](int q, const rsg_shard_batch &sb) -> uint8_t * {
        return (uint8_t *)ranks[q].d_records + sb.record_offset * kRecordBytes;
    };
    return multi_pipeline(ranks, n, seed, out, [&](std::vector<rsg_ctx *> &cs, uint64_t b) -> rsg_status {
        for (int q = 0; q < n; q++) {
            rsg_ctx *ctx = cs[(size_t)q];
            const rsg_shard_batch &sb = ranks[q].batches[b];
            const uint64_t bytes = batch_records(sb) * kRecordBytes;
            if (!bytes) continue;
            RSG_HIP(cs[0], hipSetDevice(ctx->device));
            RSG_HIP(cs[0], hipMemcpyAsync(h_records + (ranks[q].rank_record_offset + sb.record_offset) * kRecordBytes,
                                          (const uint8_t *)ranks[q].d_records + sb.record_offset * kRecordBytes, bytes,
                                          hipMemcpyDeviceToHost, ctx->side[0]));
        }
        return RSG_OK;
    });
}

rsg_status rsg_block_sums_host_multi(rsg_ctx *const *ctxs, int32_t n, const rsg_file *files, uint64_t nfiles,
                                     int32_t seed, uint8_t *records, uint64_t records_cap) {
    std::vector<rsg_ctx *> cs;
    rsg_status s = check_ctxs(ctxs, n, cs);
    if (s != RSG_OK) return s;
    if (nfiles && !files) return fail(cs[0], RSG_ERR_INVALID, "files is NULL");
    std::vector<uint64_t> lengths(nfiles);
    std::vector<int32_t> bls(nfiles);
    for (uint64_t f = 0; f < nfiles; f++) {
        lengths[f] = files[f].len;
        bls[f] = files[f].block_len;
        if (files[f].len && !files[f].data) return fail(cs[0], RSG_ERR_INVALID, "file %llu: NULL data", (unsigned long long)f);
    }
    std::vector<std::vector<Pc>> shards;
    std::vector<rsg_sum_head> heads;
    std::string err;
    if (!plan_shards(lengths.data(), bls.data(), nfiles, 0, n, shards, heads, err))
        return fail(cs[0], RSG_ERR_INVALID, "%s", err.c_str());
    uint64_t total = 0;
    std::vector<uint64_t> first(nfiles, 0);
    for (uint64_t f = 0; f < nfiles; f++) {
        first[f] = total;
        total += (uint64_t)heads[f].count;
    }
    if (total > records_cap)
        return fail(cs[0], RSG_ERR_TRUNCATED, "need %llu records, capacity %llu", (unsigned long long)total,
                    (unsigned long long)records_cap);
    if (total && !records) return fail(cs[0], RSG_ERR_INVALID, "records is NULL");
    // Every rank's pieces are files of their own with the file's B: a piece
    // starts on a block boundary, so its blocks are the reference's.
    std::vector<rsg_status> st((size_t)n, RSG_OK);
    std::vector<std::thread> th;
    for (int q = 0; q < n; q++) {
        const auto &mine = shards[(size_t)q];
        if (mine.empty()) continue;
        th.emplace_back([&, q] {
            const auto &pcs = shards[(size_t)q];
            std::vector<rsg_file> vf(pcs.size());
            uint64_t recs = 0;
            for (size_t k = 0; k < pcs.size(); k++) {
                vf[k] = rsg_file{files[pcs[k].file].data + pcs[k].offset, 0, pcs[k].length, (int32_t)pcs[k].B, 0};
                recs += pcs[k].b1 - pcs[k].b0;
            }
            const uint64_t at = first[pcs[0].file] + pcs[0].b0;
            st[(size_t)q] = rsg_block_sums_host(cs[(size_t)q], vf.data(), vf.size(), seed, records + at * kRecordBytes,
                                                recs);
        });
    }
    for (auto &t : th) t.join();
    for (int q = 0; q < n; q++)
        if (st[(size_t)q] != RSG_OK)
            return q == 0 ? st[0] : fail(cs[0], st[(size_t)q], "rank %d: %s", q, cs[(size_t)q]->err.c_str());
    return RSG_OK;
}

rsg_status rsg_generate_files_fd_multi(rsg_ctx *const *ctxs, int32_t n, const rsg_fd_file *files, uint64_t nfiles,
                                       int32_t seed, int32_t flags, rsg_write_fn write, void *user,
                                       rsg_sum_head *heads_out, uint64_t *bytes_written) {
    std::vector<rsg_ctx *> cs;
    rsg_status s = check_ctxs(ctxs, n, cs);
    if (s != RSG_OK) return s;
    rsg_ctx *c0 = cs[0];
    if (bytes_written) *bytes_written = 0;
    if (!write || (nfiles && !files)) return fail(c0, RSG_ERR_INVALID, "NULL argument");
    if (flags & ~(RSG_GEN_IDX | RSG_GEN_TERMINATE | RSG_GEN_MUX))
        return fail(c0, RSG_ERR_INVALID, "unknown flags 0x%x", flags);
    std::vector<uint64_t> lengths(nfiles);
    std::vector<int32_t> bls(nfiles);
    for (uint64_t f = 0; f < nfiles; f++) {
        if (files[f].len > (uint64_t)INT64_MAX || files[f].offset < 0)
            return fail(c0, RSG_ERR_INVALID, "file %llu: bad offset/length", (unsigned long long)f);
        lengths[f] = files[f].len;
        bls[f] = files[f].block_len;
    }
    std::vector<std::vector<Pc>> shards;
    std::vector<rsg_sum_head> heads;
    std::string err;
    if (!plan_shards(lengths.data(), bls.data(), nfiles, 0, n, shards, heads, err))
        return fail(c0, RSG_ERR_INVALID, "%s", err.c_str());
    for (uint64_t f = 0; f < nfiles; f++) {
        if (heads[f].count && files[f].fd < 0)
            return fail(c0, RSG_ERR_INVALID, "file %llu: bad descriptor", (unsigned long long)f);
        if (heads_out) heads_out[f] = heads[f];
    }
    // ranks produce records only (rsg_generate.cpp, records_only); this
    // thread puts idx + SumHead in front of each file's records
    std::atomic<bool> abort{false};
    std::vector<RankQueue> qs((size_t)n);
    std::vector<std::thread> th;
    g_queue_peak = 0;
    for (int q = 0; q < n; q++) {
        RankQueue &rq = qs[(size_t)q];
        rq.abort = &abort;
        rq.cap = g_queue_cap.load();
        if (shards[(size_t)q].empty()) {
            rq.done = true;
            continue;
        }
        th.emplace_back([&, q] {
            RankQueue &me = qs[(size_t)q];
            std::vector<rsg_fd_file> vf;
            for (const Pc &p : shards[(size_t)q]) {
                const rsg_fd_file &F = files[p.file];
                vf.push_back(rsg_fd_file{F.fd, F.idx, F.offset + (int64_t)p.offset, p.length, (int32_t)p.B, 0});
            }
            const rsg_status r = generate_files_fd_impl(cs[(size_t)q], vf.data(), vf.size(), seed, 0, push_chunk, &me,
                                                        nullptr, nullptr, true);
            std::lock_guard<std::mutex> lk(me.mu);
            me.status = r;
            if (r != RSG_OK) me.err = cs[(size_t)q]->err;
            me.done = true;
            me.cv.notify_one();
        });
    }
    std::vector<uint8_t> buf, framed;
    uint64_t written = 0;
    auto i32 = [&](int32_t v) {
        const uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
        buf.insert(buf.end(), b, b + 4);
    };
    auto flush = [&]() -> rsg_status {
        if (buf.empty()) return RSG_OK;
        const uint8_t *out = buf.data();
        uint64_t len = buf.size();
        if (flags & RSG_GEN_MUX) {  // MultiplexWriter.WriteMsg, wire.go:28-36
            constexpr uint32_t kMax = 256 * 1024;
            framed.resize(len + 4 * ((len + kMax - 1) / kMax));
            uint64_t fl = 0;
            if (rsg_mux_frame(buf.data(), len, 0, kMax, framed.data(), framed.size(), &fl) != RSG_OK)
                return fail(c0, RSG_ERR_INVALID, "mux framing");
            out = framed.data();
            len = fl;
        }
        const int32_t r = write(user, out, len);
        if (r != 0) return fail(c0, RSG_ERR_IO, "writer failed (%d) after %llu bytes", r, (unsigned long long)written);
        written += len;
        buf.clear();
        return RSG_OK;
    };
    uint64_t next_head = 0, left = 0;  // first file without its head out; records left of the current file
    auto head = [&](uint64_t f) {
        if (flags & RSG_GEN_IDX) i32(files[f].idx);  // generator.go:317
        i32(heads[f].count);                         // types.go:79-86
        i32(heads[f].block_len);
        i32(heads[f].s2len);
        i32(heads[f].rem);
    };
    auto take = [&](const uint8_t *p, uint64_t nrec) -> rsg_status {
        while (nrec) {
            while (left == 0) {
                if (next_head >= nfiles) return fail(c0, RSG_ERR_HIP, "internal: records past the last file");
                head(next_head);
                left = (uint64_t)heads[next_head++].count;
            }
            const uint64_t k = std::min(left, nrec);
            buf.insert(buf.end(), p, p + k * kRecordBytes);
            p += k * kRecordBytes;
            left -= k;
            nrec -= k;
        }
        return RSG_OK;
    };
    rsg_status first = RSG_OK;
    for (int q = 0; q < n && first == RSG_OK; q++) {
        RankQueue &rq = qs[(size_t)q];
        for (;;) {
            std::vector<uint8_t> chunk;
            bool fin = false;
            {
                std::unique_lock<std::mutex> lk(rq.mu);
                rq.cv.wait(lk, [&] { return !rq.chunks.empty() || rq.done; });
                if (!rq.chunks.empty()) {
                    chunk = std::move(rq.chunks.front());
                    rq.chunks.pop_front();
                    rq.bytes -= chunk.size();
                } else {
                    fin = true;
                }
            }
            rq.space.notify_one();
            if (fin) {
                if (rq.status != RSG_OK) first = fail(c0, rq.status, "rank %d: %s", q, rq.err.c_str());
                break;
            }
            if (chunk.size() % kRecordBytes) {
                first = fail(c0, RSG_ERR_HIP, "internal: rank %d chunk of %zu bytes", q, chunk.size());
                break;
            }
            if ((s = take(chunk.data(), chunk.size() / kRecordBytes)) != RSG_OK || (s = flush()) != RSG_OK) {
                first = s;
                break;
            }
        }
    }
    if (first != RSG_OK) {
        abort = true;
        for (RankQueue &rq : qs) {  // wake generators blocked on a full queue
            std::lock_guard<std::mutex> lk(rq.mu);
            rq.space.notify_all();
        }
    }
    for (auto &t : th) t.join();
    if (first != RSG_OK) return first;
    if (left) return fail(c0, RSG_ERR_HIP, "internal: %llu records missing", (unsigned long long)left);
    while (next_head < nfiles) head(next_head++);  // trailing files without blocks
    if (flags & RSG_GEN_TERMINATE) {  // GenerateFiles' phase markers, generator.go:31,40
        i32(-1);
        i32(-1);
    }
    if ((s = flush()) != RSG_OK) return s;
    if (bytes_written) *bytes_written = written;
    return RSG_OK;
}

rsg_status rsg_testing_multi_queue(uint64_t cap, uint64_t *peak) {
    if (peak) *peak = g_queue_peak.load();
    if (cap) g_queue_cap.store(cap);
    return RSG_OK;
}

}  // extern "C"
