// rsg_generate.cpp -- the generator's host loop around the block-sum kernel
// (SURVEY.md §8f row 1): basis files are read from open descriptors into
// pinned staging, hashed on the GPU and the sums stream is handed to the
// caller's writer, with reading, the GPU work and writing of consecutive
// batches overlapped.
//
// Replaces, for a file list whose entries all reach generateAndSendSums
// (recvGenerator with -I or a changed file, generator.go:143-322):
//   per file  Conn.WriteInt32(idx)                 generator.go:317
//             SumHead.WriteTo                      generator.go:327-330, types.go:79-86
//             per block io.ReadFull(in, b)         generator.go:335
//                       WriteInt32(sum1), Write(sum2)  generator.go:341-346
//   then      the two int32 -1 phase markers       generator.go:31,40
// The reference does one read syscall and two unbuffered writes per block
// (three mux messages on the server side, wire.go:28-36); here files are read
// in pieces of up to 2 MiB by a few threads and the stream leaves in one write
// per batch (framed in <= 256 KiB MsgData messages with RSG_GEN_MUX).
#include <errno.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "rsg_host.h"

using namespace rsgh;
using rsg::kBlockSumThreads;
using rsg::kRecordBytes;

namespace {

constexpr uint64_t kBatchRecords = 1ull << 22;

// Staging per slot: RSG_GEN_BATCH_MB (default 32 MiB; smaller batches start
// the GPU sooner and overlap more of the reads, larger ones cost fewer
// launches).
uint64_t batch_bytes() {
    const char *e = getenv("RSG_GEN_BATCH_MB");
    const long v = e ? atol(e) : 32;
    return (uint64_t)std::max(1L, std::min(v, 1024L)) << 20;
}
constexpr uint64_t kReadPiece = 2ull << 20;
constexpr uint32_t kMaxMessage = 256 * 1024;  // wire.go:46-47

struct Piece {
    uint64_t file, b0, b1;  // blocks [b0, b1) of file
    uint64_t stage_off;     // kPackAlign-aligned offset in the batch's staging arena
};
struct Batch {
    std::vector<Piece> pieces;
    uint64_t bytes = 0, recs = 0;
};

struct ReadJob {
    int fd;
    int64_t off;
    uint8_t *dst;
    uint64_t n;
    uint64_t file;
};

// io.ReadFull of n bytes at off (pread: the descriptor's position is left
// alone).  0 = done, -1 = EOF before n bytes, else errno.
int read_full(int fd, uint8_t *dst, uint64_t n, int64_t off) {
    while (n) {
        const ssize_t r = pread(fd, dst, (size_t)std::min<uint64_t>(n, 1ull << 30), (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (r == 0) return -1;
        dst += r;
        n -= (uint64_t)r;
        off += r;
    }
    return 0;
}

// Reader threads: RSG_COPY_THREADS (default 8), as the host path's copies.
int read_threads() {
    const char *e = getenv("RSG_COPY_THREADS");
    const int v = e ? atoi(e) : 8;
    return std::max(1, std::min(v, 64));
}

// All jobs on a few threads; returns the first failing job's index (or -1)
// and its read_full code.
int64_t parallel_read(const std::vector<ReadJob> &jobs, int *code) {
    std::atomic<size_t> next{0};
    std::atomic<int64_t> bad{-1};
    std::atomic<int> bad_code{0};
    std::mutex bad_mu;
    auto worker = [&] {
        for (size_t k; (k = next.fetch_add(1)) < jobs.size();) {
            // jobs are taken in index order, so every job below a recorded
            // failure is already running: finish those, skip the rest
            const int64_t b0 = bad.load();
            if (b0 >= 0 && (int64_t)k > b0) return;
            const ReadJob &j = jobs[k];
            const int r = read_full(j.fd, j.dst, j.n, j.off);
            if (r != 0) {
                // keep the LOWEST failing job, as the reference's sequential
                // loop (generator.go:332-348) would report the first file
                std::lock_guard<std::mutex> lk(bad_mu);
                const int64_t cur = bad.load();
                if (cur < 0 || (int64_t)k < cur) {
                    bad = (int64_t)k;
                    bad_code = r;
                }
            }
        }
    };
    uint64_t total = 0;
    for (const ReadJob &j : jobs) total += j.n;
    const int nt = (int)std::min<uint64_t>((uint64_t)read_threads(), std::max<uint64_t>(1, total / (4ull << 20)));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
    *code = bad_code.load();
    return bad.load();
}

// The sums stream in file order, handed to the writer once per batch.
struct Emitter {
    rsg_write_fn fn;
    void *user;
    bool mux;
    std::vector<uint8_t> buf, framed;
    uint64_t written = 0;

    void i32(int32_t v) {
        const uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
        buf.insert(buf.end(), b, b + 4);
    }
    void put(const uint8_t *p, uint64_t n) { buf.insert(buf.end(), p, p + n); }
    rsg_status flush(rsg_ctx *ctx) {
        if (buf.empty()) return RSG_OK;
        const uint8_t *out = buf.data();
        uint64_t len = buf.size();
        if (mux) {  // MultiplexWriter.WriteMsg, wire.go:28-36
            framed.resize(len + 4 * ((len + kMaxMessage - 1) / kMaxMessage));
            uint64_t fl = 0;
            if (rsg_mux_frame(buf.data(), len, 0, kMaxMessage, framed.data(), framed.size(), &fl) != RSG_OK)
                return fail(ctx, RSG_ERR_INVALID, "mux framing");
            out = framed.data();
            len = fl;
        }
        const int32_t r = fn(user, out, len);
        if (r != 0) return fail(ctx, RSG_ERR_IO, "writer failed (%d) after %llu bytes", r, (unsigned long long)written);
        written += len;
        buf.clear();
        return RSG_OK;
    }
};

}  // namespace

namespace rsgh {

// records_only: the stream carries only the 20-byte records of the files'
// blocks (no idx, SumHead, phase markers or framing): the per-rank part of
// rsg_generate_files_fd_multi (rsg_shard.cpp), whose caller thread puts the
// heads between the ranks' records.
rsg_status generate_files_fd_impl(rsg_ctx *ctx, const rsg_fd_file *files, uint64_t nfiles, int32_t seed,
                                  int32_t flags, rsg_write_fn write, void *user, rsg_sum_head *heads_out,
                                  uint64_t *bytes_written, bool records_only) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    // Whatever path leaves (a read or writer failure mid-batch included),
    // nothing stays queued on the slot streams that a later call's buffer
    // growth could free under it.
    struct Drain {
        rsg_ctx *c;
        ~Drain() {
            for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(c->side[k]);
        }
    } drain_guard{ctx};
    if (bytes_written) *bytes_written = 0;
    if (!write || (nfiles && !files)) return fail(ctx, RSG_ERR_INVALID, "NULL argument");
    if (flags & ~(RSG_GEN_IDX | RSG_GEN_TERMINATE | RSG_GEN_MUX))
        return fail(ctx, RSG_ERR_INVALID, "unknown flags 0x%x", flags);
    if (records_only) flags = 0;
    std::vector<rsg_sum_head> heads(nfiles);
    for (uint64_t i = 0; i < nfiles; i++) {
        if (files[i].len > (uint64_t)INT64_MAX || files[i].offset < 0)
            return fail(ctx, RSG_ERR_INVALID, "file %llu: bad offset/length", (unsigned long long)i);
        if (!head_for((int64_t)files[i].len, files[i].block_len, &heads[i]))  // SumSizesSqroot, generator.go:327
            return fail(ctx, RSG_ERR_INVALID, "file %llu: bad length/block_len", (unsigned long long)i);
        if (heads[i].count && files[i].fd < 0) return fail(ctx, RSG_ERR_INVALID, "file %llu: bad descriptor",
                                                           (unsigned long long)i);
        if (heads_out) heads_out[i] = heads[i];
    }
    // Batches of whole blocks, <= kBatchBytes of staging (a single block
    // larger than that travels alone), files cut on block boundaries.
    const uint64_t kBatchBytes = batch_bytes();
    std::vector<Batch> batches(1);
    for (uint64_t i = 0; i < nfiles; i++) {
        const uint64_t B = (uint64_t)heads[i].block_len, cnt = (uint64_t)heads[i].count;
        for (uint64_t b0 = 0; b0 < cnt;) {
            Batch *bt = &batches.back();
            const uint64_t room_b = bt->bytes < kBatchBytes ? (kBatchBytes - bt->bytes) / B : 0;
            uint64_t take = std::min(std::min(room_b, kBatchRecords - bt->recs), cnt - b0);
            if (take == 0) {
                if (!bt->pieces.empty()) {
                    batches.emplace_back();
                    continue;
                }
                take = 1;
            }
            const uint64_t start = b0 * B, end = std::min<uint64_t>((b0 + take) * B, files[i].len);
            bt->pieces.push_back({i, b0, b0 + take, bt->bytes});
            bt->bytes += rsg::pack_round(end - start);
            bt->recs += take;
            b0 += take;
        }
    }
    uint64_t max_bytes = 16, max_recs = 1, max_pieces = 1;
    for (const Batch &b : batches) {
        max_bytes = std::max(max_bytes, b.bytes + 16);
        max_recs = std::max(max_recs, b.recs);
        max_pieces = std::max<uint64_t>(max_pieces, b.pieces.size());
    }
    const uint64_t max_nwg = (max_recs + kBlockSumThreads - 1) / kBlockSumThreads + 1;
    const uint64_t desc_bytes = max_pieces * sizeof(rsg::DevFile) + (max_nwg + 1) * 4 + 64;
    rsg_status s;
    const bool any = batches[0].recs != 0;
    for (int k = 0; any && k < 2; k++) {
        if ((s = ensure_dev(ctx, ctx->d_in[k], max_bytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_out[k], max_recs * kRecordBytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_desc[k], desc_bytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_fb[k], rsg::block_sums_scratch_bytes(max_recs))) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_in[k], max_bytes)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_out[k], max_recs * kRecordBytes)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_desc[k], desc_bytes)) != RSG_OK) return s;
    }

    Emitter em{write, user, (flags & RSG_GEN_MUX) != 0};
    uint64_t next_head = 0;  // first file whose idx + SumHead are not out yet
    auto emit_heads_through = [&](uint64_t f) {
        if (records_only) return;
        for (; next_head <= f && next_head < nfiles; next_head++) {
            const rsg_sum_head &h = heads[next_head];
            if (flags & RSG_GEN_IDX) em.i32(files[next_head].idx);  // generator.go:317
            em.i32(h.count);                                         // types.go:79-86
            em.i32(h.block_len);
            em.i32(h.s2len);
            em.i32(h.rem);
        }
    };
    int64_t pending[2] = {-1, -1};
    // Wait for slot's batch, then append its records (wire-ready 20-byte
    // int32 sum1 || sum2[16], generator.go:341-346) behind their files' heads.
    auto drain = [&](int slot) -> rsg_status {
        if (pending[slot] < 0) return RSG_OK;
        RSG_HIP(ctx, hipEventSynchronize(ctx->side_done[slot]));
        const Batch &b = batches[(size_t)pending[slot]];
        const uint8_t *rec = (const uint8_t *)ctx->h_out[slot].p;
        for (const Piece &pc : b.pieces) {
            emit_heads_through(pc.file);
            const uint64_t n = pc.b1 - pc.b0;
            em.put(rec, n * kRecordBytes);
            rec += n * kRecordBytes;
        }
        pending[slot] = -1;
        return em.flush(ctx);
    };
    for (size_t bi = 0; bi < batches.size(); bi++) {
        const Batch &b = batches[bi];
        if (b.recs == 0) continue;
        const int slot = (int)(bi & 1);
        if ((s = drain(slot)) != RSG_OK) return s;
        uint8_t *stage = (uint8_t *)ctx->h_in[slot].p;
        std::vector<ReadJob> jobs;
        std::vector<rsg_file> vf(b.pieces.size());
        for (size_t j = 0; j < b.pieces.size(); j++) {
            const Piece &pc = b.pieces[j];
            const uint64_t B = (uint64_t)heads[pc.file].block_len;
            const uint64_t start = pc.b0 * B, end = std::min<uint64_t>(pc.b1 * B, files[pc.file].len);
            for (uint64_t o = start; o < end; o += kReadPiece)
                jobs.push_back({files[pc.file].fd, files[pc.file].offset + (int64_t)o, stage + pc.stage_off + (o - start),
                                std::min(kReadPiece, end - o), pc.file});
            vf[j].data = nullptr;
            vf[j].offset = pc.stage_off;
            vf[j].len = end - start;
            vf[j].block_len = (int32_t)B;
        }
        int code = 0;
        const int64_t badj = parallel_read(jobs, &code);
        if (badj >= 0) {
            const unsigned long long f = (unsigned long long)jobs[(size_t)badj].file;
            if (code == -1) return fail(ctx, RSG_ERR_IO, "file %llu: unexpected EOF", f);  // io.ReadFull
            return fail(ctx, RSG_ERR_IO, "file %llu: read: %s", f, strerror(code));
        }
        HostPlan plan;
        if ((s = build_plan(ctx, vf.data(), vf.size(), b.bytes, true, plan)) != RSG_OK) return s;
        uint8_t *hd = (uint8_t *)ctx->h_desc[slot].p;
        const uint64_t fbytes = plan.files.size() * sizeof(rsg::DevFile);
        const uint64_t wg_off = (fbytes + 63) & ~63ull;
        memcpy(hd, plan.files.data(), fbytes);
        memcpy(hd + wg_off, plan.wg_file.data(), plan.wg_file.size() * 4);
        hipStream_t st = ctx->side[slot];
        uint8_t *dd = (uint8_t *)ctx->d_desc[slot].p;
        RSG_HIP(ctx, hipMemcpyAsync(dd, hd, wg_off + plan.wg_file.size() * 4, hipMemcpyHostToDevice, st));
        RSG_HIP(ctx, hipMemcpyAsync(ctx->d_in[slot].p, stage, b.bytes, hipMemcpyHostToDevice, st));
        if ((s = launch_plan(ctx, plan, dd, dd + wg_off, ctx->d_in[slot].p, seed, ctx->d_out[slot].p,
                             ctx->d_fb[slot].p, st)) != RSG_OK)
            return s;
        RSG_HIP(ctx, hipMemcpyAsync(ctx->h_out[slot].p, ctx->d_out[slot].p, b.recs * kRecordBytes,
                                    hipMemcpyDeviceToHost, st));
        RSG_HIP(ctx, hipEventRecord(ctx->side_done[slot], st));
        pending[slot] = (int64_t)bi;
        // batch bi-1 (the other slot) went out before this one was read: its
        // records are written now, while this batch is on the GPU
        if ((s = drain(slot ^ 1)) != RSG_OK) return s;
    }
    if ((s = drain(0)) != RSG_OK) return s;
    if ((s = drain(1)) != RSG_OK) return s;
    emit_heads_through(nfiles);  // trailing files without blocks
    if (flags & RSG_GEN_TERMINATE) {  // GenerateFiles' phase markers, generator.go:31,40
        em.i32(-1);
        em.i32(-1);
    }
    if ((s = em.flush(ctx)) != RSG_OK) return s;
    if (bytes_written) *bytes_written = em.written;
    return RSG_OK;
}

}  // namespace rsgh

extern "C" {

rsg_status rsg_generate_files_fd(rsg_ctx *ctx, const rsg_fd_file *files, uint64_t nfiles, int32_t seed,
                                 int32_t flags, rsg_write_fn write, void *user, rsg_sum_head *heads_out,
                                 uint64_t *bytes_written) {
    return generate_files_fd_impl(ctx, files, nfiles, seed, flags, write, user, heads_out, bytes_written, false);
}

}  // extern "C"
