// rsg_api.cpp -- C-ABI of librsg.so: contexts, block-sum plans, the host
// (PCIe-inclusive) pipeline and token encoding (the RCCL gather and the
// sharded pipelines are in rsg_dist.cpp).
// Declarations and contracts: include/rsg.h.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <thread>

#include "../../include/rsg_testing.h"
#include "rsg_host.h"

using rsg::DevFile;
using rsg::kBlockSumThreads;
using rsg::kRecordBytes;

static thread_local std::string g_thread_err;

namespace rsgh {

rsg_status fail(rsg_ctx *ctx, rsg_status code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_thread_err = buf;
    return code;
}

rsg_status hip_fail(rsg_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, e == hipErrorOutOfMemory ? RSG_ERR_NOMEM : RSG_ERR_HIP, "%s: %s (%d)", what,
                hipGetErrorString(e), (int)e);
}

static bool alloc_trace() {  // RSG_TIMING: report every (re)allocation of scratch
    static const bool on = getenv("RSG_TIMING") != nullptr;
    return on;
}

// Headroom for small scratch only: a regrow frees first (hipFree waits for
// the whole device), so a buffer that grows a little per call (the sender's
// per-file candidate counts, lists and results) gets 25 % more and does not
// regrow every call.  Large buffers (arenas, record buffers, the streaming
// windows) are sized exactly, to 64 KiB, so batches that fit still fit.
static uint64_t scratch_size(uint64_t bytes) {
    if (bytes <= (16ull << 20)) return std::max<uint64_t>(bytes + bytes / 4, 4096);
    return (bytes + 0xffffull) & ~0xffffull;
}

rsg_status ensure_dev(rsg_ctx *ctx, DevBuf &b, uint64_t bytes) {
    if (bytes <= b.cap) return RSG_OK;
    if (alloc_trace()) fprintf(stderr, "[rsg] alloc dev %llu -> %llu\n", (unsigned long long)b.cap, (unsigned long long)bytes);
    if (b.p) {
        RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    const uint64_t want = scratch_size(bytes);
    RSG_HIP(ctx, hipMalloc(&b.p, want));
    b.cap = want;
    return RSG_OK;
}

rsg_status ensure_pin(rsg_ctx *ctx, PinBuf &b, uint64_t bytes) {
    if (bytes <= b.cap) return RSG_OK;
    if (alloc_trace()) fprintf(stderr, "[rsg] alloc pin %llu -> %llu\n", (unsigned long long)b.cap, (unsigned long long)bytes);
    if (b.p) {
        hipHostFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    const uint64_t want = scratch_size(bytes);
    RSG_HIP(ctx, hipHostMalloc(&b.p, want, hipHostMallocDefault));
    b.cap = want;
    return RSG_OK;
}

// rsynccommon.SumSizesSqroot, rsynccommon.go:14-37, or an explicit B.
bool head_for(int64_t len, int32_t block_len, rsg_sum_head *out) {
    if (len < 0 || block_len < 0 || block_len > RSG_MAX_BLOCK_LEN) return false;
    int32_t b = block_len;
    if (b == 0) {
        double r = sqrt((double)len);
        b = r >= 2147483647.0 ? 2147483647 : (int32_t)r;  // int32(math.Sqrt(...)), :22
        if (b < 700) b = 700;                             // blockSize, :11
    }
    int64_t count = (len + ((int64_t)b - 1)) / (int64_t)b;  // :33
    if (count > INT32_MAX) return false;
    out->count = (int32_t)count;
    out->block_len = b;
    out->s2len = 16;                      // checksumLength, :31
    out->rem = (int32_t)(len % (int64_t)b);  // :34
    return true;
}

rsg_status build_plan(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, uint64_t arena_bytes,
                      bool use_offsets, HostPlan &plan) {
    if (nfiles && !files) return fail(ctx, RSG_ERR_INVALID, "files is NULL");
    if (nfiles >= 0xFFFFFFFFull) return fail(ctx, RSG_ERR_INVALID, "too many files");
    plan.files.resize(nfiles);
    plan.max_blen = 0;
    uint64_t total = 0, off = 0;
    bool aligned = true, lines128 = true;
    for (uint64_t i = 0; i < nfiles; i++) {
        rsg_sum_head h;
        if (!head_for((int64_t)files[i].len, files[i].block_len, &h))
            return fail(ctx, RSG_ERR_INVALID, "file %llu: bad length %llu / block_len %d",
                        (unsigned long long)i, (unsigned long long)files[i].len, files[i].block_len);
        DevFile &f = plan.files[i];
        if (use_offsets) {
            f.offset = files[i].offset;
            if (files[i].offset > arena_bytes || files[i].len > arena_bytes - files[i].offset)
                return fail(ctx, RSG_ERR_INVALID, "file %llu: [%llu, +%llu) outside the arena of %llu bytes",
                            (unsigned long long)i, (unsigned long long)files[i].offset,
                            (unsigned long long)files[i].len, (unsigned long long)arena_bytes);
        } else {
            f.offset = off;
            off += rsg::pack_round(files[i].len);
        }
        f.len = files[i].len;
        f.first_block = total;
        f.blen = (uint32_t)h.block_len;
        f.nblocks = (uint32_t)h.count;
        if (h.count && f.blen > plan.max_blen) plan.max_blen = f.blen;
        if (h.count) {
            if (f.offset & 3) aligned = false;
            if (h.count > 1 && (f.blen & 3)) aligned = false;
            if ((f.offset & 127) || (h.count > 1 && (f.blen & 127))) lines128 = false;
        }
        total += (uint64_t)h.count;
    }
    plan.total_blocks = total;
    plan.aligned = aligned;
    plan.lines128 = lines128;
    plan.arena_bytes = use_offsets ? arena_bytes : off;
    const uint64_t nwg = (total + kBlockSumThreads - 1) / kBlockSumThreads;
    if (nwg >= 0x7FFFFFFFull) return fail(ctx, RSG_ERR_INVALID, "batch too large (%llu blocks)",
                                          (unsigned long long)total);
    plan.nwg = (uint32_t)nwg;
    plan.wg_file.assign(nwg + 1, 0);
    // wg_file[w] = file owning block min(w*256, total-1).
    uint64_t f = 0;
    for (uint64_t w = 0; w <= nwg && total; w++) {
        uint64_t b = std::min<uint64_t>(w * kBlockSumThreads, total - 1);
        while (f + 1 < nfiles && plan.files[f + 1].first_block <= b) f++;
        // skip zero-block files that share first_block with a later file
        plan.wg_file[w] = (uint32_t)f;
    }
    return RSG_OK;
}

rsg_status launch_plan(rsg_ctx *ctx, const HostPlan &plan, const void *d_files, const void *d_wg,
                       const void *d_arena, int32_t seed, void *d_records, void *d_scratch, hipStream_t stream) {
    if (plan.total_blocks == 0) return RSG_OK;
    if (!d_arena || !d_records) return fail(ctx, RSG_ERR_INVALID, "NULL device pointer");
    const bool aligned = plan.aligned && (((uintptr_t)d_arena & 3u) == 0);
    const bool lines128 = plan.lines128 && (((uintptr_t)d_arena & 127u) == 0);
    (void)d_scratch;
    RSG_HIP(ctx, rsg::launch_block_sums((const uint8_t *)d_arena, plan.arena_bytes, (const DevFile *)d_files,
                                        (const uint32_t *)d_wg, plan.total_blocks, plan.nwg, aligned,
                                        plan.max_blen, (uint32_t)seed, (uint8_t *)d_records, plan.lds_reserve,
                                        ctx->bs_variant, stream, lines128));
    return RSG_OK;
}

void parallel_copy(const std::vector<CopyJob> &jobs) {
    const uint64_t kPiece = 2ull << 20;
    std::vector<CopyJob> pieces;
    uint64_t total = 0;
    for (const CopyJob &j : jobs) {
        for (uint64_t o = 0; o < j.n; o += kPiece) {
            const uint64_t n = std::min(kPiece, j.n - o);
            pieces.push_back({(uint8_t *)j.dst + o, (const uint8_t *)j.src + o, n});
        }
        total += j.n;
    }
    static const int threads = [] {
        const char *e = getenv("RSG_COPY_THREADS");
        const int t = e ? atoi(e) : 8;
        return std::max(1, std::min(t, 64));
    }();
    const int nt = (int)std::min<uint64_t>((uint64_t)threads, std::max<uint64_t>(1, total / (4ull << 20)));
    if (nt <= 1) {
        for (const CopyJob &p : pieces) memcpy(p.dst, p.src, p.n);
        return;
    }
    std::atomic<size_t> next{0};
    auto worker = [&] {
        for (size_t k; (k = next.fetch_add(1)) < pieces.size();) memcpy(pieces[k].dst, pieces[k].src, pieces[k].n);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(worker);
    worker();
    for (auto &t : pool) t.join();
}

}  // namespace rsgh

using namespace rsgh;

namespace {

struct Lock {
    rsg_ctx *c;
    explicit Lock(rsg_ctx *ctx) : c(ctx) { c->mu.lock(); }
    ~Lock() { c->mu.unlock(); }
};

#define RSG_ENTER(ctx)                                                             \
    if (!(ctx)) return fail(nullptr, RSG_ERR_INVALID, "NULL context");            \
    Lock lock_((ctx));                                                             \
    RSG_HIP((ctx), hipSetDevice((ctx)->device))

hipStream_t pick_stream(rsg_ctx *ctx, void *stream) {
    return stream ? (hipStream_t)stream : ctx->stream;
}

}  // namespace

extern "C" {

int32_t rsg_abi_version(void) { return RSG_ABI_VERSION; }

int32_t rsg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int i = 0; i < n; i++) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) good++;
    }
    return good;
}

rsg_status rsg_sum_head_for(int64_t file_len, int32_t block_len, rsg_sum_head *out) {
    if (!out) return fail(nullptr, RSG_ERR_INVALID, "out is NULL");
    if (!head_for(file_len, block_len, out))
        return fail(nullptr, RSG_ERR_INVALID, "bad length %lld / block_len %d", (long long)file_len, block_len);
    return RSG_OK;
}

rsg_status rsg_ctx_create(int32_t device, rsg_ctx **out) {
    if (!out) return fail(nullptr, RSG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(nullptr, RSG_ERR_NODEV, "no HIP device visible (%s)", hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(nullptr, RSG_ERR_NODEV, "device %d of %d", device, n);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, RSG_ERR_NODEV, "device %d is %s, not gfx950 (MI355X)", device, prop.gcnArchName);
    rsg_ctx *c = new (std::nothrow) rsg_ctx();
    if (c) c->bs_variant = rsg::block_sums_variant_env();
    if (!c) return fail(nullptr, RSG_ERR_NOMEM, "context allocation");
    c->device = device;
    if ((e = hipSetDevice(device)) != hipSuccess || (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->side[0], hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->side[1], hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->confirm, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->side_done[0], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->side_done[1], hipEventDisableTiming)) != hipSuccess) {
        rsg_status s = hip_fail(nullptr, e, "context streams");
        rsg_ctx_destroy(c);
        return s;
    }
    *out = c;
    return RSG_OK;
}

void rsg_ctx_destroy(rsg_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (int i = 0; i < 2; i++)
        if (c->side[i]) hipStreamSynchronize(c->side[i]);
    if (c->confirm) hipStreamSynchronize(c->confirm);
    DevBuf *dbs[] = {&c->d_files, &c->d_wg, &c->d_in[0], &c->d_in[1], &c->d_out[0], &c->d_out[1],
                     &c->d_desc[0], &c->d_desc[1], &c->d_fb[0], &c->d_fb[1], &c->d_res};
    for (DevBuf *b : dbs)
        if (b->p) hipFree(b->p);
    for (SearchSlot &sl : c->search) {
        DevBuf *sbs[] = {&sl.agg, &sl.prefix, &sl.counts, &sl.blob, &sl.src, &sl.res,
                         &sl.cfiles, &sl.cwg, &sl.cout, &sl.cfb};
        for (DevBuf *b : sbs)
            if (b->p) hipFree(b->p);
        if (sl.count.p) hipHostFree(sl.count.p);
        if (sl.list.p) hipHostFree(sl.list.p);
        if (sl.sel.p) hipHostFree(sl.sel.p);
        if (sl.stage.p) hipHostFree(sl.stage.p);
        if (sl.hres.p) hipHostFree(sl.hres.p);
        if (sl.scanned) hipEventDestroy(sl.scanned);
        if (sl.tables_b) hipEventDestroy(sl.tables_b);
        if (sl.rolled) hipEventDestroy(sl.rolled);
        if (sl.confirmed) hipEventDestroy(sl.confirmed);
    }
    for (SmallSlot &sl : c->small) {
        if (sl.dev.p) hipFree(sl.dev.p);
        if (sl.count.p) hipFree(sl.count.p);
        PinBuf *ps[] = {&sl.stage, &sl.outs, &sl.matches};
        for (PinBuf *b : ps)
            if (b->p) hipHostFree(b->p);
        if (sl.up) hipEventDestroy(sl.up);
        if (sl.done) hipEventDestroy(sl.done);
    }
    PinBuf *pbs[] = {&c->h_in[0], &c->h_in[1], &c->h_out[0], &c->h_out[1], &c->h_desc[0], &c->h_desc[1]};
    for (PinBuf *b : pbs)
        if (b->p) hipHostFree(b->p);
    if (c->comm) ncclCommDestroy(c->comm);
    for (const rsg_ctx::TimedSpan &t : c->spans) {
        hipEventDestroy(t.a);
        hipEventDestroy(t.b);
    }
    for (int i = 0; i < 2; i++) {
        if (c->side_done[i]) hipEventDestroy(c->side_done[i]);
        if (c->side[i]) hipStreamDestroy(c->side[i]);
    }
    if (c->confirm) hipStreamDestroy(c->confirm);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

const char *rsg_last_error(const rsg_ctx *ctx) { return ctx ? ctx->err.c_str() : g_thread_err.c_str(); }

rsg_status rsg_alloc_pinned(rsg_ctx *ctx, uint64_t bytes, void **out) {
    RSG_ENTER(ctx);
    if (!out) return fail(ctx, RSG_ERR_INVALID, "out is NULL");
    RSG_HIP(ctx, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return RSG_OK;
}

rsg_status rsg_free_pinned(rsg_ctx *ctx, void *p) {
    RSG_ENTER(ctx);
    if (p) RSG_HIP(ctx, hipHostFree(p));
    return RSG_OK;
}

rsg_status rsg_alloc_device(rsg_ctx *ctx, uint64_t bytes, void **out) {
    RSG_ENTER(ctx);
    if (!out) return fail(ctx, RSG_ERR_INVALID, "out is NULL");
    RSG_HIP(ctx, hipMalloc(out, bytes ? bytes : 1));
    return RSG_OK;
}

rsg_status rsg_free_device(rsg_ctx *ctx, void *p) {
    RSG_ENTER(ctx);
    if (p) RSG_HIP(ctx, hipFree(p));
    return RSG_OK;
}

rsg_status rsg_memcpy_h2d(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    RSG_ENTER(ctx);
    if (bytes) {  // on the context's stream: ordered after its kernels (it is non-blocking)
        RSG_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return RSG_OK;
}

rsg_status rsg_memcpy_d2h(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    RSG_ENTER(ctx);
    if (bytes) {  // on the context's stream: ordered after its kernels (it is non-blocking)
        RSG_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return RSG_OK;
}

rsg_status rsg_memcpy_d2d(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    RSG_ENTER(ctx);
    if (bytes) {  // on the context's stream: ordered after its kernels (it is non-blocking)
        RSG_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return RSG_OK;
}

rsg_status rsg_synchronize(rsg_ctx *ctx, void *stream) {
    RSG_ENTER(ctx);
    RSG_HIP(ctx, hipStreamSynchronize(pick_stream(ctx, stream)));
    return RSG_OK;
}

rsg_status rsg_fill_splitmix64(rsg_ctx *ctx, void *d_dst, uint64_t n, uint64_t seed, void *stream) {
    RSG_ENTER(ctx);
    if (n && !d_dst) return fail(ctx, RSG_ERR_INVALID, "NULL destination");
    RSG_HIP(ctx, rsg::launch_fill_splitmix64((uint8_t *)d_dst, n, seed, pick_stream(ctx, stream)));
    return RSG_OK;
}

// ---------------------------------------------------------------- block sums
rsg_status rsg_plan_block_sums(const rsg_file *files, uint64_t nfiles, rsg_sum_head *heads,
                               uint64_t *first_record, uint64_t *total_records) {
    if (nfiles && !files) return fail(nullptr, RSG_ERR_INVALID, "files is NULL");
    uint64_t total = 0;
    for (uint64_t i = 0; i < nfiles; i++) {
        rsg_sum_head h;
        if (!head_for((int64_t)files[i].len, files[i].block_len, &h))
            return fail(nullptr, RSG_ERR_INVALID, "file %llu: bad length/block_len", (unsigned long long)i);
        if (heads) heads[i] = h;
        if (first_record) first_record[i] = total;
        total += (uint64_t)h.count;
    }
    if (total_records) *total_records = total;
    return RSG_OK;
}

rsg_status rsg_plan_create(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, uint64_t arena_bytes,
                           rsg_plan **out) {
    RSG_ENTER(ctx);
    if (!out) return fail(ctx, RSG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    rsg_plan *p = new (std::nothrow) rsg_plan();
    if (!p) return fail(ctx, RSG_ERR_NOMEM, "plan allocation");
    p->ctx = ctx;
    rsg_status s = build_plan(ctx, files, nfiles, arena_bytes, true, p->host);
    if (s != RSG_OK) {
        delete p;
        return s;
    }
    hipError_t e;
    if ((e = hipMalloc(&p->d_files, std::max<uint64_t>(p->host.files.size(), 1) * sizeof(DevFile))) != hipSuccess ||
        (e = hipMalloc(&p->d_wg, p->host.wg_file.size() * sizeof(uint32_t) + 4)) != hipSuccess ||
        (e = hipMalloc(&p->d_scratch, rsg::block_sums_scratch_bytes(p->host.total_blocks))) != hipSuccess ||
        (e = hipMemcpy(p->d_files, p->host.files.data(), p->host.files.size() * sizeof(DevFile),
                       hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->d_wg, p->host.wg_file.data(), p->host.wg_file.size() * sizeof(uint32_t),
                       hipMemcpyHostToDevice)) != hipSuccess) {
        rsg_plan_destroy(p);
        return hip_fail(ctx, e, "plan upload");
    }
    *out = p;
    return RSG_OK;
}

void rsg_plan_destroy(rsg_plan *p) {
    if (!p) return;
    if (p->ctx) hipSetDevice(p->ctx->device);
    if (p->d_files) hipFree(p->d_files);
    if (p->d_wg) hipFree(p->d_wg);
    if (p->d_scratch) hipFree(p->d_scratch);
    delete p;
}

uint64_t rsg_plan_total_records(const rsg_plan *p) { return p ? p->host.total_blocks : 0; }

rsg_status rsg_block_sums_planned(rsg_ctx *ctx, const rsg_plan *plan, const void *d_arena, int32_t seed,
                                  void *d_records, void *stream) {
    RSG_ENTER(ctx);
    if (!plan || plan->ctx != ctx) return fail(ctx, RSG_ERR_INVALID, "plan belongs to another context");
    return launch_plan(ctx, plan->host, plan->d_files, plan->d_wg, d_arena, seed, d_records, plan->d_scratch,
                       pick_stream(ctx, stream));
}

rsg_status rsg_set_block_sums_kernel(rsg_ctx *ctx, int32_t variant) {
    RSG_ENTER(ctx);
    if (!rsg::block_sums_variant_valid(variant))
        return fail(ctx, RSG_ERR_INVALID, "variant %d: one of -1, 0, 1, 2, 3, 4, 6, 14", variant);
    ctx->bs_variant = variant;
    return RSG_OK;
}

int32_t rsg_testing_block_sums_choice(int32_t variant, int32_t aligned, int32_t lines128, int32_t arena_align,
                                      uint32_t max_blen) {
    if (!rsg::block_sums_variant_valid(variant)) return -2;
    return rsg::block_sums_choice(variant, aligned != 0, lines128 != 0, arena_align < 0 ? 0 : arena_align > 2 ? 2 : arena_align,
                                  max_blen);
}

rsg_status rsg_block_sums_fallbacks(rsg_ctx *ctx, uint64_t counts[2], int32_t reset) {
    RSG_ENTER(ctx);
    if (!counts) return fail(ctx, RSG_ERR_INVALID, "counts is NULL");
    RSG_HIP(ctx, rsg::read_block_sums_fallbacks(counts, reset != 0));
    return RSG_OK;
}

rsg_status rsg_block_sums_device(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes, const rsg_file *files,
                                 uint64_t nfiles, int32_t seed, void *d_records, uint64_t records_cap) {
    RSG_ENTER(ctx);
    HostPlan plan;
    rsg_status s = build_plan(ctx, files, nfiles, arena_bytes, true, plan);
    if (s != RSG_OK) return s;
    if (plan.total_blocks > records_cap)
        return fail(ctx, RSG_ERR_TRUNCATED, "need %llu records, capacity %llu",
                    (unsigned long long)plan.total_blocks, (unsigned long long)records_cap);
    if ((s = ensure_dev(ctx, ctx->d_files, plan.files.size() * sizeof(DevFile) + 32)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_wg, plan.wg_file.size() * sizeof(uint32_t) + 4)) != RSG_OK) return s;
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_files.p, plan.files.data(), plan.files.size() * sizeof(DevFile),
                                hipMemcpyHostToDevice, ctx->stream));
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_wg.p, plan.wg_file.data(), plan.wg_file.size() * sizeof(uint32_t),
                                hipMemcpyHostToDevice, ctx->stream));
    if ((s = ensure_dev(ctx, ctx->d_fb[0], rsg::block_sums_scratch_bytes(plan.total_blocks))) != RSG_OK) return s;
    if ((s = launch_plan(ctx, plan, ctx->d_files.p, ctx->d_wg.p, d_arena, seed, d_records, ctx->d_fb[0].p,
                         ctx->stream)) != RSG_OK)
        return s;
    RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RSG_OK;
}

// Host path: files are cut at block boundaries into pieces, pieces are packed
// into batches of <= kBatchBytes, and two batches are in flight on two streams
// (host memcpy into pinned staging | H2D + kernel + D2H of the other slot).
rsg_status rsg_block_sums_host(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, int32_t seed,
                               uint8_t *records, uint64_t records_cap) {
    RSG_ENTER(ctx);
    struct Drain {  // no batch stays queued past an early return
        rsg_ctx *c;
        ~Drain() {
            for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(c->side[k]);
        }
    } drain_guard{ctx};
    const uint64_t kBatchBytes = 64ull << 20;
    const uint64_t kBatchRecords = 1ull << 22;
    std::vector<rsg_sum_head> heads(nfiles);
    uint64_t total = 0;
    for (uint64_t i = 0; i < nfiles; i++) {
        if (files[i].len && !files[i].data) return fail(ctx, RSG_ERR_INVALID, "file %llu: NULL data", (unsigned long long)i);
        if (!head_for((int64_t)files[i].len, files[i].block_len, &heads[i]))
            return fail(ctx, RSG_ERR_INVALID, "file %llu: bad length/block_len", (unsigned long long)i);
        total += (uint64_t)heads[i].count;
    }
    if (total > records_cap)
        return fail(ctx, RSG_ERR_TRUNCATED, "need %llu records, capacity %llu", (unsigned long long)total,
                    (unsigned long long)records_cap);
    if (total && !records) return fail(ctx, RSG_ERR_INVALID, "records is NULL");

    struct Piece { uint64_t file, b0, b1; };
    struct Batch { std::vector<Piece> pieces; uint64_t bytes = 0, recs = 0, rec_begin = 0; };
    std::vector<Batch> batches(1);
    uint64_t rec = 0;
    for (uint64_t i = 0; i < nfiles; i++) {
        const uint64_t B = (uint64_t)heads[i].block_len, cnt = (uint64_t)heads[i].count;
        uint64_t b0 = 0;
        while (b0 < cnt) {
            Batch *bt = &batches.back();
            uint64_t room_b = bt->bytes < kBatchBytes ? (kBatchBytes - bt->bytes) / B : 0;
            uint64_t room_r = kBatchRecords - bt->recs;
            uint64_t take = std::min(std::min(room_b, room_r), cnt - b0);
            if (take == 0) {
                if (bt->pieces.empty()) take = 1;  // a single block larger than a batch
                else {
                    batches.emplace_back();
                    batches.back().rec_begin = rec;
                    continue;
                }
            }
            const uint64_t start = b0 * B, end = std::min<uint64_t>((b0 + take) * B, files[i].len);
            bt->pieces.push_back({i, b0, b0 + take});
            bt->bytes += rsg::pack_round(end - start);
            bt->recs += take;
            rec += take;
            b0 += take;
        }
    }
    rsg_status s;
    uint64_t max_bytes = 16, max_recs = 1, max_pieces = 1;
    for (auto &b : batches) {
        max_bytes = std::max(max_bytes, b.bytes + 16);
        max_recs = std::max(max_recs, b.recs);
        max_pieces = std::max<uint64_t>(max_pieces, b.pieces.size());
    }
    const uint64_t max_nwg = (max_recs + kBlockSumThreads - 1) / kBlockSumThreads + 1;
    const uint64_t desc_bytes = max_pieces * sizeof(DevFile) + (max_nwg + 1) * 4 + 64;
    for (int k = 0; k < 2; k++) {
        if ((s = ensure_dev(ctx, ctx->d_in[k], max_bytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_out[k], max_recs * kRecordBytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_desc[k], desc_bytes)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_fb[k], rsg::block_sums_scratch_bytes(max_recs))) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_in[k], max_bytes)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_out[k], max_recs * kRecordBytes)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_desc[k], desc_bytes)) != RSG_OK) return s;
    }
    constexpr size_t kDirectPieces = 1024;  // per-piece DMA calls stay cheap up to here
    std::vector<int8_t> pinned(nfiles, -1);
    auto is_pinned = [&](uint64_t i) -> bool {
        if (pinned[i] < 0) {
            hipPointerAttribute_t a{};
            const hipError_t e = files[i].len ? hipPointerGetAttributes(&a, files[i].data) : hipErrorInvalidValue;
            if (e != hipSuccess) (void)hipGetLastError();  // plain pageable memory: not an error
            pinned[i] = (e == hipSuccess && a.type == hipMemoryTypeHost) ? 1 : 0;
        }
        return pinned[i] == 1;
    };
    int64_t pending[2] = {-1, -1};  // batch index in flight per slot
    auto drain = [&](int slot) -> rsg_status {
        if (pending[slot] < 0) return RSG_OK;
        RSG_HIP(ctx, hipEventSynchronize(ctx->side_done[slot]));
        const Batch &b = batches[(size_t)pending[slot]];
        memcpy(records + b.rec_begin * kRecordBytes, ctx->h_out[slot].p, b.recs * kRecordBytes);
        pending[slot] = -1;
        return RSG_OK;
    };
    for (size_t bi = 0; bi < batches.size(); bi++) {
        const Batch &b = batches[bi];
        if (b.recs == 0) continue;
        const int slot = (int)(bi & 1);
        if ((s = drain(slot)) != RSG_OK) return s;
        // stage pieces as virtual files in the pinned arena
        std::vector<rsg_file> vf(b.pieces.size());
        std::vector<CopyJob> copies(b.pieces.size());
        uint8_t *stage = (uint8_t *)ctx->h_in[slot].p;
        uint64_t off = 0;
        for (size_t j = 0; j < b.pieces.size(); j++) {
            const Piece &pc = b.pieces[j];
            const uint64_t B = (uint64_t)heads[pc.file].block_len;
            const uint64_t start = pc.b0 * B, end = std::min<uint64_t>(pc.b1 * B, files[pc.file].len);
            copies[j] = {stage + off, files[pc.file].data + start, end - start};
            vf[j].data = nullptr;
            vf[j].offset = off;
            vf[j].len = end - start;
            vf[j].block_len = (int32_t)B;
            off += rsg::pack_round(end - start);
        }
        // Pieces whose source already lies in page-locked memory (the
        // caller read the files into rsg_alloc_pinned buffers)
        // go to HBM by DMA straight from there: no staging copy.
        bool direct = b.pieces.size() <= kDirectPieces;
        for (size_t j = 0; direct && j < b.pieces.size(); j++) direct = is_pinned(b.pieces[j].file);
        if (!direct) parallel_copy(copies);
        HostPlan plan;
        if ((s = build_plan(ctx, vf.data(), vf.size(), off, true, plan)) != RSG_OK) return s;
        uint8_t *hd = (uint8_t *)ctx->h_desc[slot].p;
        const uint64_t fbytes = plan.files.size() * sizeof(DevFile);
        const uint64_t wg_off = (fbytes + 63) & ~63ull;
        memcpy(hd, plan.files.data(), fbytes);
        memcpy(hd + wg_off, plan.wg_file.data(), plan.wg_file.size() * 4);
        hipStream_t st = ctx->side[slot];
        uint8_t *dd = (uint8_t *)ctx->d_desc[slot].p;
        RSG_HIP(ctx, hipMemcpyAsync(dd, hd, wg_off + plan.wg_file.size() * 4, hipMemcpyHostToDevice, st));
        if (direct) {
            for (size_t j = 0; j < copies.size(); j++)
                RSG_HIP(ctx, hipMemcpyAsync((uint8_t *)ctx->d_in[slot].p + vf[j].offset, copies[j].src, copies[j].n,
                                            hipMemcpyHostToDevice, st));
        } else {
            RSG_HIP(ctx, hipMemcpyAsync(ctx->d_in[slot].p, stage, off, hipMemcpyHostToDevice, st));
        }
        if ((s = launch_plan(ctx, plan, dd, dd + wg_off, ctx->d_in[slot].p, seed, ctx->d_out[slot].p,
                             ctx->d_fb[slot].p, st)) != RSG_OK)
            return s;
        RSG_HIP(ctx, hipMemcpyAsync(ctx->h_out[slot].p, ctx->d_out[slot].p, b.recs * kRecordBytes,
                                    hipMemcpyDeviceToHost, st));
        RSG_HIP(ctx, hipEventRecord(ctx->side_done[slot], st));
        pending[slot] = (int64_t)bi;
    }
    if ((s = drain(0)) != RSG_OK) return s;
    if ((s = drain(1)) != RSG_OK) return s;
    return RSG_OK;
}

// ---------------------------------------------------------------- tokens
rsg_status rsg_encode_tokens(const uint8_t *src, uint64_t src_len, const rsg_sum_head *head,
                             const rsg_match *matches, uint64_t n_matches, uint8_t *out, uint64_t out_cap,
                             uint64_t *out_len) {
    if (!head || !out_len || (n_matches && !matches) || (src_len && !src))
        return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    const int64_t B = head->block_len;
    uint64_t pos = 0, last = 0;
    bool fits = true;
    auto put = [&](const void *p, uint64_t n) {
        if (out && pos + n <= out_cap) memcpy(out + pos, p, n);
        else if (out) fits = false;
        pos += n;
    };
    auto put_i32 = [&](int32_t v) {
        uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
        put(b, 4);
    };
    // simpleSendToken, token.go:4-31
    auto literal = [&](uint64_t from, uint64_t n) {
        for (uint64_t l = 0; l < n;) {
            uint64_t n1 = std::min<uint64_t>(RSG_CHUNK_SIZE, n - l);
            put_i32((int32_t)n1);
            put(src + from + l, n1);
            l += n1;
        }
    };
    for (uint64_t m = 0; m < n_matches; m++) {
        const int64_t off = matches[m].offset;
        const int32_t i = matches[m].index;
        if (i < 0 || i >= head->count || off < (int64_t)last || (uint64_t)off > src_len)
            return fail(nullptr, RSG_ERR_INVALID, "match %llu out of order or range", (unsigned long long)m);
        const int64_t len = (i == head->count - 1 && head->rem != 0) ? head->rem : B;
        if ((uint64_t)(off + len) > src_len) return fail(nullptr, RSG_ERR_INVALID, "match %llu past end", (unsigned long long)m);
        literal(last, (uint64_t)off - last);  // matched(): literal run then token
        put_i32(-(i + 1));
        last = (uint64_t)(off + len);
    }
    literal(last, src_len - last);  // matched(size, -1), match.go:212
    put_i32(0);
    *out_len = pos;
    if (!fits) return fail(nullptr, RSG_ERR_TRUNCATED, "token stream needs %llu bytes", (unsigned long long)pos);
    return RSG_OK;
}

}  // extern "C"
