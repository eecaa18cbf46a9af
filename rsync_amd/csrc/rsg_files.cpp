// rsg_files.cpp -- C-ABI of the whole-file sums (include/rsg.h, rsg_file_sums_*).
//
// Replaces the serial whole-file MD4 of a batch of files:
//   RSG_FILESUM_PLAIN  : rsyncchecksum.ReaderChecksum (rsyncchecksum.go:60-66), used for the
//                        --checksum file list (sender/flist.go:276-293) and the receiver's
//                        quick check (receiver/generator.go:82-88);
//   RSG_FILESUM_SEEDED : the transfer's whole-file sum, MD4 seeded with int32_LE(seed) before
//                        the data (match.go:52-53, sender.go:184-206, receiver.go:117-120).
// One lane per file (rsg_filesums.hip); worthwhile for many files per call.
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "rsg_host.h"

using namespace rsgh;

namespace {

rsg_status check_mode(rsg_ctx *ctx, int32_t mode) {
    if (mode != RSG_FILESUM_PLAIN && mode != RSG_FILESUM_SEEDED)
        return fail(ctx, RSG_ERR_INVALID, "mode must be RSG_FILESUM_PLAIN or RSG_FILESUM_SEEDED");
    return RSG_OK;
}

// Longest first, so the 64 lanes of a wave hash similar numbers of chunks
// (and the one-wave workgroups form an LPT schedule).  Only approximate order
// matters: a counting sort on the length in KiB (capped), stable, O(n),
// written straight into the pinned staging.  shift: the bucket width, 2^shift
// bytes (10 by default; rsg_testing_search_option 6).
void lane_order(const rsg::FileSpan *spans, uint32_t n, uint32_t *order, int shift) {
    constexpr uint32_t kKeys = 1u << 16;
    auto key = [shift](uint64_t len) { return kKeys - 1 - (uint32_t)std::min<uint64_t>(len >> shift, kKeys - 1); };
    static thread_local std::vector<uint32_t> count;
    count.assign(kKeys + 1, 0);
    uint32_t kmin = kKeys, kmax = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = key(spans[i].len);  // descending length
        count[k]++;
        kmin = std::min(kmin, k);
        kmax = std::max(kmax, k);
    }
    uint32_t at = 0;
    for (uint32_t k = kmin; k <= kmax && n; k++) {
        const uint32_t c = count[k];
        count[k] = at;
        at += c;
    }
    for (uint32_t i = 0; i < n; i++) order[count[key(spans[i].len)]++] = i;
}

}  // namespace

namespace rsgh {

// Pinned staging for n spans (and their lane order) in ctx->h_desc[slot]:
// callers write the spans there directly.
rsg_status file_spans_stage(rsg_ctx *ctx, uint64_t n, int slot, rsg::FileSpan **spans) {
    const uint64_t ooff = (n * sizeof(rsg::FileSpan) + 63) & ~63ull;
    rsg_status s;
    if ((s = ensure_dev(ctx, ctx->d_desc[slot], ooff + n * 4 + 64)) != RSG_OK) return s;
    if ((s = ensure_pin(ctx, ctx->h_desc[slot], ooff + n * 4 + 64)) != RSG_OK) return s;
    *spans = (rsg::FileSpan *)ctx->h_desc[slot].p;
    return RSG_OK;
}

// The n spans staged in ctx->h_desc[slot]: lane order next to them, one
// upload to d_desc[slot], the whole-file sums on `stream` (asynchronous; the
// slot's staging must not be reused before the stream has passed this point).
rsg_status launch_file_sums_staged(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes, uint64_t n,
                                   int32_t mode, int32_t seed, void *d_out, int slot, hipStream_t stream) {
    const uint64_t ooff = (n * sizeof(rsg::FileSpan) + 63) & ~63ull;
    uint8_t *hd = (uint8_t *)ctx->h_desc[slot].p;
    lane_order((const rsg::FileSpan *)hd, (uint32_t)n, (uint32_t *)(hd + ooff), ctx->opts.fs_key_shift);
    bool aligned4 = ((uintptr_t)d_arena & 3u) == 0;
    for (uint64_t i = 0; i < n && aligned4; i++) aligned4 = (((const rsg::FileSpan *)hd)[i].offset & 3u) == 0;
    uint8_t *dd = (uint8_t *)ctx->d_desc[slot].p;
    RSG_HIP(ctx, hipMemcpyAsync(dd, hd, ooff + n * 4, hipMemcpyHostToDevice, stream));
    hipEvent_t t0 = timed_begin(ctx, stream);
    RSG_HIP(ctx, rsg::launch_file_sums((const uint8_t *)d_arena, arena_bytes, (const rsg::FileSpan *)dd,
                                       (const uint32_t *)(dd + ooff), (uint32_t)n, (uint32_t)mode, (uint32_t)seed,
                                       (uint8_t *)d_out, aligned4, stream));
    timed_end(ctx, t0, stream, 2);
    return RSG_OK;
}

rsg_status launch_file_sums_async(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes,
                                  const std::vector<rsg::FileSpan> &spans, int32_t mode, int32_t seed, void *d_out,
                                  int slot, hipStream_t stream) {
    rsg::FileSpan *st = nullptr;
    rsg_status s;
    if ((s = file_spans_stage(ctx, spans.size(), slot, &st)) != RSG_OK) return s;
    if (!spans.empty()) memcpy(st, spans.data(), spans.size() * sizeof(rsg::FileSpan));
    return launch_file_sums_staged(ctx, d_arena, arena_bytes, spans.size(), mode, seed, d_out, slot, stream);
}

}  // namespace rsgh

namespace {

rsg_status launch(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes, const std::vector<rsg::FileSpan> &spans,
                  int32_t mode, int32_t seed, void *d_out) {
    return launch_file_sums_async(ctx, d_arena, arena_bytes, spans, mode, seed, d_out, 0, ctx->stream);
}

}  // namespace

extern "C" {

rsg_status rsg_file_sums_device(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes, const rsg_file *files,
                                uint64_t nfiles, int32_t mode, int32_t seed, void *d_out) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    rsg_status s = check_mode(ctx, mode);
    if (s != RSG_OK) return s;
    if (nfiles == 0) return RSG_OK;
    if (nfiles > 0xFFFFFFFFull) return fail(ctx, RSG_ERR_INVALID, "too many files");
    if (!files || !d_out || (arena_bytes && !d_arena)) return fail(ctx, RSG_ERR_INVALID, "NULL argument");
    rsg::FileSpan *spans = nullptr;
    if ((s = file_spans_stage(ctx, nfiles, 0, &spans)) != RSG_OK) return s;
    for (uint64_t i = 0; i < nfiles; i++) {
        if (files[i].offset > arena_bytes || files[i].len > arena_bytes - files[i].offset)
            return fail(ctx, RSG_ERR_INVALID, "file %llu lies outside the arena", (unsigned long long)i);
        spans[i] = {files[i].offset, files[i].len};
    }
    if ((s = launch_file_sums_staged(ctx, d_arena, arena_bytes, nfiles, mode, seed, d_out, 0, ctx->stream)) != RSG_OK)
        return s;
    RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RSG_OK;
}

// Host files: packed (16-byte aligned) into pinned staging in batches of at
// most kBatchBytes (a larger file travels alone), copied to the device and
// hashed there; digests come back in file order.
rsg_status rsg_file_sums_host(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, int32_t mode, int32_t seed,
                              uint8_t *out) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    rsg_status s = check_mode(ctx, mode);
    if (s != RSG_OK) return s;
    if (nfiles == 0) return RSG_OK;
    if (!files || !out) return fail(ctx, RSG_ERR_INVALID, "NULL argument");
    for (uint64_t i = 0; i < nfiles; i++)
        if (files[i].len && !files[i].data)
            return fail(ctx, RSG_ERR_INVALID, "file %llu: NULL data", (unsigned long long)i);
    const uint64_t kBatchBytes = 256ull << 20;
    uint64_t i0 = 0;
    while (i0 < nfiles) {
        uint64_t i1 = i0, bytes = 0;
        while (i1 < nfiles) {
            const uint64_t add = (files[i1].len + 15) & ~15ull;
            if (i1 > i0 && bytes + add > kBatchBytes) break;
            bytes += add;
            i1++;
        }
        if ((s = ensure_pin(ctx, ctx->h_in[0], bytes + 16)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_in[0], bytes + 16)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_out[0], (i1 - i0) * 16)) != RSG_OK) return s;
        if ((s = ensure_pin(ctx, ctx->h_out[0], (i1 - i0) * 16)) != RSG_OK) return s;
        std::vector<rsg::FileSpan> spans(i1 - i0);
        std::vector<CopyJob> copies;
        uint8_t *stage = (uint8_t *)ctx->h_in[0].p;
        uint64_t off = 0;
        for (uint64_t i = i0; i < i1; i++) {
            if (files[i].len) copies.push_back({stage + off, files[i].data, files[i].len});
            spans[i - i0] = {off, files[i].len};
            off += (files[i].len + 15) & ~15ull;
        }
        parallel_copy(copies);
        RSG_HIP(ctx, hipMemcpyAsync(ctx->d_in[0].p, stage, off, hipMemcpyHostToDevice, ctx->stream));
        if ((s = launch(ctx, ctx->d_in[0].p, off, spans, mode, seed, ctx->d_out[0].p)) != RSG_OK) return s;
        RSG_HIP(ctx, hipMemcpyAsync(ctx->h_out[0].p, ctx->d_out[0].p, (i1 - i0) * 16, hipMemcpyDeviceToHost,
                                    ctx->stream));
        RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
        memcpy(out + i0 * 16, ctx->h_out[0].p, (i1 - i0) * 16);
        i0 = i1;
    }
    return RSG_OK;
}

}  // extern "C"
