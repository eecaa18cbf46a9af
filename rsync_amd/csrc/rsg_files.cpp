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
// matters: a counting sort on the length in KiB (capped), stable, O(n).
std::vector<uint32_t> lane_order(const std::vector<rsg::FileSpan> &spans) {
    constexpr uint64_t kKeys = 1u << 16;
    auto key = [](uint64_t len) { return (uint32_t)std::min<uint64_t>(len >> 10, kKeys - 1); };
    std::vector<uint32_t> count(kKeys + 1, 0);
    for (const rsg::FileSpan &f : spans) count[kKeys - 1 - key(f.len)]++;  // descending length
    uint32_t at = 0;
    for (uint64_t k = 0; k <= kKeys; k++) {
        const uint32_t c = count[k];
        count[k] = at;
        at += c;
    }
    std::vector<uint32_t> order(spans.size());
    for (uint32_t i = 0; i < (uint32_t)spans.size(); i++) order[count[kKeys - 1 - key(spans[i].len)]++] = i;
    return order;
}

}  // namespace

namespace rsgh {

// Upload spans + order through ctx->h_desc[slot] / d_desc[slot] and launch
// the whole-file sums on `stream` (asynchronous; the slot's staging must not
// be reused before the stream has passed this point).
rsg_status launch_file_sums_async(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes,
                                  const std::vector<rsg::FileSpan> &spans, int32_t mode, int32_t seed, void *d_out,
                                  int slot, hipStream_t stream) {
    const std::vector<uint32_t> order = lane_order(spans);
    const uint64_t sbytes = spans.size() * sizeof(rsg::FileSpan);
    const uint64_t ooff = (sbytes + 63) & ~63ull;
    rsg_status s;
    if ((s = ensure_dev(ctx, ctx->d_desc[slot], ooff + order.size() * 4 + 64)) != RSG_OK) return s;
    if ((s = ensure_pin(ctx, ctx->h_desc[slot], ooff + order.size() * 4 + 64)) != RSG_OK) return s;
    uint8_t *hd = (uint8_t *)ctx->h_desc[slot].p;
    memcpy(hd, spans.data(), sbytes);
    memcpy(hd + ooff, order.data(), order.size() * 4);
    uint8_t *dd = (uint8_t *)ctx->d_desc[slot].p;
    RSG_HIP(ctx, hipMemcpyAsync(dd, hd, ooff + order.size() * 4, hipMemcpyHostToDevice, stream));
    RSG_HIP(ctx, rsg::launch_file_sums((const uint8_t *)d_arena, arena_bytes, (const rsg::FileSpan *)dd,
                                       (const uint32_t *)(dd + ooff), (uint32_t)spans.size(), (uint32_t)mode,
                                       (uint32_t)seed, (uint8_t *)d_out, stream));
    return RSG_OK;
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
    std::vector<rsg::FileSpan> spans(nfiles);
    for (uint64_t i = 0; i < nfiles; i++) {
        if (files[i].offset > arena_bytes || files[i].len > arena_bytes - files[i].offset)
            return fail(ctx, RSG_ERR_INVALID, "file %llu lies outside the arena", (unsigned long long)i);
        spans[i] = {files[i].offset, files[i].len};
    }
    if ((s = launch(ctx, d_arena, arena_bytes, spans, mode, seed, d_out)) != RSG_OK) return s;
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
