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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <unordered_map>
#include <vector>

#include "rsg_host.h"

using namespace rsgh;
using rsg::DevFile;
using rsg::kRecordBytes;
using rsg::kScanTile;
using rsg::TileAgg;
using rsg::TilePrefix;

namespace {

constexpr uint32_t kCandCap = 1u << 22;      // candidates per roll launch (32 MiB)
constexpr uint64_t kSparseBatch = 1u << 16;  // windows per verification batch

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
    PhaseTimer *pt;
    rsg_ctx *ctx;
    hipStream_t st;
    const uint8_t *d_src;
    uint64_t size;
    rsg_sum_head head;
    const uint8_t *sum2;
    int32_t seed;
    int64_t end;  // visited offsets are q < end (end >= 1: offset 0 is always visited)
    // (sum1, block) in targets order, stably sorted by sum1: each sum's blocks
    // are one run, in targets order (match.go:108 walks targets in that order)
    std::vector<std::pair<uint32_t, int32_t>> groups;
    std::vector<uint32_t> hi16;  // groups index of the first sum with a given high half (65537 entries)
    std::vector<rsg_match> out;

    int64_t len_of(int32_t i) const {
        return (i == head.count - 1 && head.rem != 0) ? head.rem : head.block_len;  // sender.go:135-139
    }
    uint32_t window(uint64_t q) const {
        return (uint32_t)std::min<uint64_t>((uint64_t)head.block_len, size - q);  // match.go:114-117
    }
};

// Candidate offsets arrive in atomic-append order: LSD radix sort on 16-bit
// digits (as many passes as the largest offset needs), std::sort for few.
void sort_offsets(std::vector<uint64_t> &C) {
    if (C.size() < 4096) {
        std::sort(C.begin(), C.end());
        return;
    }
    uint64_t mx = 0;
    for (uint64_t c : C) mx = std::max(mx, c);
    std::vector<uint64_t> tmp(C.size());
    std::vector<uint32_t> cnt(65537);
    for (int shift = 0; shift < 64 && (mx >> shift) != 0; shift += 16) {
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (uint64_t c : C) cnt[((c >> shift) & 0xffffu) + 1]++;
        for (size_t h = 1; h < cnt.size(); h++) cnt[h] += cnt[h - 1];
        for (uint64_t c : C) tmp[cnt[(c >> shift) & 0xffffu]++] = c;
        C.swap(tmp);
    }
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
    S.pt->mark("v.plan");
    if ((s = ensure_dev(ctx, ctx->d_files, plan.files.size() * sizeof(DevFile) + 32)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_wg, plan.wg_file.size() * sizeof(uint32_t) + 4)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_out[0], plan.total_blocks * kRecordBytes)) != RSG_OK) return s;
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_files.p, plan.files.data(), plan.files.size() * sizeof(DevFile),
                                hipMemcpyHostToDevice, S.st));
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_wg.p, plan.wg_file.data(), plan.wg_file.size() * sizeof(uint32_t),
                                hipMemcpyHostToDevice, S.st));
    if ((s = ensure_dev(ctx, ctx->d_fb[0], rsg::block_sums_scratch_bytes(plan.total_blocks))) != RSG_OK) return s;
    if ((s = launch_plan(ctx, plan, ctx->d_files.p, ctx->d_wg.p, S.d_src, S.seed, ctx->d_out[0].p, ctx->d_fb[0].p,
                         S.st)) != RSG_OK)
        return s;
    // Each window resolves on the GPU to the first block in targets order with
    // equal Sum1, length and sum2[:s2len] (match.go:108-136); only the block
    // indices come back.
    if ((s = ensure_dev(ctx, ctx->d_res, plan.total_blocks * 4)) != RSG_OK) return s;
    RSG_HIP(ctx, rsg::launch_resolve((const uint8_t *)ctx->d_out[0].p, (const DevFile *)ctx->d_files.p,
                                     plan.total_blocks, (const uint2 *)ctx->d_groups.p,
                                     (const uint32_t *)ctx->d_hi16.p, (const uint8_t *)ctx->d_sum2.p,
                                     S.head.count, S.head.block_len, S.head.rem, S.head.s2len,
                                     (int32_t *)ctx->d_res.p, S.st));
    if ((s = ensure_pin(ctx, ctx->h_out[0], plan.total_blocks * 4)) != RSG_OK) return s;
    const int32_t *found = (const int32_t *)ctx->h_out[0].p;
    RSG_HIP(ctx, hipMemcpyAsync(ctx->h_out[0].p, ctx->d_res.p, plan.total_blocks * 4, hipMemcpyDeviceToHost, S.st));
    RSG_HIP(ctx, hipStreamSynchronize(S.st));
    S.pt->mark("v.kernel");
    for (size_t i = 0; i < idx.size(); i++) res[idx[i]] = found[i];
    S.pt->mark("v.resolve");
    return RSG_OK;
}

// Greedy walk over one range's sorted candidates (match.go:93-210 reduced to
// the offsets where the weak sum can hit).
rsg_status walk(Search &S, const std::vector<uint64_t> &C, uint64_t &pos) {
    std::vector<int32_t> res(C.size(), -2);
    size_t i = std::lower_bound(C.begin(), C.end(), pos) - C.begin();
    std::vector<uint32_t> batch;
    while (i < C.size()) {
        const uint64_t c = C[i];
        if ((int64_t)c >= S.end) break;
        if (res[i] == -2) {
            // Batch: every pending candidate ahead while they are sparse (the
            // hashing they cost stays below twice the span they cover); in
            // dense stretches (repetitive data) follow the chain of offsets the
            // walk visits if each confirmation succeeds, plus the candidate
            // after each one in case it fails.
            batch.clear();
            uint64_t hashed = 0;
            size_t j = i;
            for (; j < C.size() && batch.size() < kSparseBatch && (int64_t)C[j] < S.end; j++) {
                if (res[j] == -2) {
                    batch.push_back((uint32_t)j);
                    hashed += S.window(C[j]);
                }
            }
            const uint64_t span = (j > i ? C[j - 1] - c : 0) + (uint64_t)S.head.block_len;
            if (hashed > 2 * span + (1u << 20)) {
                batch.clear();
                uint64_t x = c;
                for (int n = 0; n < 4096; n++) {
                    size_t a = std::lower_bound(C.begin() + i, C.end(), x) - C.begin();
                    if (a >= C.size() || (int64_t)C[a] >= S.end) break;
                    if (res[a] == -2) batch.push_back((uint32_t)a);
                    if (a + 1 < C.size() && (int64_t)C[a + 1] < S.end && res[a + 1] == -2)
                        batch.push_back((uint32_t)(a + 1));
                    x = C[a] + S.window(C[a]);
                }
                std::sort(batch.begin(), batch.end());
                batch.erase(std::unique(batch.begin(), batch.end()), batch.end());
            }
            rsg_status s = verify(S, C, res, batch);
            if (s != RSG_OK) return s;
        }
        const int32_t b = res[i];
        if (b >= 0) {
            S.out.push_back(rsg_match{(int64_t)c, b, 0});
            pos = c + (uint64_t)S.len_of(b);  // match.go:158 + the roll
            while (i < C.size() && C[i] < pos) i++;  // each candidate is stepped over once
        } else {
            pos = c + 1;
            i++;
        }
    }
    return RSG_OK;
}

rsg_status search(rsg_ctx *ctx, const uint8_t *d_src, uint64_t size, const rsg_sum_head *head, const uint32_t *sum1,
                  const uint8_t *sum2, const int32_t *targets, int32_t seed, rsg_match *matches, uint64_t match_cap,
                  uint64_t *n_matches) {
    PhaseTimer pt;
    Search S;
    S.pt = &pt;
    S.seed = seed;
    S.ctx = ctx;
    S.st = ctx->stream;
    S.d_src = d_src;
    S.size = size;
    S.head = *head;
    S.sum2 = sum2;
    const int64_t B = head->block_len;
    const int32_t count = head->count;
    const int64_t last_len = (head->rem != 0) ? head->rem : B;
    S.end = std::max<int64_t>((int64_t)size + 1 - last_len, 1);  // match.go:70 (offset 0 always visited)

    // The prefix pass over the source needs only B: it runs on the GPU while
    // the host builds the filter tables below.
    const uint64_t ntiles64 = (size + kScanTile - 1) / kScanTile;
    if (ntiles64 >= 0xFFFFFFF0ull) return fail(ctx, RSG_ERR_INVALID, "source too large");
    const uint32_t ntiles = (uint32_t)ntiles64;
    rsg_status s;
    if ((s = ensure_dev(ctx, ctx->d_agg, (uint64_t)ntiles * sizeof(TileAgg) + 64)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_prefix, ((uint64_t)ntiles + 1) * sizeof(TilePrefix) + 64)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_list, (uint64_t)kCandCap * 8)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_counts, 64)) != RSG_OK) return s;
    {
        const uint32_t r = (uint32_t)(B % kScanTile);
        RSG_HIP(ctx, rsg::launch_tile_agg(d_src, size, r, (TileAgg *)ctx->d_agg.p, ntiles, S.st));
        RSG_HIP(ctx, rsg::launch_tile_scan((const TileAgg *)ctx->d_agg.p, ntiles, (TilePrefix *)ctx->d_prefix.p, S.st));
    }

    // Basis sums grouped by Sum1 in targets order; device filter = bitmap of
    // every Sum1 + a 2-choice bucketed table {Sum1, flags: bit1 = a block of
    // length B, bit2 = the remainder block}.
    {
        // Stable LSD radix sort (two 16-bit passes) of the targets-ordered
        // (sum1, block) list: equal sums keep their targets order.
        std::vector<std::pair<uint32_t, int32_t>> tmp((size_t)count);
        S.groups.resize((size_t)count);
        for (int32_t k = 0; k < count; k++) tmp[(size_t)k] = {sum1[targets[k]], targets[k]};
        std::vector<uint32_t> cnt(65537);
        for (int pass = 0; pass < 2; pass++) {
            auto &from = pass == 0 ? tmp : S.groups;
            auto &to = pass == 0 ? S.groups : tmp;
            const int shift = 16 * pass;
            std::fill(cnt.begin(), cnt.end(), 0u);
            for (auto &e : from) cnt[((e.first >> shift) & 0xffffu) + 1]++;
            for (size_t h = 1; h < cnt.size(); h++) cnt[h] += cnt[h - 1];
            for (auto &e : from) to[cnt[(e.first >> shift) & 0xffffu]++] = e;
        }
        S.groups.swap(tmp);
        S.hi16.assign(65537, 0);
        for (auto &e : S.groups) S.hi16[(e.first >> 16) + 1]++;
        for (size_t h = 1; h < S.hi16.size(); h++) S.hi16[h] += S.hi16[h - 1];
    }
    pt.mark("groups");
    {
        // device copies for the resolve kernel: (sum1, block) pairs, hi16 index, sum2
        const uint64_t ng = S.groups.size();
        if ((s = ensure_dev(ctx, ctx->d_groups, ng * 8 + 8)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_hi16, S.hi16.size() * 4)) != RSG_OK) return s;
        if ((s = ensure_dev(ctx, ctx->d_sum2, (uint64_t)count * 16 + 16)) != RSG_OK) return s;
        static_assert(sizeof(S.groups[0]) == 8, "(sum1, block) pair must be 8 bytes");
        if (ng) {
            RSG_HIP(ctx, hipMemcpyAsync(ctx->d_groups.p, S.groups.data(), ng * 8, hipMemcpyHostToDevice, S.st));
            RSG_HIP(ctx, hipMemcpyAsync(ctx->d_sum2.p, sum2, (uint64_t)count * 16, hipMemcpyHostToDevice, S.st));
        }
        RSG_HIP(ctx, hipMemcpyAsync(ctx->d_hi16.p, S.hi16.data(), S.hi16.size() * 4, hipMemcpyHostToDevice, S.st));
    }
    std::vector<std::pair<uint32_t, uint32_t>> keys;  // distinct sum1 -> flags
    for (size_t i = 0; i < S.groups.size(); i++) {
        const uint32_t f = 1u | ((S.len_of(S.groups[i].second) == B) ? 2u : 4u);
        if (!keys.empty() && keys.back().first == S.groups[i].first) keys.back().second |= f;
        else keys.push_back({S.groups[i].first, f});
    }
    std::vector<uint32_t> bitmap(rsg::kFilterBits / 32, 0);
    for (auto &kv : keys) {
        const uint32_t h = rsg::filter_hash(kv.first);
        bitmap[rsg::filter_word(h)] |= rsg::filter_mask(h);
    }
    uint32_t nb = 16;
    while (nb < keys.size() / 2) nb <<= 1;
    std::vector<uint64_t> table;
    for (;;) {
        table.assign((size_t)nb * rsg::kBucketWays, 0);
        std::vector<uint8_t> fill(nb, 0);
        bool ok = true;
        for (auto &kv : keys) {
            const uint32_t h1 = rsg::bucket_hash1(kv.first) & (nb - 1), h2 = rsg::bucket_hash2(kv.first) & (nb - 1);
            const uint32_t h = fill[h2] < fill[h1] ? h2 : h1;
            if (fill[h] == rsg::kBucketWays) { ok = false; break; }
            table[(size_t)h * rsg::kBucketWays + fill[h]++] = ((uint64_t)kv.first << 32) | kv.second;
        }
        if (ok) break;
        nb <<= 1;
    }
    pt.mark("tables");
    if ((s = ensure_dev(ctx, ctx->d_filter, bitmap.size() * 4)) != RSG_OK) return s;
    if ((s = ensure_dev(ctx, ctx->d_table, table.size() * 8)) != RSG_OK) return s;
    const uint32_t bmask = nb - 1;
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_filter.p, bitmap.data(), bitmap.size() * 4, hipMemcpyHostToDevice, S.st));
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_table.p, table.data(), table.size() * 8, hipMemcpyHostToDevice, S.st));

    if (pt.on) {
        RSG_HIP(ctx, hipStreamSynchronize(S.st));
        pt.mark("agg+scan");
    }
    int dev_cus = 256;
    hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, ctx->device);
    const uint64_t scan_end = std::min<uint64_t>((uint64_t)S.end, size);
    const uint32_t tile_end = (uint32_t)((scan_end + kScanTile - 1) / kScanTile);
    uint32_t lo = 0, span = tile_end;
    uint64_t pos = 0;
    std::vector<uint64_t> C;
    while (lo < tile_end) {
        const uint32_t hi = std::min(tile_end, lo + span);
        if ((uint64_t)hi * kScanTile <= pos) {  // the walk already jumped past this range
            lo = hi;
            continue;
        }
        RSG_HIP(ctx, hipMemsetAsync(ctx->d_counts.p, 0, 4, S.st));
        RSG_HIP(ctx, rsg::launch_roll(d_src, size, (uint32_t)B, (uint32_t)head->rem, (uint64_t)S.end, lo, hi,
                                      (const TileAgg *)ctx->d_agg.p, (const TilePrefix *)ctx->d_prefix.p, ntiles,
                                      (const uint32_t *)ctx->d_filter.p, (const uint64_t *)ctx->d_table.p, bmask,
                                      (uint64_t *)ctx->d_list.p, kCandCap, (uint32_t *)ctx->d_counts.p,
                                      (uint32_t)dev_cus, S.st));
        uint32_t n = 0;
        RSG_HIP(ctx, hipMemcpyAsync(&n, ctx->d_counts.p, 4, hipMemcpyDeviceToHost, S.st));
        RSG_HIP(ctx, hipStreamSynchronize(S.st));
        if (n > kCandCap) {  // dense range (repetitive data): halve it and retry
            if (hi - lo == 1) return fail(ctx, RSG_ERR_INVALID, "internal: candidate overflow in one tile");
            span = std::max<uint32_t>(1, (hi - lo) / 2);
            continue;
        }
        C.resize(n);
        if (n) {
            RSG_HIP(ctx, hipMemcpyAsync(C.data(), ctx->d_list.p, (uint64_t)n * 8, hipMemcpyDeviceToHost, S.st));
            RSG_HIP(ctx, hipStreamSynchronize(S.st));
        }
        pt.mark("roll");
        sort_offsets(C);
        C.erase(std::unique(C.begin(), C.end()), C.end());
        if ((s = walk(S, C, pos)) != RSG_OK) return s;
        pt.mark("walk");
        lo = hi;
    }
    *n_matches = S.out.size();
    const uint64_t ncopy = std::min<uint64_t>(S.out.size(), match_cap);
    if (ncopy) memcpy(matches, S.out.data(), ncopy * sizeof(rsg_match));
    if (S.out.size() > match_cap)
        return fail(ctx, RSG_ERR_TRUNCATED, "%llu matches, capacity %llu", (unsigned long long)S.out.size(),
                    (unsigned long long)match_cap);
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

}  // namespace

extern "C" {

rsg_status rsg_hash_search_device(rsg_ctx *ctx, const void *d_src, uint64_t src_len, const rsg_sum_head *head,
                                  const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                  rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    rsg_status s = check_args(ctx, head, sum1, sum2, targets, matches, match_cap, n_matches);
    if (s != RSG_OK) return s;
    *n_matches = 0;
    if (head->count == 0 || src_len == 0) return RSG_OK;  // sendFile path / empty source: no matches
    if (!d_src) return fail(ctx, RSG_ERR_INVALID, "NULL source");
    const uint8_t *src = (const uint8_t *)d_src;
    if ((uintptr_t)src & 15u) {  // the scan kernels read 16-byte vectors at 16-byte strides
        if ((s = ensure_dev(ctx, ctx->d_misc, src_len + 64)) != RSG_OK) return s;
        RSG_HIP(ctx, hipMemcpyAsync(ctx->d_misc.p, src, src_len, hipMemcpyDeviceToDevice, ctx->stream));
        src = (const uint8_t *)ctx->d_misc.p;
    }
    return search(ctx, src, src_len, head, sum1, sum2, targets, seed, matches, match_cap, n_matches);
}

rsg_status rsg_hash_search_host(rsg_ctx *ctx, const uint8_t *src, uint64_t src_len, const rsg_sum_head *head,
                                const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    rsg_status s = check_args(ctx, head, sum1, sum2, targets, matches, match_cap, n_matches);
    if (s != RSG_OK) return s;
    *n_matches = 0;
    if (head->count == 0 || src_len == 0) return RSG_OK;
    if (!src) return fail(ctx, RSG_ERR_INVALID, "NULL source");
    if ((s = ensure_dev(ctx, ctx->d_misc, src_len + 64)) != RSG_OK) return s;
    RSG_HIP(ctx, hipMemcpyAsync(ctx->d_misc.p, src, src_len, hipMemcpyHostToDevice, ctx->stream));
    return search(ctx, (const uint8_t *)ctx->d_misc.p, src_len, head, sum1, sum2, targets, seed, matches,
                  match_cap, n_matches);
}

}  // extern "C"
