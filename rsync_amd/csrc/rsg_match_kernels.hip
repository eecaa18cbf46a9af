// rsg_match_kernels.hip -- sender search kernels (internal/sender/match.go:21-230).
//
// The reference slides a block-length window one byte at a time over the
// source, rolling the weak sum (match.go:171-196) and looking every offset up
// in a 16-bit tag table (match.go:95-108).  Here every offset is independent:
// the weak sum of the window [q, e), e = min(q + B, size), is
//     S1 = P[e] - P[q],  S2 = e*(P[e] - P[q]) - (Q[e] - Q[q])   (mod 2^16)
// with P[j] = sum_{i<j} x_i and Q[j] = sum_{i<j} i*x_i over sign-extended
// bytes (SignExtend, rsyncchecksum.go:24-27).  Three kernels:
//   tile_agg   one pass over the source: per 32 KiB tile, (sum x, sum i*x) of
//              the whole tile and of its first r = B mod 32768 bytes;
//   tile_scan  exclusive prefix of the tile sums (P, Q at every tile start);
//   roll       per tile, 1024 lanes x 32 consecutive offsets: initial window
//              from the prefixes plus a workgroup scan, then the reference's
//              own rolling update; each offset is tested against an exact-
//              equivalent filter (128 KiB LDS blocked Bloom filter keyed on the full 32-bit
//              sum, then an L2-resident hash table of the basis sums with the
//              block lengths present) and survivors are appended as
//              candidates.  Candidates are confirmed on the host side of the
//              C-ABI with the strong-sum kernel (rsg_blocksums.hip) in the
//              greedy order of match.go (rsg_match.cpp).
//   roll_packed  the default for B <= kFusedMaxB: the same roll with two
//              windows per lane in the 16-bit halves of each register
//              (v_pk_* updates), a 2^16 x 16-bit LDS filter and a key-only
//              probe table; its range's last tiles on a scalar edge path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "rsg_internal.h"

namespace rsg {

typedef uint32_t u32x4a4m __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ int32_t sx8(uint32_t w, int b) {
    return (int32_t)(w << (24 - 8 * b)) >> 24;  // SignExtend of byte b of w
}

// sx8(a, b) - sx8(c, b) and k * sx8(c, b) (k a 24-bit signed value) in one
// VALU instruction each: SDWA operand byte selects with sign extension
// (SignExtend, rsyncchecksum.go:24-27).  b must fold to a constant.
__device__ __forceinline__ int32_t sub_sx8(uint32_t a, uint32_t c, int b) { return sx8(a, b) - sx8(c, b); }
__device__ __forceinline__ int32_t mul_sx8(int32_t k, uint32_t c, int b) { return k * sx8(c, b); }


// Four little-endian words of src[pos, pos+16); bytes at or past `size` read 0.
// The fast path needs pos 4-byte aligned (the caller guarantees it).
__device__ __forceinline__ void load_vec(const uint8_t *src, uint64_t size, uint64_t pos, uint32_t w[4]) {
    if (pos + 16 <= size) {
        const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(src + pos);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint64_t p = pos + 4 * q + b;
                if (p < size) x |= (uint32_t)src[p] << (8 * b);
            }
            w[q] = x;
        }
    }
}

// sum x and sum k*x (k = 0..15) of one 16-byte vector, signed bytes.
__device__ __forceinline__ void vec_sums(const uint32_t w[4], int32_t &v1, int32_t &v2) {
    v1 = 0;
    v2 = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int wt = (4 * q) | ((4 * q + 1) << 8) | ((4 * q + 2) << 16) | ((4 * q + 3) << 24);
        v1 = __builtin_amdgcn_sdot4((int)w[q], 0x01010101, v1, false);
        v2 = __builtin_amdgcn_sdot4((int)w[q], wt, v2, false);
    }
}

// Inclusive wave64 prefix sum with DPP (row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast 15 / 31 across rows): VALU only, where __shfl_up
// lowers to one ds_bpermute (an LDS instruction) per step.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Sum over the 16 lanes of each row (every row holds the same 16 values):
// DPP row scan, then lane 15's value, wave-uniform.
__device__ __forceinline__ uint32_t row16_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
}

template <typename T>
__device__ __forceinline__ T block_reduce_add(T v, T *scratch) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    T tot = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) tot += scratch[i];
    __syncthreads();
    return tot;
}

// --------------------------------------------------------------- tile_agg
__global__ __launch_bounds__(256) void tile_agg_kernel(const uint8_t *__restrict__ src, uint64_t size, uint32_t r,
                                                       TileAgg *__restrict__ out) {
    __shared__ uint32_t scratch[4][4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
    uint32_t a1 = 0, a2 = 0, r1 = 0, r2 = 0;
#pragma unroll 2
    for (uint32_t j = 0; j < kScanTile / (256 * 16); j++) {
        const uint32_t loc = 16u * (256u * j + threadIdx.x);
        uint32_t w[4];
        load_vec(src, size, t0 + loc, w);
        int32_t v1, v2;
        vec_sums(w, v1, v2);
        a1 += (uint32_t)v1;
        a2 += (uint32_t)v2 + loc * (uint32_t)v1;
        if (loc + 16 <= r) {
            r1 += (uint32_t)v1;
            r2 += (uint32_t)v2 + loc * (uint32_t)v1;
        } else if (loc < r) {  // the vector holding byte r: keep bytes < r only
            const uint32_t keep = r - loc;  // 1..15
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint32_t k = 4 * q + b;
                    if (k < keep) {
                        const int32_t x = sx8(w[q], b);
                        r1 += (uint32_t)x;
                        r2 += (loc + k) * (uint32_t)x;
                    }
                }
        }
    }
    uint32_t (*s)[4] = scratch;
    a1 = block_reduce_add(a1, &s[0][0]);
    a2 = block_reduce_add(a2, &s[1][0]);
    r1 = block_reduce_add(r1, &s[2][0]);
    r2 = block_reduce_add(r2, &s[3][0]);
    if (threadIdx.x == 0) out[blockIdx.x] = TileAgg{a1, a2, r1, r2};
}

// --------------------------------------------------------------- tile_scan
// One workgroup: pre[t] = (P, Q) at the start of tile t (global byte index in
// Q), pre[ntiles] = totals.  Tile t contributes (a1, a2 + t*T*a1).  Rounds of
// 1024 x 32 tiles; a thread owns 32 consecutive tiles of a round, loads them
// all at once (independent loads: one memory latency per round, not one per
// tile) and keeps them in registers for the write-out.
constexpr uint32_t kScanPer = 32;
__global__ __launch_bounds__(1024) void tile_scan_kernel(const TileAgg *__restrict__ agg, uint32_t ntiles,
                                                         TilePrefix *__restrict__ pre) {
    __shared__ uint32_t sp[16], sq[16];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t carry_p = 0, carry_q = 0;
    for (uint64_t base = 0; base < ntiles; base += 1024ull * kScanPer) {
        const uint64_t b = base + (uint64_t)threadIdx.x * kScanPer;
        uint32_t c1[kScanPer], c2[kScanPer];
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            // branch-free: clamped loads, out-of-range tiles contribute 0
            const uint64_t t = b + k;
            const uint2 v = *reinterpret_cast<const uint2 *>(&agg[t < ntiles ? t : ntiles - 1]);
            const uint32_t a1 = t < ntiles ? v.x : 0u, a2 = t < ntiles ? v.y : 0u;
            c1[k] = a1;
            c2[k] = a2 + (uint32_t)t * kScanTile * a1;
        }
        uint32_t p = 0, q = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) { p += c1[k]; q += c2[k]; }
        // inclusive wave scan, then across the 16 waves
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t vp = __shfl_up(p, d, 64), vq = __shfl_up(q, d, 64);
            if (lane >= d) { p += vp; q += vq; }
        }
        if (lane == 63) { sp[wave] = p; sq[wave] = q; }
        __syncthreads();
        uint32_t wp = carry_p, wq = carry_q, tp = carry_p, tq = carry_q;
        for (uint32_t w = 0; w < 16; w++) {
            if (w < wave) { wp += sp[w]; wq += sq[w]; }
            tp += sp[w];
            tq += sq[w];
        }
        __syncthreads();
        // exclusive prefix of this thread's first tile
        uint32_t xp = wp + __shfl_up(p, 1, 64), xq = wq + __shfl_up(q, 1, 64);
        if (lane == 0) { xp = wp; xq = wq; }
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint64_t t = b + k;
            if (t < ntiles) pre[t] = TilePrefix{xp, xq};
            xp += c1[k];
            xq += c2[k];
        }
        carry_p = tp;
        carry_q = tq;
    }
    if (threadIdx.x == 0) pre[ntiles] = TilePrefix{carry_p, carry_q};
}

// --------------------------------------------------------------- roll

// Exact membership of a weak sum in the basis: 2-choice table of buckets of
// kBucketWays entries {sum1 << 32 | flags} (flags: bit0 used, bit1 = a block
// of length B has this sum, bit2 = the remainder block has it).  Two 32-byte
// bucket loads, no probe chains.
__device__ __forceinline__ uint32_t table_flags(const uint64_t *__restrict__ table, uint32_t bmask, uint32_t sum) {
    const uint32_t h1 = bucket_hash1(sum) & bmask, h2 = bucket_hash2(sum) & bmask;
    const uint64_t *b1 = table + (uint64_t)h1 * kBucketWays;
    const uint64_t *b2 = table + (uint64_t)h2 * kBucketWays;
    uint64_t e[2 * kBucketWays];
#pragma unroll
    for (uint32_t i = 0; i < kBucketWays; i++) { e[i] = b1[i]; e[kBucketWays + i] = b2[i]; }
    uint32_t fl = 0;
#pragma unroll
    for (uint32_t i = 0; i < 2 * kBucketWays; i++)
        if ((uint32_t)(e[i] >> 32) == sum && (uint32_t)e[i] != 0) fl |= (uint32_t)e[i];
    return fl;
}

// Whether sum is a basis Sum1, from the key-only copy of the bucket table
// (same buckets; empty slots hold an existing key): two 16-byte loads, eight
// compares.  The block length is not checked here: the confirmation resolves
// a window only to blocks of its own length (match.go:118).
__device__ __forceinline__ bool table_has(uint4 a, uint4 b, uint32_t sum) {
    return (a.x == sum) | (a.y == sum) | (a.z == sum) | (a.w == sum) | (b.x == sum) | (b.y == sum) | (b.z == sum) |
           (b.w == sum);
}
__device__ __forceinline__ void table_buckets(const uint32_t *__restrict__ keys, uint32_t bmask, uint32_t sum,
                                              uint4 &a, uint4 &b) {
    a = *reinterpret_cast<const uint4 *>(keys + (uint64_t)(bucket_hash1(sum) & bmask) * kBucketWays);
    b = *reinterpret_cast<const uint4 *>(keys + (uint64_t)(bucket_hash2(sum) & bmask) * kBucketWays);
}

// The filter word of sum s, and whether both of s's bits are set in it.
template <bool SEL>
__device__ __forceinline__ uint32_t filt_index(uint32_t s) {
    return SEL ? sel_word(s) : filter_word(filter_hash(s));
}
template <bool SEL>
__device__ __forceinline__ bool filt_hit(uint32_t word, uint32_t s) {
    if constexpr (SEL) {
        const uint32_t x = word >> ((s >> 24) & 31u);
        const uint32_t y = word >> (__builtin_amdgcn_alignbit(s, s, 29) & 31u);  // rotr(s, 29)[0..4]
        uint32_t z = x & y & 1u;
        asm("" : "+v"(z));  // one compare serves both the ballot and the lane's own test
        return z != 0;
    } else {
        const uint32_t m = filter_mask(filter_hash(s));
        return (word & m) == m;
    }
}

constexpr uint32_t kQueueCap = 96;  // bitmap hits parked per wave and tile before the exact probes

// SEL: the filter's bit-selection layout (sel_word / sel_mask: 5 VALU per
// test) instead of the rotate-xor hash (8).
template <bool SEL>
__global__ __launch_bounds__(kRollThreads) void roll_kernel(
    const uint8_t *__restrict__ src, uint64_t size, uint32_t B, uint32_t rem, uint64_t end, uint32_t tile_lo,
    uint32_t tile_hi, const TileAgg *__restrict__ agg, const TilePrefix *__restrict__ pre, uint32_t ntiles,
    const uint32_t *__restrict__ bitmap_g, const uint64_t *__restrict__ table, uint32_t bmask,
    uint64_t *__restrict__ cand, uint32_t cap, uint32_t *__restrict__ count, uint32_t fused,
    const uint32_t *__restrict__ ovf) {
    constexpr uint32_t kWaves = kRollThreads / 64;
    constexpr uint32_t P = kRollPerThread;     // offsets per lane
    constexpr int OW = (int)P / 4;             // words of a lane's own bytes
    constexpr int NV = (int)P / 16;            // 16-byte vectors of them
    static_assert(P % 16 == 0 && kWaves <= 16, "lane layout");
    __shared__ uint32_t bitmap[kFilterBits / 32];       // 128 KiB
    __shared__ uint2 queue[kWaves][2][kQueueCap];        // (tile-local offset, sum), per tile parity
    __shared__ uint4 wsum[2][kWaves];                     // scan partials, double-buffered per tile
    __shared__ uint2 carry[2];                            // fused prefix: next tile's (D1, DM), per tile parity
    for (uint32_t i = threadIdx.x; i < kFilterBits / 32; i += kRollThreads) bitmap[i] = bitmap_g[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t Bt = B / kScanTile;
    const TilePrefix tot = fused ? TilePrefix{0, 0} : pre[ntiles];
    const uint32_t rem_flag = (rem != 0 && rem != B) ? 4u : 2u;
    // a table the GPU build could not complete (build_tables_kernel): every
    // filter hit is a candidate, the confirmation sorts them out
    const uint32_t all_flags = __builtin_amdgcn_readfirstlane(*ovf) ? 7u : 0u;
    uint32_t parity = 0;

    // Exact probes of a wave's parked hits (one queue half = one tile); true
    // candidates go to `cand`.  The probes of tile t are issued while tile
    // t+1 is scanned (their L2 latency hides under the offset loop): one
    // entry per lane is prefetched, any further ones are probed in place.
    auto probe = [&](uint64_t q, uint32_t sum, uint32_t fl) {
        const uint32_t k = (uint32_t)min<uint64_t>((uint64_t)B, size - q);
        const uint32_t need = (k == B) ? 2u : ((k == rem) ? rem_flag : 0u);
        if ((fl | all_flags) & need) {
            const uint32_t at = atomicAdd(count, 1u);
            if (at < cap) cand[at] = q;
        }
    };
    auto drain_rest = [&](uint32_t qh, uint64_t q0, uint32_t from, uint32_t n) {
        for (uint32_t i = from + lane; i < n; i += 64) {
            const uint2 e = queue[wave][qh][i];
            probe(q0 + e.x, e.y, table_flags(table, bmask, e.y));
        }
    };
    uint32_t prev_n = 0, qh = 0;  // entries parked by the previous tile, in queue half qh ^ 1
    uint64_t prev_q0 = 0;
    // Each workgroup takes a contiguous run of tiles: the shifted window
    // bytes [q + B, ...) it reads for tile t are tile t + B/32K's own bytes,
    // which the same workgroup reads a few tiles later, so they come from its
    // XCD's L2 instead of HBM (with tiles dealt round-robin the two reads
    // land on different XCDs).
    const uint32_t per = (tile_hi - tile_lo + gridDim.x - 1) / gridDim.x;
    const uint32_t t_begin = tile_lo + blockIdx.x * per;
    const uint32_t t_end = min(tile_hi, t_begin + per);
    const uint32_t lo = threadIdx.x * P;  // local offset of this lane's first offset
    const uint32_t sh = B & 3u;  // (q0 + lo + B) & 3: q0, lo are multiples of 32
    // Fused prefix (B <= kFusedMaxB, no tile_agg / tile_scan passes): the
    // window at tile start q0 needs only D1 = sum x and DM = sum i*x (absolute
    // i, mod 2^32) over [q0, q0 + B), bytes past the source's end reading 0.
    // The run's first tile reduces them directly; each further tile follows
    //   D1(q0 + T) = D1(q0) + sum(shifted bytes) - sum(own bytes)
    // (and the same for DM) from totals the tile's scan produces anyway.
    uint32_t D1 = 0, DM = 0;
    if (fused && t_begin < t_end) {
        const uint64_t qb = (uint64_t)t_begin * kScanTile;
        uint32_t a1 = 0, a2 = 0;
        for (uint32_t off = threadIdx.x * 16u; off < B; off += kRollThreads * 16u) {
            uint32_t w[4];
            load_vec(src, size, qb + off, w);
            if (off + 16u > B) {  // keep bytes < B only
                const uint32_t keep = B - off;
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const uint32_t nb = keep > 4 * q ? min(keep - 4 * q, 4u) : 0u;
                    w[q] &= nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
                }
            }
            int32_t v1, v2;
            vec_sums(w, v1, v2);
            a1 += (uint32_t)v1;
            a2 += (uint32_t)v2 + (uint32_t)(qb + off) * (uint32_t)v1;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            a1 += __shfl_xor(a1, m, 64);
            a2 += __shfl_xor(a2, m, 64);
        }
        if (lane == 0) wsum[0][wave] = make_uint4(a1, a2, 0, 0);
        __syncthreads();
#pragma unroll
        for (uint32_t w = 0; w < kWaves; w++) {
            D1 += __builtin_amdgcn_readfirstlane(wsum[0][w].x);
            DM += __builtin_amdgcn_readfirstlane(wsum[0][w].y);
        }
        __syncthreads();
    }
    // own bytes [qt, qt+32) and the 4-byte aligned shifted bytes around
    // [qt+B, qt+B+32) of tile t; the next tile's are loaded while this one
    // is scanned (one workgroup per CU: nothing else would hide the latency)
    uint32_t O[OW], A[OW + 4], On[OW];
    // Plain 16-byte loads (no end-of-source guards): for tiles whose own and
    // shifted bytes lie inside the source.
    auto fetch_plain = [&](uint32_t tt, uint32_t *o, uint32_t *a) {
        const uint8_t *p = src + (uint64_t)tt * kScanTile + lo;
#pragma unroll
        for (int q = 0; q < NV; q++) {
            const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(p + 16 * q);
            o[4 * q] = v.x; o[4 * q + 1] = v.y; o[4 * q + 2] = v.z; o[4 * q + 3] = v.w;
        }
        const uint8_t *pa = p + B - sh;
#pragma unroll
        for (int q = 0; q < NV + 1; q++) {
            const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(pa + 16 * q);
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
    };
    auto interior = [&](uint32_t tt) { return (uint64_t)(tt + 1) * kScanTile + B + 48 <= size; };
    bool have = false;  // O, A already hold tile t's bytes (prefetched)
    for (uint32_t t = t_begin; t < t_end; t++) {
        const uint64_t q0 = (uint64_t)t * kScanTile;
        if (q0 >= end) break;  // uniform
        const uint64_t qt = q0 + lo;
        if (!have) {
#pragma unroll
            for (int q = 0; q < NV; q++) load_vec(src, size, qt + 16 * q, O + 4 * q);
            const uint64_t pa = qt + B - sh;
#pragma unroll
            for (int q = 0; q < NV + 1; q++) load_vec(src, size, pa + 16 * q, A + 4 * q);
        }
        uint32_t S[OW];
#pragma unroll
        for (int k = 0; k < OW; k++) S[k] = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sh);
        // the next tile's bytes load while this one is scanned (one workgroup
        // per CU: nothing else would hide the latency); A is dead once S is
        // built, so it takes the next tile's shifted bytes
        const bool next = t + 1 < t_end && (uint64_t)(t + 1) * kScanTile < end && interior(t + 1);
        if (next) fetch_plain(t + 1, On, A);
        // the previous tile's first 64 parked hits: entry and bucket loads now
        uint2 pe = make_uint2(0, 0);
        uint64_t pb[2 * kBucketWays];
        const bool pv = lane < prev_n;
        if (pv) {
            pe = queue[wave][qh ^ 1][lane];
            const uint64_t *b1 = table + (uint64_t)(bucket_hash1(pe.y) & bmask) * kBucketWays;
            const uint64_t *b2 = table + (uint64_t)(bucket_hash2(pe.y) & bmask) * kBucketWays;
#pragma unroll
            for (uint32_t i = 0; i < kBucketWays; i++) { pb[i] = b1[i]; pb[kBucketWays + i] = b2[i]; }
        }
        int32_t o1, o2, s1, s2, v1, v2;
        vec_sums(O, o1, o2);
        vec_sums(S, s1, s2);
#pragma unroll
        for (int c = 1; c < NV; c++) {
            vec_sums(O + 4 * c, v1, v2);
            o2 += v2 + 16 * c * v1;
            o1 += v1;
            vec_sums(S + 4 * c, v1, v2);
            s2 += v2 + 16 * c * v1;
            s1 += v1;
        }
        // one workgroup scan of four values: prefixes (within the tile) of the
        // own and shifted byte sums, sum x and sum (local index) * x
        uint32_t v[4] = {(uint32_t)o1, (uint32_t)o2 + lo * (uint32_t)o1, (uint32_t)s1,
                         (uint32_t)s2 + lo * (uint32_t)s1};
        // Only two combinations of the four prefixes enter an interior window
        // (W1 = exA + a tile constant, M = exB + a tile constant):
        //   exA = ex(s1) - ex(o1),  exB = ex(s2') + (q0+B) ex(s1) - ex(o2') - q0 ex(o1)
        // so a tile whose windows are all interior (always, with the fused
        // prefix) scans two values; only a long-block tile near the source's
        // end scans all four (its last windows need the own prefix alone).
        uint32_t exA, exB, ex0 = 0, ex1 = 0;
        const bool two = fused || q0 + kScanTile + B <= size;  // tile-uniform
        {
            const uint32_t a = v[2] - v[0];
            const uint32_t b = (v[3] + (uint32_t)(q0 + B) * v[2]) - (v[1] + (uint32_t)q0 * v[0]);
            uint32_t incl[4];
            if (two) {
                incl[0] = wave_incl_scan(a);
                incl[1] = wave_incl_scan(b);
                if (lane == 63) wsum[parity][wave] = make_uint4(incl[0], incl[1], 0, 0);
            } else {
#pragma unroll
                for (int c = 0; c < 4; c++) incl[c] = wave_incl_scan(v[c]);
                if (lane == 63) wsum[parity][wave] = make_uint4(incl[0], incl[1], incl[2], incl[3]);
            }
            __syncthreads();
            // the partials of the waves before this one: lane l of every row
            // reads wave l's (zero for l >= wave), each row sums its 16 lanes
            const uint32_t w = lane & 15u;
            uint4 p = wsum[parity][min(w, kWaves - 1)];
            if (w >= wave) p = make_uint4(0, 0, 0, 0);
            if (two) {
                exA = incl[0] - a + row16_sum(p.x);
                exB = incl[1] - b + row16_sum(p.y);
            } else {
                uint32_t ex[4];
                const uint32_t add[4] = {row16_sum(p.x), row16_sum(p.y), row16_sum(p.z), row16_sum(p.w)};
#pragma unroll
                for (int c = 0; c < 4; c++) ex[c] = incl[c] - v[c] + add[c];
                exA = ex[2] - ex[0];
                exB = (ex[3] + (uint32_t)(q0 + B) * ex[2]) - (ex[1] + (uint32_t)q0 * ex[0]);
                ex0 = ex[0];
                ex1 = ex[1];
            }
        }
        if (fused && t != t_begin) {  // the previous tile's last lane left this tile's start window
            const uint2 c = carry[parity];
            D1 = __builtin_amdgcn_readfirstlane(c.x);
            DM = __builtin_amdgcn_readfirstlane(c.y);
        }
        parity ^= 1u;
        // Lanes past `end` stay in the loop (they never hit): the probes spread the
        // wave's parked hits over all 64 lanes.
        uint32_t W1, W2, k;
        if (fused) {
            // window [qt, qt + B) = [q0, q0 + B) - [q0, qt) + [q0 + B, qt + B)
            W1 = D1 + exA;
            const uint32_t M = DM + exB;
            k = qt + B <= size ? B : (qt < size ? (uint32_t)(size - qt) : 0u);
            W2 = (uint32_t)(qt + k) * W1 - M;
        } else if (qt + B <= size) {
            // W1 = P[qt + B] - P[qt], Q likewise: the tile constants P[q0 + B] -
            // P[q0] (Q[...]) plus the in-tile prefix differences exA (exB)
            const uint32_t u = min(t + Bt, ntiles);  // tile holding q0 + B
            const uint32_t ur1 = u < ntiles ? agg[u].r1 : 0u, ur2 = u < ntiles ? agg[u].r2 : 0u;
            const uint32_t Pb = pre[u].p + ur1;                                              // P[q0 + B]
            const uint32_t Qb = pre[u].q + ur2 + (uint32_t)((uint64_t)u * kScanTile) * ur1;  // Q[q0 + B]
            W1 = (Pb - pre[t].p) + exA;
            W2 = (uint32_t)(qt + B) * W1 - ((Qb - pre[t].q) + exB);
            k = B;
        } else {
            const uint32_t Pq = pre[t].p + ex0;
            const uint32_t Qq = pre[t].q + ex1 + (uint32_t)q0 * ex0;
            W1 = tot.p - Pq;
            W2 = (uint32_t)size * W1 - (tot.q - Qq);
            k = qt < size ? (uint32_t)(size - qt) : 0u;
        }
        // An opaque copy of lo: without it the compiler hoists lo + j for all
        // 32 offsets out of the tile loop (64 live registers, spilled).
        uint32_t lol = lo;
        asm volatile("" : "+v"(lol));
        uint32_t nq = 0;  // wave-uniform queue fill
        // Park one offset's filter hit in the wave's LDS queue (wave-uniform
        // branch on the ballot).  When the queue is full (repetitive data: most
        // offsets hit) the hit goes straight to the candidate list unprobed;
        // the host-side confirmation re-checks Checksum1 exactly anyway.
        auto park = [&](bool hit, uint32_t j, uint32_t sum) {
            const uint64_t bal = __ballot(hit);
            if (bal) {
                const uint32_t nb = __popcll(bal);
                if (nq + nb <= kQueueCap) {
                    if (hit) {
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                        queue[wave][qh][nq + below] = make_uint2(lol + j, sum);
                    }
                    nq += nb;
                } else if (hit) {
                    const uint32_t at = atomicAdd(count, 1u);
                    if (at < cap) cand[at] = q0 + lol + j;
                }
            }
        };
        // Offsets go in groups of 8: the 8 sums and their bitmap words are
        // computed and fetched first (one LDS wait per group, not per offset),
        // then the hits are parked.
        constexpr int G = 8;
        if (q0 + kScanTile <= end && q0 + kScanTile + B <= size) {
            // Interior tile: every offset is visited and every window has its
            // full length B and a byte entering (match.go:175-191 "more").
            // S2 only matters mod 2^16, so -B*x uses (2^16 - B) mod 2^16, a
            // non-negative 24-bit factor (one v_mul_i32_i24 with an SDWA byte
            // operand, then v_add3: no negation for the compiler to turn into
            // a subtraction).
            const int32_t negB16 = (int32_t)((0x10000u - (B & 0xffffu)) & 0xffffu);
#pragma unroll
            for (int g0 = 0; g0 < (int)P; g0 += G) {
                uint32_t sum[G], word[G];
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    const int j = g0 + jj;
                    sum[jj] = __builtin_amdgcn_perm(W2, W1, 0x05040100u);  // (W1 & 0xffff) | W2 << 16, match.go:106
                    word[jj] = bitmap[filt_index<SEL>(sum[jj])];
                    // W1 += xi - xo; W2 += W1 - B * xo (4 VALU, SDWA byte selects)
                    W1 += (uint32_t)sub_sx8(S[j >> 2], O[j >> 2], j & 3);
                    W2 = W2 + (uint32_t)mul_sx8(negB16, O[j >> 2], j & 3) + W1;
                }
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    const bool hit = filt_hit<SEL>(word[jj], sum[jj]);
                    park(hit, (uint32_t)(g0 + jj), sum[jj]);
                }
                __builtin_amdgcn_sched_barrier(0);  // groups stay apart: registers for the next tile's bytes
            }
        } else {
            // Edge tile (the file's end is near): 32-bit offsets relative to q0.
            const uint32_t end_rel = (uint32_t)min<uint64_t>(end - q0, 0xFFFFFFFFull);
            const uint32_t size_rel = (uint32_t)min<uint64_t>(size > q0 ? size - q0 : 0, 0xFFFFFFFFull);
#pragma unroll
            for (int g0 = 0; g0 < (int)P; g0 += G) {
                uint32_t sum[G], word[G];
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    const int j = g0 + jj;
                    const uint32_t qr = lol + j;
                    sum[jj] = __builtin_amdgcn_perm(W2, W1, 0x05040100u);
                    word[jj] = bitmap[filt_index<SEL>(sum[jj])];
                    // rolling update, match.go:171-196
                    const int32_t xo = sx8(O[j >> 2], j & 3);
                    const bool more = qr + k < size_rel;
                    const int32_t xi = more ? sx8(S[j >> 2], j & 3) : 0;
                    W1 = W1 - (uint32_t)xo + (uint32_t)xi;
                    W2 = W2 - k * (uint32_t)xo + (more ? W1 : 0u);
                    if (!more) k--;
                }
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    const bool hit = filt_hit<SEL>(word[jj], sum[jj]) && (lol + g0 + jj < end_rel);
                    park(hit, (uint32_t)(g0 + jj), sum[jj]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // Fused prefix: after its 32 updates the tile's last lane holds the
        // window at q0 + T (length k): the next tile's D1 = W1 and
        // DM = (q0 + T + k) W1 - W2 (only their low 16 bits matter).
        if (fused && threadIdx.x == kRollThreads - 1)
            carry[parity] = make_uint2(W1, (uint32_t)(q0 + kScanTile + k) * W1 - W2);
        if (pv) {
            uint32_t fl = 0;
#pragma unroll
            for (uint32_t i = 0; i < 2 * kBucketWays; i++)
                if ((uint32_t)(pb[i] >> 32) == pe.y && (uint32_t)pb[i] != 0) fl |= (uint32_t)pb[i];
            probe(prev_q0 + pe.x, pe.y, fl);
        }
        if (prev_n > 64) drain_rest(qh ^ 1, prev_q0, 64, prev_n);
        prev_n = nq;
        prev_q0 = q0;
        qh ^= 1u;
        if (next) {
#pragma unroll
            for (int k = 0; k < OW; k++) O[k] = On[k];
        }
        have = next;
    }
    drain_rest(qh ^ 1, prev_q0, 0, prev_n);  // the last tile's hits
}

// --------------------------------------------------------------- roll, packed
// Interior tiles of the fused mode (every window has length B, every offset
// is visited), two offsets per VALU instruction.  S1 and S2 only matter mod
// 2^16 (match.go:106), so a lane rolls two windows at once in 16-bit halves:
// stream a = its offsets 0..15, stream b = its offsets 16..31.
//   P1 = (W1_a + 128B, W1_b + 128B)   P2 = (W2_a, W2_b)          (mod 2^16)
// over bytes u = x ^ 0x80 (SignExtend(x) = u - 128, rsyncchecksum.go:24-27):
//   P1 += u_in - u_out;  P2 += P1 - B u_out      (= match.go:175-191's update:
//   W1 += x_in - x_out;  W2 += W1 - B x_out, the 128B in P1 absorbs the -128s)
// one v_perm per operand pair and four v_pk_* per two offsets.  The filter is
// 2^16 16-bit words indexed by P1 ^ P2 (word ((W1 + 128B) ^ W2) mod 2^16, the
// host builds it shifted; one v_xor for both windows), bits W2[0..3],
// W2[4..7] and W2[8..11]: a 16-bit shift of both halves at once
// (v_pk_lshlrev_b16, the bits stored at 15 - s) per bit.  About 0.6 % of non-matching window sums pass
// with 32768 basis sums (1.0 % with the first two bits only).
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// v_pk_lshlrev_b16: each half of w shifted left by the low 4 bits of the
// same half of s (the hardware's own masking; a C shift needs an explicit
// `& 15` the compiler keeps).
__device__ __forceinline__ u16x2 pk_shl(u16x2 w, u16x2 s) {
    uint32_t d;
    asm("v_pk_lshlrev_b16 %0, %1, %2" : "=v"(d) : "v"(as_u32(s)), "v"(as_u32(w)));
    return as_u16x2(d);
}

// Byte p of wa in the low half, byte p of wb in the high half (zero-extended).
__device__ __forceinline__ u16x2 pair_bytes(uint32_t wa, uint32_t wb, int p) {
    const uint32_t sel = 0x0c000c00u | ((4u + (uint32_t)p) << 16) | (uint32_t)p;
    return as_u16x2(__builtin_amdgcn_perm(wb, wa, sel));
}

// NBITS: filter bits per sum, S2[0..3], S2[4..7] (and S2[8..11]); EDGE: the
// kernel rolls the range's edge tiles itself (else the host leaves them to
// roll_kernel and passes t_int = tile_hi); BT: B is the tile length (the
// reference's block length for a 1 GiB file, sqrt(2^30)): the bytes a lane
// shifts in over tile t are the ones it shifts out over tile t + 1, so their
// sums and their xor-ed copy carry over instead of being loaded and summed
// again (16 v_dot4, 8 v_alignbyte, 8 v_xor and two 16-byte loads per lane
// and tile fewer).
template <int NBITS, bool EDGE, bool BT>
__global__ __launch_bounds__(kRollThreads) void roll_packed_kernel(
    const uint8_t *__restrict__ src, uint64_t size, uint32_t B, uint32_t rem, uint64_t end, uint32_t tile_lo,
    uint32_t t_int, uint32_t tile_hi, const uint16_t *__restrict__ filter_g, const uint32_t *__restrict__ keys,
    uint32_t bmask, uint64_t *__restrict__ cand, uint32_t cap, uint32_t *__restrict__ count,
    const uint32_t *__restrict__ ovf) {
    constexpr uint32_t kWaves = kRollThreads / 64;
    constexpr uint32_t P = kRollPerThread;  // offsets per lane (2 streams of P/2)
    constexpr int OW = (int)P / 4;
    constexpr int NV = (int)P / 16;
    constexpr int H = (int)P / 2;           // offsets per stream
    static_assert(P == 32 && kWaves <= 16, "two streams of 16 offsets per lane");
    __shared__ uint16_t filt[1u << 16];                   // 128 KiB
    __shared__ uint2 queue[kWaves][2][kQueueCap];        // (tile-local offset, raw packed sum), per tile parity
    __shared__ uint2 wsum[2][kWaves];                     // scan partials, double-buffered per tile
    __shared__ uint2 carry[2];                            // next tile's (D1, DM), per tile parity
    {
        const uint4 *fg = reinterpret_cast<const uint4 *>(filter_g);
        uint4 *fl = reinterpret_cast<uint4 *>(filt);
        for (uint32_t i = threadIdx.x; i < (1u << 16) / 8; i += kRollThreads) fl[i] = fg[i];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t C128 = (128u * B) & 0xffffu;  // the filter index offset of P1
    const bool all = __builtin_amdgcn_readfirstlane(*ovf) != 0;  // incomplete table (roll_kernel's all_flags)
    uint32_t parity = 0;

    // Exact probes of a wave's parked hits: the window at q (length k =
    // min(B, size - q); interior windows k = B) is a candidate when its sum
    // is a basis Sum1 and some block has length k.
    auto probe = [&](uint64_t q, bool present) {
        const uint32_t k = (uint32_t)min<uint64_t>((uint64_t)B, size - q);
        if ((present || all) && (k == B || k == rem)) {
            const uint32_t at = atomicAdd(count, 1u);
            if (at < cap) cand[at] = q;
        }
    };
    auto unraw = [&](uint32_t raw) { return (raw & 0xffff0000u) | ((raw - C128) & 0xffffu); };
    auto drain_rest = [&](uint32_t qh, uint64_t q0, uint32_t from, uint32_t n) {
        for (uint32_t i = from + lane; i < n; i += 64) {
            const uint2 e = queue[wave][qh][i];
            const uint32_t sum = unraw(e.y);
            uint4 ba, bb;
            table_buckets(keys, bmask, sum, ba, bb);
            probe(q0 + e.x, table_has(ba, bb, sum));
        }
    };
    uint32_t prev_n = 0, qh = 0;
    uint64_t prev_q0 = 0;
    const uint32_t per = (tile_hi - tile_lo + gridDim.x - 1) / gridDim.x;
    const uint32_t t_begin = tile_lo + blockIdx.x * per;
    const uint32_t t_end = min(tile_hi, t_begin + per);
    const uint32_t lo = threadIdx.x * P;
    const uint32_t sh = B & 3u;
    // The run's first window [q0, q0 + B): D1 = sum x, DM = sum i*x (absolute i).
    uint32_t D1 = 0, DM = 0;
    if (t_begin < t_end) {
        const uint64_t qb = (uint64_t)t_begin * kScanTile;
        uint32_t a1 = 0, a2 = 0;
        for (uint32_t off = threadIdx.x * 16u; off < B; off += kRollThreads * 16u) {
            uint32_t w[4];
            load_vec(src, size, qb + off, w);
            if (off + 16u > B) {
                const uint32_t keep = B - off;
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const uint32_t nb = keep > 4 * q ? min(keep - 4 * q, 4u) : 0u;
                    w[q] &= nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
                }
            }
            int32_t v1, v2;
            vec_sums(w, v1, v2);
            a1 += (uint32_t)v1;
            a2 += (uint32_t)v2 + (uint32_t)(qb + off) * (uint32_t)v1;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            a1 += __shfl_xor(a1, m, 64);
            a2 += __shfl_xor(a2, m, 64);
        }
        if (lane == 0) wsum[0][wave] = make_uint2(a1, a2);
        __syncthreads();
#pragma unroll
        for (uint32_t w = 0; w < kWaves; w++) {
            D1 += __builtin_amdgcn_readfirstlane(wsum[0][w].x);
            DM += __builtin_amdgcn_readfirstlane(wsum[0][w].y);
        }
        __syncthreads();
    }
    uint32_t O[OW], A[OW + 4], On[OW];
    // BT: the previous tile's shifted bytes = this tile's outgoing ones, kept
    // as the pair step's operands (xor-ed, the two streams' bytes in 16-bit
    // halves: the v_perm of the step that shifted them in), and their sums
    u16x2 Uo[BT ? H : 1];
    int32_t c1 = 0, c2 = 0, c1a = 0, c2a = 0;
    if constexpr (BT) {
#pragma unroll
        for (int k = 0; k < H; k++) Uo[k] = u16x2{0, 0};
    }
    auto fetch_shifted = [&](uint32_t tt, uint32_t *a) {  // BT: the next tile's shifted bytes only (sh = 0)
        const uint8_t *pa = src + (uint64_t)tt * kScanTile + lo + B;
#pragma unroll
        for (int q = 0; q < NV; q++) {
            const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(pa + 16 * q);
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
    };
    auto fetch_plain = [&](uint32_t tt, uint32_t *o, uint32_t *a) {
        const uint8_t *p = src + (uint64_t)tt * kScanTile + lo;
#pragma unroll
        for (int q = 0; q < NV; q++) {
            const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(p + 16 * q);
            o[4 * q] = v.x; o[4 * q + 1] = v.y; o[4 * q + 2] = v.z; o[4 * q + 3] = v.w;
        }
        const uint8_t *pa = p + B - sh;
#pragma unroll
        for (int q = 0; q < NV + 1; q++) {
            const u32x4a4m v = *reinterpret_cast<const u32x4a4m *>(pa + 16 * q);
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
    };
    const u16x2 negB = as_u16x2(((0x10000u - (B & 0xffffu)) & 0xffffu) * 0x10001u);
    bool have = false;  // O, A already hold tile t's bytes (prefetched)
    for (uint32_t t = t_begin; t < t_end; t++) {
        const uint64_t q0 = (uint64_t)t * kScanTile;
        if (q0 >= end) break;  // uniform
        const uint64_t qt = q0 + lo;
        if (!have) {  // the run's first tile, or an edge tile: guarded loads
#pragma unroll
            for (int q = 0; q < NV; q++) load_vec(src, size, qt + 16 * q, O + 4 * q);
#pragma unroll
            for (int q = 0; q < NV + 1; q++) load_vec(src, size, qt + B - sh + 16 * q, A + 4 * q);
        }
        const bool edge = EDGE && t >= t_int;  // windows shorter than B or offsets past end: the scalar path
        uint32_t S[OW];
#pragma unroll
        for (int k = 0; k < OW; k++) S[k] = BT ? A[k] : __builtin_amdgcn_alignbyte(A[k + 1], A[k], sh);
        const bool next = t + 1 < t_end && t + 1 < t_int;
        // BT: the shifted bytes' sums and xor-ed copy before the prefetch reuses A
        int32_t s1, s2, v1, v2, s1a = 0, s2a = 0;
        uint32_t Sx[OW];
        if constexpr (BT) {
            vec_sums(S, s1, s2);
            s1a = s1;
            s2a = s2;
#pragma unroll
            for (int c = 1; c < NV; c++) {
                vec_sums(S + 4 * c, v1, v2);
                s2 += v2 + 16 * c * v1;
                s1 += v1;
            }
#pragma unroll
            for (int k = 0; k < OW; k++) Sx[k] = S[k] ^ 0x80808080u;
            if (next) fetch_shifted(t + 1, A);
        } else {
            if (next) fetch_plain(t + 1, On, A);
        }
        uint2 pe = make_uint2(0, 0);
        uint4 pba, pbb;
        const bool pv = lane < prev_n;
        if (pv) {
            pe = queue[wave][qh ^ 1][lane];
            pe.y = unraw(pe.y);
            table_buckets(keys, bmask, pe.y, pba, pbb);
        }
        // lane totals, and the first 16 bytes' own (stream a's range) for
        // stream b's start window
        int32_t o1, o2, o1a, o2a;
        if (BT && have) {  // tile t - 1's shifted bytes, summed there
            o1 = c1; o2 = c2; o1a = c1a; o2a = c2a;
        } else {
            vec_sums(O, o1, o2);
            o1a = o1;
            o2a = o2;
#pragma unroll
            for (int c = 1; c < NV; c++) {
                vec_sums(O + 4 * c, v1, v2);
                o2 += v2 + 16 * c * v1;
                o1 += v1;
            }
            if constexpr (BT) {  // in this (uniform) branch, so the loop's uo = Uo needs no per-lane select
#pragma unroll
                for (int j = 0; j < H; j++)
                    Uo[j] = pair_bytes(O[j >> 2] ^ 0x80808080u, O[(j >> 2) + OW / 2] ^ 0x80808080u, j & 3);
            }
        }
        if constexpr (!BT) {
            vec_sums(S, s1, s2);
            s1a = s1;
            s2a = s2;
#pragma unroll
            for (int c = 1; c < NV; c++) {
                vec_sums(S + 4 * c, v1, v2);
                s2 += v2 + 16 * c * v1;
                s1 += v1;
            }
        }
        // one workgroup scan of exA = ex(s1) - ex(o1), exB (roll_kernel's
        // two-value form: every window here is interior)
        uint32_t exA, exB;
        {
            const uint32_t so2 = (uint32_t)s2 + lo * (uint32_t)s1, oo2 = (uint32_t)o2 + lo * (uint32_t)o1;
            const uint32_t a = (uint32_t)s1 - (uint32_t)o1;
            const uint32_t b = (so2 + (uint32_t)(q0 + B) * (uint32_t)s1) - (oo2 + (uint32_t)q0 * (uint32_t)o1);
            const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
            if (lane == 63) wsum[parity][wave] = make_uint2(ia, ib);
            __syncthreads();
            const uint32_t w = lane & 15u;
            uint2 p = wsum[parity][min(w, kWaves - 1)];
            if (w >= wave) p = make_uint2(0, 0);
            exA = ia - a + row16_sum(p.x);
            exB = ib - b + row16_sum(p.y);
        }
        if (t != t_begin) {
            const uint2 c = carry[parity];
            D1 = __builtin_amdgcn_readfirstlane(c.x);
            DM = __builtin_amdgcn_readfirstlane(c.y);
        }
        parity ^= 1u;
        uint32_t lol = lo;
        asm volatile("" : "+v"(lol));
        uint32_t nq = 0;
        auto park_m = [&](uint64_t bal, bool hit, uint32_t j, uint32_t raw) {  // bal = __ballot(hit)
            if (bal) {
                const uint32_t nb = __popcll(bal);
                if (nq + nb <= kQueueCap) {
                    if (hit) {
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                        queue[wave][qh][nq + below] = make_uint2(lol + j, raw);
                    }
                    nq += nb;
                } else if (hit) {
                    const uint32_t at = atomicAdd(count, 1u);
                    if (at < cap) cand[at] = q0 + lol + j;
                }
            }
        };
        auto park = [&](bool hit, uint32_t j, uint32_t raw) { park_m(__ballot(hit), hit, j, raw); };
        if constexpr (!EDGE) {
        } else if (edge) {
            // The source's last tiles (roll_kernel's edge path, with this
            // kernel's filter): 32-bit offsets relative to q0, the window at
            // qt of length k = min(B, size - qt), bytes past the end read 0.
            uint32_t W1 = D1 + exA;
            const uint32_t M = DM + exB;
            uint32_t k = qt + B <= size ? B : (qt < size ? (uint32_t)(size - qt) : 0u);
            uint32_t W2 = (uint32_t)(qt + k) * W1 - M;
            const uint32_t end_rel = (uint32_t)min<uint64_t>(end - q0, 0xFFFFFFFFull);
            const uint32_t size_rel = (uint32_t)min<uint64_t>(size > q0 ? size - q0 : 0, 0xFFFFFFFFull);
            constexpr int GE = 8;
#pragma unroll
            for (int g0 = 0; g0 < (int)P; g0 += GE) {
                uint32_t raw[GE], word[GE];
#pragma unroll
                for (int jj = 0; jj < GE; jj++) {
                    const int j = g0 + jj;
                    const uint32_t qr = lol + j;
                    raw[jj] = ((W1 + C128) & 0xffffu) | (W2 << 16);           // unraw() gives the sum
                    word[jj] = filt[((W1 + C128) ^ W2) & 0xffffu];           // f16_word
                    const int32_t xo = sx8(O[j >> 2], j & 3);                // match.go:171-196
                    const bool more = qr + k < size_rel;
                    const int32_t xi = more ? sx8(S[j >> 2], j & 3) : 0;
                    W1 = W1 - (uint32_t)xo + (uint32_t)xi;
                    W2 = W2 - k * (uint32_t)xo + (more ? W1 : 0u);
                    if (!more) k--;
                }
#pragma unroll
                for (int jj = 0; jj < GE; jj++) {
                    const uint32_t s2 = raw[jj] >> 16;  // bits at 15 - s (f16_mask)
                    uint32_t bits = (word[jj] << (s2 & 15u)) & (word[jj] << ((s2 >> 4) & 15u));
                    if constexpr (NBITS == 3) bits &= word[jj] << ((s2 >> 8) & 15u);
                    park((bits & 0x8000u) && (lol + g0 + jj < end_rel), (uint32_t)(g0 + jj), raw[jj]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            if (threadIdx.x == kRollThreads - 1)
                carry[parity] = make_uint2(W1, (uint32_t)(q0 + kScanTile + k) * W1 - W2);
        }
        if (!edge) {
        // window at the lane's first offset, then at its 17th (16 rolling
        // steps in closed form: W1 + sum d, W2 + 16 W1 + sum (16 - j) d_j - B sum x_out)
        const uint32_t W1 = D1 + exA;
        const uint32_t W2 = (uint32_t)(qt + B) * W1 - (DM + exB);
        const uint32_t da = (uint32_t)(s1a - o1a);
        const uint32_t W1b = W1 + da;
        const uint32_t W2b = W2 + 16u * W1 + 16u * da - (uint32_t)(s2a - o2a) - B * (uint32_t)o1a;
        u16x2 P1 = as_u16x2(((W1 + C128) & 0xffffu) | ((W1b + C128) << 16));
        u16x2 P2 = as_u16x2((W2 & 0xffffu) | (W2b << 16));
        uint32_t Ox[BT ? 1 : OW];
        if constexpr (!BT) {
#pragma unroll
            for (int k = 0; k < OW; k++) {
                Ox[k] = O[k] ^ 0x80808080u;
                Sx[k] = S[k] ^ 0x80808080u;
            }
        }
        constexpr int G = 4;  // pair steps per group: 8 filter reads in flight
        uint32_t one16 = 1;  // the SDWA shift count of the filter addresses (a VGPR operand)
        asm("" : "+v"(one16));
#pragma unroll
        for (int g0 = 0; g0 < H; g0 += G) {
            u16x2 p1[G], p2[G], wd[G];
            uint32_t wl[G], wh[G];  // the two filter words of each step, joined after the group's loads
#pragma unroll
            for (int jj = 0; jj < G; jj++) {
                const int j = g0 + jj;
                p1[jj] = P1;
                p2[jj] = P2;
                const u16x2 X = P1 ^ P2;  // the word index of both windows
                {
                    // the filter words' LDS byte addresses 2 X.x, 2 X.y: one SDWA
                    // shift each (the compiler's form takes three VALU for the
                    // pair), plus the filter's LDS base (0: the add folds away).
                    // (d16 loads into the two halves of one VGPR would save the
                    // v_perm too, but with SRAM ECC on gfx950 a d16 load zeroes
                    // the other half: measured, the parity tests failed.)
                    const uint32_t fb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint16_t *)filt;
                    const uint32_t xa = as_u32(X);
                    uint32_t alo, ahi;
                    asm("v_lshlrev_b32_sdwa %0, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
                        "v_lshlrev_b32_sdwa %1, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                        : "=&v"(alo), "=&v"(ahi) : "v"(xa), "v"(one16));
                    typedef __attribute__((address_space(3))) const uint16_t lds16;
                    wl[jj] = *(lds16 *)(uintptr_t)(alo + fb);
                    wh[jj] = *(lds16 *)(uintptr_t)(ahi + fb);
                }
                if constexpr (BT) {
                    // uo's last uses, then ui written over it in place (a tied
                    // asm operand): the pair carried to the next tile keeps
                    // its register, no copies at the tile loop's back edge
                    const u16x2 uo = Uo[j];
                    P1 = P1 - uo;
                    P2 = P2 + uo * negB;
                    uint32_t r = as_u32(uo);
                    const uint32_t sel = 0x0c000c00u | ((4u + (uint32_t)(j & 3)) << 16) | (uint32_t)(j & 3);
                    asm("v_perm_b32 %0, %1, %2, %3" : "+v"(r) : "v"(Sx[(j >> 2) + OW / 2]), "v"(Sx[j >> 2]), "s"(sel));
                    Uo[j] = as_u16x2(r);  // this step's ui: the next tile's outgoing pair
                    P1 = P1 + Uo[j];
                    P2 = P2 + P1;
                } else {
                    const u16x2 uo = pair_bytes(Ox[j >> 2], Ox[(j >> 2) + OW / 2], j & 3);
                    const u16x2 ui = pair_bytes(Sx[j >> 2], Sx[(j >> 2) + OW / 2], j & 3);
                    P1 = P1 + ui - uo;
                    P2 = P2 + uo * negB + P1;
                }
            }
            // The group's eight filter reads are all issued before the first
            // is used: the words are joined into pairs only here, so the first
            // join waits for its own two reads while the other six are in
            // flight (joined right after each pair of reads, every step waited
            // out the whole LDS latency).
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int jj = 0; jj < G; jj++) wd[jj] = as_u16x2(__builtin_amdgcn_perm(wh[jj], wl[jj], 0x05040100u));
            // the group's eight hit masks first, then its parks: each park's
            // branch then tests a mask computed several instructions earlier
            // instead of waiting on the compare right before it
            uint64_t mk[2 * G];
#pragma unroll
            for (int jj = 0; jj < G; jj++) {
                // every tested bit shifted into bit 15 of its half (f16_mask):
                // the AND is the test, its two sign bits the two hits (no
                // mask; the low half by a 16-bit compare, which reads bits
                // 0..15 only)
                const u16x2 x = pk_shl(wd[jj], p2[jj]);
                const u16x2 y = pk_shl(wd[jj], p2[jj] >> (uint16_t)4);
                u16x2 xy = x & y;
                if constexpr (NBITS == 3) xy &= pk_shl(wd[jj], p2[jj] >> (uint16_t)8);
                uint32_t z = as_u32(xy);
                asm("" : "+v"(z));
                uint64_t mlo;
                asm("v_cmp_gt_i16_e64 %0, 0, %1" : "=s"(mlo) : "v"(z));
                mk[2 * jj] = mlo;
                mk[2 * jj + 1] = __ballot((int32_t)z < 0);
            }
            // room in the queue for the whole group (nearly always): parks
            // without a per-park capacity test; else park_m's own
            uint32_t gn = 0;
#pragma unroll
            for (int k = 0; k < 2 * G; k++) gn += (uint32_t)__popcll(mk[k]);
            if (nq + gn <= kQueueCap) {
#pragma unroll
                for (int k = 0; k < 2 * G; k++) {
                    const int jj = k >> 1;
                    const uint64_t bal = mk[k];
                    if (bal) {
                        if (__builtin_amdgcn_inverse_ballot_w64(bal)) {
                            const uint32_t r1 = as_u32(p1[jj]), r2 = as_u32(p2[jj]);
                            const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                            queue[wave][qh][nq + below] =
                                make_uint2(lol + (uint32_t)((k & 1) * H + g0 + jj),
                                           __builtin_amdgcn_perm(r2, r1, (k & 1) ? 0x07060302u : 0x05040100u));
                        }
                        nq += (uint32_t)__popcll(bal);
                    }
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < G; jj++) {
                    const int j = g0 + jj;
                    const uint32_t r1 = as_u32(p1[jj]), r2 = as_u32(p2[jj]);
                    park_m(mk[2 * jj], __builtin_amdgcn_inverse_ballot_w64(mk[2 * jj]), (uint32_t)j,
                           __builtin_amdgcn_perm(r2, r1, 0x05040100u));
                    park_m(mk[2 * jj + 1], __builtin_amdgcn_inverse_ballot_w64(mk[2 * jj + 1]), (uint32_t)(H + j),
                           __builtin_amdgcn_perm(r2, r1, 0x07060302u));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // the tile's last lane ends at the next tile's first window
        if (threadIdx.x == kRollThreads - 1) {
            const uint32_t w1 = ((as_u32(P1) >> 16) - C128) & 0xffffu, w2 = as_u32(P2) >> 16;
            carry[parity] = make_uint2(w1, (uint32_t)(q0 + kScanTile + B) * w1 - w2);
        }
        if constexpr (BT) {  // this tile's shifted bytes are the next tile's outgoing ones (Uo set in the loop)
            c1 = s1; c2 = s2; c1a = s1a; c2a = s2a;
        }
        }  // interior tile
        if (pv) probe(prev_q0 + pe.x, table_has(pba, pbb, pe.y));
        if (prev_n > 64) drain_rest(qh ^ 1, prev_q0, 64, prev_n);
        prev_n = nq;
        prev_q0 = q0;
        qh ^= 1u;
        if (!BT && next) {
#pragma unroll
            for (int k = 0; k < OW; k++) O[k] = On[k];
        }
        have = next;
    }
    drain_rest(qh ^ 1, prev_q0, 0, prev_n);
}

// --------------------------------------------------------------- confirm plan
// One DevFile per candidate window, in the roll's append order: window
// [q, q + min(B, size - q)) is record i (match.go:114-117).  The confirmation
// of a sparse range starts as soon as the roll's count is known, without the
// candidates' round trip through the host (rsg_match.cpp: confirm_all).
__global__ __launch_bounds__(256) void confirm_plan_kernel(const uint64_t *__restrict__ cand, uint32_t n,
                                                           uint64_t size, uint32_t B, DevFile *__restrict__ files,
                                                           uint32_t *__restrict__ wg_file, uint32_t nwg) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        const uint64_t q = cand[i];
        const uint32_t k = (uint32_t)min<uint64_t>((uint64_t)B, size - q);
        files[i] = DevFile{q, k, i, k, 1};
    }
    if (i <= nwg) wg_file[i] = min(i * 256u, n - 1);  // plan layout of rsg_match.cpp verify()
}

hipError_t launch_confirm_plan(const uint64_t *cand, uint32_t n, uint64_t size, uint32_t B, DevFile *files,
                               uint32_t *wg_file, uint32_t nwg, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t threads = max(n, nwg + 1);
    hipLaunchKernelGGL(confirm_plan_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, cand, n, size, B, files,
                       wg_file, nwg);
    return hipGetLastError();
}

// --------------------------------------------------------------- resolve
__global__ __launch_bounds__(256) void resolve_kernel(const uint8_t *__restrict__ records,
                                                      const DevFile *__restrict__ files, uint64_t n,
                                                      const uint2 *__restrict__ groups,
                                                      const uint32_t *__restrict__ hi16,
                                                      const uint8_t *__restrict__ sum2, int32_t count, int32_t blen,
                                                      int32_t rem, int32_t s2len, int32_t *__restrict__ res) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t *r = reinterpret_cast<const uint32_t *>(records + i * kRecordBytes);
    const uint32_t w = r[0];
    const uint32_t d[4] = {r[1], r[2], r[3], r[4]};
    const uint64_t k = files[i].len;
    int32_t found = -1;
    for (uint32_t j = hi16[w >> 16], stop = hi16[(w >> 16) + 1]; j < stop; j++) {
        const uint2 gb = groups[j];
        if (gb.x < w) continue;
        if (gb.x > w) break;
        const int32_t b = (int32_t)gb.y;
        const uint64_t len = (b == count - 1 && rem != 0) ? (uint64_t)rem : (uint64_t)blen;  // sender.go:135-139
        if (len != k) continue;                                                                // match.go:118
        const uint8_t *want = sum2 + 16 * (uint64_t)b;
        bool eq = true;
        for (int32_t q = 0; q < s2len; q++)                                                    // match.go:133
            eq = eq && (want[q] == (uint8_t)(d[q >> 2] >> (8 * (q & 3))));
        if (eq) { found = b; break; }
    }
    res[i] = found;
}

hipError_t launch_resolve(const uint8_t *records, const DevFile *files, uint64_t n, const uint2 *groups,
                          const uint32_t *hi16, const uint8_t *sum2, int32_t count, int32_t blen, int32_t rem,
                          int32_t s2len, int32_t *res, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(resolve_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, records, files, n,
                       groups, hi16, sum2, count, blen, rem, s2len, res);
    return hipGetLastError();
}

hipError_t launch_tile_agg(const uint8_t *src, uint64_t size, uint32_t r, TileAgg *out, uint32_t ntiles,
                           hipStream_t stream) {
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_agg_kernel, dim3(ntiles), dim3(256), 0, stream, src, size, r, out);
    return hipGetLastError();
}

hipError_t launch_tile_scan(const TileAgg *agg, uint32_t ntiles, TilePrefix *pre, hipStream_t stream) {
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, stream, agg, ntiles, pre);
    return hipGetLastError();
}

// ------------------------------------------------------------- roll tables
// Part A of the basis tables (rsg_match.cpp: tables_roll) built on the GPU
// from the uploaded Sum1 array, one lane per block k: the Bloom filter bits,
// the packed roll's 16-bit filter bits and the 2-choice bucket table entry
// {Sum1 << 32 | flags} (flags: 1, and 2 = a block of length B, 4 = the
// shorter last block).  An entry goes into the first free slot of the less
// filled bucket by a 64-bit CAS (slots fill in order, so a scan stops at the
// first empty one); an equal key already present gets its flags OR-ed in,
// as the host build merges them.  Both buckets full: *ovf = 1, and the rolls
// take every filter hit as a candidate (the confirmation and resolve, from
// the host-built exact groups, keep the result exact).  The table has at
// least 2 buckets per key (4 ways each), so that is reserved for pathological
// key sets.
__global__ __launch_bounds__(256) void build_tables_kernel(const uint32_t *__restrict__ sum1, int32_t count,
                                                           uint32_t B, uint32_t rem, int packed,
                                                           uint32_t *__restrict__ bitmap,
                                                           uint32_t *__restrict__ filter16w,
                                                           unsigned long long *__restrict__ table, uint32_t bmask,
                                                           uint32_t *__restrict__ ovf) {
    const int32_t k = (int32_t)(blockIdx.x * 256u + threadIdx.x);
    if (k >= count) return;
    const uint32_t v = sum1[k];
    atomicOr(&bitmap[sel_word(v)], sel_mask(v));
    if (packed) {
        const uint32_t w = f16_word(v, B);
        atomicOr(&filter16w[w >> 1], (f16_mask(v) & 0xffffu) << (16u * (w & 1u)));
    }
    const uint32_t len = (k == count - 1 && rem != 0) ? rem : B;  // types.go: the last block may be short
    const unsigned long long f = 1u | (len == B ? 2u : 4u);
    const unsigned long long e = ((unsigned long long)v << 32) | f;
    const uint32_t hb[2] = {bucket_hash1(v) & bmask, bucket_hash2(v) & bmask};
    const int nbk = hb[1] == hb[0] ? 1 : 2;
    for (int attempt = 0; attempt < 64; attempt++) {
        uint32_t fill[2] = {kBucketWays, kBucketWays};
        for (int b = 0; b < nbk; b++) {
            unsigned long long *bk = table + (uint64_t)hb[b] * kBucketWays;
            uint32_t i = 0;
            for (; i < kBucketWays; i++) {
                const unsigned long long x = __hip_atomic_load(&bk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (x == 0) break;
                if ((uint32_t)(x >> 32) == v) {
                    atomicOr(&bk[i], f);
                    return;
                }
            }
            fill[b] = i;
        }
        const int b = (nbk == 2 && fill[1] < fill[0]) ? 1 : 0;
        if (fill[b] >= kBucketWays) break;
        unsigned long long *slot = table + (uint64_t)hb[b] * kBucketWays + fill[b];
        const unsigned long long old = atomicCAS(slot, 0ull, e);
        if (old == 0) return;
        if ((uint32_t)(old >> 32) == v) {
            atomicOr(slot, f);
            return;
        }
        // another key took the slot: scan again
    }
    atomicOr(ovf, 1u);
}

// The packed roll's key-only copy of the table (empty slots: an existing key).
__global__ __launch_bounds__(256) void table_keys_kernel(const unsigned long long *__restrict__ table, uint32_t n,
                                                         const uint32_t *__restrict__ sum1,
                                                         uint32_t *__restrict__ keys) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const unsigned long long e = table[i];
    keys[i] = (uint32_t)e != 0 ? (uint32_t)(e >> 32) : sum1[0];
}

hipError_t launch_build_tables(const uint32_t *sum1, int32_t count, uint32_t B, uint32_t rem, bool packed,
                               uint32_t *bitmap, uint16_t *filter16, uint64_t *table, uint32_t *keys, uint32_t nb,
                               uint32_t *ovf, bool force_ovf, hipStream_t stream) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(build_tables_kernel, dim3(((uint32_t)count + 255) / 256), dim3(256), 0, stream, sum1, count, B,
                       rem, packed ? 1 : 0, bitmap,
                       reinterpret_cast<uint32_t *>(filter16), reinterpret_cast<unsigned long long *>(table), nb - 1,
                       ovf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint32_t n = nb * kBucketWays;
    hipLaunchKernelGGL(table_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, stream,
                       reinterpret_cast<const unsigned long long *>(table), n, sum1, keys);
    e = hipGetLastError();
    // force_ovf (rsg_testing_search_option): report an incomplete table
    // anyway (tests of the rolls' every-filter-hit fallback)
    if (e == hipSuccess && force_ovf) e = hipMemsetAsync(ovf, 1, 4, stream);
    return e;
}

__global__ void roll_count_out_kernel(uint32_t *__restrict__ count, uint32_t *__restrict__ host) {
    if (threadIdx.x == 0) {
        *host = *count;  // pinned host word, read by the host after the stream's event
        *count = 0;
    }
}

hipError_t launch_roll_count_out(uint32_t *count, uint32_t *host, hipStream_t stream) {
    hipLaunchKernelGGL(roll_count_out_kernel, dim3(1), dim3(64), 0, stream, count, host);
    return hipGetLastError();
}

hipError_t launch_roll(const uint8_t *src, uint64_t size, uint32_t B, uint32_t rem, uint64_t end, uint32_t tile_lo,
                       uint32_t tile_hi, const TileAgg *agg, const TilePrefix *pre, uint32_t ntiles,
                       const uint32_t *bitmap, const uint16_t *filter16, const uint64_t *table,
                       const uint32_t *table_keys, uint32_t bmask, uint64_t *cand, uint32_t cap, uint32_t *count,
                       const uint32_t *ovf, uint32_t grid, bool fused, hipStream_t stream) {
    if (tile_hi <= tile_lo) return hipSuccess;
    if (fused && filter16) {
        // Interior tiles [tile_lo, t_int): every offset of tile t visited
        // ((t+1) T <= end) and its window and shifted-byte loads inside the
        // source ((t+1) T + B + 48 <= size).  The packed kernel takes the
        // whole range and rolls the rest -- the source's last B bytes or so --
        // with its scalar edge path (one launch; a separate roll_kernel
        // launch for the edge measured the same).  A range
        // with no interior tile is roll_kernel's.
        const uint64_t lim = std::min<uint64_t>(end, size >= (uint64_t)B + 48 ? size - B - 48 : 0);
        const uint32_t t_int = (uint32_t)std::max<uint64_t>(tile_lo, std::min<uint64_t>(tile_hi, lim / kScanTile));
        if (t_int > tile_lo) {
            const uint32_t ga = min(grid, tile_hi - tile_lo);
            // B = the tile length (the reference's B for a 1 GiB file): a
            // tile's shifted bytes are carried into the next tile
            auto kern = B == kScanTile ? roll_packed_kernel<3, true, true> : roll_packed_kernel<3, true, false>;
            hipLaunchKernelGGL(kern, dim3(ga), dim3(kRollThreads), 0, stream, src, size, B, rem, end, tile_lo, t_int,
                               tile_hi, filter16, table_keys, bmask, cand, cap, count, ovf);
            return hipGetLastError();
        }
    }
    const uint32_t g = min(grid, tile_hi - tile_lo);
    hipLaunchKernelGGL(roll_kernel<true>, dim3(g), dim3(kRollThreads), 0, stream, src, size, B, rem, end, tile_lo, tile_hi, agg,
                       pre, ntiles, bitmap, table, bmask, cand, cap, count, fused ? 1u : 0u, ovf);
    return hipGetLastError();
}

}  // namespace rsg
