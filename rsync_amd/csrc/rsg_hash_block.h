// rsg_hash_block.h -- per-lane block hashing shared by the block-sum kernels
// (rsg_blocksums.hip) and the small-file sender (rsg_search_small.hip):
// Checksum1 (rsyncchecksum.go:29-51) and MD4(block || int32_LE(seed))
// (rsyncchecksum.go:53-58) of one block at any byte offset, one lane per block.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rsg_internal.h"
#include "rsg_md4.h"

namespace rsg {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// 16 message words from a 4-byte-aligned address known to lie inside the arena.
__device__ __forceinline__ void load16(const uint8_t *p, uint32_t w[16]) {
    const u32x4a4 *q = reinterpret_cast<const u32x4a4 *>(p);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        u32x4a4 v = q[j];
        w[4 * j + 0] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
}

static __device__ __noinline__ uint32_t load_word_slow(const uint8_t *p, uintptr_t end) {
    uint32_t w = 0;
    for (int i = 0; i < 4; i++)
        if ((uintptr_t)(p + i) < end) w |= (uint32_t)p[i] << (8 * i);
    return w;
}

// Same, but never touches a byte at or past `end` (reads there yield 0).  Only
// used for the chunk holding a block's tail, which may run past the arena.
__device__ __forceinline__ void load16_guarded(const uint8_t *p, uintptr_t end, uint32_t w[16]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint8_t *pj = p + 16 * j;
        if ((uintptr_t)pj + 16 <= end) {
            u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(pj);
            w[4 * j + 0] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) w[4 * j + i] = load_word_slow(pj + 4 * i, end);
        }
    }
}

__device__ __forceinline__ uint32_t load_word_guarded(const uint8_t *p, uintptr_t end) {
    if ((uintptr_t)p + 4 <= end) return *reinterpret_cast<const uint32_t *>(p);
    return load_word_slow(p, end);
}

// Hash data chunk c of a block: message words (funnel-shifted when the block
// is not 4-byte aligned; w16 is the first aligned word of the next chunk),
// then the weak-sum terms and one MD4 compression.
template <bool ALIGNED>
__device__ __forceinline__ void hash_chunk(const uint32_t W[16], uint32_t w16, uint32_t sh, uint32_t c,
                                           uint32_t h[4], int32_t &s1, uint32_t &t) {
    uint32_t X[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        X[k] = ALIGNED ? W[k] : __builtin_amdgcn_alignbyte(k < 15 ? W[k + 1] : w16, W[k], sh);
    const int32_t s1b = s1;
    int32_t tl = 0;
    weak_chunk(X, s1, tl);
    t += (uint32_t)tl + (c << 6) * (uint32_t)(s1 - s1b);
    md4_compress(h, X);
}

// Tail of a block: chunk `nfull` holds the last r = n % 64 data bytes (words W,
// plus w16 = the next aligned word when not ALIGNED), then the 4 seed bytes
// (rsyncchecksum.go:56), then RFC 1320 padding (0x80, zeros, 64-bit bit length).
// Word kd = r/4 holds the last rb = r%4 data bytes followed by seed bytes, word
// kd+1 the rest of the seed and the 0x80; everything after is zero up to the
// length words.  One or two compressions (two when r >= 52).
template <bool ALIGNED>
__device__ __forceinline__ void hash_tail(const uint32_t W[16], uint32_t w16, uint32_t sh, uint32_t n,
                                          uint32_t seed, uint32_t h[4], int32_t &s1, uint32_t &t) {
    const uint32_t nfull = n >> 6;
    const uint32_t r = n & 63u, kd = r >> 2, rb = r & 3u;
    const uint32_t mask = rb ? ((1u << (8 * rb)) - 1u) : 0u;
    const uint32_t wB = rb ? ((seed >> (32 - 8 * rb)) | (0x80u << (8 * rb))) : 0x80u;
    const uint32_t lenlo = (n + 4u) << 3, lenhi = (n + 4u) >> 29;
    const bool two = r >= 52;
    uint32_t X[16], XD[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t dk = ALIGNED ? W[k] : __builtin_amdgcn_alignbyte(k < 15 ? W[k + 1] : w16, W[k], sh);
        const uint32_t wA = rb ? ((dk & mask) | (seed << (8 * rb))) : seed;
        const uint32_t uk = (uint32_t)k;
        X[k] = uk < kd ? dk : (uk == kd ? wA : (uk == kd + 1 ? wB : 0u));
        XD[k] = uk < kd ? dk : (uk == kd ? (dk & mask) : 0u);
    }
    if (!two) { X[14] = lenlo; X[15] = lenhi; }
    {
        const int32_t s1b = s1;
        int32_t tl = 0;
        weak_chunk(XD, s1, tl);
        t += (uint32_t)tl + (nfull << 6) * (uint32_t)(s1 - s1b);
    }
    md4_compress(h, X);
    if (two) {
#pragma unroll
        for (int k = 0; k < 16; k++) X[k] = 0;
        X[0] = (kd + 1 == 16) ? wB : 0u;
        X[14] = lenlo; X[15] = lenhi;
        md4_compress(h, X);
    }
}

// One lane hashes its whole block with its own 16-byte loads (one chunk of
// prefetch).  ALIGNED: the block starts 4-byte aligned, so message words are
// plain loads; otherwise each word is funnel-shifted out of two aligned words.
template <bool ALIGNED>
__device__ __forceinline__ void hash_block_direct(const uint8_t *arena, uintptr_t end, uint64_t off, uint32_t n,
                                                  uint32_t seed, uint32_t h[4], int32_t &s1, uint32_t &t) {
    const uint8_t *p = arena + off;
    const uint32_t sh = ALIGNED ? 0u : (uint32_t)((uintptr_t)p & 3u);
    const uint8_t *p0 = p - sh;
    const uint32_t nfull = n >> 6;
    uint32_t A[16], B[16];
    // Chunks 0..nfull-1 hold only file bytes.  Chunk c+1 is loaded before chunk
    // c is hashed; every load except the one of the tail chunk stays inside the
    // block, so only that one is guarded.  Unrolled by two so the double buffer
    // needs no register copies.
    uint32_t c = 0;
    if (nfull == 0) {
        load16_guarded(p0, end, A);
    } else {
        load16(p0, A);
        for (; c + 2 < nfull; c += 2) {
            load16(p0 + 64u * (c + 1), B);
            hash_chunk<ALIGNED>(A, B[0], sh, c, h, s1, t);
            load16(p0 + 64u * (c + 2), A);
            hash_chunk<ALIGNED>(B, A[0], sh, c + 1, h, s1, t);
        }
        if (c + 1 < nfull) {
            load16(p0 + 64u * (c + 1), B);
            hash_chunk<ALIGNED>(A, B[0], sh, c, h, s1, t);
            load16_guarded(p0 + 64u * nfull, end, A);
            hash_chunk<ALIGNED>(B, A[0], sh, c + 1, h, s1, t);
        } else {
            load16_guarded(p0 + 64u * nfull, end, B);
            hash_chunk<ALIGNED>(A, B[0], sh, c, h, s1, t);
#pragma unroll
            for (int k = 0; k < 16; k++) A[k] = B[k];
        }
    }
    const uint32_t extra = ALIGNED ? 0u : load_word_guarded(p0 + 64u * nfull + 64u, end);
    hash_tail<ALIGNED>(A, extra, sh, n, seed, h, s1, t);
}

}  // namespace rsg
