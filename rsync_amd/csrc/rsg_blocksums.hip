// rsg_blocksums.hip -- receiver block-sum kernel (weak + seeded MD4) for gfx950.
//
// Replaces the per-block loop of (*receiver.Transfer).generateAndSendSums,
// internal/receiver/generator.go:332-348:
//     sum1 = Checksum1(block)            rsyncchecksum.go:29-51
//     sum2 = Checksum2(seed, block)      rsyncchecksum.go:53-58  (MD4(block || seed_LE))
//     write int32 LE sum1, then sum2[16] generator.go:341-346
// for every block of every file of a batch, one lane per block.
//
// Layout in HBM: the files of a batch sit in one byte arena (any offsets);
// output records are RSG_RECORD_BYTES = 20 bytes each, record g = global block
// g (blocks numbered file by file, in file order), so each file's records are
// contiguous and wire-ready.
//
// Memory: every byte of the arena is read once from HBM (each lane walks its
// own block front to back with 16-byte loads; neighbouring lanes' blocks are
// adjacent, so every cache line is fully consumed by at most two lanes of one
// wave); 20 bytes written per block.  Roofline: HBM read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rsg_internal.h"
#include "rsg_md4.h"

namespace rsg {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// 16 message words from a 4-byte-aligned address known to lie inside the arena.
__device__ __forceinline__ void load16(const uint8_t *p, uint32_t w[16]) {
    const u32x4a4 *q = reinterpret_cast<const u32x4a4 *>(p);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        u32x4a4 v = q[j];
        w[4 * j + 0] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
    }
}

__device__ __noinline__ uint32_t load_word_slow(const uint8_t *p, uintptr_t end) {
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

// ALIGNED: every block starts 4-byte aligned (all file offsets and block
// lengths are multiples of 4), so message words are plain loads; otherwise
// each word is funnel-shifted out of two aligned words (v_alignbyte_b32).
template <bool ALIGNED>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_kernel(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlockSumThreads + threadIdx.x;
    if (g >= total_blocks) return;

    // File of block g: the largest f in [wg_file[wg], wg_file[wg+1]] with
    // first_block <= g (zero-length files own no blocks and are skipped).
    uint32_t lo = wg_file[blockIdx.x], hi = wg_file[blockIdx.x + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
    }
    const DevFile F = files[lo];
    const uint64_t bi = g - F.first_block;
    const uint64_t boff = bi * F.blen;
    const uint64_t left = F.len - boff;
    const uint32_t n = left < F.blen ? (uint32_t)left : F.blen;  // generator.go:334

    const uint8_t *p = arena + F.offset + boff;
    const uintptr_t end = (uintptr_t)(arena + arena_bytes);
    const uint32_t sh = ALIGNED ? 0u : (uint32_t)((uintptr_t)p & 3u);
    const uint8_t *p0 = p - sh;
    const uint32_t nfull = n >> 6;

    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;  // sum x_i (wrapping, as the reference's uint32)
    uint32_t t = 0;  // sum i*x_i
    uint32_t A[16], B[16];
    // Chunks 0..nfull-1 hold only file bytes.  Chunk c+1 is loaded before chunk
    // c is hashed (one chunk of prefetch per lane); every load except the one
    // of the tail chunk stays inside the block, so only that one is guarded.
    // Unrolled by two so the double buffer needs no register copies.
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
    const uint32_t *cur = A;

    // Tail: r data bytes, then the 4 seed bytes (rsyncchecksum.go:56), then
    // RFC 1320 padding (0x80, zeros, 64-bit bit length).  Word kd holds the
    // last rb data bytes followed by seed bytes; word kd+1 the rest of the seed
    // and the 0x80; everything after is zero up to the length words.
    const uint32_t extra = ALIGNED ? 0u : load_word_guarded(p0 + 64u * nfull + 64u, end);
    const uint32_t r = n & 63u, kd = r >> 2, rb = r & 3u;
    const uint32_t mask = rb ? ((1u << (8 * rb)) - 1u) : 0u;
    const uint32_t wB = rb ? ((seed >> (32 - 8 * rb)) | (0x80u << (8 * rb))) : 0x80u;
    const uint32_t lenlo = (n + 4u) << 3, lenhi = (n + 4u) >> 29;
    const bool two = r >= 52;
    uint32_t X[16], XD[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t dk = ALIGNED ? cur[k] : __builtin_amdgcn_alignbyte(k < 15 ? cur[k + 1] : extra, cur[k], sh);
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

    const uint32_t s2 = n * (uint32_t)s1 - t;  // sum (n - i) x_i
    const uint32_t sum1 = ((uint32_t)s1 & 0xffffu) | (s2 << 16);  // rsyncchecksum.go:50
    uint32_t *o = reinterpret_cast<uint32_t *>(out + g * kRecordBytes);
    o[0] = sum1;
    o[1] = h[0]; o[2] = h[1]; o[3] = h[2]; o[4] = h[3];
}

hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t seed, uint8_t *out, hipStream_t stream) {
    if (total_blocks == 0) return hipSuccess;
    dim3 grid(nwg), block(kBlockSumThreads);
    if (aligned)
        hipLaunchKernelGGL(block_sums_kernel<true>, grid, block, 0, stream, arena, arena_bytes, files,
                           wg_file, total_blocks, seed, out);
    else
        hipLaunchKernelGGL(block_sums_kernel<false>, grid, block, 0, stream, arena, arena_bytes, files,
                           wg_file, total_blocks, seed, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ synthetic data
__global__ void fill_splitmix64_kernel(uint8_t *dst, uint64_t n, uint64_t seed) {
    const uint64_t words = (n + 7) / 8;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        uint8_t *q = dst + 8 * i;
        if (8 * i + 8 <= n && (((uintptr_t)q) & 7) == 0) {
            *reinterpret_cast<uint64_t *>(q) = z;
        } else {
            for (int b = 0; b < 8 && 8 * i + b < n; b++) q[b] = (uint8_t)(z >> (8 * b));
        }
    }
}

hipError_t launch_fill_splitmix64(uint8_t *dst, uint64_t n, uint64_t seed, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t words = (n + 7) / 8;
    uint64_t blocks = (words + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fill_splitmix64_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, dst, n, seed);
    return hipGetLastError();
}

}  // namespace rsg
