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
#include <stdlib.h>
#include <string.h>

#include <algorithm>

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

// Record g = int32 LE Checksum1 then the 16 MD4 digest bytes (generator.go:341-346).
__device__ __forceinline__ void store_record(uint8_t *out, uint64_t g, uint32_t n, int32_t s1, uint32_t t,
                                             const uint32_t h[4]) {
    const uint32_t s2 = n * (uint32_t)s1 - t;  // sum (n - i) x_i
    const uint32_t sum1 = ((uint32_t)s1 & 0xffffu) | (s2 << 16);  // rsyncchecksum.go:50
    uint32_t *o = reinterpret_cast<uint32_t *>(out + g * kRecordBytes);
    o[0] = sum1;
    o[1] = h[0]; o[2] = h[1]; o[3] = h[2]; o[4] = h[3];
}

// File of block g: the largest f in [wg_file[wg], wg_file[wg+1]] with
// first_block <= g (zero-length files own no blocks and are skipped).
// Returns the block's arena offset and length (generator.go:334).
__device__ __forceinline__ void locate_block(const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file,
                                             uint64_t g, uint64_t &off, uint32_t &n) {
    uint32_t lo = wg_file[blockIdx.x], hi = wg_file[blockIdx.x + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
    }
    const DevFile F = files[lo];
    const uint64_t bi = g - F.first_block;
    const uint64_t boff = bi * F.blen;
    const uint64_t left = F.len - boff;
    n = left < F.blen ? (uint32_t)left : F.blen;
    off = F.offset + boff;
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

// Variant "direct": one lane per block, per-lane loads.  Handles any
// alignment; the staged kernel below falls back to it for edge waves.
template <bool ALIGNED>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_direct(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlockSumThreads + threadIdx.x;
    if (g >= total_blocks) return;
    uint64_t off;
    uint32_t n;
    locate_block(files, wg_file, g, off, n);
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;  // sum x_i (wrapping, as the reference's uint32)
    uint32_t t = 0;  // sum i*x_i
    hash_block_direct<ALIGNED>(arena, (uintptr_t)(arena + arena_bytes), off, n, seed, h, s1, t);
    store_record(out, g, n, s1, t, h);
}

// ---------------------------------------------------------------- long-block variant
// Few long blocks (the sender's 32 KiB confirmation windows, 128 KiB blocks):
// there are too few lanes to hide HBM latency by occupancy, so each lane keeps
// P chunks of its own block in flight (P x 16 VGPRs; one wave per SIMD is
// plenty here).  Chunk c lives in buffer c % P; after chunk c is hashed its
// buffer is refilled with chunk c + P.
template <int P, bool ALIGNED>
__device__ __forceinline__ void hash_block_deep(const uint8_t *arena, uintptr_t end, uint64_t off, uint32_t n,
                                                uint32_t seed, uint32_t h[4], int32_t &s1, uint32_t &t) {
    const uint8_t *p = arena + off;
    const uint32_t sh = ALIGNED ? 0u : (uint32_t)((uintptr_t)p & 3u);
    const uint8_t *p0 = p - sh;
    const uint32_t nfull = n >> 6;
    // Fast path: chunks 0..nfull+1 lie inside the arena, so every load in the
    // ring is a plain unconditional load (branch-free loop: the compiler can
    // keep P - 1 chunks in flight).  Blocks ending near the arena's end take
    // the guarded single-chunk path.
    if ((uintptr_t)p0 + 64u * (uint64_t)(nfull + 2) + (ALIGNED ? 0u : 4u) > end) {
        hash_block_direct<ALIGNED>(arena, end, off, n, seed, h, s1, t);
        return;
    }
    const uint32_t last = nfull + 1;  // loads are clamped to this chunk
    // buf[u] = chunk words; nxt[u] = the next aligned word after the chunk
    // (funnel-shift input when not ALIGNED), loaded with it so that a chunk
    // never waits on a younger load.
    uint32_t buf[P][16], nxt[P];
#define RSG_FETCH(U, CHUNK)                                                        \
    do {                                                                           \
        const uint8_t *q_ = p0 + 64u * (CHUNK);                                    \
        load16(q_, buf[U]);                                                        \
        if (!ALIGNED) nxt[U] = *reinterpret_cast<const uint32_t *>(q_ + 64);       \
    } while (0)
#pragma unroll
    for (int u = 0; u < P; u++) RSG_FETCH(u, min((uint32_t)u, last));
    uint32_t c = 0;
#pragma unroll 1
    for (; c + P <= nfull; c += P) {
#pragma unroll
        for (int u = 0; u < P; u++) {
            hash_chunk<ALIGNED>(buf[u], ALIGNED ? 0u : nxt[u], sh, c + u, h, s1, t);
            RSG_FETCH(u, min(c + (uint32_t)u + P, last));
        }
    }
#undef RSG_FETCH
    // Fewer than P data chunks left: they and the tail chunk (chunk c+u sits in
    // buffer u) are already in the ring; one last predicated round, no loads.
#pragma unroll
    for (int u = 0; u < P; u++) {
        const uint32_t cc = c + (uint32_t)u;
        if (cc < nfull) hash_chunk<ALIGNED>(buf[u], ALIGNED ? 0u : nxt[u], sh, cc, h, s1, t);
        else if (cc == nfull) hash_tail<ALIGNED>(buf[u], ALIGNED ? 0u : nxt[u], sh, n, seed, h, s1, t);
    }
}

template <bool ALIGNED>
__global__ __launch_bounds__(64) void block_sums_long(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (g >= total_blocks) return;
    // wg_file is indexed per 256-lane workgroup of the plan
    uint32_t lo = wg_file[g / kBlockSumThreads], hi = wg_file[g / kBlockSumThreads + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
    }
    const DevFile F = files[lo];
    const uint64_t boff = (g - F.first_block) * F.blen;
    const uint64_t left = F.len - boff;
    const uint32_t n = left < F.blen ? (uint32_t)left : F.blen;  // generator.go:334
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    hash_block_deep<8, ALIGNED>(arena, (uintptr_t)(arena + arena_bytes), F.offset + boff, n, seed, h, s1, t);
    store_record(out, g, n, s1, t, h);
}

// ---------------------------------------------------------------- staged variant
// Coalesced HBM reads: a wave owns 64 consecutive blocks (one per lane) and
// streams them through a private LDS slab 256 bytes (4 MD4 chunks) of every
// block at a time.  The slab is filled by buffer_load_dwordx4 ... lds (LDS DMA,
// no VGPRs in flight): each DMA wave-instruction fetches 4 contiguous 256-byte
// pieces, so every cache line is consumed by one instruction instead of by 64
// scattered per-lane loads.  Piece j (lane j's block) sits at j*272 in the slab:
// the 16-byte pad makes the per-lane ds_read_b128 of one unit conflict-free
// (bank = 4*(j + unit) mod 64 inside every 16-lane group).  While the wave
// hashes segment s out of registers, segment s+1 is already in flight.
constexpr uint32_t kSegBytes = 256;
constexpr uint32_t kPiece = kSegBytes + 16;          // padded piece stride in LDS
constexpr uint32_t kWaveSlab = 64 * kPiece;          // 17408 bytes per wave
constexpr uint32_t kDmaPerSeg = kWaveSlab / 1024;    // 17 DMA instructions per segment
static_assert(kWaveSlab % 1024 == 0, "slab must be a whole number of DMA instructions");

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return v;
}

// MODE 0 = the product kernel.  Timing diagnostics (outputs meaningless):
// MODE 1 = DMA + LDS reads only (memory ceiling of this access pattern),
// MODE 2 = hashing only, no DMA (compute ceiling),
// MODE 3 = as MODE 1 with every piece rounded down to a 128-byte line,
// MODE 4 = as MODE 1 with the wave's blocks packed back to back (768 B apart).
//
// K = consecutive blocks per lane.  A line that straddles two blocks is
// needed by the end of one block and the start of the next; when both blocks
// belong to the same lane the two uses are one segment apart and the second
// is an L2 hit, whereas across lanes they are a whole block apart and the line
// is often refetched from HBM.  K = 4 cuts those refetches by 4x.
template <int K, int MODE, bool TRIM = false, int DEPTH = 1, bool A16 = false>
__device__ __forceinline__ void staged_tile(
    uint32_t tile, uint8_t *slab_all, const uint8_t *__restrict__ arena, uint64_t arena_bytes,
    const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file, uint32_t nwg256,
    uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    // readfirstlane: provably wave-uniform values keep the LDS base (M0) and
    // the buffer descriptor in SGPRs (no waterfall loops around the DMA).
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * kWaveSlab * DEPTH;
    const uint64_t wave_first = ((uint64_t)tile * (kBlockSumThreads / 64) + wave) * 64u * K;
    const uint64_t g0 = wave_first + (uint64_t)lane * K;

    // Locate the lane's K blocks: binary search for the first, then walk.
    uint64_t off[K];
    uint32_t n[K];
    {
        uint32_t lo = wg_file[tile * K];
        uint32_t hi = wg_file[min((tile + 1) * K, nwg256)];
        const uint64_t gq = g0 < total_blocks ? g0 : total_blocks - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (files[mid].first_block <= gq) lo = mid; else hi = mid - 1;
        }
        DevFile F = files[lo];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t g = g0 + k;
            if (g < total_blocks) {
                while (g >= F.first_block + F.nblocks) F = files[++lo];
                const uint64_t boff = (g - F.first_block) * F.blen;
                const uint64_t left = F.len - boff;
                n[k] = left < F.blen ? (uint32_t)left : F.blen;  // generator.go:334
                off[k] = F.offset + boff;
            } else {
                n[k] = 0;
                off[k] = 0;
            }
        }
    }

    // Wave-uniform choice of path: the staged path needs all 64*K blocks,
    // every DMA read inside the arena and the wave's span addressable by a
    // 32-bit buffer offset.  Otherwise (last partial wave, a file ending at
    // the arena's end, giant spans) the wave runs the direct path.
    uint32_t S[K];
    uint64_t lo_off = ~0ull, hi_end = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t nseg = n[k] ? ((n[k] >> 6) >> 2) + 1 : 0;  // segments through the tail chunk
        S[k] = __builtin_amdgcn_readfirstlane((uint32_t)wave_max_u64(nseg));
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (n[k]) {
            lo_off = off[k] < lo_off ? off[k] : lo_off;
            const uint64_t e = off[k] + (uint64_t)kSegBytes * S[k] + (A16 ? 16u : 0u);
            hi_end = e > hi_end ? e : hi_end;
        }
    }
    const uint64_t base_v = wave_min_u64(lo_off) & (A16 ? ~15ull : ~0ull);
    const uint64_t base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base_v >> 32)) << 32) |
                          __builtin_amdgcn_readfirstlane((uint32_t)base_v);
    const uint64_t top = wave_max_u64(hi_end);
    const bool staged = (wave_first + 64u * K - 1 < total_blocks) && top <= arena_bytes &&
                        (top - base) <= 0x7FFFFFFFull;
    if (!staged) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (n[k] == 0) continue;
            uint32_t h[4];
            md4_init(h);
            int32_t s1 = 0;
            uint32_t t = 0;
            hash_block_direct<true>(arena, (uintptr_t)(arena + arena_bytes), off[k], n[k], seed, h, s1, t);
            store_record(out, g0 + k, n[k], s1, t, h);
        }
        return;
    }

    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + (MODE == 3 ? base & ~127ull : base)), (short)0,
                                          0x7FFFFFFF, 0x00020000);
    uint32_t rel[K];
#pragma unroll
    for (int k = 0; k < K; k++) rel[k] = MODE == 3 ? (uint32_t)(off[k] - (base & ~127ull)) & ~127u
                                       : MODE == 4 ? (lane * K + k) * 768u
                                                   : (uint32_t)(off[k] - base);

    // DMA instruction i, lane t fills slab bytes [16*(64 i + t), +16): piece
    // j = (64 i + t) / 17 (lane j's block), unit u = (64 i + t) % 17.  u == 16
    // is the pad: its offset is past num_records, so the buffer range check
    // drops it without a memory request.
    uint32_t voff[kDmaPerSeg];
    auto build_voff = [&](uint32_t kb) {
        uint32_t r = rel[0];
#pragma unroll
        for (int k = 1; k < K; k++) r = (kb == (uint32_t)k) ? rel[k] : r;
#pragma unroll
        for (uint32_t i = 0; i < kDmaPerSeg; i++) {
            const uint32_t idx = 64u * i + lane;
            const uint32_t j = idx / 17u, u = idx - 17u * j;
            const uint32_t v = __shfl(A16 ? (r & ~15u) : r, (int)j, 64) + 16u * u;
            // pad slot: out of range, no memory request.  A16: pieces start
            // on the 16-byte unit below the block's bytes, so every DMA lane
            // is one aligned 16-byte request, and the 17th unit is data.
            voff[i] = (A16 || u < 16u) ? v : 0x80000000u;
        }
    };
    // TRIM: the last segment of a block is cut at the block's end (16-byte
    // units at or past n_j are dropped like the pad).  Without the cut, lane
    // j's last piece runs up to 68 bytes into block j+1, whose first line was
    // fetched by lane j+1 a whole block earlier and is usually gone from L2.
    auto trim_voff = [&](uint32_t kb, uint32_t s) {
        uint32_t nn = n[0];
#pragma unroll
        for (int k = 1; k < K; k++) nn = (kb == (uint32_t)k) ? n[k] : nn;
#pragma unroll
        for (uint32_t i = 0; i < kDmaPerSeg; i++) {
            const uint32_t idx = 64u * i + lane;
            const uint32_t j = idx / 17u, u = idx - 17u * j;
            const uint32_t nj = (uint32_t)__shfl((int)nn, (int)j, 64);
            voff[i] = (16u * u + kSegBytes * s < nj) ? voff[i] : 0x80000000u;
        }
    };
    auto dma_segment = [&](uint32_t s) {
#pragma unroll
        for (uint32_t i = 0; i < kDmaPerSeg; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsrc, (__attribute__((address_space(3))) void *)(slab + 1024u * i), 16, voff[i], kSegBytes * s, 0, 0);
    };
    uint32_t R[64];
    if constexpr (DEPTH == 2) {
        // Two slabs per wave: while segment s is hashed, segments s+1 and s+2
        // are both in flight (the single-slab schedule below keeps only s+1
        // in flight, so a wave's queue runs dry while it hashes).  K == 1.
        static_assert(K == 1 && MODE == 0 && !TRIM, "depth-2 schedule: K = 1 product kernel only");
        static_assert(kDmaPerSeg == 17, "the vmcnt immediate below is kDmaPerSeg");
        const uint32_t S0 = S[0], nk = n[0], nfull = nk >> 6;
        build_voff(0);
        auto dma_into = [&](uint32_t s, uint8_t *dst) {
#pragma unroll
            for (uint32_t i = 0; i < kDmaPerSeg; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * i), 16, voff[i], kSegBytes * s, 0, 0);
        };
        dma_into(0, slab);
        if (S0 > 1) dma_into(1, slab + kWaveSlab);
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
#pragma unroll 1
        for (uint32_t cs = 0; cs < S0; cs++) {
            uint8_t *buf = slab + (cs & 1u) * kWaveSlab;
            if (cs + 1 < S0) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");  // segment cs landed, cs+1 may fly
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint8_t *mine2 = buf + lane * kPiece;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine2 + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab read out before it is refilled
            if (cs + 2 < S0) dma_into(cs + 2, buf);
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t c = 4u * cs + i;
                if (c < nfull) hash_chunk<true>(R + 16 * i, 0u, 0u, c, h, s1, t);
                else if (c == nfull) hash_tail<true>(R + 16 * i, 0u, 0u, nk, seed, h, s1, t);
            }
        }
        store_record(out, g0, nk, s1, t, h);
        return;
    }
    const uint8_t *mine = slab + lane * kPiece + (A16 ? (rel[0] & 15u) : 0u);
    auto read_segment = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (A16) {
            static_assert(K == 1, "A16: one block per lane");
            const uint32_t *w = reinterpret_cast<const uint32_t *>(mine);
#pragma unroll
            for (int q = 0; q < 64; q++) R[q] = w[q];
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };

    // Flattened schedule over (block k, segment s); the DMA cursor runs one
    // step ahead of the compute cursor.
    uint32_t dk = 0, ds = 0;
    auto next_cursor = [&](uint32_t &k, uint32_t &s) {
        uint32_t sk = S[0];
#pragma unroll
        for (int q = 1; q < K; q++) sk = (k == (uint32_t)q) ? S[q] : sk;
        if (++s >= sk) { s = 0; k++; }
    };
    build_voff(0);
    if (TRIM && S[0] == 1) trim_voff(0, 0);
    if (MODE != 2) dma_segment(0);
    next_cursor(dk, ds);
    read_segment();
#pragma unroll 1
    for (uint32_t ck = 0; ck < (uint32_t)K; ck++) {
        uint32_t nk = n[0];
        uint32_t sk = S[0];
#pragma unroll
        for (int q = 1; q < K; q++) {
            nk = (ck == (uint32_t)q) ? n[q] : nk;
            sk = (ck == (uint32_t)q) ? S[q] : sk;
        }
        const uint32_t nfull = nk >> 6;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
#pragma unroll 1
        for (uint32_t cs = 0; cs < sk; cs++) {
            const bool more = dk < (uint32_t)K;
            if (more) {
                if (ds == 0) build_voff(dk);
                if (TRIM) {
                    uint32_t sk2 = S[0];
#pragma unroll
                    for (int q = 1; q < K; q++) sk2 = (dk == (uint32_t)q) ? S[q] : sk2;
                    if (ds + 1 == sk2) trim_voff(dk, ds);
                }
                if (MODE != 2) dma_segment(ds);
                next_cursor(dk, ds);
            }
            if (MODE == 1 || MODE == 3 || MODE == 4) {
#pragma unroll
                for (int q = 0; q < 64; q++) h[q & 3] ^= R[q];
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    const uint32_t c = 4u * cs + i;
                    if (c < nfull) hash_chunk<true>(R + 16 * i, 0u, 0u, c, h, s1, t);
                    else if (c == nfull) hash_tail<true>(R + 16 * i, 0u, 0u, nk, seed, h, s1, t);
                }
            }
            if (more) read_segment();
        }
        store_record(out, g0 + ck, nk, s1, t, h);
    }
}


template <int K, int MODE, bool TRIM = false>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab];
    staged_tile<K, MODE, TRIM>(blockIdx.x, slab_all, arena, arena_bytes, files, wg_file, nwg256, total_blocks, seed, out);
}

// ---------------------------------------------------------------- chunk-ring variant
// Occupancy first.  The staged kernel above holds 4 chunks of every lane's
// block in VGPRs (R[64]) and a 17 KiB slab per wave, so it runs at 2 waves per
// SIMD -- and MD4's serial chain then leaves the VALU idle most of the time
// (hashing alone: ~4.9 cycles per wave-instruction per SIMD against a 2-cycle
// issue rate).  Here a lane keeps only the chunk it is hashing in VGPRs; the
// wave's LDS is a ring of R slots, slot = SEGC 64-byte chunks of each of the
// 64 blocks (4 KiB per chunk), filled by LDS DMA R segments ahead.  Small
// slots buy waves: R = 1, SEGC = 1 is 4 KiB per wave.
//
// Slot layout: lane j's piece at j * 64 * SEGC, its 16-byte quads rotated by
// f(j) (quad q of the block's segment sits at position (q + f(j)) % Q) so the
// per-lane ds_read_b128 of one quad is conflict-free in every 16-lane group.
// The rotation is applied on the DMA side: the DMA lane writing position p of
// lane j's piece fetches quad (p - f(j)) % Q of the block.
template <int SEGC>
struct CRing {
    static constexpr uint32_t kQ = 4 * SEGC;                 // quads per lane piece
    static constexpr uint32_t kPieceB = 64 * SEGC;           // bytes per lane piece
    static constexpr uint32_t kSlotB = 64 * kPieceB;         // bytes per slot (64 lanes)
    static constexpr uint32_t kDma = kSlotB / 1024;          // DMA instructions per slot
    static constexpr uint32_t kShift = SEGC == 1 ? 2 : SEGC == 2 ? 1 : 0;  // f(j) = (j >> kShift) % kQ
    __device__ static uint32_t rot(uint32_t j) { return (j >> kShift) & (kQ - 1); }
};

// Segment S_ of the wave's 64 blocks into ring slot S_ % R (C::kDma LDS-DMA
// instructions; the segment advance rides in the scalar offset).  Every
// builtin argument is of a non-dependent type: hipcc 7.2's host pass silently
// drops the kernel stub of a template whose builtin call has a
// type-dependent argument (e.g. C::kPieceB * s).
#define RSG_CRING_DMA(S_)                                                                                   \
    do {                                                                                                    \
        uint8_t *slot_ = ring + ((S_) % R) * C::kSlotB;                                                     \
        const uint32_t so_ = (uint32_t)(C::kPieceB * (S_));                                                 \
        _Pragma("unroll") for (uint32_t i_ = 0; i_ < C::kDma; i_++)                                         \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                       \
                rsrc, (__attribute__((address_space(3))) void *)(slot_ + 1024u * i_), 16, (uint32_t)voff[i_], so_, 0, 0); \
    } while (0)

// MODE 0 = product; timing diagnostics (outputs meaningless): 1 = DMA + LDS
// reads only, 2 = hashing only (no DMA).  WPS = waves per SIMD the launch
// bound asks for (the LDS of the ring must allow as many workgroups).
template <int R, int SEGC, int MODE, int WPS>
__global__ __launch_bounds__(kBlockSumThreads, WPS) void block_sums_cring(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    using C = CRing<SEGC>;
    constexpr uint32_t kWaveB = R * C::kSlotB;
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[(kBlockSumThreads / 64) * kWaveB];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *ring = ring_all + wave * kWaveB;
    const uint64_t wave_first = (uint64_t)blockIdx.x * kBlockSumThreads + wave * 64u;
    const uint64_t g = wave_first + lane;

    uint64_t off = 0;
    uint32_t n = 0;
    if (g < total_blocks) locate_block(files, wg_file, g, off, n);
    (void)nwg256;
    const uint32_t nfull = n >> 6;
    // segments through the tail chunk (chunk nfull holds the last n % 64 bytes)
    const uint32_t nseg = n ? (nfull + SEGC) / SEGC : 0;
    const uint32_t S = __builtin_amdgcn_readfirstlane((uint32_t)wave_max_u64(nseg));
    const uint64_t lo_v = wave_min_u64(n ? off : ~0ull);
    const uint64_t base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo_v >> 32)) << 32) |
                          __builtin_amdgcn_readfirstlane((uint32_t)lo_v);
    const uint64_t top = wave_max_u64(n ? off + (uint64_t)C::kPieceB * nseg : 0);
    if (S == 0) return;
    // Every DMA'd byte must lie inside the arena and the span must fit a 31-bit
    // buffer offset; otherwise (the wave at the arena's end, giant spans) the
    // lanes hash their blocks with per-lane loads.
    if (!(top <= arena_bytes && top - base <= 0x7FFFFFFFull)) {
        // one chunk at a time (few VGPRs: this path must not raise the
        // kernel's register budget); only the tail chunk's load is guarded
        if (n == 0) return;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
        const uint8_t *p = arena + off;
        const uintptr_t end = (uintptr_t)(arena + arena_bytes);
        uint32_t X[16];
#pragma unroll 1
        for (uint32_t c = 0; c < nfull; c++) {
            load16(p + 64u * c, X);
            hash_chunk<true>(X, 0u, 0u, c, h, s1, t);
        }
        load16_guarded(p + 64u * nfull, end, X);
        hash_tail<true>(X, 0u, 0u, n, seed, h, s1, t);
        store_record(out, g, n, s1, t, h);
        return;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
    // idle lanes (past the batch) alias the wave's first block: valid addresses
    const uint32_t rel = n ? (uint32_t)(off - base) : 0u;

    // DMA instruction i, lane l fills slot bytes [1024 i + 16 l, +16): lane
    // j's piece, position p -> the block's quad (p - f(j)) % Q.
    uint32_t voff[C::kDma];
#pragma unroll
    for (uint32_t i = 0; i < C::kDma; i++) {
        const uint32_t pos = 1024u * i + 16u * lane;
        const uint32_t j = pos / C::kPieceB;
        const uint32_t p = (pos % C::kPieceB) / 16u;
        const uint32_t q = (p - C::rot(j)) & (C::kQ - 1);
        voff[i] = (uint32_t)__shfl((int)rel, (int)j, 64) + 16u * q;
    }
    const uint32_t rj = C::rot(lane);
    const uint8_t *mine = ring + lane * C::kPieceB;

    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    if (MODE != 2) {
#pragma unroll
        for (uint32_t s = 0; s < (uint32_t)R; s++)
            if (s < S) RSG_CRING_DMA(s);
    }
#pragma unroll 1
    for (uint32_t s = 0; s < S; s++) {
        if (MODE != 2) {
            // segment s has landed once at most the younger in-flight ones remain
            if (s + R <= S) {
                if constexpr (R == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::kDma) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C::kDma) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        const uint8_t *slot = mine + (s % R) * C::kSlotB;
        uint32_t X[16 * SEGC];
#pragma unroll
        for (uint32_t q = 0; q < C::kQ; q++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(slot + 16u * ((q + rj) & (C::kQ - 1)));
            X[4 * q + 0] = v.x; X[4 * q + 1] = v.y; X[4 * q + 2] = v.z; X[4 * q + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read out: it may be refilled
        if (MODE != 2 && s + R < S) RSG_CRING_DMA(s + R);
        if (MODE == 1) {
#pragma unroll
            for (int q = 0; q < 16 * SEGC; q++) h[q & 3] ^= X[q];
        } else {
#pragma unroll
            for (uint32_t cc = 0; cc < (uint32_t)SEGC; cc++) {
                const uint32_t c = SEGC * s + cc;
                if (c < nfull) hash_chunk<true>(X + 16 * cc, 0u, 0u, c, h, s1, t);
                else if (c == nfull) hash_tail<true>(X + 16 * cc, 0u, 0u, n, seed, h, s1, t);
            }
        }
    }
    if (n) store_record(out, g, n, s1, t, h);
}
#undef RSG_CRING_DMA

// Variant 21: depth 2 at the single-slab LDS budget.  Segments are 128 bytes
// (2 MD4 chunks) of every block, two of them per wave in flight in two
// 64 x 144-byte slabs (18 KiB per wave, as the 256-byte single slab), so the
// workgroup keeps two waves per SIMD while the queue never runs dry.
constexpr uint32_t kHSeg = 128;
constexpr uint32_t kHPiece = kHSeg + 16;
constexpr uint32_t kHSlab = 64 * kHPiece;     // 9216 bytes
constexpr uint32_t kHDma = kHSlab / 1024;     // 9 DMA instructions per segment
static_assert(kHSlab % 1024 == 0 && kHDma == 9, "vmcnt immediate below is kHDma");

__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged_half(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kHSlab * 2];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * kHSlab * 2;
    const uint64_t g = ((uint64_t)blockIdx.x * (kBlockSumThreads / 64) + wave) * 64u + lane;
    uint64_t off = 0;
    uint32_t n = 0;
    {
        uint32_t lo = wg_file[blockIdx.x], hi = wg_file[min(blockIdx.x + 1, nwg256)];
        const uint64_t gq = g < total_blocks ? g : total_blocks - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (files[mid].first_block <= gq) lo = mid; else hi = mid - 1;
        }
        const DevFile F = files[lo];
        if (g < total_blocks) {
            const uint64_t boff = (g - F.first_block) * F.blen;
            const uint64_t left = F.len - boff;
            n = left < F.blen ? (uint32_t)left : F.blen;  // generator.go:334
            off = F.offset + boff;
        }
    }
    const uint32_t S = __builtin_amdgcn_readfirstlane((uint32_t)wave_max_u64(n ? (n >> 7) + 1 : 0));
    const uint64_t base_v = wave_min_u64(n ? off : ~0ull);
    const uint64_t base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base_v >> 32)) << 32) |
                          __builtin_amdgcn_readfirstlane((uint32_t)base_v);
    const uint64_t top = wave_max_u64(n ? off + (uint64_t)kHSeg * S : 0);
    const uint64_t wave_first = g - lane;
    const bool staged = (wave_first + 63 < total_blocks) && top <= arena_bytes && (top - base) <= 0x7FFFFFFFull;
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    if (!staged) {
        if (n) {
            hash_block_direct<true>(arena, (uintptr_t)(arena + arena_bytes), off, n, seed, h, s1, t);
            store_record(out, g, n, s1, t, h);
        }
        return;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t rel = (uint32_t)(off - base);
    uint32_t voff[kHDma];
#pragma unroll
    for (uint32_t i = 0; i < kHDma; i++) {
        const uint32_t idx = 64u * i + lane;
        const uint32_t j = idx / 9u, u = idx - 9u * j;
        const uint32_t v = __shfl(rel, (int)j, 64) + 16u * u;
        voff[i] = u < 8u ? v : 0x80000000u;  // pad slot: out of range, no memory request
    }
    auto dma_into = [&](uint32_t s, uint8_t *dst) {
#pragma unroll
        for (uint32_t i = 0; i < kHDma; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * i), 16, voff[i], kHSeg * s, 0, 0);
    };
    dma_into(0, slab);
    if (S > 1) dma_into(1, slab + kHSlab);
    const uint32_t nfull = n >> 6;
    uint32_t R[32];
#pragma unroll 1
    for (uint32_t cs = 0; cs < S; cs++) {
        uint8_t *buf = slab + (cs & 1u) * kHSlab;
        if (cs + 1 < S) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // segment cs landed, cs+1 may fly
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint8_t *mine = buf + lane * kHPiece;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
            R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab read out before it is refilled
        if (cs + 2 < S) dma_into(cs + 2, buf);
#pragma unroll
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t c = 2u * cs + i;
            if (c < nfull) hash_chunk<true>(R + 16 * i, 0u, 0u, c, h, s1, t);
            else if (c == nfull) hash_tail<true>(R + 16 * i, 0u, 0u, n, seed, h, s1, t);
        }
    }
    if (n) store_record(out, g, n, s1, t, h);
}

// Variant 22 (timing diagnostic, outputs meaningless): the memory pattern of
// a whole-block tile.  A one-wave workgroup DMAs its 64 blocks (B <= 704) in a
// single pass into a 64 x 720-byte LDS tile -- every byte of the wave's span
// is requested in one burst of 45 instructions -- then folds the tile.  Asks
// whether reading a span in one pass restores the linear read's DRAM
// efficiency that the three-pass staged pattern loses.
constexpr uint32_t kTPiece = 720;
constexpr uint32_t kTDma = 64 * kTPiece / 1024;  // 45
static_assert(64 * kTPiece % 1024 == 0, "tile must be whole DMA instructions");

__global__ __launch_bounds__(64) void block_sums_diag_tile(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[64 * kTPiece];
    const uint32_t lane = threadIdx.x;
    const uint64_t g = (uint64_t)blockIdx.x * 64u + lane;
    const uint32_t wg256 = (uint32_t)(g / 256u);
    uint64_t off = 0;
    uint32_t n = 0;
    {
        uint32_t lo = wg_file[wg256], hi = wg_file[min(wg256 + 1, nwg256)];
        const uint64_t gq = g < total_blocks ? g : total_blocks - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (files[mid].first_block <= gq) lo = mid; else hi = mid - 1;
        }
        const DevFile F = files[lo];
        if (g < total_blocks) {
            const uint64_t boff = (g - F.first_block) * F.blen;
            const uint64_t left = F.len - boff;
            n = left < F.blen ? (uint32_t)left : F.blen;
            off = F.offset + boff;
        }
    }
    const uint64_t base_v = wave_min_u64(n ? off : ~0ull);
    const uint64_t base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base_v >> 32)) << 32) |
                          __builtin_amdgcn_readfirstlane((uint32_t)base_v);
    const uint64_t top = wave_max_u64(n ? off + 704u : 0);
    if (!(g - lane + 63 < total_blocks && top <= arena_bytes && n <= 704u)) return;  // diagnostic: skip edge waves
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t rel = (uint32_t)(off - base);
#pragma unroll 5
    for (uint32_t i = 0; i < kTDma; i++) {
        const uint32_t idx = 64u * i + lane;
        const uint32_t j = idx / 45u, u = idx - 45u * j;
        const uint32_t v = __shfl(rel, (int)j, 64) + 16u * u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(tile + 1024u * i), 16,
                                                 u < 44u ? v : 0x80000000u, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t h[4] = {0, 0, 0, 0};
    const uint8_t *mine = tile + lane * kTPiece;
#pragma unroll
    for (int q = 0; q < 44; q++) {
        const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
        h[0] ^= v.x; h[1] ^= v.y; h[2] ^= v.z; h[3] ^= v.w;
    }
    store_record(out, g, n, (int32_t)seed, 0u, h);
}

// Variant 23: the staged kernel with 16-byte aligned DMA units (A16).
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged_a16(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab];
    staged_tile<1, 0, false, 1, true>(blockIdx.x, slab_all, arena, arena_bytes, files, wg_file, nwg256, total_blocks,
                                      seed, out);
}

// Variant 20: the depth-2 schedule (two slabs per wave, 136 KiB of LDS per
// 4-wave workgroup, so one workgroup = one wave per SIMD per CU).
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged2(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab * 2];
    staged_tile<1, 0, false, 2>(blockIdx.x, slab_all, arena, arena_bytes, files, wg_file, nwg256, total_blocks, seed, out);
}

// ---------------------------------------------------------------- line-ring layout
// A line step of a wave in LDS: 64 lanes x (128-byte line + 16-byte pad); the
// pad spreads the lanes' realigned reads over the banks.
constexpr uint32_t kRingLane = 144;                    // 128-byte line + 16-byte pad
constexpr uint32_t kRingSlot = 64 * kRingLane;         // 9216 B: one line step of the wave

// ---------------------------------------------------------------- loaded-line-ring variant
// Same line stream as the ring above (every line requested once, whole
// aligned lines), but the lines travel HBM -> VGPRs with plain coalesced
// buffer loads (each wave instruction = 8 lanes' line t = 8 whole lines, the
// linear-read pattern), so the bytes in flight sit in the register file, not
// in LDS.  Each lane then writes its 16-byte piece into a 2-slot LDS ring
// (slot = one line step of the wave's 64 blocks) and reads back its own
// block's 32 words for the step, realigned by d_j, exactly as in the DMA ring.
// LDS: 2 x 9 KiB per wave, so two waves per SIMD; two line steps (16 KiB per
// wave) are in flight while a step hashes.
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
constexpr uint32_t kLrSlots = 2;
constexpr uint32_t kLrWave = kLrSlots * kRingSlot;   // 18432 B per wave
constexpr uint32_t kLrLoads = 8;                     // load instructions per line step

// 0 = product; timing diagnostics (outputs meaningless): 1 = loads + LDS round trip, 2 = loads only
// SHARE: block j's last line is usually block j+1's first line (blocks are
// contiguous and rarely end on a line boundary).  Without sharing, lane j+1
// fetches it at step 0 and lane j again ~6 steps later, long evicted from L2:
// ~1 extra line per block (6.5 instead of 5.5 for 700-byte blocks).  With
// SHARE, lane j copies that line out of lane j+1's slot right after step 0's
// store into 32 VGPRs and writes it into its own slot when its stream reaches
// it, so the line is requested once.
template <int MODE, bool SHARE = false>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_lring(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    // 128-byte guard in front: line-(i+1) bases are formed 128 bytes below a slot.
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[128 + (kBlockSumThreads / 64) * kLrWave];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave_first = (uint64_t)blockIdx.x * kBlockSumThreads + wave * 64u;
    const uint64_t g = wave_first + lane;
    uint64_t off = 0;
    uint32_t n = 0;
    locate_block(files, wg_file, g < total_blocks ? g : total_blocks - 1, off, n);

    const uintptr_t abs = (uintptr_t)(arena + off);
    const uint64_t lo = wave_min_u64(abs);
    const uint64_t hi = wave_max_u64(abs + n);
    const uint64_t base = (((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo >> 32)) << 32) |
                           __builtin_amdgcn_readfirstlane((uint32_t)lo)) & ~127ull;
    if (!(wave_first + 63 < total_blocks) || hi - base > 0x7FFFFF00ull) {
        if (g >= total_blocks) return;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
        hash_block_direct<true>(arena, (uintptr_t)(arena + arena_bytes), off, n, seed, h, s1, t);
        store_record(out, g, n, s1, t, h);
        return;
    }
    const uint64_t avail = (uint64_t)(uintptr_t)(arena + arena_bytes) - base;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)base, (short)0, (int)(avail < 0x7FFFFFFFull ? avail : 0x7FFFFFFFull), 0x00020000);
    const uint32_t rel = (uint32_t)(abs - base);
    const uint32_t d = rel & 127u;
    const uint32_t nl = (d + n + 127u) >> 7;
    const uint32_t l0 = rel >> 7;  // first line, relative to base
    const uint32_t next_l0 = __shfl(l0, (int)((lane + 1) & 63u), 64);
    const bool share0 = SHARE && lane < 63u && next_l0 == l0 + nl - 1u;
    // lane j+1 must load its first line itself (not when that line is also
    // its last and shared onward: a one-line block between two neighbours)
    const uint32_t next_self = __shfl((uint32_t)(!share0 || nl > 1u), (int)((lane + 1) & 63u), 64);
    const bool share = share0 && next_self;
    const uint32_t nl_load = nl - (share ? 1u : 0u);  // lines this lane's stream loads itself
    const uint32_t nfull = n >> 6;
    const uint32_t steps = (nfull + 2u) >> 1;
    const uint32_t T = __builtin_amdgcn_readfirstlane((uint32_t)wave_max_u64(steps));

    // Load instruction q, lane t: block j = 8 q + t / 8, bytes 16 (t % 8) of
    // its line; written to slot offset j * 144 + 16 (t % 8).
    uint32_t voff[kLrLoads], vnl[kLrLoads], wpos[kLrLoads];
#pragma unroll
    for (uint32_t q = 0; q < kLrLoads; q++) {
        const uint32_t j = 8u * q + (lane >> 3), u = lane & 7u;
        voff[q] = __shfl(rel & ~127u, (int)j, 64) + 16u * u;
        vnl[q] = __shfl(nl_load, (int)j, 64);
        wpos[q] = j * kRingLane + 16u * u;
    }
    uint8_t *ring = ring_all + 128 + wave * kLrWave;
    auto load_line = [&](uint32_t t, u32x4v buf[kLrLoads]) {
        // Unconditional (lines past a lane's block are out-of-range loads, no
        // memory request): a skipped load would make the compiler's vmcnt
        // bookkeeping wait for every outstanding line at the next write.
#pragma unroll
        for (uint32_t q = 0; q < kLrLoads; q++)
            buf[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, t < vnl[q] ? voff[q] : 0x80000000u, 128u * t, 0);
    };
    auto store_line = [&](uint32_t slot, const u32x4v buf[kLrLoads]) {
#pragma unroll
        for (uint32_t q = 0; q < kLrLoads; q++)
            *reinterpret_cast<u32x4v *>(ring + slot * kRingSlot + wpos[q]) = buf[q];
    };
    u32x4v tail[SHARE ? 8 : 1];
    auto fetch_tail = [&]() {  // lane j+1's first line, now in slot 0
        if (SHARE) {
#pragma unroll
            for (uint32_t u = 0; u < 8; u++)
                tail[u] = *reinterpret_cast<const u32x4v *>(ring + (lane + 1u) * kRingLane + 16u * u);
        }
    };
    auto put_tail = [&](uint32_t t, uint32_t slot) {  // line t just stored into slot
        if (SHARE && share && t == nl - 1u) {
#pragma unroll
            for (uint32_t u = 0; u < 8; u++)
                *reinterpret_cast<u32x4v *>(ring + slot * kRingSlot + lane * kRingLane + 16u * u) = tail[u];
        }
    };
    const uint8_t *mine = ring + lane * kRingLane + d;
    const uint32_t split = (128u - d) >> 2;  // words 0..split-1 from line i, the rest from line i+1

    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t tw = 0;
    auto step = [&](uint32_t i, uint32_t sa) {  // chunks 2i, 2i+1; line i in slot sa
        // SHARE makes the slot index opaque: the 64 per-word addresses are
        // recomputed each step (one select per word) instead of being held in
        // 64 VGPRs, which the tail line needs
        uint32_t so = sa;
        if (SHARE) asm volatile("" : "+s"(so));
        const uint8_t *pA = mine + so * kRingSlot;
        const uint8_t *pB = mine + (so ^ 1u) * kRingSlot - 128;
        uint32_t X[32];
#pragma unroll
        for (uint32_t k = 0; k < 32; k++)
            X[k] = *reinterpret_cast<const uint32_t *>((k < split ? pA : pB) + 4 * k);
        return [=, &h, &s1, &tw]() mutable {
            if (MODE == 1) {
#pragma unroll
                for (int k = 0; k < 32; k++) h[k & 3] ^= X[k];
            } else {
#pragma unroll
                for (uint32_t c2 = 0; c2 < 2; c2++) {
                    const uint32_t c = 2u * i + c2;
                    if (c < nfull) hash_chunk<true>(X + 16 * c2, 0u, 0u, c, h, s1, tw);
                    else if (c == nfull) hash_tail<true>(X + 16 * c2, 0u, 0u, n, seed, h, s1, tw);
                }
            }
        };
    };
    // Two line steps in flight in VGPR buffers; buffer (t % 2) carries line t.
    u32x4v buf[2][kLrLoads];
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
        for (uint32_t q = 0; q < kLrLoads; q++) buf[b][q] = (u32x4v){0u, 0u, 0u, 0u};
    load_line(0, buf[0]);
    load_line(1, buf[1]);
    store_line(0, buf[0]);
    fetch_tail();
    put_tail(0, 0);
    store_line(1, buf[1]);
    put_tail(1, 1);
    // The scheduler must not interleave these groups: the loop relies on the
    // loads of line 2 being older than those of line 3 (vmcnt is in order).
    load_line(2, buf[0]);
    __builtin_amdgcn_sched_barrier(0);
    load_line(3, buf[1]);
    __builtin_amdgcn_sched_barrier(0);
    // Two steps per trip (slots and buffers alternate); an odd T runs one
    // extra step whose chunks are past every block (it hashes nothing).
#pragma unroll 1
    for (uint32_t i0 = 0; i0 < T; i0 += 2) {
#pragma unroll
        for (uint32_t st = 0; st < 2; st++) {
            const uint32_t i = i0 + st;
            auto hash = step(i, st);      // lines i (slot st), i+1 (the other slot)
            store_line(st, buf[st]);      // line i+2 -> slot st
            put_tail(i + 2, st);
            load_line(i + 4, buf[st]);
            hash();
        }
    }
    store_record(out, g, n, s1, tw, h);
}

// ---------------------------------------------------------------- register-block variant
// For blocks of at most kRegMaxBytes (the reference's default 700-byte blocks,
// SumSizesSqroot for every file up to 490 000 bytes): each lane loads its whole
// block into VGPRs with back-to-back 16-byte loads, so a wave requests its
// entire 44.8 KB tile in one burst (every shared cache line is requested by
// neighbouring lanes of the same burst, and DRAM rows are opened once), then
// hashes from registers.  Two waves per SIMD alternate load and hash phases.
constexpr uint32_t kRegChunks = 11;                  // data chunks held per lane
constexpr uint32_t kRegMaxBytes = 64 * kRegChunks - 1;  // 703: tail chunk index <= 10

template <int MODE>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_regblock(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlockSumThreads + threadIdx.x;
    if (g >= total_blocks) return;
    uint64_t off;
    uint32_t n;
    locate_block(files, wg_file, g, off, n);
    const uint8_t *p = arena + off;
    const uintptr_t end = (uintptr_t)(arena + arena_bytes);
    const uint32_t nvec = (n + 15) >> 4;  // 16-byte loads covering the block
    uint32_t R[16 * kRegChunks];
    if ((uintptr_t)p + 16u * nvec <= end) {
#pragma unroll
        for (uint32_t j = 0; j < 4 * kRegChunks; j++) {
            if (j < nvec) {
                const u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(p + 16 * j);
                R[4 * j + 0] = v.x; R[4 * j + 1] = v.y; R[4 * j + 2] = v.z; R[4 * j + 3] = v.w;
            } else {
                R[4 * j + 0] = R[4 * j + 1] = R[4 * j + 2] = R[4 * j + 3] = 0;
            }
        }
    } else {  // the block's last vector would cross the arena end
#pragma unroll
        for (uint32_t j = 0; j < 4 * kRegChunks; j++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                R[4 * j + q] = j < nvec ? load_word_guarded(p + 16 * j + 4 * q, end) : 0u;
    }
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    const uint32_t nfull = n >> 6;
    if (MODE == 1) {
#pragma unroll
        for (int q = 0; q < 16 * (int)kRegChunks; q++) h[q & 3] ^= R[q];
    } else {
#pragma unroll
        for (uint32_t c = 0; c < kRegChunks; c++) {
            if (c < nfull) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, t);
            else if (c == nfull) hash_tail<true>(R + 16 * c, 0u, 0u, n, seed, h, s1, t);
        }
    }
    store_record(out, g, n, s1, t, h);
}

// ---------------------------------------------------------------- read ceilings
// Timing diagnostics only: the fastest way to read the same arena with no
// hashing, i.e. the empirical HBM-read roofline of this box for DESIGN.md.
// LDS = false: coalesced global_load_dwordx4, 4 in flight per lane;
// LDS = true: the same bytes through buffer_load_dwordx4 ... lds.
template <bool LDS>
__global__ __launch_bounds__(256) void diag_linear_read(const uint8_t *__restrict__ arena, uint64_t bytes,
                                                        uint32_t *__restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4 * 4096];
    const uint64_t per_iter = (uint64_t)gridDim.x * 256 * 64;  // 4 x 16 B per lane
    uint32_t acc = 0;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * 64; base + 256 * 64 <= bytes; base += per_iter) {
        if (LDS) {
            const uint64_t wb = base + wave * 4096;
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(arena + ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wb >> 32)) << 32 |
                                  __builtin_amdgcn_readfirstlane((uint32_t)wb))),
                (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
            for (int i = 0; i < 4; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    r, (__attribute__((address_space(3))) void *)(buf + wave * 4096 + 1024 * i), 16,
                    (threadIdx.x & 63) * 16, 1024 * i, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= *reinterpret_cast<const uint32_t *>(buf + wave * 4096 + (threadIdx.x & 63) * 4);
        } else {
            const u32x4a4 *q = reinterpret_cast<const u32x4a4 *>(arena + base + threadIdx.x * 16);
            u32x4a4 v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = q[256 * i];
#pragma unroll
            for (int i = 0; i < 4; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keep the loads alive
}

// ---------------------------------------------------------------- register-tile variant
// For blocks of at most kRegMaxBytes (the reference's default 700-byte blocks):
// a wave's 64 consecutive blocks are fetched as ONE near-linear stream of
// 1 KiB LDS-DMA instructions (block j lands at j*720 in an LDS tile, so each
// instruction covers ~1.4 contiguous blocks: full cache lines, DRAM rows read
// once), then every lane copies its block into VGPRs with 16-byte-aligned
// ds_read_b128 (stride 720 B = 180 dwords: conflict-free) and hashes it from
// registers.  A persistent 8-wave workgroup per CU shares kRtBufs LDS tiles:
// the waves of one tile buffer take turns in a fixed order (an LDS ticket),
// so while some waves hash, others keep the HBM stream busy.
constexpr uint32_t kRtPiece = 720;                 // LDS bytes per block (45 x 16 B)
constexpr uint32_t kRtTile = 64 * kRtPiece;        // 46080 B per wave tile
constexpr uint32_t kRtDma = kRtTile / 1024;        // 45 DMA instructions per tile
constexpr uint32_t kRtBufs = 3;
constexpr uint32_t kRtWaves = 8;
constexpr uint32_t kRtThreads = 64 * kRtWaves;
static_assert(kRtTile % 1024 == 0, "tile must be whole DMA instructions");

// Follow-up to the register-tile kernel: the tiles (64 blocks) it could not
// stage (the arena's last partial tile, a tile whose 720-byte reads would run
// past the arena, giant spans) are hashed here with per-lane loads.
// fb[0] = count, fb[1..] = tile indices.
__global__ __launch_bounds__(64) void block_sums_tile_fallback(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out, const uint32_t *__restrict__ fb) {
    const uint32_t count = fb[0];
    const uintptr_t aend = (uintptr_t)(arena + arena_bytes);
    for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
        const uint64_t t = fb[1 + i];
        const uint64_t g = t * 64 + threadIdx.x;
        if (g >= total_blocks) continue;
        const uint64_t wlo = t * 64 / 256, whi = (t * 64 + 63) / 256 + 1;
        uint32_t lo = wg_file[wlo < nwg256 ? wlo : nwg256];
        uint32_t hi = wg_file[whi < nwg256 ? whi : nwg256];
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
        }
        const DevFile F = files[lo];
        const uint64_t boff = (g - F.first_block) * F.blen;
        const uint64_t left = F.len - boff;
        const uint32_t n = left < F.blen ? (uint32_t)left : F.blen;
        const uint64_t off = F.offset + boff;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t tw = 0;
        if (((uintptr_t)(arena + off) & 3u) == 0) hash_block_direct<true>(arena, aend, off, n, seed, h, s1, tw);
        else hash_block_direct<false>(arena, aend, off, n, seed, h, s1, tw);
        store_record(out, g, n, s1, tw, h);
    }
}

template <int MODE>  // 0 = product, 1 = memory only (diagnostic)
__global__ __launch_bounds__(kRtThreads) void block_sums_regtile(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out, uint32_t *__restrict__ fb) {
    __shared__ __attribute__((aligned(16))) uint8_t tiles[kRtBufs][kRtTile];
    __shared__ uint32_t turn[kRtBufs];
    if (threadIdx.x < kRtBufs) turn[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t buf = wave % kRtBufs;
    const uint32_t users = (kRtWaves - buf + kRtBufs - 1) / kRtBufs;  // waves sharing this buffer
    const uint32_t order = wave / kRtBufs;                             // this wave's turn within a round
    uint8_t *tile = &tiles[buf][0];
    const uint64_t ntile = (total_blocks + 63) / 64;
    const uint64_t per_round = (uint64_t)gridDim.x * kRtWaves;
    const uint32_t rounds = (uint32_t)((ntile + per_round - 1) / per_round);

    for (uint32_t r = 0; r < rounds; r++) {
        const uint64_t t = (uint64_t)r * per_round + (uint64_t)blockIdx.x * kRtWaves + wave;
        const uint64_t g = t * 64 + lane;
        const bool valid = g < total_blocks;
        uint64_t off = 0;
        uint32_t n = 0;
        if (valid) {
            const uint64_t gq = g;
            const uint64_t wlo = t * 64 / 256, whi = (t * 64 + 63) / 256 + 1;
            uint32_t lo = wg_file[wlo < nwg256 ? wlo : nwg256];
            uint32_t hi = wg_file[whi < nwg256 ? whi : nwg256];
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (files[mid].first_block <= gq) lo = mid; else hi = mid - 1;
            }
            const DevFile F = files[lo];
            const uint64_t boff = (g - F.first_block) * F.blen;
            const uint64_t left = F.len - boff;
            n = left < F.blen ? (uint32_t)left : F.blen;
            off = F.offset + boff;
        }
        // wave-uniform: staged through the LDS tile, or per-lane fallback
        const uint64_t base_v = wave_min_u64(valid ? off : ~0ull);
        const uint64_t base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base_v >> 32)) << 32) |
                              __builtin_amdgcn_readfirstlane((uint32_t)base_v);
        const uint64_t top = wave_max_u64(valid ? off + kRtPiece : 0);
        const uint32_t nmax = (uint32_t)wave_max_u64(n);
        const bool fast = (t * 64 + 63 < total_blocks) && nmax <= kRegMaxBytes && top <= arena_bytes &&
                          (top - base) <= 0x7FFFFFFFull;

        // take this wave's turn on its tile buffer
        const uint32_t ticket = r * users + order;
        while (__hip_atomic_load(&turn[buf], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != ticket)
            __builtin_amdgcn_s_sleep(1);
        uint32_t R[16 * kRegChunks];
        if (fast) {
            const __amdgpu_buffer_rsrc_t rsrc =
                __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
            const uint32_t rel = (uint32_t)(off - base);
#pragma unroll 5
            for (uint32_t i = 0; i < kRtDma; i++) {
                const uint32_t idx = 64u * i + lane;
                const uint32_t j = idx / 45u, u = idx - 45u * j;
                const uint32_t voff = __shfl(rel, (int)j, 64) + 16u * u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)(tile + 1024u * i), 16, voff, 0, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint8_t *mine = tile + lane * kRtPiece;
#pragma unroll
            for (uint32_t q = 0; q < 4 * kRegChunks; q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        // release the buffer to the next wave in line
        if (lane == 0) __hip_atomic_fetch_add(&turn[buf], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);

        if (fast) {
            uint32_t h[4];
            md4_init(h);
            int32_t s1 = 0;
            uint32_t tw = 0;
            const uint32_t nfull = n >> 6;
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < 16 * (int)kRegChunks; q++) h[q & 3] ^= R[q];
            } else {
#pragma unroll
                for (uint32_t c = 0; c < kRegChunks; c++) {
                    if (c < nfull) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
                    else if (c == nfull) hash_tail<true>(R + 16 * c, 0u, 0u, n, seed, h, s1, tw);
                }
            }
            store_record(out, g, n, s1, tw, h);
        } else if (valid && lane == 0 && MODE == 0) {
            // irregular wave: the follow-up kernel hashes its blocks per lane
            const uint32_t at = atomicAdd(&fb[0], 1u);
            fb[1 + at] = (uint32_t)t;
        }
    }
}

// ---------------------------------------------------------------- loader / register-park variant
// For blocks of at most kRegMaxBytes (703: the reference's 700-byte blocks).
// Every byte should cross HBM once, in long runs: a tile = 64 consecutive
// blocks (45 KiB) is fetched as one near-linear LDS-DMA burst, and each
// block then parks in its lane's VGPRs (176 registers) while it is hashed,
// so LDS only holds tiles in transit.  One persistent 8-wave workgroup per CU:
//   wave 0 (loader) locates the tiles of this workgroup (scalar loads, no
//     vmcnt coupling with its DMA), writes their block lengths to LDS and
//     keeps up to three tiles' DMA in flight in a 3-slot ring;
//   waves 1..7 (hashers) take tiles in order by an LDS ticket, copy the slot
//     into registers, free it, hash 64 blocks and store the records.
// LDS handshake per slot: full[s] = the ticket it holds (set by the loader
// after its covering vmcnt), freeq[s] = the ticket it may take next (set by
// the hasher once its ds_reads of the slot completed).  Tiles that cannot be
// staged (the batch's partial last tile, a tile whose 704-byte reads would
// run past the arena, a span past a 31-bit offset) are marked direct: the
// hasher locates and loads its blocks itself.
constexpr uint32_t kPkPiece = 720;                // LDS bytes per block (44 data quads + 1 pad quad)
constexpr uint32_t kPkTile = 64 * kPkPiece;       // 46080 B
constexpr uint32_t kPkDma = kPkTile / 1024;       // 45 DMA instructions per tile
constexpr uint32_t kPkSlots = 3;
constexpr uint32_t kPkWaves = 8;
constexpr uint32_t kPkThreads = 64 * kPkWaves;
static_assert(kPkTile % 1024 == 0 && kPkPiece % 16 == 0, "tile = whole DMA instructions");

struct PkShared {
    uint8_t tile[kPkSlots][kPkTile];
    uint32_t n[kPkSlots][64];  // block lengths of the slot's tile
    uint32_t full[kPkSlots];
    uint32_t freeq[kPkSlots];
    uint32_t kind[kPkSlots];   // 1 = staged in the slot, 0 = direct
    uint32_t ticket;
};

__device__ __forceinline__ uint32_t pk_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void pk_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Tile descriptor (64 blocks = one tile).  Regular tile = all 64 blocks in
// one file: block j at base + B j, length B except the file's last block
// (lane jl, length nl).  Otherwise per-lane (off, n), DMA offsets by
// ds_bpermute.  Every load here is wave-uniform (scalar loads: they do not
// queue behind the caller's LDS DMA in vmcnt).
struct PkDesc {
    uint64_t base;
    uint32_t B, jl, nl;
    bool regular, staged;
    bool fast;  // staged and every block has its tail in chunk 10 (640 <= n <= 703)
    uint64_t off;  // per lane
    uint32_t n;    // per lane
};

__device__ __forceinline__ void pk_locate(uint64_t t, PkDesc &d, uint32_t lane, const DevFile *__restrict__ files,
                                          const uint32_t *__restrict__ wg_file, uint32_t nwg256,
                                          uint64_t total_blocks, uint64_t arena_bytes) {
    const uint64_t g0 = t * 64;
    const uint32_t w = (uint32_t)(g0 >> 8);
    uint32_t lo = wg_file[w], hi = wg_file[min(w + 1, nwg256)];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= g0) lo = mid; else hi = mid - 1;
    }
    const DevFile F0 = files[__builtin_amdgcn_readfirstlane(lo)];
    const uint64_t fend = F0.first_block + F0.nblocks;
    d.regular = g0 >= F0.first_block && g0 + 64 <= fend;
    const uint64_t g = g0 + lane;
    if (d.regular) {
        const uint64_t b0 = g0 - F0.first_block;
        d.base = F0.offset + b0 * F0.blen;
        d.B = F0.blen;
        d.jl = (uint32_t)min<uint64_t>(fend - 1 - g0, 64);
        d.nl = (uint32_t)(F0.len - (uint64_t)(F0.nblocks - 1) * F0.blen);
        d.n = lane == d.jl ? d.nl : d.B;
        d.off = d.base + (uint64_t)d.B * lane;
        const uint64_t top = d.base + (uint64_t)d.B * 63 + 704u;
        d.staged = d.B <= kRegMaxBytes && top <= arena_bytes && top - d.base <= 0x7FFFFFFFull;
        d.fast = d.staged && d.B >= 640 && (d.jl >= 64 || d.nl >= 640);
        return;
    }
    const uint64_t gend = min(g0 + 64, total_blocks);
    uint64_t off = 0;
    uint32_t n = 0;
#pragma unroll 1
    for (uint32_t f = __builtin_amdgcn_readfirstlane(lo);; f++) {
        const DevFile F = files[f];
        if (g >= F.first_block && g < F.first_block + F.nblocks) {
            const uint64_t boff = (g - F.first_block) * F.blen;
            const uint64_t left = F.len - boff;
            n = left < F.blen ? (uint32_t)left : F.blen;  // generator.go:334
            off = F.offset + boff;
        }
        if (F.first_block + F.nblocks >= gend) break;
    }
    const uint64_t lo_v = wave_min_u64(n ? off : ~0ull);
    d.base = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo_v >> 32)) << 32) |
             __builtin_amdgcn_readfirstlane((uint32_t)lo_v);
    const uint64_t top = wave_max_u64(n ? off + 704u : 0);
    const uint32_t nmax = (uint32_t)wave_max_u64(n);
    d.staged = (g0 + 64 <= total_blocks) && nmax <= kRegMaxBytes && top <= arena_bytes &&
               top - d.base <= 0x7FFFFFFFull;
    d.fast = d.staged && (uint32_t)wave_min_u64(n) >= 640u;
    d.off = off;
    d.n = n;
    d.B = 0;
}

// MODE 0 = product; 1 = memory only (diagnostic: DMA + copy, no hashing).
// AUX = cache policy of the tile DMA (0 default, 2 = nt: read once).
template <int MODE, int AUX, int NL>
__global__ __launch_bounds__(kPkThreads) void block_sums_park(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) PkShared sh;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < kPkSlots) {
        sh.full[threadIdx.x] = ~0u;
        sh.freeq[threadIdx.x] = threadIdx.x;
    }
    if (threadIdx.x == 0) sh.ticket = 0;
    __syncthreads();
    const uint64_t ntiles = (total_blocks + 63) / 64;
    const uint32_t G = gridDim.x;

    if (wave < NL) {
        // ------------------------------------------------------------ loaders
        // DMA instruction i, lane l fills tile bytes [1024 i + 16 l, +16):
        // block j = (64 i + l) / 45, quad u = (64 i + l) % 45 (u = 44: pad,
        // marked by an offset no block length reaches).
        uint32_t jj[kPkDma], uu[kPkDma];
#pragma unroll
        for (uint32_t i = 0; i < kPkDma; i++) {
            const uint32_t idx = 64u * i + lane;
            jj[i] = idx / 45u;
            const uint32_t u = idx - 45u * jj[i];
            uu[i] = u < 44u ? 16u * u : 0x40000000u;  // the pad quad: no block length reaches it
        }
        PkDesc cur;
        uint32_t k = wave;  // loader L takes tickets L, L + NL, ...
        uint64_t t = blockIdx.x + (uint64_t)wave * G;
        bool any = false;
        if (t < ntiles) pk_locate(t, cur, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
#pragma unroll 1
        for (; t < ntiles; t += (uint64_t)NL * G, k += NL) {
            const uint32_t slot = k % kPkSlots;
            // the slot's previous tile must have been copied out by its hasher
            while (pk_load(&sh.freeq[slot]) != k) __builtin_amdgcn_s_sleep(1);
            sh.n[slot][lane] = cur.n;
            if (lane == 0) sh.kind[slot] = cur.staged ? 1u : 0u;
            const bool staged = cur.staged;
            if (staged) pk_issue<AUX, true>(arena, &sh.tile[slot][0], cur, lane, jj, uu);
            // next tile's descriptor while this one and the previous are in flight
            if (t + (uint64_t)NL * G < ntiles)
                pk_locate(t + (uint64_t)NL * G, cur, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
            // publish this loader's previous tile once its DMA has landed
            if (any) {
                if (staged) asm volatile("s_waitcnt vmcnt(45)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) pk_store(&sh.full[(k - NL) % kPkSlots], k - NL);
            }
            any = true;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (any && lane == 0) pk_store(&sh.full[(k - NL) % kPkSlots], k - NL);
        return;
    }

    // ---------------------------------------------------------------- hashers
#pragma unroll 1
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = __hip_atomic_fetch_add(&sh.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        k = __builtin_amdgcn_readfirstlane(k);
        const uint64_t t = blockIdx.x + (uint64_t)k * G;
        if (t >= ntiles) break;
        const uint32_t slot = k % kPkSlots;
        while (pk_load(&sh.full[slot]) != k) __builtin_amdgcn_s_sleep(1);
        const uint32_t n = sh.n[slot][lane];
        const uint32_t kind = __builtin_amdgcn_readfirstlane(sh.kind[slot]);
        const uint64_t g = t * 64 + lane;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t tw = 0;
        if (kind) {
            uint32_t R[16 * kRegChunks];
            const uint8_t *mine = &sh.tile[slot][0] + lane * kPkPiece;
#pragma unroll
            for (uint32_t q = 0; q < 4 * kRegChunks; q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) pk_store(&sh.freeq[slot], k + kPkSlots);
            const uint32_t nfull = n >> 6;
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < 16 * (int)kRegChunks; q++) h[q & 3] ^= R[q];
            } else {
#pragma unroll
                for (uint32_t c = 0; c < kRegChunks; c++) {
                    if (c < nfull) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
                    else if (c == nfull) hash_tail<true>(R + 16 * c, 0u, 0u, n, seed, h, s1, tw);
                }
            }
            store_record(out, g, n, s1, tw, h);
        } else {
            if (lane == 0) pk_store(&sh.freeq[slot], k + kPkSlots);
            if (g < total_blocks) {
                uint64_t off;
                uint32_t nn;
                const uint32_t w = (uint32_t)(g >> 8);
                uint32_t lo = wg_file[w], hi = wg_file[min(w + 1, nwg256)];
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) >> 1;
                    if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
                }
                const DevFile F = files[lo];
                const uint64_t boff = (g - F.first_block) * F.blen;
                const uint64_t left = F.len - boff;
                nn = left < F.blen ? (uint32_t)left : F.blen;
                off = F.offset + boff;
                const uint8_t *p = arena + off;
                const uintptr_t end = (uintptr_t)(arena + arena_bytes);
                const uint32_t nf = nn >> 6;
                uint32_t X[16];
#pragma unroll 1
                for (uint32_t c = 0; c < nf; c++) {
                    load16(p + 64u * c, X);
                    hash_chunk<true>(X, 0u, 0u, c, h, s1, tw);
                }
                load16_guarded(p + 64u * nf, end, X);
                hash_tail<true>(X, 0u, 0u, nn, seed, h, s1, tw);
                store_record(out, g, nn, s1, tw, h);
            }
        }
    }
}

// Issue the 45 LDS-DMA instructions of a staged tile into dst.  Instruction
// i, lane l fills dst bytes [1024 i + 16 l, +16): block j = (64 i + l) / 45,
// quad u = (64 i + l) % 45 (u = 44 is the pad).  Quads past the block's
// bytes and the pad get an offset past num_records: no memory request.
// jj/uu: per-lane block index and byte offset (0x40000000 for the pad) of
// each instruction, precomputed by a caller with registers to spare (UNROLL);
// otherwise computed on the fly.
template <int AUX, bool UNROLL>
__device__ __forceinline__ void pk_issue(const uint8_t *arena, uint8_t *dst, const PkDesc &d, uint32_t lane,
                                         const uint32_t *jj = nullptr, const uint32_t *uu = nullptr) {
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + d.base), (short)0, 0x7FFFFFFF, 0x00020000);
    const int rel = (int)(uint32_t)(d.off - d.base);
#define RSG_PK_ONE(I_, REG)                                                                                     \
    do {                                                                                                        \
        uint32_t j_, u16_;                                                                                      \
        if (UNROLL) {                                                                                           \
            j_ = jj[I_];                                                                                        \
            u16_ = uu[I_];                                                                                      \
        } else {                                                                                                \
            const uint32_t idx_ = 64u * (I_) + lane;                                                            \
            j_ = idx_ / 45u;                                                                                    \
            const uint32_t u_ = idx_ - 45u * j_;                                                                \
            u16_ = u_ < 44u ? 16u * u_ : 0x40000000u;                                                           \
        }                                                                                                       \
        uint32_t vo_;                                                                                           \
        if (REG) {                                                                                              \
            const uint32_t nj_ = j_ == d.jl ? d.nl : d.B;                                                       \
            vo_ = u16_ < nj_ ? d.B * j_ + u16_ : 0x80000000u;                                                   \
        } else {                                                                                                \
            const uint32_t rj_ = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j_), rel);                  \
            const uint32_t nj_ = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j_), (int)d.n);             \
            vo_ = u16_ < nj_ ? rj_ + u16_ : 0x80000000u;                                                        \
        }                                                                                                       \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * (I_)), \
                                                 16, vo_, 0, 0, AUX);                                           \
    } while (0)
    // the regular/irregular choice is made once per tile (a branch per
    // instruction costs an lgkmcnt wait per instruction); UNROLL = false when
    // the caller holds a parked block (176 VGPRs)
    if (d.regular) {
        if constexpr (UNROLL) {
#pragma unroll
            for (uint32_t i = 0; i < kPkDma; i++) RSG_PK_ONE(i, true);
        } else {
#pragma unroll 1
            for (uint32_t i = 0; i < kPkDma; i++) RSG_PK_ONE(i, true);
        }
    } else {
        if constexpr (UNROLL) {
#pragma unroll
            for (uint32_t i = 0; i < kPkDma; i++) RSG_PK_ONE(i, false);
        } else {
#pragma unroll 1
            for (uint32_t i = 0; i < kPkDma; i++) RSG_PK_ONE(i, false);
        }
    }
#undef RSG_PK_ONE
}

// Hash a parked block (R = its 704 bytes, chunks 0..10) from chunk C_LO up to
// C_HI (exclusive).
template <uint32_t C_LO, uint32_t C_HI>
__device__ __forceinline__ void pk_hash(const uint32_t *R, uint32_t n, uint32_t seed, uint32_t h[4], int32_t &s1,
                                        uint32_t &tw) {
    const uint32_t nfull = n >> 6;
#pragma unroll
    for (uint32_t c = C_LO; c < C_HI; c++) {
        if (c < nfull) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
        else if (c == nfull) hash_tail<true>(R + 16 * c, 0u, 0u, n, seed, h, s1, tw);
    }
}

// A block of a direct tile: the lane locates and loads it itself.
__device__ __forceinline__ void pk_direct(const uint8_t *__restrict__ arena, uint64_t arena_bytes,
                                       const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file,
                                       uint32_t nwg256, uint64_t g, uint32_t seed, uint8_t *__restrict__ out) {
    const uint32_t w = (uint32_t)(g >> 8);
    uint32_t lo = wg_file[w], hi = wg_file[min(w + 1, nwg256)];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= g) lo = mid; else hi = mid - 1;
    }
    const DevFile F = files[lo];
    const uint64_t boff = (g - F.first_block) * F.blen;
    const uint64_t left = F.len - boff;
    const uint32_t nn = left < F.blen ? (uint32_t)left : F.blen;
    const uint8_t *p = arena + F.offset + boff;
    const uintptr_t end = (uintptr_t)(arena + arena_bytes);
    const uint32_t nf = nn >> 6;
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t tw = 0;
    uint32_t X[16];
#pragma unroll 1
    for (uint32_t c = 0; c < nf; c++) {
        load16(p + 64u * c, X);
        hash_chunk<true>(X, 0u, 0u, c, h, s1, tw);
    }
    load16_guarded(p + 64u * nf, end, X);
    hash_tail<true>(X, 0u, 0u, nn, seed, h, s1, tw);
    store_record(out, g, nn, s1, tw, h);
}

// ---------------------------------------------------------------- relay variant
// The loader wave above is capped by its 6-bit vmcnt: at most 63 DMA
// instructions (63 KiB) in flight per wave, i.e. per CU.  Here there is no
// loader: all 8 waves hash, and each one relays the ring forward.  The wave
// that takes ticket k copies slot k % 3 into its registers and immediately
// refills that slot with tile k + 3 (its own DMA, at most 45 instructions in
// its own vmcnt), hashes chunks 0..C0-1 of its blocks while the DMA flies,
// then waits for it, publishes tile k + 3 and hashes the rest.  Up to three
// tiles (138 KiB) are in flight per CU, spread over three waves' counters.
template <int AUX, uint32_t C0>
__global__ __launch_bounds__(kPkThreads) void block_sums_relay(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) PkShared sh;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < kPkSlots) sh.full[threadIdx.x] = ~0u;
    if (threadIdx.x == 0) sh.ticket = 0;
    __syncthreads();
    const uint64_t ntiles = (total_blocks + 63) / 64;
    const uint32_t G = gridDim.x;
    // prologue: waves 0..2 load tickets 0..2
    if (wave < kPkSlots && blockIdx.x + (uint64_t)wave * G < ntiles) {
        PkDesc d;
        pk_locate(blockIdx.x + (uint64_t)wave * G, d, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
        sh.n[wave][lane] = d.n;
        if (lane == 0) sh.kind[wave] = d.fast ? 1u : (d.staged ? 2u : 0u);
        if (d.staged) pk_issue<AUX, false>(arena, &sh.tile[wave][0], d, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) pk_store(&sh.full[wave], wave);
    }
#pragma unroll 1
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = __hip_atomic_fetch_add(&sh.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        k = __builtin_amdgcn_readfirstlane(k);
        const uint64_t t = blockIdx.x + (uint64_t)k * G;
        if (t >= ntiles) break;
        const uint32_t slot = k % kPkSlots;
        const uint64_t tn = t + (uint64_t)kPkSlots * G;  // the tile this wave relays
        const bool relay = tn < ntiles;
        PkDesc d;
        if (relay) pk_locate(tn, d, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
        while (pk_load(&sh.full[slot]) != k) __builtin_amdgcn_s_sleep(1);
        const uint32_t n = sh.n[slot][lane];
        const uint32_t kind = __builtin_amdgcn_readfirstlane(sh.kind[slot]);
        const uint64_t g = t * 64 + lane;
        // refill the slot with tile k + 3 (its descriptor first: the slot's
        // own n/kind have been read)
#define RSG_RELAY_ISSUE()                                                      \
    do {                                                                       \
        sh.n[slot][lane] = d.n;                                                \
        if (lane == 0) sh.kind[slot] = d.fast ? 1u : (d.staged ? 2u : 0u);     \
        if (d.staged) pk_issue<AUX, false>(arena, &sh.tile[slot][0], d, lane);        \
    } while (0)
#define RSG_RELAY_PUBLISH()                                                    \
    do {                                                                       \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                       \
        if (lane == 0) pk_store(&sh.full[slot], k + kPkSlots);                 \
    } while (0)
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t tw = 0;
        if (kind == 1) {
            // every block ends in chunk 10: park it, refill the slot at once,
            // publish the refill after chunk C0
            uint32_t R[16 * kRegChunks];
            const uint8_t *mine = &sh.tile[slot][0] + lane * kPkPiece;
#pragma unroll
            for (uint32_t q = 0; q < 4 * kRegChunks; q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read out
            if (relay) RSG_RELAY_ISSUE();
#pragma unroll
            for (uint32_t c = 0; c < C0; c++) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
            if (relay) RSG_RELAY_PUBLISH();
#pragma unroll
            for (uint32_t c = C0; c < kRegChunks - 1; c++) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
            hash_tail<true>(R + 16 * (kRegChunks - 1), 0u, 0u, n, seed, h, s1, tw);
            store_record(out, g, n, s1, tw, h);
        } else if (kind == 2) {
            // ragged block lengths: hash straight out of the slot (few
            // VGPRs), then refill it
            const uint8_t *mine = &sh.tile[slot][0] + lane * kPkPiece;
            const uint32_t nfull = n >> 6;
            uint32_t X[16];
#pragma unroll 1
            for (uint32_t c = 0; c <= nfull; c++) {
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(mine + 64 * c + 16 * q);
                    X[4 * q + 0] = v.x; X[4 * q + 1] = v.y; X[4 * q + 2] = v.z; X[4 * q + 3] = v.w;
                }
                if (c < nfull) hash_chunk<true>(X, 0u, 0u, c, h, s1, tw);
                else hash_tail<true>(X, 0u, 0u, n, seed, h, s1, tw);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (relay) {
                RSG_RELAY_ISSUE();
                RSG_RELAY_PUBLISH();
            }
            store_record(out, g, n, s1, tw, h);
        } else {
            if (relay) {
                RSG_RELAY_ISSUE();
                RSG_RELAY_PUBLISH();
            }
            if (g < total_blocks) pk_direct(arena, arena_bytes, files, wg_file, nwg256, g, seed, out);
        }
#undef RSG_RELAY_ISSUE
#undef RSG_RELAY_PUBLISH
    }
}

// Kernel variants (rsg_set_block_sums_kernel): -1 = automatic, 0 = direct,
// 1 = staged K=1, 2 = staged K=4, 3 = register-block, 4 = register-tile,
// 5 = loaded line ring, 6 = line ring with shared boundary lines, 7/8 = 1/2
// with the last segment cut at the block end, 9 = long blocks with deep
// per-lane prefetch (automatic for unaligned blocks >= kLongBlockBytes).  Timing
// diagnostics with meaningless outputs: 10 = staged K=1 memory only, 11 =
// staged K=1 hashing only, 12 = register-block memory only, 13/14 = linear
// read of the arena (plain loads / LDS DMA), 15 = staged with line-aligned
// pieces (memory only), 16 = staged with packed pieces (memory only), 17 =
// register-tile memory only, 18 = line ring memory only.
static int g_variant = -2;  // -2 = not yet read from RSG_BLOCKSUMS_KERNEL

hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t max_blen, uint32_t seed, uint8_t *out, uint32_t *scratch, hipStream_t stream) {
    if (total_blocks == 0) return hipSuccess;
    if (g_variant == -2) {
        const char *e = getenv("RSG_BLOCKSUMS_KERNEL");
        g_variant = e ? atoi(e) : -1;
    }
    int v = g_variant;
    // automatic: staged for aligned batches (also the faster one for long
    // aligned blocks, tools/blocklen_sweep.py); unaligned batches (the sender's
    // confirmation windows) take the deep-prefetch kernel when blocks are long
    if (v == -1) v = aligned ? 1 : (max_blen >= kLongBlockBytes ? 9 : 0);
    if (!aligned && ((v < 13 && v != 9) || v >= 20)) v = 0;
    if ((v == 3 || v == 4 || v == 12 || v == 17 || (v >= 34 && v <= 41)) && max_blen > kRegMaxBytes) v = 1;
    if ((v == 4 || v == 17) && !scratch) v = 1;
    dim3 grid(nwg), block(kBlockSumThreads);
#define RSG_LAUNCH(KERNEL, GRID) \
    hipLaunchKernelGGL(KERNEL, GRID, block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out)
#define RSG_STAGED(KK, MM, ...)                                                                                 \
    hipLaunchKernelGGL((block_sums_staged<KK, MM, ##__VA_ARGS__>), dim3((uint32_t)((total_blocks + 256u * KK - 1) / (256u * KK))), \
                       block, 0, stream, arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out)
#define RSG_CRING(RR, SS, MM, WW)                                                                             \
    hipLaunchKernelGGL((block_sums_cring<RR, SS, MM, WW>), dim3((uint32_t)((total_blocks + 255u) / 256u)), block, 0, \
                       stream, arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out)
    switch (v) {
        case 38:
        case 39:
        case 40:
        case 41: {
            int dev = 0, cus = 256;
            if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            const uint64_t ntile = (total_blocks + 63) / 64;
            const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus, ntile));
            if (v == 38)
                hipLaunchKernelGGL((block_sums_relay<2, 4>), dim3(g), dim3(kPkThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out);
            else if (v == 39)
                hipLaunchKernelGGL((block_sums_relay<2, 2>), dim3(g), dim3(kPkThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out);
            else if (v == 40)
                hipLaunchKernelGGL((block_sums_relay<2, 6>), dim3(g), dim3(kPkThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out);
            else
                hipLaunchKernelGGL((block_sums_relay<2, 8>), dim3(g), dim3(kPkThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out);
            break;
        }
        case 34:
        case 35:
        case 36:
        case 37: {
            int dev = 0, cus = 256;
            if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            const uint64_t ntile = (total_blocks + 63) / 64;
            const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus, ntile));
#define RSG_PARK(MM, AA, NN)                                                                                 \
    hipLaunchKernelGGL((block_sums_park<MM, AA, NN>), dim3(g), dim3(kPkThreads), 0, stream, arena, arena_bytes, files, \
                       wg_file, nwg, total_blocks, seed, out)
            if (v == 34) RSG_PARK(0, 2, 2);
            else if (v == 35) RSG_PARK(1, 2, 2);
            else if (v == 36) RSG_PARK(0, 2, 1);
            else RSG_PARK(1, 2, 1);
#undef RSG_PARK
            break;
        }
        case 24: RSG_CRING(1, 1, 0, 8); break;
        case 25: RSG_CRING(2, 1, 0, 5); break;
        case 26: RSG_CRING(3, 1, 0, 3); break;
        case 27: RSG_CRING(1, 2, 0, 5); break;
        case 28: RSG_CRING(2, 2, 0, 2); break;
        case 29: RSG_CRING(1, 1, 1, 8); break;
        case 30: RSG_CRING(1, 1, 2, 8); break;
        case 31: RSG_CRING(2, 1, 1, 5); break;
        case 32: RSG_CRING(2, 1, 2, 5); break;
        case 33: RSG_CRING(1, 2, 1, 5); break;
        case 0:
            if (aligned) RSG_LAUNCH(block_sums_direct<true>, grid);
            else RSG_LAUNCH(block_sums_direct<false>, grid);
            break;
        case 2: RSG_STAGED(4, 0); break;
        case 23:
            hipLaunchKernelGGL(block_sums_staged_a16, dim3((uint32_t)((total_blocks + 255u) / 256u)), block, 0, stream,
                               arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 22:
            hipLaunchKernelGGL(block_sums_diag_tile, dim3((uint32_t)((total_blocks + 63u) / 64u)), dim3(64), 0, stream,
                               arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 21:
            hipLaunchKernelGGL(block_sums_staged_half, dim3((uint32_t)((total_blocks + 255u) / 256u)), block, 0, stream,
                               arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 20:
            hipLaunchKernelGGL(block_sums_staged2, dim3((uint32_t)((total_blocks + 255u) / 256u)), block, 0, stream,
                               arena, arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 9: {
            dim3 g64((uint32_t)((total_blocks + 63) / 64)), b64(64);
            if (aligned)
                hipLaunchKernelGGL(block_sums_long<true>, g64, b64, 0, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
            else
                hipLaunchKernelGGL(block_sums_long<false>, g64, b64, 0, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
            break;
        }
        case 3: RSG_LAUNCH(block_sums_regblock<0>, grid); break;
        case 4:
        case 17: {
            int cus = 256;
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
            const uint64_t ntile = (total_blocks + 63) / 64;
            const uint32_t g = (uint32_t)std::min<uint64_t>((uint64_t)cus, (ntile + kRtWaves - 1) / kRtWaves);
            hipError_t e = hipMemsetAsync(scratch, 0, 4, stream);
            if (e != hipSuccess) return e;
            if (v == 4)
                hipLaunchKernelGGL(block_sums_regtile<0>, dim3(g), dim3(kRtThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out, scratch);
            else
                hipLaunchKernelGGL(block_sums_regtile<1>, dim3(g), dim3(kRtThreads), 0, stream, arena, arena_bytes,
                                   files, wg_file, nwg, total_blocks, seed, out, scratch);
            hipLaunchKernelGGL(block_sums_tile_fallback, dim3(256), dim3(64), 0, stream, arena, arena_bytes, files,
                               wg_file, nwg, total_blocks, seed, out, (const uint32_t *)scratch);
            break;
        }
        case 5: RSG_LAUNCH(block_sums_lring<0>, grid); break;
        case 6: RSG_LAUNCH((block_sums_lring<0, true>), grid); break;
        case 18: RSG_LAUNCH(block_sums_lring<1>, grid); break;
        case 10: RSG_STAGED(1, 1); break;
        case 11: RSG_STAGED(1, 2); break;
        case 15: RSG_STAGED(1, 3); break;
        case 7: RSG_STAGED(1, 0, true); break;
        case 8: RSG_STAGED(4, 0, true); break;
        case 19: RSG_STAGED(1, 1, true); break;
        case 16: RSG_STAGED(1, 4); break;
        case 12: RSG_LAUNCH(block_sums_regblock<1>, grid); break;
        case 13:
            hipLaunchKernelGGL(diag_linear_read<false>, dim3(2048), dim3(256), 0, stream, arena, arena_bytes,
                               (uint32_t *)out);
            break;
        case 14:
            hipLaunchKernelGGL(diag_linear_read<true>, dim3(2048), dim3(256), 0, stream, arena, arena_bytes,
                               (uint32_t *)out);
            break;
        default: RSG_STAGED(1, 0); break;
    }
#undef RSG_LAUNCH
#undef RSG_STAGED
#undef RSG_CRING
    return hipGetLastError();
}

void set_block_sums_variant(int v) { g_variant = v; }

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
