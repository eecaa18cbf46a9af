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
#include "rsg_hash_block.h"
#include "rsg_md4.h"

namespace rsg {


// Fallback census (rsg_block_sums_fallbacks): [0] full 64-block waves of the
// staged kernels, [1] full 64-block tiles of the park kernel that could not
// take the LDS-DMA path and were hashed with per-lane loads.  The records are
// the same either way, only speed differs, so this is how a test tells that
// the fast path was really taken.  One atomic per fallback wave (vector
// atomic from lane 0), nothing on the fast path.
__device__ unsigned long long g_fallbacks[2];
__device__ __forceinline__ void count_fallback(int k) { atomicAdd(&g_fallbacks[k], 1ull); }

// Record g = int32 LE Checksum1 then the 16 MD4 digest bytes (generator.go:341-346).
__device__ __forceinline__ void store_record(uint8_t *out, uint64_t g, uint32_t n, int32_t s1, uint32_t t,
                                             const uint32_t h[4]) {
    const uint32_t s2 = n * (uint32_t)s1 - t;  // sum (n - i) x_i
    const uint32_t sum1 = ((uint32_t)s1 & 0xffffu) | (s2 << 16);  // rsyncchecksum.go:50
    uint32_t *o = reinterpret_cast<uint32_t *>(out + g * kRecordBytes);
    o[0] = sum1;
    o[1] = h[0]; o[2] = h[1]; o[3] = h[2]; o[4] = h[3];
}

// The 64 records of a staged tile (blocks t*64 .. t*64+63: 1280 contiguous
// bytes of the output) through the hasher's LDS area, so they leave as
// full 16-byte lanes of 1 KiB runs (64 + 16 quads) instead of 64 lanes each
// writing 20 bytes at a 20-byte stride: those strided partial-line stores
// cost the kernel its streaming rate (park memory only with
// and without its record stores: 0.187 against 0.155 ms per cfg2 launch).
// REC = 2: the stores are nontemporal (the records are not read again here).
template <int REC>
__device__ __forceinline__ void store_tile_records(uint8_t *out, uint64_t t, uint32_t lane, uint32_t *rec, uint32_t n,
                                                   int32_t s1, uint32_t tw, const uint32_t h[4]) {
    const uint32_t s2 = n * (uint32_t)s1 - tw;                    // sum (n - i) x_i
    const uint32_t sum1 = ((uint32_t)s1 & 0xffffu) | (s2 << 16);  // rsyncchecksum.go:50
    rec[5 * lane + 0] = sum1;
    rec[5 * lane + 1] = h[0];
    rec[5 * lane + 2] = h[1];
    rec[5 * lane + 3] = h[2];
    rec[5 * lane + 4] = h[3];
    // other lanes' records are read back: the wave's LDS operations run in
    // order, so only the compiler must not move the reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const u32x4v a = reinterpret_cast<const u32x4v *>(rec)[lane];
    uint8_t *tile_out = out + t * (64ull * kRecordBytes);
    if constexpr (REC >= 4) {
        // buffer stores with an explicit cache policy: 4 = nt | sc1, 5 = nt | sc0 | sc1
        constexpr int aux = REC == 4 ? (2 | 16) : (1 | 2 | 16);
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)tile_out, (short)0, 1280, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(a, r, 16u * lane, 0, aux);
        if (lane < 16) {
            const u32x4v b = reinterpret_cast<const u32x4v *>(rec)[64 + lane];
            __builtin_amdgcn_raw_buffer_store_b128(b, r, 1024u + 16u * lane, 0, aux);
        }
        return;
    }
    u32x4a4 *dst = reinterpret_cast<u32x4a4 *>(tile_out);
    if (REC == 2) __builtin_nontemporal_store(u32x4a4{a.x, a.y, a.z, a.w}, dst + lane);
    else dst[lane] = u32x4a4{a.x, a.y, a.z, a.w};
    if (lane < 16) {
        const u32x4v b = reinterpret_cast<const u32x4v *>(rec)[64 + lane];
        if (REC == 2) __builtin_nontemporal_store(u32x4a4{b.x, b.y, b.z, b.w}, dst + 64 + lane);
        else dst[64 + lane] = u32x4a4{b.x, b.y, b.z, b.w};
    }
}

// A lane's own record with nontemporal stores (park REC = 3).
__device__ __forceinline__ void store_record_nt(uint8_t *out, uint64_t g, uint32_t n, int32_t s1, uint32_t t,
                                                const uint32_t h[4]) {
    const uint32_t s2 = n * (uint32_t)s1 - t;
    const uint32_t sum1 = ((uint32_t)s1 & 0xffffu) | (s2 << 16);
    u32x4a4 *o = reinterpret_cast<u32x4a4 *>(out + g * kRecordBytes);
    __builtin_nontemporal_store(u32x4a4{sum1, h[0], h[1], h[2]}, o);
    __builtin_nontemporal_store(h[3], reinterpret_cast<uint32_t *>(out + g * kRecordBytes + 16));
}

// File of block g: the largest f in [wg_file[wg], wg_file[wg+1]] with
// first_block <= g (zero-length files own no blocks and are skipped).
// Returns the block's arena offset and length (generator.go:334).
// wg: the 256-block workgroup slot g belongs to (wg_file's index; the
// launch's blockIdx.x unless a persistent workgroup loops over slots)
__device__ __forceinline__ void locate_block(const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file,
                                             uint64_t g, uint64_t &off, uint32_t &n, uint64_t wg) {
    uint32_t lo = wg_file[wg], hi = wg_file[wg + 1];
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
__device__ __forceinline__ void locate_block(const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file,
                                             uint64_t g, uint64_t &off, uint32_t &n) {
    locate_block(files, wg_file, g, off, n, blockIdx.x);
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

// Workgroups of W waves.  With few windows (the sender's ~23 K confirmation
// windows) W = 2 puts the two waves of a CU on separate SIMDs: one-wave
// workgroups took 0.31 or 0.55-0.60 ms depending on whether two landed on one
// SIMD, four-wave workgroups 0.46 ms (four waves share the CU's memory
// pipeline).  With more waves than 2 per CU, W = 1 spreads them better.
template <bool ALIGNED, int W>
__global__ __launch_bounds__(64 * W) void block_sums_long(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    constexpr uint32_t kLongThreads = 64 * W;
    const uint64_t g = (uint64_t)blockIdx.x * kLongThreads + threadIdx.x;
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
// Coalesced HBM reads for blocks of any length: a wave owns 64 consecutive
// blocks (one per lane) and streams them through a private LDS slab 256 bytes
// (4 MD4 chunks) of every block at a time.  The slab is filled by
// buffer_load_dwordx4 ... lds (LDS DMA, no VGPRs in flight): each DMA
// wave-instruction fetches 4 contiguous 256-byte pieces.  Piece j (lane j's
// block) sits at j*272 in the slab: the 16-byte pad makes the per-lane
// ds_read_b128 of one unit conflict-free (bank = 4*(j + unit) mod 64 inside
// every 16-lane group).  While the wave hashes segment s out of registers,
// segment s+1 is already in flight.  The default for aligned batches whose
// blocks are longer than the park kernel's 703 bytes.
// SEG = bytes of every block per segment (256 by default; 128 and 512 are
// variants 4 and 5 for long blocks: more waves per CU vs longer pieces).
template <uint32_t SEG>
struct Seg {
    static constexpr uint32_t kSegBytes = SEG;
    static constexpr uint32_t kUnits = SEG / 16 + 1;           // 16-byte units per padded piece
    static constexpr uint32_t kPiece = SEG + 16;               // padded piece stride in LDS
    static constexpr uint32_t kWaveSlab = 64 * kPiece;         // 17408 bytes per wave at SEG = 256
    static constexpr uint32_t kDmaPerSeg = kWaveSlab / 1024;   // 17 DMA instructions per segment
    static constexpr uint32_t kChunks = SEG / 64;              // MD4 chunks per segment
    static_assert(kWaveSlab % 1024 == 0, "slab must be a whole number of DMA instructions");
};

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
// A 64-block group's layout, wave-uniform when the whole group lies in one
// file (every lane's block full-length except perhaps lane 63's, the file's
// last): the file is found with g = the group's first block, so the loads
// are uniform (scalar loads: no wait on the vector-memory counter, which
// the in-flight DMA also holds).  Otherwise (the group spans files or runs
// past the batch) the lanes locate their own blocks (locate_block).
struct GroupDesc {
    uint64_t off;   // this lane's block
    uint32_t n;
    uint64_t base;  // lane 0's block (uniform)
    uint32_t S;     // segments through the longest block's tail chunk (uniform)
    bool staged;    // the staged path applies (uniform)
};

template <uint32_t SEG>
__device__ __forceinline__ void locate_group(const uint8_t *arena, uint64_t arena_bytes,
                                             const DevFile *__restrict__ files, const uint32_t *__restrict__ wg_file,
                                             uint64_t total_blocks, uint64_t wave_first, uint32_t lane, GroupDesc &d) {
    constexpr uint32_t kChunks = SEG / 64;
    (void)arena;
    const uint64_t wg = wave_first / kBlockSumThreads;
    uint32_t lo = rfl32(wg_file[wg]), hi = rfl32(wg_file[wg + 1]);
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[mid].first_block <= wave_first) lo = mid; else hi = mid - 1;
    }
    const uint64_t F_off = rfl64(files[lo].offset), F_len = rfl64(files[lo].len), F_first = rfl64(files[lo].first_block);
    const uint32_t F_blen = rfl32(files[lo].blen), F_nb = rfl32(files[lo].nblocks);
    const bool full = wave_first + 63 < total_blocks;
    if (full && wave_first + 63 - F_first < F_nb) {
        const uint64_t bi = wave_first + lane - F_first, boff = bi * F_blen, left = F_len - boff;
        d.n = left < F_blen ? (uint32_t)left : F_blen;
        d.off = F_off + boff;
        d.base = F_off + (wave_first - F_first) * F_blen;
        d.S = (F_blen >> 6) / kChunks + 1;
        const uint64_t top = d.base + 63ull * F_blen + (uint64_t)SEG * d.S;
        d.staged = top <= arena_bytes && (top - d.base) <= 0x7FFFFFFFull;
        return;
    }
    const uint64_t g = wave_first + lane;
    d.off = 0;
    d.n = 0;
    if (g < total_blocks) locate_block(files, wg_file, g, d.off, d.n, wg);
    const uint32_t nseg = d.n ? (d.n >> 6) / kChunks + 1 : 0;
    d.S = rfl32((uint32_t)wave_max_u64(nseg));
    d.base = rfl64(wave_min_u64(d.n ? d.off : ~0ull));
    const uint64_t top = rfl64(wave_max_u64(d.n ? d.off + (uint64_t)SEG * d.S : 0));
    d.staged = full && top <= arena_bytes && (top - d.base) <= 0x7FFFFFFFull;
}

// KIND % 10: 0 = the product kernel; timing diagnostics (outputs
// meaningless): 1 = DMA + LDS reads only (the memory cost of this access
// pattern), 2 = hashing only, no DMA (the compute cost).  (KIND / 10) % 10
// picks the segment: 0 = 256 bytes, 1 = 128, 2 = 512.  KIND >= 100: blocks
// start at any byte (the sender's confirmation windows; the arena itself
// 4-byte aligned): each piece is fetched from the block's start rounded down
// to 4 bytes, one 16-byte unit longer (the pad unit carries data), and the
// lane funnel-shifts its words (alignbyte) as the direct kernel does.
// (Wave priority 3 from the segment wait through the next DMA issue, 0 while
// hashing, as park does: no gain at B = 1024 / 4096 / 128 KiB,
// profiles/r04g_blocklen_sweep.jsonl, so not kept.)
template <int KIND>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    constexpr bool UNAL = (KIND % 1000) >= 100;
    constexpr bool DB = (KIND / 1000) % 2 == 1;  // two slabs per wave: segment s+2's DMA issues while s+1 lands
    constexpr bool PERSIST = KIND >= 2000;       // each wave loops over 64-block groups (grid = resident waves)
    // nt policy on the DMA: every byte is read once (A/B against the default
    // policy, profiles/r02f_blocklen_sweep_nt.jsonl: B = 4096 0.239 -> 0.219 ms,
    // cfg5 6.48 -> 6.25 ms, B = 1024 and the sender's confirmation unchanged)
    constexpr int DMA_AUX = 2;
    constexpr int MODE = KIND % 10;
    constexpr uint32_t SEG = (KIND % 100) >= 20 ? 512u : ((KIND % 100) >= 10 ? 128u : 256u);
    constexpr uint32_t kSegBytes = Seg<SEG>::kSegBytes, kUnits = Seg<SEG>::kUnits, kPiece = Seg<SEG>::kPiece;
    constexpr uint32_t kWaveSlab = Seg<SEG>::kWaveSlab, kDmaPerSeg = Seg<SEG>::kDmaPerSeg;
    constexpr uint32_t kChunks = Seg<SEG>::kChunks;
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab * (DB ? 2 : 1)];
    const uint32_t lane = threadIdx.x & 63u;
    // readfirstlane: provably wave-uniform values keep the LDS base (M0) and
    // the buffer descriptor in SGPRs (no waterfall loops around the DMA).
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * kWaveSlab * (DB ? 2 : 1);
    // one 64-block group: the wave's blocks [wave_first, wave_first + 64)
    auto group = [&](const uint64_t wave_first) {
    const uint64_t g = wave_first + lane;
    uint64_t off = 0;
    uint32_t n = 0;
    if (g < total_blocks) locate_block(files, wg_file, g, off, n, wave_first / kBlockSumThreads);
    const uint32_t sh = UNAL ? (uint32_t)(off & 3u) : 0u;
    const uint64_t loff = off - sh;  // 4-byte aligned fetch start
    const uint32_t nseg = n ? (n >> 6) / kChunks + 1 : 0;  // segments through the tail chunk
    const uint32_t S = rfl32((uint32_t)wave_max_u64(nseg));
    const uint64_t base = rfl64(wave_min_u64(n ? loff : ~0ull));
    const uint64_t top = rfl64(wave_max_u64(n ? loff + (uint64_t)kSegBytes * S + (UNAL ? 16u : 0u) : 0));
    // Wave-uniform choice of path: the staged path needs all 64 blocks, every
    // DMA read inside the arena and the span addressable by a 31-bit buffer
    // offset.  Otherwise (last partial wave, a file ending at the arena's end,
    // giant spans) the lanes hash with per-lane loads.
    const bool full = wave_first + 63 < total_blocks;
    const bool staged = full && top <= arena_bytes && (top - base) <= 0x7FFFFFFFull;
    if (!staged) {
        if (MODE == 0 && full && lane == 0) count_fallback(0);
        if (n == 0) return;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
        hash_block_direct<!UNAL>(arena, (uintptr_t)(arena + arena_bytes), off, n, seed, h, s1, t);
        store_record(out, g, n, s1, t, h);
        return;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t rel = (uint32_t)(loff - base);
    // DMA instruction i, lane t fills slab bytes [16*(64 i + t), +16): piece
    // j = (64 i + t) / kUnits (lane j's block), unit u = (64 i + t) % kUnits.
    // u == kUnits - 1 is the pad: its offset is past num_records, so the
    // buffer range check drops it without a memory request.
    // (fixed bound: an array sized by a template-dependent local makes hipcc's
    // host pass drop this kernel's launch stubs; entries past kDmaPerSeg are dead)
    uint32_t voff[Seg<512>::kDmaPerSeg];
#pragma unroll
    for (uint32_t i = 0; i < kDmaPerSeg; i++) {
        const uint32_t idx = 64u * i + lane;
        const uint32_t j = idx / kUnits, u = idx - kUnits * j;
        const uint32_t v = (uint32_t)__shfl((int)rel, (int)j, 64) + 16u * u;
        voff[i] = (UNAL || u + 1 < kUnits) ? v : 0x80000000u;
    }
    uint32_t R[Seg<512>::kSegBytes / 4 + 4];  // fixed bound, as voff
    const uint8_t *mine = slab + lane * kPiece;
#define RSG_DMA_SEGMENT(S_)                                                                                      \
    do {                                                                                                         \
        const uint32_t so_ = kSegBytes * (S_);                                                                   \
        uint8_t *sb_ = slab + (DB ? kWaveSlab * ((S_) & 1u) : 0u);                                               \
        _Pragma("unroll") for (uint32_t i_ = 0; i_ < kDmaPerSeg; i_++)                                           \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(sb_ + 1024u * i_), \
                                                     16, voff[i_], so_, 0, DMA_AUX);                             \
    } while (0)
#define RSG_READ_SEGMENT()                                                                                       \
    do {                                                                                                         \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                         \
        _Pragma("unroll") for (int q_ = 0; q_ < (int)(SEG / 16) + (UNAL ? 1 : 0); q_++) {                        \
            const uint4 v_ = *reinterpret_cast<const uint4 *>(mine + 16 * q_);                                  \
            R[4 * q_ + 0] = v_.x; R[4 * q_ + 1] = v_.y; R[4 * q_ + 2] = v_.z; R[4 * q_ + 3] = v_.w;              \
        }                                                                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
    } while (0)
    const uint32_t nfull = n >> 6;
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    if constexpr (DB) {
        // segment cs sits in slab half cs & 1; at the top of iteration cs the
        // DMAs of cs and cs+1 are outstanding (vmcnt counts instructions, in
        // order): wait for cs's, read it, refill its half with cs+2, hash cs
        if (MODE != 2) {
            RSG_DMA_SEGMENT(0u);
            if (S > 1) RSG_DMA_SEGMENT(1u);
        }
#pragma unroll 1
        for (uint32_t cs = 0; cs < S; cs++) {
            if (cs + 1 < S) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDmaPerSeg) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint8_t *mh = mine + kWaveSlab * (cs & 1u);
#pragma unroll
            for (int q = 0; q < (int)(SEG / 16) + (UNAL ? 1 : 0); q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mh + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (MODE != 2 && cs + 2 < S) RSG_DMA_SEGMENT(cs + 2);
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < (int)(SEG / 4); q++) h[q & 3] ^= R[q];
            } else {
#pragma unroll
                for (uint32_t i = 0; i < kChunks; i++) {
                    const uint32_t c = kChunks * cs + i;
                    if (c < nfull) hash_chunk<!UNAL>(R + 16 * i, R[16 * i + 16], sh, c, h, s1, t);
                    else if (c == nfull) hash_tail<!UNAL>(R + 16 * i, R[16 * i + 16], sh, n, seed, h, s1, t);
                }
            }
        }
        if (MODE == 0) store_tile_records<2>(out, wave_first / 64, lane, reinterpret_cast<uint32_t *>(slab), n, s1, t, h);
        else store_record(out, g, n, s1, t, h);
        return;
    }
    if (MODE != 2) RSG_DMA_SEGMENT(0);
    RSG_READ_SEGMENT();
#pragma unroll 1
    for (uint32_t cs = 0; cs < S; cs++) {
        const bool more = cs + 1 < S;
        if (MODE != 2 && more) RSG_DMA_SEGMENT(cs + 1);  // in flight while segment cs hashes
        if (MODE == 1) {
#pragma unroll
            for (int q = 0; q < (int)(SEG / 4); q++) h[q & 3] ^= R[q];
        } else {
#pragma unroll
            for (uint32_t i = 0; i < kChunks; i++) {
                const uint32_t c = kChunks * cs + i;
                if (c < nfull) hash_chunk<!UNAL>(R + 16 * i, R[16 * i + 16], sh, c, h, s1, t);
                else if (c == nfull) hash_tail<!UNAL>(R + 16 * i, R[16 * i + 16], sh, n, seed, h, s1, t);
            }
        }
        if (more) RSG_READ_SEGMENT();
    }
#undef RSG_DMA_SEGMENT
#undef RSG_READ_SEGMENT
    // a full wave's 64 records are contiguous (blocks wave_first ..): staged
    // in the wave's slab (its last segment has been read) and written as
    // coalesced nontemporal stores, as the park kernel does (round 5)
    if (MODE == 0) store_tile_records<2>(out, wave_first / 64, lane, reinterpret_cast<uint32_t *>(slab), n, s1, t, h);
    else store_record(out, g, n, s1, t, h);
    };
    if constexpr (PERSIST) {
        const uint64_t groups = (total_blocks + 63) / 64, stride = (uint64_t)gridDim.x * (kBlockSumThreads / 64);
#pragma unroll 1
        for (uint64_t gw = (uint64_t)blockIdx.x * (kBlockSumThreads / 64) + wave; gw < groups; gw += stride) {
            group(gw * 64);
            // the next group's DMA rewrites the slab: the records' LDS
            // staging reads (store_tile_records) must be done
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    } else {
        group((uint64_t)blockIdx.x * kBlockSumThreads + wave * 64u);
    }
}

// Variants 13 / 14 (round 5): the persistent staged kernel with each wave's
// group boundary hidden.  Diagnostics showed the staged pattern's cost is
// its temporal order, not the piece length alone (`diag_stream_read` PAT 4 /
// 5), and that a persistent wave pays a full memory round trip plus the
// block lookup at every group start with nothing of its own in flight.  Here
// the next group is located (uniform loads) while the current group's last
// segment is in flight, its segment 0 is requested as soon as the slab is
// free (before the current group's last segment is hashed), and the current
// group's records leave after the next group's first segment has landed.
// KIND % 10: 0 product, 1 memory only (outputs meaningless); (KIND / 10) % 10
// picks the segment as the staged kernel does (0 = 256, 1 = 128, 2 = 512).
// Measured (profiles/r05am, r05ao sweeps, ms per GiB): memory only 0.179
// against the staged kernel's 0.200 at B = 1024 (0.180 / 0.186 at 2048,
// 0.218 / 0.219 at 4096); the product holds 153 VGPRs (3 waves per SIMD
// against staged's 4), so it gains only at B = 4096: 0.212-0.214 against
// 0.214-0.216.  Held to 4 waves per SIMD it spills (0.236 at B = 1024).
// With 512-byte segments (variant 14: one wave per SIMD, LDS-bound anyway)
// it is the automatic choice for most lengths from 704 to 8192 bytes (see
// launch_block_sums).
template <int KIND>
__device__ __forceinline__ void pipe_body(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    constexpr int MODE = KIND % 10;
    constexpr uint32_t SEG = (KIND % 100) >= 20 ? 512u : ((KIND % 100) >= 10 ? 128u : 256u);
    constexpr uint32_t kUnits = Seg<SEG>::kUnits, kPiece = Seg<SEG>::kPiece;
    constexpr uint32_t kWaveSlab = Seg<SEG>::kWaveSlab, kDmaPerSeg = Seg<SEG>::kDmaPerSeg;
    constexpr uint32_t kChunks = Seg<SEG>::kChunks;
    constexpr int DMA_AUX = 2;
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * kWaveSlab;
    const uint8_t *mine = slab + lane * kPiece;
    const uint64_t groups = (total_blocks + 63) / 64, stride = (uint64_t)gridDim.x * (kBlockSumThreads / 64);
    uint64_t gw = (uint64_t)blockIdx.x * (kBlockSumThreads / 64) + wave;
    if (gw >= groups) return;
    uint32_t voff[Seg<512>::kDmaPerSeg];  // fixed bound (see block_sums_staged)
    __amdgpu_buffer_rsrc_t rsrc;
    // the lane offsets and buffer of group d's DMA (valid until the next call)
    auto point = [&](const GroupDesc &d) {
        rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(arena + d.base), (short)0, 0x7FFFFFFF, 0x00020000);
        const uint32_t rel = (uint32_t)(d.off - d.base);
#pragma unroll
        for (uint32_t i = 0; i < kDmaPerSeg; i++) {
            const uint32_t idx = 64u * i + lane;
            const uint32_t j = idx / kUnits, u = idx - kUnits * j;
            const uint32_t v = (uint32_t)__shfl((int)rel, (int)j, 64) + 16u * u;
            voff[i] = u + 1 < kUnits ? v : 0x80000000u;
        }
    };
    auto dma = [&](uint32_t s) {
#pragma unroll
        for (uint32_t i = 0; i < kDmaPerSeg; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + 1024u * i),
                                                     16, voff[i], SEG * s, 0, DMA_AUX);
    };
    uint32_t R[Seg<512>::kSegBytes / 4 + 4];
    auto read_segment = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < (int)(SEG / 16); q++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
            R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    GroupDesc cur, nxt;
    locate_group<SEG>(arena, arena_bytes, files, wg_file, total_blocks, gw * 64, lane, cur);
    if (cur.staged) {
        point(cur);
        if (MODE != 2) dma(0);
    }
    // the previous group's records, stored once the next group's first
    // segment has landed (the slab is free then)
    bool pend = false;
    uint64_t pend_tile = 0;
    uint32_t pn = 0, ph[4] = {0, 0, 0, 0}, pt = 0;
    int32_t ps1 = 0;
#pragma unroll 1
    for (;;) {
        const uint64_t nw = gw + stride;
        const bool has_next = nw < groups;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
        const uint32_t n = cur.n, nfull = n >> 6;
        bool next_located = false;
        if (!cur.staged) {
            if (pend) {
                store_record(out, pend_tile * 64 + lane, pn, ps1, pt, ph);
                pend = false;
            }
            if (n) {
                hash_block_direct<true>(arena, (uintptr_t)(arena + arena_bytes), cur.off, n, seed, h, s1, t);
                store_record(out, gw * 64 + lane, n, s1, t, h);
            }
            if (!has_next) break;
            gw = nw;
            locate_group<SEG>(arena, arena_bytes, files, wg_file, total_blocks, gw * 64, lane, cur);
            if (cur.staged) {
                point(cur);
                dma(0);
            }
            continue;
        }
        read_segment();
        if (pend) {
            if (MODE == 0) store_tile_records<2>(out, pend_tile, lane, reinterpret_cast<uint32_t *>(slab), pn, ps1, pt, ph);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before the slab is refilled
            pend = false;
        }
        const uint32_t S = cur.S;
        if (S == 1 && has_next) {
            locate_group<SEG>(arena, arena_bytes, files, wg_file, total_blocks, nw * 64, lane, nxt);
            next_located = true;
        }
#pragma unroll 1
        for (uint32_t cs = 0; cs < S; cs++) {
            const bool more = cs + 1 < S;
            if (more) {
                dma(cs + 1);
            } else if (next_located && nxt.staged) {
                point(nxt);  // the slab is free: segment cs is in R
                dma(0);
            }
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < (int)(SEG / 4); q++) h[q & 3] ^= R[q];
            } else {
#pragma unroll
                for (uint32_t i = 0; i < kChunks; i++) {
                    const uint32_t c = kChunks * cs + i;
                    if (c < nfull) hash_chunk<true>(R + 16 * i, R[16 * i + 16], 0, c, h, s1, t);
                    else if (c == nfull) hash_tail<true>(R + 16 * i, R[16 * i + 16], 0, n, seed, h, s1, t);
                }
            }
            if (more) {
                if (cs + 2 == S && has_next) {
                    // the wave would wait for segment cs + 1 here anyway
                    locate_group<SEG>(arena, arena_bytes, files, wg_file, total_blocks, nw * 64, lane, nxt);
                    next_located = true;
                }
                read_segment();
            }
        }
        pend = true;
        pend_tile = gw;
        pn = n;
        ps1 = s1;
        pt = t;
#pragma unroll
        for (int k = 0; k < 4; k++) ph[k] = h[k];
        if (!has_next) break;
        gw = nw;
        cur = nxt;  // if staged, its segment 0 is in flight (pointed above)
    }
    if (pend) {
        // no DMA in flight: the slab is free
        if (MODE == 0) store_tile_records<2>(out, pend_tile, lane, reinterpret_cast<uint32_t *>(slab), pn, ps1, pt, ph);
        else store_record(out, pend_tile * 64 + lane, pn, ps1, pt, ph);
    }
}
template <int KIND>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_pipe(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    pipe_body<KIND>(arena, arena_bytes, files, wg_file, total_blocks, seed, out);
}

// ---------------------------------------------------------------- read ceilings
// Timing diagnostics only: the fastest way to read the same arena with no
// hashing, i.e. the empirical HBM-read roofline of this box for DESIGN.md.
// LDS = false: coalesced global_load_dwordx4, 4 in flight per lane;
// LDS = true: the same bytes through buffer_load_dwordx4 ... lds.
// MIS: every lane's 16-byte request shifted by 4 bytes (LDS only): the same
// linear stream, misaligned as most quads of 700-byte blocks are.
template <bool LDS, uint32_t MIS = 0>
__global__ __launch_bounds__(256) void diag_linear_read(const uint8_t *__restrict__ arena, uint64_t bytes,
                                                        uint32_t *__restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4 * 4096];
    const uint64_t per_iter = (uint64_t)gridDim.x * 256 * 64;  // 4 x 16 B per lane
    uint32_t acc = 0;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * 64; base + 256 * 64 + MIS <= bytes; base += per_iter) {
        if (LDS) {
            const uint64_t wb = base + wave * 4096;
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void *)(arena + rfl64(wb)), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
            for (int i = 0; i < 4; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    r, (__attribute__((address_space(3))) void *)(buf + wave * 4096 + 1024 * i), 16,
                    (threadIdx.x & 63) * 16 + MIS, 1024 * i, 0, 0);
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

// Timing diagnostic: the park kernel's memory pattern without its hand-off.
// One persistent workgroup per CU (as park), NW streaming waves; chunk c =
// PER KiB of contiguous arena (PER LDS-DMA instructions), chunk c of the
// arena belongs to workgroup c % G and wave (c / G) % NW; a wave keeps DEPTH
// chunks in flight (DEPTH * PER <= 63, the vmcnt cap).  The LDS content is
// discarded (every wave DMAs into the same 64 KiB).
__device__ __forceinline__ uint32_t park_quad_offset(uint32_t idx) {
    const uint32_t j = idx / 45u, u = idx - 45u * j;
    return u < 44u ? 700u * j + 16u * u : 0x80000000u;
}
// PAT = 1: the chunk is a park tile of 64 blocks of 700 bytes (44 800 bytes),
// requested as park requests it (quad u of block j at 700 j + 16 u, the pad
// quad not requested).
template <int NW, int PER, int DEPTH, int PAT = 0>
__global__ __launch_bounds__(512) void diag_stream_read(const uint8_t *__restrict__ arena, uint64_t bytes,
                                                           uint32_t *__restrict__ sink) {
    static_assert(PER * DEPTH <= 63 && PER <= 64, "vmcnt cap");
    static_assert(PAT != 1 || PER == 45, "park tiles are 45 requests");
    // PAT 2 / 3: the staged kernel's pattern at B = 4096 -- chunk = 64
    // pieces of L = 512 / 128 bytes, 4096 bytes apart (segment seg of 64
    // consecutive 4 KiB blocks); PER = 64 L / 1024 requests.  Chunks are
    // dealt round-robin over the chip, so a group's K segments are read at
    // once by K waves.  PAT 4 / 5: the same pieces, but each wave walks one
    // group's segments in order (the staged kernel's temporal order).
    constexpr bool SEQ = PAT >= 4;
    constexpr uint32_t L = (PAT == 2 || PAT == 4) ? 512u : 128u, K = 4096u / L, UPP = L / 16u;
    static_assert(PAT < 2 || PER * 1024 == 64 * L, "one chunk = 64 pieces");
    __shared__ __attribute__((aligned(16))) uint8_t buf[64 * 1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= NW) return;  // idle waves (a launch of more waves than streams)
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t chunk = PAT == 1 ? 64ull * 700 : (uint64_t)PER * 1024;
    const uint64_t nch = PAT >= 2 ? bytes / (64ull * 4096) * K : bytes / chunk;
    const uint32_t G = gridDim.x;
    uint32_t issued = 0;
#pragma unroll 1
    for (uint64_t it = 0;; it++) {
        const uint64_t W = blockIdx.x + (uint64_t)G * wave, T = (uint64_t)G * NW;
        const uint64_t c = SEQ ? (W + T * (it / K)) * K + it % K : W + T * it;
        if (c >= nch) break;
        const uint64_t at = PAT >= 2 ? (c / K) * (64ull * 4096) + (c % K) * L : c * chunk;
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)(arena + rfl64(at)), (short)0, 0x7FFFFFFF, 0x00020000);
        if constexpr (PAT >= 2) {
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const uint32_t idx = 64u * i + lane;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(buf + 1024 * i),
                                                         16, (idx / UPP) * 4096u + (idx % UPP) * 16u, 0, 0, 2);
            }
        } else if constexpr (PAT != 0) {
#pragma unroll
            for (int i = 0; i < PER; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(buf + 1024 * i),
                                                         16, park_quad_offset(64u * i + lane), 0, 0, 2);
        } else {
#pragma unroll
            for (int i = 0; i < PER; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(buf + 1024 * i),
                                                         16, lane * 16 + 1024 * i, 0, 0, 2);
        }
        if (++issued >= DEPTH) {
            if constexpr (DEPTH == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if constexpr (DEPTH == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (buf[threadIdx.x] == 0x5a && buf[threadIdx.x + 1] == 0xa5 && bytes == 1) sink[0] = 1;
}

// Timing diagnostic: the stream above plus the records' write stream.  3
// waves, chunk = one park tile (64 x 700 bytes, 45 DMA instructions); per
// chunk 1280 bytes of "records" are due at out + 1280 * chunk.  ASSIGN 0:
// chunk c belongs to workgroup c % G (park's order); 1: workgroup w owns the
// contiguous chunks [w n / G, (w + 1) n / G).  WB: chunks whose records a wave
// writes at once (coalesced nt 16-byte stores; with ASSIGN 1 they are
// contiguous in the output, with ASSIGN 0 they are 1280-byte pieces).
template <int ASSIGN, int WB>
__global__ __launch_bounds__(512) void diag_stream_rw(const uint8_t *__restrict__ arena, uint64_t bytes,
                                                      uint8_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[64 * 1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 3) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t chunk = 64ull * 700;
    const uint64_t nch = bytes / chunk;
    const uint32_t G = gridDim.x;
    // ASSIGN 1: the workgroup's range split again into one contiguous range per wave
    const uint64_t w0 = nch * blockIdx.x / G, w1 = nch * (blockIdx.x + 1) / G;
    const uint64_t c0 = ASSIGN ? w0 + (w1 - w0) * wave / 3 : blockIdx.x + (uint64_t)G * wave;
    const uint64_t c1 = ASSIGN ? w0 + (w1 - w0) * (wave + 1) / 3 : nch;
    const uint64_t step = ASSIGN ? 1 : 3ull * G;
    uint32_t pending = 0;
    uint64_t first = 0;
#pragma unroll 1
    for (uint64_t c = c0; c < c1; c += step) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)(arena + rfl64(c * chunk)), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int i = 0; i < 45; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(buf + 1024 * i), 16,
                                                     park_quad_offset(64u * i + lane), 0, 0, 2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (pending == 0) first = c;
        if (++pending == WB || c + step >= c1) {
            // this wave's records of its `pending` last chunks
            const u32x4v v = reinterpret_cast<const u32x4v *>(buf)[lane];
            if (ASSIGN) {  // the pending chunks are consecutive: one contiguous burst
                u32x4a4 *o = reinterpret_cast<u32x4a4 *>(out + first * 1280ull);
                for (uint32_t q = lane; q < 80u * pending; q += 64)
                    __builtin_nontemporal_store(u32x4a4{v.x, v.y, v.z, v.w}, o + q);
            } else {
                for (uint32_t k = 0; k < pending; k++) {
                    u32x4a4 *o = reinterpret_cast<u32x4a4 *>(out + (first + (uint64_t)k * step) * 1280ull);
                    __builtin_nontemporal_store(u32x4a4{v.x, v.y, v.z, v.w}, o + lane);
                    if (lane < 16) __builtin_nontemporal_store(u32x4a4{v.x, v.y, v.z, v.w}, o + 64 + lane);
                }
            }
            pending = 0;
        }
    }
}

// ---------------------------------------------------------------- park variant (loader + register park)
// For blocks of at most kRegMaxBytes (703: the reference's 700-byte blocks).
// Every byte should cross HBM once, in long runs: a tile = 64 consecutive
// blocks (45 KiB) is fetched as one near-linear LDS-DMA burst, and each
// block then parks in its lane's VGPRs (176 registers) while it is hashed,
// so LDS only holds tiles in transit.  One persistent 8-wave workgroup per CU:
//   waves 0..NL-1 (loaders; NL = 3: one per slot of the 3-slot ring) locate
//     their tiles (scalar loads, no vmcnt coupling with the DMA), write the
//     block lengths to LDS and DMA the tile.  A wave's vmcnt is a 6-bit
//     counter (at most 63 DMA instructions = 63 KiB in flight per wave), so
//     one loader cannot keep the ring full: three loaders keep up to three
//     tiles (135 KiB) in flight per CU;
//   the other waves (hashers) take tiles in order by an LDS ticket, copy the
//     slot into registers, free it, hash 64 blocks and store the records.
// LDS handshake per slot: full[s] = the ticket it holds (set by the loader
// after its covering vmcnt), freeq[s] = the ticket it may take next (set by
// the hasher once its ds_reads of the slot completed).  Tiles that cannot be
// staged (the batch's partial last tile, a tile whose 704-byte reads would
// run past the arena, a span past a 31-bit offset) are marked direct: the
// hasher locates and loads its blocks itself.
constexpr uint32_t kRegChunks = 11;                      // data chunks parked per lane
constexpr uint32_t kRegMaxBytes = 64 * kRegChunks - 1;   // 703: tail chunk index <= 10
constexpr uint32_t kParkMinBytes = 512;                  // shorter blocks waste the 720-byte slots
constexpr uint32_t kPkPiece = 720;                // LDS bytes per block (44 data quads + 1 pad quad)
constexpr uint32_t kPkTile = 64 * kPkPiece;       // 46080 B
constexpr uint32_t kPkDma = kPkTile / 1024;       // 45 DMA instructions per tile
constexpr uint32_t kPkSlots = 3;
constexpr uint32_t kPkWaves = 8;
constexpr uint32_t kPkThreads = 64 * kPkWaves;
static_assert(kPkTile % 1024 == 0 && kPkPiece % 16 == 0, "tile = whole DMA instructions");

constexpr uint32_t kRecRing = 16;  // tiles of records the workgroup stages (REC 6); two groups of 8
struct PkShared {
    uint8_t tile[kPkSlots][kPkTile];
    // REC 1..5: wave w's 64 records (20 B each) at rec[320 w]; REC 6: a ring
    // of kRecRing tiles' records, ticket k's at rec[320 (k % kRecRing)]
    uint32_t rec[kRecRing * 64 * 5];
    uint32_t ring_kind[kRecRing];  // REC 6: 1 = flush the slot's records, 0 = written directly
    uint32_t ring_done[2];         // REC 6: tiles of the group (8 tickets) whose records are in
    uint32_t ring_flushed[2];      // REC 6: the last group flushed from each half of the ring
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
        return;
    }
    const uint64_t gend = min(g0 + 64, total_blocks);
    const uint32_t fmax = wg_file[nwg256];  // the batch's last block's file: no tile needs a later one
    uint64_t off = 0;
    uint32_t n = 0;
    // The tile's lowest block offset, its highest block offset + 704 and its
    // largest block length, from the descriptors (wave-uniform, scalar
    // arithmetic: no cross-lane reductions, whose serialized bpermutes cost
    // the loader ~1 us per tile).  Within a file, offsets grow with the block
    // index; the largest B bounds every n.
    uint64_t lo_off = ~0ull, top = 0;
    uint32_t bmax = 0;
    // Small files (cfg4: 4-64 KiB) put up to ~11 files in a tile: four
    // descriptors per step, their scalar loads issued together.
    bool done = false;
#pragma unroll 1
    for (uint32_t f = __builtin_amdgcn_readfirstlane(lo); !done; f += 4) {
        DevFile F[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) F[i] = files[min(f + i, fmax)];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            if (done) break;
            const uint64_t fb = F[i].first_block, fe = fb + F[i].nblocks;
            if (g >= fb && g < fe) {
                const uint64_t boff = (g - fb) * F[i].blen;
                const uint64_t left = F[i].len - boff;
                n = left < F[i].blen ? (uint32_t)left : F[i].blen;  // generator.go:334
                off = F[i].offset + boff;
            }
            if (fe > fb && fe > g0 && fb < gend) {  // the file has blocks in this tile
                const uint64_t b_first = (g0 > fb ? g0 : fb) - fb, b_last = (gend < fe ? gend : fe) - 1 - fb;
                const uint64_t o_first = F[i].offset + b_first * F[i].blen;
                const uint64_t o_top = F[i].offset + b_last * F[i].blen + 704u;
                lo_off = o_first < lo_off ? o_first : lo_off;
                top = o_top > top ? o_top : top;
                bmax = F[i].blen > bmax ? F[i].blen : bmax;
            }
            done = fe >= gend || f + i >= fmax;
        }
    }
    d.base = rfl64(lo_off);
    top = rfl64(top);
    bmax = rfl32(bmax);
    d.staged = (g0 + 64 <= total_blocks) && bmax <= kRegMaxBytes && top <= arena_bytes &&
               top - d.base <= 0x7FFFFFFFull;
    d.off = off;
    d.n = n;
    d.B = 0;
}

// Issue the 45 LDS-DMA instructions of a staged tile into dst.  Instruction
// i, lane l fills dst bytes [1024 i + 16 l, +16): block j = (64 i + l) / 45,
// quad u = (64 i + l) % 45 (u = 44 is the pad).  Quads past the block's
// bytes and the pad get an offset past num_records: no memory request.
// jj/uu: per-lane block index and byte offset (0x40000000 for the pad) of
// each instruction, precomputed by the loader (UNROLL); otherwise computed on
// the fly (a caller short of VGPRs).
template <int AUX, bool UNROLL, bool ALN = false>
__device__ __forceinline__ void pk_issue(const uint8_t *arena, uint8_t *dst, const PkDesc &d, uint32_t lane,
                                         const uint32_t *jj = nullptr, const uint32_t *uu = nullptr) {
    // ALN (timing diagnostic only): every quad request rounded down to a
    // 16-byte boundary of the arena -- the same bytes per tile, naturally
    // aligned, to price the misaligned quads of blocks at a 700-byte stride
    const uint32_t amis = ALN ? (uint32_t)(d.base & 15u) : 0u;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + (d.base - amis)), (short)0, 0x7FFFFFFF, 0x00020000);
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
            vo_ = u16_ < nj_ ? (ALN ? ((d.B * j_ + u16_ + amis) & ~15u) : d.B * j_ + u16_) : 0x80000000u;     \
        } else {                                                                                                \
            const uint32_t rj_ = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j_), rel);                  \
            const uint32_t nj_ = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j_), (int)d.n);             \
            vo_ = u16_ < nj_ ? rj_ + u16_ : 0x80000000u;                                                        \
        }                                                                                                       \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * (I_)), \
                                                 16, vo_, 0, 0, AUX);                                           \
    } while (0)
    // the regular/irregular choice is made once per tile (a branch per
    // instruction costs an lgkmcnt wait per instruction)
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
            // Irregular tile: each instruction's offsets come from two
            // ds_bpermutes.  Issued one instruction at a time, every DMA waits
            // for its own bpermutes (an lgkmcnt wait per instruction, the LDS
            // busy with DMA writes and the hashers' copy-out); in batches of 9
            // the 18 bpermutes go out back to back and the 9 DMAs follow.
            constexpr uint32_t kBatch = 9;
            static_assert(kPkDma % kBatch == 0, "whole batches");
#pragma unroll
            for (uint32_t i0 = 0; i0 < kPkDma; i0 += kBatch) {
                uint32_t rj[kBatch], nj[kBatch];
#pragma unroll
                for (uint32_t k = 0; k < kBatch; k++) {
                    rj[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * jj[i0 + k]), rel);
                    nj[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * jj[i0 + k]), (int)d.n);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (uint32_t k = 0; k < kBatch; k++) {
                    const uint32_t u16 = uu[i0 + k];
                    const uint32_t vo = u16 < nj[k] ? (ALN ? ((rj[k] + u16 + amis) & ~15u) : rj[k] + u16) : 0x80000000u;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * (i0 + k)), 16, vo, 0, 0, AUX);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll 1
            for (uint32_t i = 0; i < kPkDma; i++) RSG_PK_ONE(i, false);
        }
    }
#undef RSG_PK_ONE
}

// Register-staged tile (park LDR = 1): the same 45 requests as pk_issue, but
// into the loader's VGPRs (R[i] = the 16 bytes DMA instruction i would put at
// slot bytes [1024 i + 16 l, +16)), so a tile can be in flight while the
// loader's slot still holds the previous one; pk_reg_store writes it to the
// slot once that is freed.  Block j / quad offset u16 of request i are stepped
// instead of tabulated (the tables would cost 90 VGPRs next to R's 180):
// index 64 i + l advances by 64 = 45 + 19 per request.  Out-of-range requests
// (quads past the block, the pad) return zeros and fetch nothing.
template <int AUX>
__device__ __forceinline__ void pk_reg_issue(const uint8_t *arena, const PkDesc &d, uint32_t lane, u32x4v R[kPkDma]) {
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + d.base), (short)0, 0x7FFFFFFF, 0x00020000);
    uint32_t j = lane / 45u;
    uint32_t u16 = 16u * (lane - 45u * j);
    // opaque to the optimiser: the stepped (j, u16) sequence is the same for
    // every tile, and hoisting all 45 steps out of the loader's loop costs
    // ~90 registers (spills) to save ~5 VALU per request
    asm volatile("" : "+v"(j), "+v"(u16));
    if (d.regular) {
        uint32_t off = d.B * j + u16;  // = B j + u16, stepped with j and u16
#pragma unroll
        for (uint32_t i = 0; i < kPkDma; i++) {
            const uint32_t nj = j == d.jl ? d.nl : d.B;
            R[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, u16 < nj ? off : 0x80000000u, 0, AUX);
            const bool wrap = u16 >= 720u - 304u;
            u16 = wrap ? u16 - 416u : u16 + 304u;
            j += wrap ? 2u : 1u;
            off += wrap ? 2u * d.B - 416u : d.B + 304u;
        }
    } else {
        const int rel = (int)(uint32_t)(d.off - d.base);
        constexpr uint32_t kBatch = 9;  // bpermutes issued back to back, then the loads (pk_issue)
#pragma unroll
        for (uint32_t i0 = 0; i0 < kPkDma; i0 += kBatch) {
            uint32_t rj[kBatch], nj[kBatch], uq[kBatch];
#pragma unroll
            for (uint32_t k = 0; k < kBatch; k++) {
                rj[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j), rel);
                nj[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * j), (int)d.n);
                uq[k] = u16;
                const bool wrap = u16 >= 720u - 304u;
                u16 = wrap ? u16 - 416u : u16 + 304u;
                j += wrap ? 2u : 1u;
            }
#pragma unroll
            for (uint32_t k = 0; k < kBatch; k++)
                R[i0 + k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, uq[k] < nj[k] ? rj[k] + uq[k] : 0x80000000u,
                                                                   0, AUX);
        }
    }
    __builtin_amdgcn_sched_barrier(0);  // the loads stay here, ahead of the caller's slot wait
}

__device__ __forceinline__ void pk_reg_store(uint8_t *dst, uint32_t lane, const u32x4v R[kPkDma]) {
#pragma unroll
    for (uint32_t i = 0; i < kPkDma; i++) *reinterpret_cast<u32x4v *>(dst + 1024u * i + 16u * lane) = R[i];
}

// LDR = 2: store R (the landed tile) into the slot request by request, each
// register refilled with the next tile's request as soon as it is stored, so
// the loader's 45 requests stay in flight across the hand-off.
template <int AUX>
__device__ __forceinline__ void pk_reg_swap(uint8_t *dst, const uint8_t *arena, const PkDesc &d, uint32_t lane,
                                            u32x4v R[kPkDma]) {
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + d.base), (short)0, 0x7FFFFFFF, 0x00020000);
    uint32_t j = lane / 45u;
    uint32_t u16 = 16u * (lane - 45u * j);
    asm volatile("" : "+v"(j), "+v"(u16));
    uint32_t off = d.B * j + u16;
#pragma unroll
    for (uint32_t i = 0; i < kPkDma; i++) {
        *reinterpret_cast<u32x4v *>(dst + 1024u * i + 16u * lane) = R[i];
        const uint32_t nj = j == d.jl ? d.nl : d.B;
        R[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, u16 < nj ? off : 0x80000000u, 0, AUX);
        const bool wrap = u16 >= 720u - 304u;
        u16 = wrap ? u16 - 416u : u16 + 304u;
        j += wrap ? 2u : 1u;
        off += wrap ? 2u * d.B - 416u : d.B + 304u;
    }
    __builtin_amdgcn_sched_barrier(0);
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

// REC 6: the workgroup's records leave in bursts of 8 tiles.  Writing them
// tile by tile interleaves a small write with the reads every ~2 us per CU,
// and HBM pays for every read/write switch (a bare
// 3-wave reader with 1 280 bytes of records per tile 0.185 ms, the same
// records written 8 tiles at a time 0.169, reads alone 0.150).  Ticket k's
// records go to ring slot k % 16 (a group = tickets 8m .. 8m + 7, its half
// m % 2); the hasher that completes a group writes its tiles' records (8
// separate 1 280-byte pieces of the output) as coalesced nt stores and
// releases the half.  A hasher waits for its half's previous group (m - 2)
// to be flushed before writing into it: groups complete in ticket order up
// to the hashers in flight, so that wait is on older tickets only.
// put = false: a direct tile whose lanes stored their records themselves.
__device__ __forceinline__ void pk_ring_put(PkShared &sh, uint32_t k, uint64_t t, uint32_t G, uint64_t ntiles,
                                            uint32_t lane, uint32_t n, int32_t s1, uint32_t tw, const uint32_t h[4],
                                            uint8_t *__restrict__ out, bool put) {
    const uint32_t r = k % kRecRing, m = k / 8u, half = m & 1u;
    while (pk_load(&sh.ring_flushed[half]) != m - 2u) __builtin_amdgcn_s_sleep(1);
    if (put) {
        const uint32_t s2 = n * (uint32_t)s1 - tw;
        uint32_t *rec = &sh.rec[320u * r + 5u * lane];
        rec[0] = ((uint32_t)s1 & 0xffffu) | (s2 << 16);  // rsyncchecksum.go:50
        rec[1] = h[0];
        rec[2] = h[1];
        rec[3] = h[2];
        rec[4] = h[3];
    }
    // Every branch below is on wave-uniform scalars and the single-lane
    // stores are written by all lanes (same value): a lane-0-only store next
    // to the early return let the compiler split the wave at the loop exit
    // (lanes 1-63 ran on into the next ticket without lane 0: deadlock).
    sh.ring_kind[r] = put ? 1u : 0u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&sh.ring_done[half], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    // this workgroup's tickets: t = blockIdx.x + k G < ntiles
    const uint64_t nk = (ntiles - blockIdx.x + G - 1) / G;
    const uint64_t left = nk - 8ull * m;
    const uint32_t gsize = __builtin_amdgcn_readfirstlane(left < 8 ? (uint32_t)left : 8u);
    if (old + 1 != gsize) return;
    // the group's last tile: flush the group
    for (uint32_t j = 0; j < gsize; j++) {
        const uint32_t kk = 8u * m + j, rr = kk % kRecRing;
        if (!__builtin_amdgcn_readfirstlane(sh.ring_kind[rr])) continue;
        const uint64_t tt = blockIdx.x + (uint64_t)kk * G;
        const u32x4v* src = reinterpret_cast<const u32x4v *>(&sh.rec[320u * rr]);
        u32x4a4 *dst = reinterpret_cast<u32x4a4 *>(out + tt * (64ull * kRecordBytes));
        const u32x4v a = src[lane];
        __builtin_nontemporal_store(u32x4a4{a.x, a.y, a.z, a.w}, dst + lane);
        if (lane < 16) {
            const u32x4v b = src[64 + lane];
            __builtin_nontemporal_store(u32x4a4{b.x, b.y, b.z, b.w}, dst + 64 + lane);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the ring's reads are done before the half is released
    sh.ring_done[half] = 0;
    pk_store(&sh.ring_flushed[half], m);
}

// MODE 0 = product; diagnostics: 1 = memory only (DMA + copy, no hashing),
// 2 = hashing only (no DMA: the hashers hash whatever the slots hold),
// 3 = memory only with every quad request 16-byte aligned (ALN above).
// The tile DMA uses the nt cache policy (aux = 2): every byte is read once.
// (A/B, profiles/r02f_ab_park_cache_policy*.json: the default policy, sc0 or
// sc1 alone cost 6-9 %; nt combined with sc0 / sc1 equals nt.)
// NL = loader waves (1 or 2); the other 8 - NL waves hash.
// PRIO: wave priorities (s_setprio) -- 0 = none; 3 (the product) = loader
// waves at priority 3 (a slot's next DMA issues ahead of the hasher sharing
// the SIMD) and hashers at 3 while they copy a slot out (the slot frees
// sooner), 0 while they hash.  (8-round A/B, profiles/r04f_ab_park_prio.json:
// none 0.1984 ms, loaders only 0.1962, copy-out at 2 0.1950, at 3 0.1942;
// raising the hasher already while it waits for its slot: no gain,
// profiles/r04g_ab_park_prio_ticket.json.)
// LDR: 0 = each loader DMAs its tile into the slot once the slot is freed;
// 1 = register-staged loaders (pk_reg_issue): a loader's next tile is loaded
// into its VGPRs right after it publishes the current one, so the HBM latency
// overlaps the slot's hand-off to a hasher, and a freed slot is refilled by
// 45 ds_write_b128 instead of waiting out a DMA.
// REC: 0 = each lane stores its own 20-byte record (store_record); 1 / 2 =
// a staged tile's 64 records through LDS as coalesced 16-byte stores
// (store_tile_records; 2 = nontemporal).
template <int MODE, int NL, int AUX, int PRIO = 0, int LDR = 0, int REC = 0>
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
    if (threadIdx.x < 2) {
        sh.ring_done[threadIdx.x] = 0;
        sh.ring_flushed[threadIdx.x] = threadIdx.x - 2u;  // "group -2 / -1 flushed": both halves free
    }
    if (threadIdx.x == 0) sh.ticket = 0;
    __syncthreads();
    const uint64_t ntiles = (total_blocks + 63) / 64;
    const uint32_t G = gridDim.x;  // one persistent workgroup per CU; tile t belongs to workgroup t % G

    if (LDR >= 1 && wave < NL) {
        static_assert(LDR == 0 || NL == (int)kPkSlots, "register-staged loaders own one slot each");
        if (PRIO >= 3) __builtin_amdgcn_s_setprio(3);
        // loader L owns slot L and the tickets k = L mod 3
        const uint32_t slot = wave;
        uint32_t k = wave;
        uint64_t t = blockIdx.x + (uint64_t)k * G;
        PkDesc cur, nxt;
        u32x4v R[kPkDma];
        bool held = false;  // R holds (or is loading) cur's tile
        if (t < ntiles) {
            pk_locate(t, cur, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
            if (cur.staged && MODE != 2) {
                pk_reg_issue<AUX>(arena, cur, lane, R);
                held = true;
            }
        }
#pragma unroll 1
        while (t < ntiles) {
            const uint64_t tn = t + (uint64_t)kPkSlots * G;
            // the next tile's descriptor (scalar loads) while this one is in flight
            if (tn < ntiles) pk_locate(tn, nxt, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
            while (pk_load(&sh.freeq[slot]) != k) __builtin_amdgcn_s_sleep(1);
            sh.n[slot][lane] = cur.n;
            if (lane == 0) sh.kind[slot] = cur.staged ? 1u : 0u;
            bool swapped = false;
            if (LDR == 2 && held && tn < ntiles && nxt.staged && nxt.regular) {
                pk_reg_swap<AUX>(&sh.tile[slot][0], arena, nxt, lane, R);
                swapped = true;
            } else if (held) {
                pk_reg_store(&sh.tile[slot][0], lane, R);
            }
            if (LDR == 2) {
                // only the slot's LDS writes must land before the publish; the
                // next tile's requests stay in flight
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(&sh.full[slot], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                if (lane == 0) pk_store(&sh.full[slot], k);
            }
            k += kPkSlots;
            t = tn;
            cur = nxt;
            held = swapped;
            if (!swapped && t < ntiles && cur.staged && MODE != 2) {
                pk_reg_issue<AUX>(arena, cur, lane, R);
                held = true;
            }
        }
        return;
    }
    if (wave < NL) {
        if (PRIO >= 3) __builtin_amdgcn_s_setprio(3);
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
        // Loader L owns the slots s with s % NL == L and loads the tickets k
        // whose slot k % 3 it owns (NL = 2: loader 0 slots 0 and 2, loader 1
        // slot 1), so each loader's tiles sit in its own vmcnt.
        auto owned = [&](uint32_t kk) { return (kk % kPkSlots) % NL == wave; };
        uint32_t nown = 0;  // slots this loader owns
        for (uint32_t sl = 0; sl < kPkSlots; sl++) nown += (sl % NL == wave) ? 1u : 0u;
        const bool single = nown == 1;
        uint32_t k = 0;
        while (!owned(k)) k++;
        PkDesc cur;
        uint64_t t = blockIdx.x + (uint64_t)k * G;
        if (t < ntiles) pk_locate(t, cur, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
        bool have_prev = false;
        uint32_t prev = 0;
#pragma unroll 1
        while (t < ntiles) {
            const uint32_t slot = k % kPkSlots;
            // the slot's previous tile must have been copied out by its hasher
            while (pk_load(&sh.freeq[slot]) != k) __builtin_amdgcn_s_sleep(1);
            sh.n[slot][lane] = cur.n;
            if (lane == 0) sh.kind[slot] = cur.staged ? 1u : 0u;
            const bool staged = cur.staged;
            if (staged && MODE != 2) pk_issue<AUX, true, MODE == 3>(arena, &sh.tile[slot][0], cur, lane, jj, uu);
            uint32_t kn = k + 1;
            while (!owned(kn)) kn++;
            const uint64_t tn = blockIdx.x + (uint64_t)kn * G;
            // next tile's descriptor (scalar loads) while this one and the
            // previous one are in flight
            if (tn < ntiles) pk_locate(tn, cur, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
            if (single) {
                // one slot: publish this tile before waiting for the slot again
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) pk_store(&sh.full[slot], k);
            } else if (have_prev) {
                // publish the previous tile once its DMA has landed.  vmcnt is
                // a 6-bit counter: a wave cannot have more than 63 DMA
                // instructions (63 KiB) in flight, so waiting for an older
                // tile instead stalls the issue of this one (measured slower).
                if (staged) asm volatile("s_waitcnt vmcnt(45)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) pk_store(&sh.full[prev % kPkSlots], prev);
            }
            have_prev = true;
            prev = k;
            k = kn;
            t = tn;
        }
        if (!single && have_prev) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) pk_store(&sh.full[prev % kPkSlots], prev);
        }
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
        if (PRIO >= 3) __builtin_amdgcn_s_setprio(3);
        const uint32_t n = sh.n[slot][lane];
        const uint32_t kind = __builtin_amdgcn_readfirstlane(sh.kind[slot]);
        const uint64_t g = t * 64 + lane;
        if (kind) {
            uint32_t h[4];
            md4_init(h);
            int32_t s1 = 0;
            uint32_t tw = 0;
            uint32_t R[16 * kRegChunks];
            const uint8_t *mine = &sh.tile[slot][0] + lane * kPkPiece;
#pragma unroll
            for (uint32_t q = 0; q < (MODE == 4 ? 1 : 4 * kRegChunks); q++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * q);
                R[4 * q + 0] = v.x; R[4 * q + 1] = v.y; R[4 * q + 2] = v.z; R[4 * q + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) pk_store(&sh.freeq[slot], k + kPkSlots);
            if (PRIO >= 3) __builtin_amdgcn_s_setprio(0);
            const uint32_t nfull = n >> 6;
            if (MODE == 1 || MODE == 3 || MODE == 5) {
#pragma unroll
                for (int q = 0; q < 16 * (int)kRegChunks; q++) h[q & 3] ^= R[q];
            } else if (MODE == 4) {
                h[0] ^= R[0];
            } else {
#pragma unroll
                for (uint32_t c = 0; c < kRegChunks; c++) {
                    if (c < nfull) hash_chunk<true>(R + 16 * c, 0u, 0u, c, h, s1, tw);
                    else if (c == nfull) hash_tail<true>(R + 16 * c, 0u, 0u, n, seed, h, s1, tw);
                }
            }
            if (MODE == 5 && h[0] != 0x9e3779b9u) {
                // diagnostic: no record stores
            } else if (REC == 6) {
                pk_ring_put(sh, k, t, G, ntiles, lane, n, s1, tw, h, out, true);
            } else if (REC == 3) {
                store_record_nt(out, g, n, s1, tw, h);
            } else if (REC >= 1) {
                store_tile_records<REC>(out, t, lane, &sh.rec[320u * wave], n, s1, tw, h);
            } else {
                store_record(out, g, n, s1, tw, h);
            }
        } else {
            if (PRIO >= 3) __builtin_amdgcn_s_setprio(0);
            if (lane == 0) {
                pk_store(&sh.freeq[slot], k + kPkSlots);
                if (MODE == 0 && t * 64 + 64 <= total_blocks) count_fallback(1);
            }
            if (g < total_blocks) pk_direct(arena, arena_bytes, files, wg_file, nwg256, g, seed, out);
            if (REC == 6) {
                const uint32_t z[4] = {0, 0, 0, 0};
                pk_ring_put(sh, k, t, G, ntiles, lane, 0, 0, 0, z, out, false);  // its records are out already
            }
        }
    }
}

// ------------------------------------------------------------- long park
// Park's streaming ring for blocks longer than a slot (B > 703, variant 12).
// The staged kernel reads such blocks 128 or 256 bytes of each of a wave's 64
// blocks at a time, and at B = 4096 those short pieces bound it (0.22 ms per
// GiB; a bare reader with 512-byte pieces of the same 64 blocks 4 KiB apart
// takes 0.149, profiles/r05y_b4096_stream_patterns.jsonl).  Here a tile is
// segment s (704 bytes: 11 chunks) of each of a 64-block group's blocks,
// streamed through park's three LDS slots by its three loader waves; a
// hasher copies its lane's 704 bytes out as park's do.  A block's MD4 state
// crosses tiles in LDS: a workgroup keeps kLpGroups groups in flight, and
// its tickets run segment-major over them (batch b, segment s, group slot q:
// k = (b S + s) kLpGroups + q), so consecutive tickets are different groups
// and the hasher of (q, s) waits only for (q, s - 1), finished kLpGroups
// tickets earlier (done[q] counts the slot's finished tickets).  S =
// segments of the batch's longest block (max_blen): tiles of shorter blocks
// request no bytes past them and hash nothing.  A group of several files'
// blocks takes per-lane offsets (ds_bpermute per request, as park's
// irregular tiles); only a partial last group, or one whose span does not
// fit a buffer offset, takes the per-lane path at its segment 0.
constexpr uint32_t kLpSeg = 64 * kRegChunks;  // 704 bytes of each block per tile
constexpr uint32_t kLpGroups = 6;
struct LpShared {
    uint8_t tile[kPkSlots][kPkTile];
    uint32_t rec[kPkWaves - 3][320];        // hashers' record staging (store_tile_records)
    uint32_t st[kLpGroups][6][64];          // per group slot: h0..h3, s1, t of each lane's block
    uint32_t n[kPkSlots][64];
    uint32_t full[kPkSlots], freeq[kPkSlots], kind[kPkSlots];
    uint32_t done[kLpGroups];
    uint32_t ticket;
};

template <int MODE>
__global__ __launch_bounds__(kPkThreads) void block_sums_lpark(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t max_blen, uint32_t seed,
    uint8_t *__restrict__ out) {
    constexpr uint32_t NL = 3;
    __shared__ __attribute__((aligned(16))) LpShared sh;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < kPkSlots) {
        sh.full[threadIdx.x] = ~0u;
        sh.freeq[threadIdx.x] = threadIdx.x;
    }
    if (threadIdx.x < kLpGroups) sh.done[threadIdx.x] = 0;
    if (threadIdx.x == 0) sh.ticket = 0;
    __syncthreads();
    const uint64_t ngroups = (total_blocks + 63) / 64;
    const uint32_t G = gridDim.x;
    // this workgroup's groups: gw = blockIdx.x + G m, m < M
    // 32-bit ticket arithmetic: the launch checks that every count fits
    const uint32_t M = ngroups > blockIdx.x ? (uint32_t)((ngroups - blockIdx.x + G - 1) / G) : 0u;
    const uint32_t S = (max_blen >> 6) / kRegChunks + 1;  // segments through the longest block's tail chunk
    const uint32_t SG = S * kLpGroups;
    const uint32_t ntk = (M + kLpGroups - 1) / kLpGroups * SG;
    auto decode = [&](uint32_t k, uint32_t &sg, uint32_t &q, uint32_t &m, uint32_t &b) {
        b = k / SG;
        const uint32_t r = k - b * SG;
        sg = r / kLpGroups;
        q = r - sg * kLpGroups;
        m = b * kLpGroups + q;
    };

    if (wave < NL) {
        __builtin_amdgcn_s_setprio(3);
        // loader L fills slot L with the tickets k = L mod 3.  The next
        // ticket's descriptor (pk_locate: a chain of scalar loads, a few us)
        // is built while this ticket's DMA is in flight, as park's loaders do.
        auto prepare = [&](uint32_t k, PkDesc &d, uint32_t &kind, uint32_t &sg) {
            uint32_t q, m, b;
            decode(k, sg, q, m, b);
            kind = 2;  // nothing to load or hash
            d.n = 0;
            if (m < M) {
                const uint64_t gw = blockIdx.x + (uint64_t)G * m;
                pk_locate(gw, d, lane, files, wg_file, nwg256, total_blocks, arena_bytes);
                const bool full = gw * 64 + 64 <= total_blocks;
                bool ok;
                // every 16-byte request inside the arena: a block's last
                // request may run up to 15 bytes past its end
                if (d.regular) {
                    const uint32_t n63 = d.jl == 63 ? d.nl : d.B;  // lane 63's block: the file's last, or a whole one
                    ok = full && (uint64_t)d.B * 64 <= 0x7FFFFFFFull &&
                         d.base + (uint64_t)d.B * 63 + ((n63 + 15u) & ~15u) <= arena_bytes;
                } else {
                    // blocks of several files: per-lane offsets (pk_locate's base is the lowest)
                    const uint64_t top = rfl64(wave_max_u64(d.n ? d.off + ((d.n + 15u) & ~15u) : 0));
                    ok = full && top <= arena_bytes && top - d.base <= 0x7FFFFFFFull;
                }
                kind = ok ? 1u : (sg == 0 ? 0u : 2u);
            }
        };
        // request i, lane l: block j = (64 i + l) / 45, 16-byte unit u (44 = the pad)
        uint32_t jj[kPkDma], uu[kPkDma];
#pragma unroll
        for (uint32_t i = 0; i < kPkDma; i++) {
            const uint32_t idx = 64u * i + lane;
            jj[i] = idx / 45u;
            const uint32_t u = idx - 45u * jj[i];
            uu[i] = u < 44u ? 16u * u : 0x40000000u;  // past every block length
        }
        uint32_t k = wave;
        PkDesc cur, nxt;
        uint32_t kind = 2, sg = 0;
        if (k < ntk) prepare(k, cur, kind, sg);
#pragma unroll 1
        while (k < ntk) {
            const uint32_t slot = k % kPkSlots;
            while (pk_load(&sh.freeq[slot]) != k) __builtin_amdgcn_s_sleep(1);
            sh.n[slot][lane] = cur.n;
            if (lane == 0) sh.kind[slot] = kind;
            if (kind == 1 && MODE != 2) {
                // segment sg of block j: bytes [sg 704, +704) of the block, none past its end
                const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(arena + cur.base + (uint64_t)sg * kLpSeg), (short)0, 0x7FFFFFFF, 0x00020000);
                const uint32_t so = sg * kLpSeg;
                const int rel = (int)(uint32_t)(cur.off - cur.base);
                if (cur.regular) {
                    // the bytes of block j left from segment sg on (0 past its end)
                    const uint32_t nB = cur.B > so ? cur.B - so : 0u, nL = cur.nl > so ? cur.nl - so : 0u;
#pragma unroll
                    for (uint32_t i = 0; i < kPkDma; i++) {
                        const uint32_t left = jj[i] == cur.jl ? nL : nB;
                        const uint32_t vo = uu[i] < left ? cur.B * jj[i] + uu[i] : 0x80000000u;
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rsrc, (__attribute__((address_space(3))) void *)(&sh.tile[slot][0] + 1024u * i), 16, vo, 0, 0, 2);
                    }
                } else {
                    // (unrolled: a dynamically indexed jj / uu would live in scratch memory)
#pragma unroll
                    for (uint32_t i = 0; i < kPkDma; i++) {
                        const uint32_t rj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * jj[i]), rel);
                        const uint32_t nj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * jj[i]), (int)cur.n);
                        const uint32_t vo = (uu[i] < 0x40000000u && so + uu[i] < nj) ? rj + uu[i] : 0x80000000u;
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rsrc, (__attribute__((address_space(3))) void *)(&sh.tile[slot][0] + 1024u * i), 16, vo, 0, 0, 2);
                    }
                }
            }
            const uint32_t kn = k + kPkSlots;
            uint32_t kind_n = 2, sg_n = 0;
            if (kn < ntk) prepare(kn, nxt, kind_n, sg_n);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            if (lane == 0) pk_store(&sh.full[slot], k);
            k = kn;
            cur = nxt;
            kind = kind_n;
            sg = sg_n;
        }
        return;
    }

    // ---------------------------------------------------------------- hashers
    uint32_t *rec = &sh.rec[wave - NL][0];
#pragma unroll 1
    for (;;) {
        uint32_t kk = 0;
        if (lane == 0) kk = __hip_atomic_fetch_add(&sh.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t k = __builtin_amdgcn_readfirstlane(kk);
        if (k >= ntk) break;
        const uint32_t slot = k % kPkSlots;
        uint32_t sg, q, m, b;
        decode(k, sg, q, m, b);
        while (pk_load(&sh.full[slot]) != k) __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_s_setprio(3);
        const uint32_t n = sh.n[slot][lane];
        const uint32_t kind = __builtin_amdgcn_readfirstlane(sh.kind[slot]);
        uint32_t R[16 * kRegChunks];
        if (kind == 1) {
            const uint8_t *mine = &sh.tile[slot][0] + lane * kPkPiece;
#pragma unroll
            for (uint32_t qd = 0; qd < 4 * kRegChunks; qd++) {
                const uint4 v = *reinterpret_cast<const uint4 *>(mine + 16 * qd);
                R[4 * qd + 0] = v.x; R[4 * qd + 1] = v.y; R[4 * qd + 2] = v.z; R[4 * qd + 3] = v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if (lane == 0) pk_store(&sh.freeq[slot], k + kPkSlots);
        __builtin_amdgcn_s_setprio(0);
        // this group slot's previous ticket (its segment sg - 1, or the last
        // segment of the slot's previous group) must be done
        const uint32_t want = b * S + sg;
        while (pk_load(&sh.done[q]) != want) __builtin_amdgcn_s_sleep(1);
        const uint64_t gw = blockIdx.x + (uint64_t)G * m;
        if (kind == 1) {
            uint32_t h[4];
            int32_t s1;
            uint32_t tw;
            if (sg == 0) {
                md4_init(h);
                s1 = 0;
                tw = 0;
            } else {
                h[0] = sh.st[q][0][lane]; h[1] = sh.st[q][1][lane]; h[2] = sh.st[q][2][lane]; h[3] = sh.st[q][3][lane];
                s1 = (int32_t)sh.st[q][4][lane];
                tw = sh.st[q][5][lane];
            }
            const uint32_t nfull = n >> 6;
            if (MODE == 1) {
#pragma unroll
                for (int qd = 0; qd < 16 * (int)kRegChunks; qd++) h[qd & 3] ^= R[qd];
            } else {
#pragma unroll
                for (uint32_t c0 = 0; c0 < kRegChunks; c0++) {
                    const uint32_t c = sg * kRegChunks + c0;
                    if (c < nfull) hash_chunk<true>(R + 16 * c0, 0u, 0u, c, h, s1, tw);
                    else if (c == nfull) hash_tail<true>(R + 16 * c0, 0u, 0u, n, seed, h, s1, tw);
                }
            }
            if (sg + 1 == S) {
                store_tile_records<2>(out, gw, lane, rec, n, s1, tw, h);
            } else {
                sh.st[q][0][lane] = h[0]; sh.st[q][1][lane] = h[1]; sh.st[q][2][lane] = h[2]; sh.st[q][3][lane] = h[3];
                sh.st[q][4][lane] = (uint32_t)s1;
                sh.st[q][5][lane] = tw;
            }
        } else if (kind == 0) {
            if (MODE == 0 && lane == 0 && gw * 64 + 64 <= total_blocks) count_fallback(1);
            const uint64_t g = gw * 64 + lane;
            if (g < total_blocks) pk_direct(arena, arena_bytes, files, wg_file, nwg256, g, seed, out);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the state stores land before the hand-on
        if (lane == 0) pk_store(&sh.done[q], want + 1);
    }
}

// Kernel variants (rsg_set_block_sums_kernel; identical results, only speed
// differs): -1 = automatic, 0 = direct per-lane loads, 1 = staged LDS-DMA
// slabs (256-byte segments), 2 = park (three loader waves + five hashers with
// register-parked blocks, blocks <= 703 bytes), 3 = long blocks with deep
// per-lane prefetch, 4 / 5 = staged with 128- / 512-byte segments, 6 = staged
// for blocks at any byte offset (funnel-shifted pieces), 7 = park with
// register-staged loaders, 8 / 9 = staged with two slabs per wave, 10 / 11 =
// staged in persistent workgroups, 12 = long park (rsg.h has the details).
// Automatic (launch_block_sums below): aligned batches take park when
// 512 <= max block <= 703, 4 when the max block is 704..2048, 10 up to
// 4096, else 1; unaligned batches take 6 (3 for blocks >= 8 KiB, else 0,
// when the arena itself is not 4-byte aligned).
//
// Timing diagnostics (rsg_testing_block_sums_diagnostic, a test-only knob of
// one context, so the product knob can never select one; their "records" are
// meaningless):
// 1 = staged memory only, 2 = staged hashing only, 3 = park memory only,
// 4 = park hashing only, 5 = linear read with plain loads, 6 = linear read
// with LDS DMA, 7 = the same with every request 4 bytes off a 16-byte
// boundary, 8 = park memory only with 16-byte aligned quad requests.
constexpr int kParkLoaders = 3;  // 1 / 2 / 3 loaders measured
// Record stores of the park kernel: a tile's 64 records staged in LDS and
// written as coalesced nontemporal 16-byte stores (DESIGN.md §4.1, round 5:
// 0.1864-0.1893 ms against 0.1943-0.1946 for per-lane 20-byte stores).
constexpr int kParkRec = 2;
int block_sums_variant_env() {
    static const int v = [] {
        const char *e = getenv("RSG_BLOCKSUMS_KERNEL");
        const int x = e ? atoi(e) : -1;
        return (x < -1 || x > kBlockSumsVariantMax) ? -1 : x;
    }();
    return v;
}

static uint32_t park_grid(uint64_t total_blocks) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t ntile = (total_blocks + 63) / 64;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus, ntile));
}

// Persistent staged kernels: every resident workgroup (LDS-limited: 4 per CU
// at 128-byte segments, 2 at 256, 1 at 512) loops over the waves' 64-block groups.
static dim3 staged_persist_grid(uint32_t seg, uint32_t nwg) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t per_cu = seg == 128 ? 4u : (seg == 256 ? 2u : 1u);
    return dim3(std::max(1u, std::min<uint32_t>(nwg, (uint32_t)cus * per_cu)));
}

hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t max_blen, uint32_t seed, uint8_t *out, uint32_t *scratch,
                             uint32_t lds_reserve, int variant, int diag, hipStream_t stream, bool lines128) {
    (void)scratch;
    if (total_blocks == 0) return hipSuccess;
    const dim3 block(kBlockSumThreads), grid(nwg);
    const dim3 pgrid(park_grid(total_blocks)), pblock(kPkThreads);
    if (diag > 0 && aligned) {
        switch (diag) {
            case 1:
                hipLaunchKernelGGL((block_sums_staged<1>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
                break;
            case 2:
                hipLaunchKernelGGL((block_sums_staged<2>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
                break;
            case 3:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<1, kParkLoaders, 2, 3>), pgrid, pblock, 0, stream, arena, arena_bytes,
                                       files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 4:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<2, kParkLoaders, 2, 3>), pgrid, pblock, 0, stream, arena, arena_bytes,
                                       files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 5:
                hipLaunchKernelGGL(diag_linear_read<false>, dim3(2048), dim3(256), 0, stream, arena, arena_bytes,
                                   (uint32_t *)out);
                break;
            case 6:
                hipLaunchKernelGGL(diag_linear_read<true>, dim3(2048), dim3(256), 0, stream, arena, arena_bytes,
                                   (uint32_t *)out);
                break;
            case 7:
                hipLaunchKernelGGL((diag_linear_read<true, 4>), dim3(2048), dim3(256), 0, stream, arena, arena_bytes,
                                   (uint32_t *)out);
                break;
            case 8:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<3, kParkLoaders, 2, 3>), pgrid, pblock, 0, stream, arena, arena_bytes,
                                       files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 10: hipLaunchKernelGGL((diag_stream_read<3, 45, 1>), pgrid, dim3(192), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 11: hipLaunchKernelGGL((diag_stream_read<3, 21, 3>), pgrid, dim3(192), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 12: hipLaunchKernelGGL((diag_stream_read<3, 31, 2>), pgrid, dim3(192), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 13: hipLaunchKernelGGL((diag_stream_read<8, 8, 1>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 14: hipLaunchKernelGGL((diag_stream_read<8, 16, 2>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 15: hipLaunchKernelGGL((diag_stream_read<8, 31, 2>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 16: hipLaunchKernelGGL((diag_stream_read<4, 45, 1>), pgrid, dim3(256), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 17:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<1, kParkLoaders, 2, 3, 2>), pgrid, pblock, 0, stream, arena,
                                       arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 18:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<0, kParkLoaders, 2, 3, 2>), pgrid, pblock, 0, stream, arena,
                                       arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 19: hipLaunchKernelGGL((diag_stream_read<3, 45, 1, 1>), pgrid, dim3(192), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 20:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<4, kParkLoaders, 2, 3>), pgrid, pblock, 0, stream, arena, arena_bytes,
                                       files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 21:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<5, kParkLoaders, 2, 3>), pgrid, pblock, 0, stream, arena, arena_bytes,
                                       files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 22: hipLaunchKernelGGL((diag_stream_read<3, 45, 1>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 23:
            case 24:
            case 25:
            case 26:
                if (max_blen <= kRegMaxBytes) {
                    auto kern = diag == 23   ? block_sums_park<1, kParkLoaders, 2, 3, 0, 1>
                                : diag == 24 ? block_sums_park<0, kParkLoaders, 2, 3, 0, 1>
                                : diag == 25 ? block_sums_park<0, kParkLoaders, 2, 3, 0, 2>
                                             : block_sums_park<1, kParkLoaders, 2, 3, 0, 2>;
                    hipLaunchKernelGGL(kern, pgrid, pblock, 0, stream, arena, arena_bytes, files, wg_file, nwg,
                                       total_blocks, seed, out);
                }
                break;
            case 33: hipLaunchKernelGGL((diag_stream_rw<0, 1>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 34: hipLaunchKernelGGL((diag_stream_rw<1, 1>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 35: hipLaunchKernelGGL((diag_stream_rw<1, 8>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 36: hipLaunchKernelGGL((diag_stream_read<3, 45, 1, 1>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 37: hipLaunchKernelGGL((diag_stream_rw<1, 4>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 38: hipLaunchKernelGGL((diag_stream_rw<1, 16>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 39: hipLaunchKernelGGL((diag_stream_rw<1, 32>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 40: hipLaunchKernelGGL((diag_stream_rw<0, 8>), pgrid, dim3(512), 0, stream, arena, arena_bytes, out); break;
            case 54: hipLaunchKernelGGL((block_sums_lpark<1>), pgrid, pblock, 0, stream, arena, arena_bytes, files, wg_file, nwg, total_blocks, max_blen, seed, out); break;
            case 52: hipLaunchKernelGGL((block_sums_staged<2011>), staged_persist_grid(128, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 53: hipLaunchKernelGGL((block_sums_staged<2001>), staged_persist_grid(256, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 46: hipLaunchKernelGGL((diag_stream_read<3, 32, 1, 0>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 47: hipLaunchKernelGGL((diag_stream_read<3, 32, 1, 2>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 48: hipLaunchKernelGGL((diag_stream_read<3, 8, 3, 3>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 49: hipLaunchKernelGGL((diag_stream_read<8, 32, 1, 2>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 50: hipLaunchKernelGGL((diag_stream_read<8, 8, 3, 3>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 51: hipLaunchKernelGGL((diag_stream_read<8, 32, 1, 0>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 55: hipLaunchKernelGGL((diag_stream_read<8, 32, 1, 4>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 56: hipLaunchKernelGGL((diag_stream_read<8, 8, 3, 5>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 57: hipLaunchKernelGGL((diag_stream_read<3, 32, 1, 4>), pgrid, dim3(512), 0, stream, arena, arena_bytes, (uint32_t *)out); break;
            case 58: hipLaunchKernelGGL((block_sums_staged<21>), grid, block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 59: hipLaunchKernelGGL((block_sums_staged<2021>), staged_persist_grid(512, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 60: hipLaunchKernelGGL((block_sums_staged<2020>), staged_persist_grid(512, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 61: hipLaunchKernelGGL((block_sums_pipe<11>), staged_persist_grid(128, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 62: hipLaunchKernelGGL((block_sums_pipe<21>), staged_persist_grid(512, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 63: hipLaunchKernelGGL((block_sums_pipe<1>), staged_persist_grid(256, nwg), block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 43: hipLaunchKernelGGL((block_sums_staged<1011>), grid, block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 44: hipLaunchKernelGGL((block_sums_staged<1001>), grid, block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 45: hipLaunchKernelGGL((block_sums_staged<11>), grid, block, 0, stream, arena, arena_bytes, files, wg_file, total_blocks, seed, out); break;
            case 41:
            case 42:
                if (max_blen <= kRegMaxBytes) {
                    auto kern = diag == 41 ? block_sums_park<0, kParkLoaders, 2, 3, 0, 6>
                                           : block_sums_park<1, kParkLoaders, 2, 3, 0, 6>;
                    hipLaunchKernelGGL(kern, pgrid, pblock, 0, stream, arena, arena_bytes, files, wg_file, nwg,
                                       total_blocks, seed, out);
                }
                break;
            case 32:  // the round-4 product: per-lane record stores
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<0, kParkLoaders, 2, 3, 0, 0>), pgrid, pblock, 0, stream, arena,
                                       arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
                break;
            case 27:
            case 28:
            case 29:
            case 30:
            case 31:
                if (max_blen <= kRegMaxBytes) {
                    auto kern = diag == 27   ? block_sums_park<0, kParkLoaders, 2, 3, 0, 3>
                                : diag == 28 ? block_sums_park<0, kParkLoaders, 2, 3, 1, 2>
                                : diag == 29 ? block_sums_park<1, kParkLoaders, 2, 3, 1, 2>
                                : diag == 30 ? block_sums_park<0, kParkLoaders, 2, 3, 0, 4>
                                             : block_sums_park<0, kParkLoaders, 2, 3, 0, 5>;
                    hipLaunchKernelGGL(kern, pgrid, pblock, 0, stream, arena, arena_bytes, files, wg_file, nwg,
                                       total_blocks, seed, out);
                }
                break;
            case 9:
                if (max_blen <= kRegMaxBytes)
                    hipLaunchKernelGGL((block_sums_park<1, kParkLoaders, 2, 3, 1>), pgrid, pblock, 0, stream, arena,
                                       arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
                break;
        }
        return hipGetLastError();
    }
    int v = variant;
    // Aligned: park for 512..703-byte blocks, 128-byte segments when every
    // block starts on a 128-byte line up to 8192, otherwise (below) 512-byte
    // pipelined segments up to 8192 bytes.  History: 128-byte segments up to 4096
    // (B = 1024: 0.197-0.204 ms against 0.207-0.224 for 256-byte segments in
    // three sweeps; B = 2048 0.186 against 0.197, B = 4096 equal,
    // profiles/r04x_blocklen_sweep.jsonl), in persistent workgroups above
    // 2048 (B = 4096: 0.215-0.216 ms against 0.222-0.223, but B = 1024 / 2048
    // slower, profiles/r05af_blocklen_lpark.jsonl and the r05aa sweep), with
    // each wave's next group requested early (variant 13: 0.212-0.214 at
    // B = 4096, profiles/r05ao_blocklen_sweep_pipe.jsonl),
    // 256-byte segments beyond 4096 (12 % better at 128 KiB).  Unaligned: the
    // staged kernel wins at every block length measured.
    // Block lengths that are not multiples of 128 (most SumSizesSqroot
    // lengths: sqrt(len) rounded to 8) put most 128-byte pieces across two
    // 128-byte lines: there 512-byte segments with the group boundary hidden
    // (variant 14) win at every length measured from 1000 to 8000 bytes,
    // unless the segments through a block's tail chunk over-read it by more
    // than a fifth (B = 1224: 1536 bytes; then 256-byte segments).  Blocks
    // that all start on 128-byte lines (lines128: lengths and file offsets
    // multiples of 128; the library packs its arenas so) keep 128-byte segments (B = 2176..8192: 0.184-0.203
    // ms against 0.196-0.228 for variant 14, r05av; B = 4096 over files of
    // mixed lengths 0.181 against 0.202, r05ay, though 4 MiB files 4 MiB apart
    // favour variant 14, 0.215 against 0.223), up to 32768 (B = 16384 0.172
    // against 0.200, r05bb).  Above 8192 (to 24576) variant 14 also wins unless the
    // persistent grid's rounds run mostly empty (r05as: B = 9000 0.214
    // against 0.246, 20000 0.224 against 0.253; 16000 0.292 against 0.275)
    // (profiles/r05aq_blocklen_sweep_realistic.jsonl: B = 1000 0.240 ms
    // against 0.340 for 128-byte segments, B = 4000 0.227 against 0.300).
    if (v == -1) {
        const uint64_t seg512_bytes = (uint64_t)((max_blen >> 6) / 8 + 1) * 512;  // read per block
        if (!aligned) v = 6;
        else if (max_blen >= kParkMinBytes && max_blen <= kRegMaxBytes) v = 2;
        else if (max_blen > kRegMaxBytes && max_blen <= 32768 && lines128) v = 4;
        else if (max_blen > kRegMaxBytes && max_blen <= 8192) {
            v = seg512_bytes * 5 <= (uint64_t)max_blen * 6 ? 14 : 1;
        } else if (max_blen > 8192 && max_blen <= 24576) {
            // longer groups: the persistent grid's last round can run nearly
            // empty (B = 16000 on 256 x 4 MiB: 1052 groups on 1024 waves),
            // so variant 14 only when the rounds are at least 60 % full
            const uint64_t waves = (uint64_t)staged_persist_grid(512, nwg).x * (kBlockSumThreads / 64);
            const uint64_t groups = (total_blocks + 63) / 64;
            const uint64_t rounds = (groups + waves - 1) / waves;
            v = groups * 5 >= rounds * waves * 3 ? 14 : 1;
        } else v = 1;
    }
    // the aligned LDS-DMA kernels need 4-byte aligned blocks; the unaligned
    // staged kernel (6) needs a 4-byte aligned arena
    if (!aligned && (v == 1 || v == 2 || v == 4 || v == 5 || (v >= 8 && v <= 15))) v = 0;
    if (v == 6 && ((uintptr_t)arena & 3u)) v = max_blen >= kLongBlockBytes ? 3 : 0;
    if ((v == 2 || v == 7) && max_blen > kRegMaxBytes) v = 1;
    if (v == 7 && !aligned) v = 0;
    switch (v) {
        case 1:
            hipLaunchKernelGGL((block_sums_staged<0>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                               total_blocks, seed, out);
            break;
        case 2:
            hipLaunchKernelGGL((block_sums_park<0, kParkLoaders, 2, 3, 0, kParkRec>), pgrid, pblock, 0, stream, arena, arena_bytes,
                               files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 7:
            hipLaunchKernelGGL((block_sums_park<0, kParkLoaders, 2, 3, 1>), pgrid, pblock, 0, stream, arena, arena_bytes,
                               files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 6:  // blocks at any byte offset; an aligned batch takes the aligned kernel
            if (aligned)
                hipLaunchKernelGGL((block_sums_staged<0>), grid, block, lds_reserve, stream, arena, arena_bytes, files,
                                   wg_file, total_blocks, seed, out);
            else
                hipLaunchKernelGGL((block_sums_staged<100>), grid, block, lds_reserve, stream, arena, arena_bytes,
                                   files, wg_file, total_blocks, seed, out);
            break;
        case 4:
            hipLaunchKernelGGL((block_sums_staged<10>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                               total_blocks, seed, out);
            break;
        case 5:
            hipLaunchKernelGGL((block_sums_staged<20>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                               total_blocks, seed, out);
            break;
        case 8:  // 128-byte segments, two slabs per wave
            hipLaunchKernelGGL((block_sums_staged<1010>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                               total_blocks, seed, out);
            break;
        case 12:  // long park: 704-byte segments of 64-block groups through park's ring
            // (its ticket counts are 32-bit: per workgroup groups x segments)
            if (aligned && ((total_blocks + 63) / 64 / pgrid.x + kLpGroups) * ((max_blen >> 6) / kRegChunks + 1) * kLpGroups <
                               (1ull << 31))
                hipLaunchKernelGGL((block_sums_lpark<0>), pgrid, pblock, 0, stream, arena, arena_bytes, files, wg_file,
                                   nwg, total_blocks, max_blen, seed, out);
            else
                hipLaunchKernelGGL((block_sums_staged<2010>), staged_persist_grid(128, nwg), block, 0, stream, arena,
                                   arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 13:  // persistent, group boundaries hidden: 128 / 512 / 256-byte segments
            hipLaunchKernelGGL((block_sums_pipe<10>), staged_persist_grid(128, nwg), block, 0, stream, arena,
                               arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 14:
            hipLaunchKernelGGL((block_sums_pipe<20>), staged_persist_grid(512, nwg), block, 0, stream, arena,
                               arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 15:
            hipLaunchKernelGGL((block_sums_pipe<0>), staged_persist_grid(256, nwg), block, 0, stream, arena,
                               arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 10:  // 128-byte segments, persistent workgroups
            hipLaunchKernelGGL((block_sums_staged<2010>), staged_persist_grid(128, nwg), block, 0, stream, arena,
                               arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 11:  // 256-byte segments, persistent workgroups
            hipLaunchKernelGGL((block_sums_staged<2000>), staged_persist_grid(256, nwg), block, 0, stream, arena,
                               arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 9:  // 256-byte segments, two slabs per wave
            hipLaunchKernelGGL((block_sums_staged<1000>), grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                               total_blocks, seed, out);
            break;
        case 3: {
            const uint64_t waves = (total_blocks + 63) / 64;
            const bool two = waves <= 2ull * park_grid(~0ull >> 8);  // at most two waves per CU
            const uint32_t lt = two ? 128u : 64u;
            const dim3 lg((uint32_t)((total_blocks + lt - 1) / lt)), lb(lt);
            if (aligned && two)
                hipLaunchKernelGGL((block_sums_long<true, 2>), lg, lb, lds_reserve, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
            else if (aligned)
                hipLaunchKernelGGL((block_sums_long<true, 1>), lg, lb, lds_reserve, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
            else if (two)
                hipLaunchKernelGGL((block_sums_long<false, 2>), lg, lb, lds_reserve, stream, arena, arena_bytes, files,
                                   wg_file, total_blocks, seed, out);
            else
                hipLaunchKernelGGL((block_sums_long<false, 1>), lg, lb, lds_reserve, stream, arena, arena_bytes, files,
                                   wg_file, total_blocks, seed, out);
            break;
        }
        default:
            if (aligned)
                hipLaunchKernelGGL(block_sums_direct<true>, grid, block, 0, stream, arena, arena_bytes, files, wg_file,
                                   total_blocks, seed, out);
            else
                hipLaunchKernelGGL(block_sums_direct<false>, grid, block, 0, stream, arena, arena_bytes, files,
                                   wg_file, total_blocks, seed, out);
            break;
    }
    return hipGetLastError();
}


hipError_t read_block_sums_fallbacks(uint64_t out[2], bool reset) {
    unsigned long long v[2] = {0, 0};
    hipError_t e = hipDeviceSynchronize();  // the counters are bumped on any of the context's streams
    if (e == hipSuccess) e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_fallbacks), sizeof v, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
        const unsigned long long z[2] = {0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_fallbacks), z, sizeof z, 0, hipMemcpyHostToDevice);
    }
    out[0] = v[0];
    out[1] = v[1];
    return e;
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
