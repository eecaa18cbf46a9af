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
// The stores are nontemporal (the records are not read again here).
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
    u32x4a4 *dst = reinterpret_cast<u32x4a4 *>(out + t * (64ull * kRecordBytes));
    __builtin_nontemporal_store(u32x4a4{a.x, a.y, a.z, a.w}, dst + lane);
    if (lane < 16) {
        const u32x4v b = reinterpret_cast<const u32x4v *>(rec)[64 + lane];
        __builtin_nontemporal_store(u32x4a4{b.x, b.y, b.z, b.w}, dst + 64 + lane);
    }
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

// SEG = bytes of every block per segment: 256 (variant 1) or 128 (variant
// 4: more waves per CU, and whole 128-byte lines when blocks start on them).
// UNAL (variant 6): blocks start at any byte (the sender's confirmation
// windows; the arena itself 4-byte aligned): each piece is fetched from the
// block's start rounded down to 4 bytes, one 16-byte unit longer (the pad
// unit carries data), and the lane funnel-shifts its words (alignbyte) as
// the direct kernel does.
// (Wave priority 3 from the segment wait through the next DMA issue, 0 while
// hashing, as park does: no gain at B = 1024 / 4096 / 128 KiB,
// profiles/r04g_blocklen_sweep.jsonl, so not kept.)
template <uint32_t SEG, bool UNAL>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_staged(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    // Aligned: nt policy on the DMA, every byte is read once (A/B against the
    // default policy, profiles/r02f_blocklen_sweep_nt.jsonl: B = 4096 0.239 ->
    // 0.219 ms, cfg5 6.48 -> 6.25 ms).  UNAL: the default policy.  A piece
    // starting mid-line shares its first and last 128-byte lines with the
    // block's previous and next segments, requested one segment apart; nt
    // lines were gone by then (FETCH 1.51x the block bytes at B = 1773,
    // 1.31x with the default policy) -- round 6,
    // profiles/r06o_blocklen_policy_ab.txt: B = 1773 / 2289 / 4222 / 5882
    // 0.262 / 0.260 / 0.257 / 0.253 -> 0.222 / 0.227 / 0.234 / 0.235 ms per
    // GiB, cfg3's confirmation windows 1112 -> 1161 GiB/s.
    constexpr int DMA_AUX = UNAL ? 0 : 2;
    constexpr uint32_t kSegBytes = Seg<SEG>::kSegBytes, kUnits = Seg<SEG>::kUnits, kPiece = Seg<SEG>::kPiece;
    constexpr uint32_t kWaveSlab = Seg<SEG>::kWaveSlab, kDmaPerSeg = Seg<SEG>::kDmaPerSeg;
    constexpr uint32_t kChunks = Seg<SEG>::kChunks;
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * kWaveSlab];
    const uint32_t lane = threadIdx.x & 63u;
    // readfirstlane: provably wave-uniform values keep the LDS base (M0) and
    // the buffer descriptor in SGPRs (no waterfall loops around the DMA).
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * kWaveSlab;
    // the wave's 64-block group: blocks [wave_first, wave_first + 64)
    const uint64_t wave_first = (uint64_t)blockIdx.x * kBlockSumThreads + wave * 64u;
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
        if (full && lane == 0) count_fallback(0);
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
    // UNAL: volatile keeps one ds_read_b128 per unit (conflict-free at the
    // 272-byte stride); left to itself the compiler split the funnel-shifted
    // reads into ds_read2_b32, whose 32-bank groups conflict 4-way there
    typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));
#define RSG_DMA_SEGMENT(S_)                                                                                      \
    do {                                                                                                         \
        const uint32_t so_ = kSegBytes * (S_);                                                                   \
        _Pragma("unroll") for (uint32_t i_ = 0; i_ < kDmaPerSeg; i_++)                                           \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + 1024u * i_), \
                                                     16, voff[i_], so_, 0, DMA_AUX);                             \
    } while (0)
#define RSG_READ_SEGMENT()                                                                                       \
    do {                                                                                                         \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                         \
        _Pragma("unroll") for (int q_ = 0; q_ < (int)(SEG / 16) + (UNAL ? 1 : 0); q_++) {                        \
            if constexpr (UNAL) {                                                                                \
                const U32x4 v_ = *(const volatile __attribute__((address_space(3))) U32x4 *)(mine + 16 * q_);    \
                R[4 * q_ + 0] = v_.x; R[4 * q_ + 1] = v_.y; R[4 * q_ + 2] = v_.z; R[4 * q_ + 3] = v_.w;          \
            } else {                                                                                             \
                const uint4 v_ = *reinterpret_cast<const uint4 *>(mine + 16 * q_);                              \
                R[4 * q_ + 0] = v_.x; R[4 * q_ + 1] = v_.y; R[4 * q_ + 2] = v_.z; R[4 * q_ + 3] = v_.w;          \
            }                                                                                                    \
        }                                                                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
    } while (0)
    const uint32_t nfull = n >> 6;
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    RSG_DMA_SEGMENT(0);
    RSG_READ_SEGMENT();
#pragma unroll 1
    for (uint32_t cs = 0; cs < S; cs++) {
        const bool more = cs + 1 < S;
        if (more) RSG_DMA_SEGMENT(cs + 1);  // in flight while segment cs hashes
#pragma unroll
        for (uint32_t i = 0; i < kChunks; i++) {
            const uint32_t c = kChunks * cs + i;
            if (c < nfull) hash_chunk<!UNAL>(R + 16 * i, R[16 * i + 16], sh, c, h, s1, t);
            else if (c == nfull) hash_tail<!UNAL>(R + 16 * i, R[16 * i + 16], sh, n, seed, h, s1, t);
        }
        if (more) RSG_READ_SEGMENT();
    }
#undef RSG_DMA_SEGMENT
#undef RSG_READ_SEGMENT
    // a full wave's 64 records are contiguous (blocks wave_first ..): staged
    // in the wave's slab (its last segment has been read) and written as
    // coalesced nontemporal stores, as the park kernel does (round 5)
    store_tile_records(out, wave_first / 64, lane, reinterpret_cast<uint32_t *>(slab), n, s1, t, h);
}

// Variant 7 (round 6): line windows.  The staged kernels fetch each block's
// segments from the block's own start, so a block that does not start on a
// 128-byte line reads, every segment, a line it read (partly) the segment
// before: 3 lines per 256-byte segment, 1.3-1.5x the block bytes in FETCH_SIZE
// (B = 1773, profiles/r06o_blocklen_policy_ab.txt).  Here lane j's windows are
// the 128-byte lines from the one holding its first byte: window w =
// [A_j + 128 w, +128), A_j = that line, delta_j = off_j - A_j < 128.  Step s
// hashes chunks 2s and 2s+1, whose 33 words (32 + the funnel word) start at
// word delta_j / 4 of window s and end in window s+1, so windows s and s+1
// sit in the wave's two slabs (144-byte pieces: 8 data units + a pad unit the
// buffer range check drops) and window s+2 is requested into window s's slab
// once its words are in registers.  The words are read with one ds_read_b32
// each from a per-lane base chosen per word (window s or s+1: a compare and a
// select, ~15 % more VALU than the staged kernel's 17 ds_read_b128 per four
// chunks).  ALN: every block 4-byte aligned (no funnel shift).  The arena
// must start on a 128-byte line (launch_block_sums checks).
// DMA_AUX: nt (2): every line is fetched once per block now; nt measured
// 3-9 % faster than the default policy (B = 1448 / 1773 / 4222 / 5882: 0.208 /
// 0.200 / 0.181 / 0.188 against 0.209 / 0.204 / 0.195 / 0.206 ms per GiB,
// profiles/r06v_lines_policy_ab.txt)
// PU: 16-byte units per piece (8 data + 1 or 2 dropped pads).  Lane j's word
// k sits in bank (PU*4*j + delta_j/4 + k) mod 32, and consecutive blocks of
// one file have delta_j = (j B + c) mod 128: with PU = 9, B = 6000 put all 32
// lanes on one bank (0.50 ms per GiB against 0.21); the launcher picks the PU
// whose 4 PU + B/4 has the fewest factors of 2 mod 32.
template <bool ALN, int DMA_AUX, uint32_t PU>
__global__ __launch_bounds__(kBlockSumThreads) void block_sums_lines(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint64_t total_blocks, uint32_t seed, uint8_t *__restrict__ out) {
    constexpr uint32_t kWin = 128, kUnits = PU, kPiece = 16 * kUnits, kSlab = 64 * kPiece, kDma = kSlab / 1024;
    static_assert(PU == 9 || PU == 10, "nine or ten units per piece");
    __shared__ __attribute__((aligned(16))) uint8_t slab_all[(kBlockSumThreads / 64) * 2 * kSlab];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slab = slab_all + wave * 2 * kSlab;
    const uint64_t wave_first = (uint64_t)blockIdx.x * kBlockSumThreads + wave * 64u;
    const uint64_t g = wave_first + lane;
    uint64_t off = 0;
    uint32_t n = 0;
    if (g < total_blocks) locate_block(files, wg_file, g, off, n, wave_first / kBlockSumThreads);
    const uint32_t sh = ALN ? 0u : (uint32_t)(off & 3u);
    const uint32_t delta = (uint32_t)(off & (kWin - 1));
    const uint64_t aoff = off - delta;                      // line-aligned fetch start
    const uint32_t nfull = n >> 6;
    const uint32_t steps = n ? nfull / 2 + 1 : 0;           // step s: chunks 2s, 2s+1 (through the tail chunk)
    const uint32_t S = rfl32((uint32_t)wave_max_u64(steps));
    const uint64_t base = rfl64(wave_min_u64(n ? aoff : ~0ull));
    // windows 0..S of every lane (the last one only for the funnel word)
    const uint64_t top = rfl64(wave_max_u64(n ? aoff + (uint64_t)kWin * (S + 1) : 0));
    const bool full = wave_first + 63 < total_blocks;
    const bool staged = full && top <= arena_bytes && (top - base) <= 0x7FFFFFFFull;
    if (!staged) {
        if (full && lane == 0) count_fallback(0);
        if (n == 0) return;
        uint32_t h[4];
        md4_init(h);
        int32_t s1 = 0;
        uint32_t t = 0;
        hash_block_direct<ALN>(arena, (uintptr_t)(arena + arena_bytes), off, n, seed, h, s1, t);
        store_record(out, g, n, s1, t, h);
        return;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + base), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t rel = (uint32_t)(aoff - base);
    // DMA instruction i, lane t: piece j = (64 i + t) / 9 (lane j's window),
    // unit u = (64 i + t) % 9; u == 8 is the dropped pad
    uint32_t voff[10];  // fixed bound (a template-dependent one drops the host launch stub, as in staged)
#pragma unroll
    for (uint32_t i = 0; i < kDma; i++) {
        const uint32_t idx = 64u * i + lane;
        const uint32_t j = idx / kUnits, u = idx - kUnits * j;
        const uint32_t v = (uint32_t)__shfl((int)rel, (int)j, 64) + 16u * u;
        voff[i] = u < 8 ? v : 0x80000000u;
    }
#define RSG_DMA_WINDOW(W_)                                                                                       \
    do {                                                                                                         \
        uint8_t *d_ = slab + ((W_) & 1u) * kSlab;                                                                \
        _Pragma("unroll") for (uint32_t i_ = 0; i_ < kDma; i_++)                                                 \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(d_ + 1024u * i_), \
                                                     16, voff[i_], kWin * (W_), 0, DMA_AUX);                     \
    } while (0)
    // word k of step s: word dw + k of window s, or of window s+1 past its 32 words
    const uint32_t dw = delta >> 2;
    const uint32_t mine = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)(slab + lane * kPiece) + 4u * dw;
    constexpr int NW = ALN ? 32 : 33;
    uint32_t R[33];
    R[32] = 0;  // ALN: the funnel word is never read
    const uint32_t nfull_c = nfull;
    uint32_t h[4];
    md4_init(h);
    int32_t s1 = 0;
    uint32_t t = 0;
    RSG_DMA_WINDOW(0u);
    RSG_DMA_WINDOW(1u);
#pragma unroll 1
    for (uint32_t s = 0; s < S; s++) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t a0 = mine + (s & 1u) * kSlab;               // window s
        const uint32_t a1 = mine + ((s + 1u) & 1u) * kSlab - kWin;  // window s+1, minus its 32 words
        typedef __attribute__((address_space(3))) const volatile uint32_t lds32;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t a = dw + (uint32_t)k < 32u ? a0 : a1;
            R[k] = *(lds32 *)(uintptr_t)(a + 4u * (uint32_t)k);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (s + 2 <= S) RSG_DMA_WINDOW(s + 2);  // into window s's slab, in flight while s hashes
#pragma unroll
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t c = 2 * s + i;
            if (c < nfull_c) hash_chunk<ALN>(R + 16 * i, R[16 * i + 16], sh, c, h, s1, t);
            else if (c == nfull_c) hash_tail<ALN>(R + 16 * i, R[16 * i + 16], sh, n, seed, h, s1, t);
        }
    }
#undef RSG_DMA_WINDOW
    store_tile_records(out, wave_first / 64, lane, reinterpret_cast<uint32_t *>(slab), n, s1, t, h);
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

struct PkShared {
    uint8_t tile[kPkSlots][kPkTile];
    uint32_t rec[kPkWaves * 64 * 5];  // wave w's 64 records (20 B each) at rec[320 w] (store_tile_records)
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
// each instruction, precomputed by the loader.
template <int AUX>
__device__ __forceinline__ void pk_issue(const uint8_t *arena, uint8_t *dst, const PkDesc &d, uint32_t lane,
                                         const uint32_t *jj, const uint32_t *uu) {
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(arena + d.base), (short)0, 0x7FFFFFFF, 0x00020000);
    const int rel = (int)(uint32_t)(d.off - d.base);
    // the regular/irregular choice is made once per tile (a branch per
    // instruction costs an lgkmcnt wait per instruction)
    if (d.regular) {
#pragma unroll
        for (uint32_t i = 0; i < kPkDma; i++) {
            const uint32_t j = jj[i], u16 = uu[i];
            const uint32_t nj = j == d.jl ? d.nl : d.B;
            const uint32_t vo = u16 < nj ? d.B * j + u16 : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * i),
                                                     16, vo, 0, 0, AUX);
        }
    } else {
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
                const uint32_t vo = u16 < nj[k] ? rj[k] + u16 : 0x80000000u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)(dst + 1024u * (i0 + k)), 16, vo, 0, 0, AUX);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
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

// The tile DMA uses the nt cache policy (aux = 2): every byte is read once.
// (A/B, profiles/r02f_ab_park_cache_policy*.json: the default policy, sc0 or
// sc1 alone cost 6-9 %; nt combined with sc0 / sc1 equals nt.)
// Three loader waves, one per slot (1 / 2 / 3 loaders
// measured); the other five waves hash.
// Wave priorities (s_setprio): loaders at 3 (a slot's next DMA issues ahead
// of the hasher sharing the SIMD), hashers at 3 while they copy a slot out
// (the slot frees sooner), 0 while they hash.  (8-round A/B,
// profiles/r04f_ab_park_prio.json: none 0.1984 ms, loaders only 0.1962,
// copy-out at 2 0.1950, at 3 0.1942.)
// Records: a staged tile's 64 records through the hasher's LDS area as
// coalesced nontemporal 16-byte stores (store_tile_records; DESIGN.md §4.1,
// round 5: 0.1864-0.1893 ms against 0.1943-0.1946 for per-lane 20-byte
// stores).
constexpr uint32_t kParkLoaders = kPkSlots;
constexpr int kParkAux = 2;
__global__ __launch_bounds__(kPkThreads) void block_sums_park(
    const uint8_t *__restrict__ arena, uint64_t arena_bytes, const DevFile *__restrict__ files,
    const uint32_t *__restrict__ wg_file, uint32_t nwg256, uint64_t total_blocks, uint32_t seed,
    uint8_t *__restrict__ out) {
    constexpr int MODE = 0, NL = (int)kParkLoaders, AUX = kParkAux, PRIO = 3, REC = 2;
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
    const uint32_t G = gridDim.x;  // one persistent workgroup per CU; tile t belongs to workgroup t % G

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
            if (staged && MODE != 2) pk_issue<AUX>(arena, &sh.tile[slot][0], cur, lane, jj, uu);
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
            static_assert(REC == 2, "records through LDS, nontemporal");
            store_tile_records(out, t, lane, &sh.rec[320u * wave], n, s1, tw, h);
        } else {
            if (PRIO >= 3) __builtin_amdgcn_s_setprio(0);
            if (lane == 0) {
                pk_store(&sh.freeq[slot], k + kPkSlots);
                if (MODE == 0 && t * 64 + 64 <= total_blocks) count_fallback(1);
            }
            if (g < total_blocks) pk_direct(arena, arena_bytes, files, wg_file, nwg256, g, seed, out);
        }
    }
}

// Kernel variants (rsg_set_block_sums_kernel; identical results, only speed
// differs): -1 = automatic, 0 = direct per-lane loads, 1 = staged LDS-DMA
// slabs (256-byte segments), 2 = park (three loader waves + five hashers with
// register-parked blocks, blocks <= 703 bytes), 3 = long blocks with deep
// per-lane prefetch, 4 = staged with 128-byte segments, 6 = staged for
// blocks at any byte offset (funnel-shifted pieces), 7 = line windows (each
// block's bytes as the 128-byte lines that hold them, every line once).  (7
// was a dropped ABI-3 variant's number, reused from ABI 5; the other dropped ones -- 5,
// 8..15, 14 the persistent 512-byte kernel until round 6 -- are not reused;
// tools/build_ab.sh rebuilds them from the history.)
int block_sums_variant_env() {
    static const int v = [] {
        const char *e = getenv("RSG_BLOCKSUMS_KERNEL");
        const int x = e ? atoi(e) : -1;
        return block_sums_variant_valid(x) ? x : -1;
    }();
    return v;
}

bool block_sums_variant_valid(int v) {
    return v == -1 || v == 0 || v == 1 || v == 2 || v == 3 || v == 4 || v == 6 || v == 7;
}

// The automatic rule, in two lines (rsg.h; tests/test_abi.py pins its
// boundaries, DESIGN.md §4.1 has the measurements behind each):
//   unaligned blocks, or blocks of >= 704 bytes off the 128-byte lines -> line
//   windows (7); 512..703 -> park (2); on the lines up to 32 KiB -> 4; else 1.
// A variant the batch cannot take falls back: the LDS-DMA kernels need
// 4-byte aligned blocks (else 0), line windows a 128-byte aligned arena (else
// 6 for unaligned blocks, 1 for aligned ones), the any-offset kernel a 4-byte
// aligned arena (else 3 for blocks >= 8 KiB, 0 below), park blocks <= 703
// bytes (else 1).  arena_align: 0 = not 4-byte aligned, 1 = 4-byte, 2 = 128-byte.
int block_sums_choice(int variant, bool aligned, bool lines128, int arena_align, uint32_t max_blen) {
    int v = variant;
    if (v == -1) {
        if (!aligned) v = 7;
        else if (max_blen >= kParkMinBytes && max_blen <= kRegMaxBytes) v = 2;
        else if (max_blen > kRegMaxBytes && lines128 && max_blen <= 32768) v = 4;
        else if (max_blen > kRegMaxBytes && !lines128) v = 7;
        else v = 1;
    }
    if (!aligned && (v == 1 || v == 2 || v == 4)) v = 0;
    if (v == 7 && arena_align < 2) v = aligned ? 1 : 6;
    if (v == 6 && arena_align < 1) v = max_blen >= kLongBlockBytes ? 3 : 0;
    if (v == 2 && max_blen > kRegMaxBytes) v = 1;
    return v;
}

static uint32_t park_grid(uint64_t total_blocks) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t ntile = (total_blocks + 63) / 64;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus, ntile));
}

hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t max_blen, uint32_t seed, uint8_t *out, uint32_t lds_reserve, int variant,
                             hipStream_t stream, bool lines128) {
    if (total_blocks == 0) return hipSuccess;
    const dim3 block(kBlockSumThreads), grid(nwg);
    const uintptr_t ab = (uintptr_t)arena;
    const int v = block_sums_choice(variant, aligned, lines128, (ab & 127u) == 0 ? 2 : (ab & 3u) == 0 ? 1 : 0, max_blen);
    switch (v) {
        case 1:
            hipLaunchKernelGGL((block_sums_staged<256, false>), grid, block, 0, stream, arena, arena_bytes, files,
                               wg_file, total_blocks, seed, out);
            break;
        case 2:
            hipLaunchKernelGGL(block_sums_park, dim3(park_grid(total_blocks)), dim3(kPkThreads), 0, stream, arena,
                               arena_bytes, files, wg_file, nwg, total_blocks, seed, out);
            break;
        case 4:
            hipLaunchKernelGGL((block_sums_staged<128, false>), grid, block, 0, stream, arena, arena_bytes, files,
                               wg_file, total_blocks, seed, out);
            break;
        case 6:  // blocks at any byte offset; an aligned batch takes the aligned kernel
            if (aligned)
                hipLaunchKernelGGL((block_sums_staged<256, false>), grid, block, lds_reserve, stream, arena,
                                   arena_bytes, files, wg_file, total_blocks, seed, out);
            else
                hipLaunchKernelGGL((block_sums_staged<256, true>), grid, block, lds_reserve, stream, arena,
                                   arena_bytes, files, wg_file, total_blocks, seed, out);
            break;
        case 7:  // line windows (the arena on a 128-byte line, checked by block_sums_choice)
        {
            auto tz = [](uint32_t x) { return x == 0 ? 5 : std::min(5, __builtin_ctz(x)); };  // factors of 2 mod 32
            const uint32_t bw = (max_blen / 4) & 31u;
            const bool ten = tz((36u + bw) & 31u) > tz((40u + bw) & 31u);
            auto kern = aligned ? (ten ? block_sums_lines<true, 2, 10> : block_sums_lines<true, 2, 9>)
                                : (ten ? block_sums_lines<false, 2, 10> : block_sums_lines<false, 2, 9>);
            hipLaunchKernelGGL(kern, grid, block, lds_reserve, stream, arena, arena_bytes, files, wg_file, total_blocks,
                               seed, out);
        }
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
