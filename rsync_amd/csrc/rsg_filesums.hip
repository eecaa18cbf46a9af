// rsg_filesums.hip -- whole-file MD4 sums, one lane per file.
//
//   mode 0: MD4(file)                   rsyncchecksum.ReaderChecksum, rsyncchecksum.go:60-66
//           (the --checksum file-list sums: sender/flist.go:276-293, receiver/generator.go:82-88)
//   mode 1: MD4(int32_LE(seed) || file) the transfer's whole-file sum, seeded BEFORE the data
//           (match.go:52-53 + matched :262-269, sender.go:184-206, receiver.go:117-120)
//
// MD4 is a serial chain per message, so the parallelism is across files: a
// batch of many files (cfg4: 100 000 files of 4-64 KiB) hashes one file per
// lane.  Files are assigned to lanes longest first so the lanes of a wave run
// for similar numbers of chunks.  Memory: each lane streams its own file with
// 16-byte loads (any alignment, funnel-shifted), eight chunks in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "rsg_internal.h"
#include "rsg_md4.h"

namespace rsg {

typedef uint32_t fs_u32x4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __noinline__ uint32_t fs_word_slow(const uint8_t *p, uintptr_t end) {
    uint32_t w = 0;
    for (int i = 0; i < 4; i++)
        if ((uintptr_t)(p + i) < end) w |= (uint32_t)p[i] << (8 * i);
    return w;
}

// 16 message words starting at byte pointer q (any alignment).  Bytes at or
// past `end` (the arena's end) read as 0 and are never touched.
__device__ __forceinline__ void fs_load_chunk(const uint8_t *q, uintptr_t end, uint32_t X[16]) {
    const uint32_t sh = (uint32_t)((uintptr_t)q & 3u);
    const uint8_t *p0 = q - sh;
    uint32_t W[17];
    if ((uintptr_t)p0 + 68 <= end) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const fs_u32x4 v = reinterpret_cast<const fs_u32x4 *>(p0)[j];
            W[4 * j + 0] = v.x; W[4 * j + 1] = v.y; W[4 * j + 2] = v.z; W[4 * j + 3] = v.w;
        }
        W[16] = sh ? *reinterpret_cast<const uint32_t *>(p0 + 64) : 0u;
    } else {
#pragma unroll
        for (int k = 0; k < 17; k++) {
            const uint8_t *pk = p0 + 4 * k;
            W[k] = (uintptr_t)pk + 4 <= end ? *reinterpret_cast<const uint32_t *>(pk) : fs_word_slow(pk, end);
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) X[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sh);
}

// The first message chunk when the seed is prepended: seed, then data[0..60).
__device__ __forceinline__ void fs_seeded_head(const uint8_t *d, uintptr_t end, uint32_t seed, uint32_t X[16]) {
    uint32_t D[16];
    fs_load_chunk(d, end, D);
    X[0] = seed;
#pragma unroll
    for (int k = 1; k < 16; k++) X[k] = D[k - 1];
}

// Ring of P chunks in flight per lane (a chunk = the 17 aligned words its
// realignment needs), so the MD4 chain of a lane does not wait on one HBM
// round trip per 64 bytes: with ~1.5 waves per SIMD (100 000 files) nothing
// else hides that latency.  Chunk cc's words start at p0 + 64 cc.
template <int P>
__device__ __forceinline__ void fs_ring(const uint8_t *p0, uint32_t sh, uint64_t c, uint64_t nfull, uint32_t h[4],
                                        uint32_t X[16]) {
    uint32_t buf[P][17];
#define RSG_FS_FETCH(U, CC)                                                                                     \
    do {                                                                                                        \
        const uint8_t *q_ = p0 + 64 * (CC);                                                                     \
        _Pragma("unroll") for (int j_ = 0; j_ < 4; j_++) {                                                      \
            const fs_u32x4 v_ = reinterpret_cast<const fs_u32x4 *>(q_)[j_];                                     \
            buf[U][4 * j_ + 0] = v_.x; buf[U][4 * j_ + 1] = v_.y; buf[U][4 * j_ + 2] = v_.z; buf[U][4 * j_ + 3] = v_.w; \
        }                                                                                                       \
        buf[U][16] = *reinterpret_cast<const uint32_t *>(q_ + 64);                                              \
    } while (0)
#pragma unroll
    for (int u = 0; u < P; u++) RSG_FS_FETCH(u, min(c + (uint64_t)u, nfull));
#pragma unroll 1
    for (; c + P <= nfull; c += P) {
#pragma unroll
        for (int u = 0; u < P; u++) {
#pragma unroll
            for (int k = 0; k < 16; k++) X[k] = __builtin_amdgcn_alignbyte(buf[u][k + 1], buf[u][k], sh);
            md4_compress(h, X);
            RSG_FS_FETCH(u, min(c + (uint64_t)u + P, nfull));
        }
    }
#undef RSG_FS_FETCH
    // fewer than P data chunks left: they and the tail chunk nfull sit in
    // buffers 0 .. nfull - c; the tail's words are left in X
#pragma unroll
    for (int u = 0; u < P; u++) {
        const uint64_t cc = c + (uint64_t)u;
        if (cc <= nfull) {
#pragma unroll
            for (int k = 0; k < 16; k++) X[k] = __builtin_amdgcn_alignbyte(buf[u][k + 1], buf[u][k], sh);
            if (cc < nfull) md4_compress(h, X);
        }
        if (cc >= nfull) break;
    }
}

// Tail of a message of L bytes whose last chunk's words are in X: r = L % 64
// message bytes, 0x80, zeros, the 64-bit bit length (RFC 1320); one or two
// compressions.
__device__ __forceinline__ void fs_tail(uint32_t X[16], uint64_t L, uint32_t h[4]) {
    const uint32_t r = (uint32_t)(L & 63u), kd = r >> 2, rb = r & 3u;
    const uint32_t keep = rb ? ((1u << (8 * rb)) - 1u) : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        X[k] = k < kd ? X[k] : (k == kd ? ((X[k] & keep) | (0x80u << (8 * rb))) : 0u);
    const uint64_t bits = L << 3;
    if (r < 56) {
        X[14] = (uint32_t)bits;
        X[15] = (uint32_t)(bits >> 32);
        md4_compress(h, X);
    } else {
        md4_compress(h, X);
#pragma unroll
        for (int k = 0; k < 14; k++) X[k] = 0;
        X[14] = (uint32_t)bits;
        X[15] = (uint32_t)(bits >> 32);
        md4_compress(h, X);
    }
}

// Whole message of one file with the lane's own loads: MD4(file) (pre = 0) or
// MD4(int32_LE(seed) || file) (pre = 4).  The ring path for most files; the
// guarded single-chunk path for a file ending at the arena's very end.
__device__ __forceinline__ void fs_hash_lane(const uint8_t *__restrict__ arena, uint64_t arena_bytes, FileSpan F,
                                             uint64_t pre, uint32_t seed, uint32_t h[4]) {
    const uint8_t *d = arena + F.offset;
    const uintptr_t end = (uintptr_t)(arena + arena_bytes);
    const uint64_t L = F.len + pre;             // message length
    const uint64_t nfull = L >> 6;
    md4_init(h);
    uint32_t X[16];
    uint64_t c = 0;
    if (pre && nfull > 0) {
        fs_seeded_head(d, end, seed, X);
        md4_compress(h, X);
        c = 1;
    }
    // message chunk c = data bytes [64 c - pre, 64 c - pre + 64); for c >= 1
    // (or no prefix) its aligned words start at p0 + 64 c, inside the file's
    // allocation.  Fast path: every word through the tail chunk's lies inside
    // the arena (all but a file ending at the arena's very end).
    const uint32_t sh = (uint32_t)((uintptr_t)(d - pre) & 3u);
    const uint8_t *p0 = d - pre - sh;
    if (c <= nfull && (uintptr_t)p0 + 64 * (nfull + 1) + 4 <= end && !(pre && nfull == 0)) {
        fs_ring<8>(p0, sh, c, nfull, h, X);
    } else {
        for (; c < nfull; c++) {
            fs_load_chunk(d + 64 * c - pre, end, X);
            md4_compress(h, X);
        }
        if (pre && nfull == 0) fs_seeded_head(d, end, seed, X);
        else fs_load_chunk(d + 64 * nfull - pre, end, X);
    }
    fs_tail(X, L, h);
}

// ---------------------------------------------------------------- staged variant
// The ring kernel above gathers every 16-byte load from 64 different files
// (64 cache lines per wave instruction): the CU's address path, not HBM,
// bounds it (27 % of 8 TB/s on cfg4's files).  Here a wave's 64 files
// stream through a private LDS slab, 128 bytes of every file per segment, by
// LDS DMA: instruction i, lane l fills slab bytes [1024 i + 16 l, +16) =
// slot (64 i + l) % U of file j = (64 i + l) / U's piece of U units (U = 8
// or 9 below; a piece starts at the file's first byte rounded down to 4).
// global_load_lds takes a 64-bit address per lane, so a wave's files may lie
// anywhere in an arena of any size (a buffer descriptor's 31-bit offsets
// would confine them to 2 GiB).  Waves with a file whose needed bytes run
// past the arena's end hash with the ring path above.  A unit a lane does not
// need (its file is done) re-reads the file's last segment, lines fetched a
// segment earlier (segment 0, read back at the end, counted ~2 % of extra
// traffic from the Infinity Cache, round 6).
// Seeded mode: message word 0 is the seed, word w >= 1 is data word w - 1,
// so message chunk c = (carry, data words 16 c .. 16 c + 14) with carry =
// the data word before them -- the data stream is read from the file's own
// start, never before it.
// ALN: every file of the launch starts 4-byte aligned (the library's own
// arenas pack files at 16 or 128 bytes), so a segment is exactly the file's
// next 256 bytes: no funnel shift, and the 17th unit of each piece -- kept
// so the per-lane ds_read_b128 of a 272-byte stride stays conflict-free --
// re-reads the segment's own last 16 bytes, a line just fetched, instead of
// the next segment's first 16 bytes.
// Measured alternatives (round 6, profiles/r06k_filesums_ab.txt, kernel ms
// on cfg4's 100 000 files): 128-byte segments (8 waves per CU) 0.88,
// three slabs in flight 0.82-0.86, 512-byte segments 1.07, 256-byte
// segments with the 16 units rotated instead of padded (5 waves per CU)
// 0.84, against 0.80 for this layout: neither occupancy nor prefetch depth
// bounds it (the 64 files' interleaved 256-byte pieces do, as for the
// block-sum kernels' staged order, §4.1 of DESIGN.md).
struct FsShape {
    static constexpr uint32_t kChunks = 4;                  // MD4 chunks per segment
    static constexpr uint32_t kSeg = 64 * kChunks;          // file bytes per segment
    static constexpr uint32_t kUnits = 4 * kChunks + 1;     // 16-byte units per piece (272 bytes)
    static constexpr uint32_t kPiece = 16 * kUnits;         // LDS bytes per file
    static constexpr uint32_t kSlab = 64 * kPiece;          // LDS bytes per wave and segment
    static constexpr uint32_t kDma = kUnits;                // DMA instructions per segment
};

template <bool SEEDED, int AUX, bool ALN>
__global__ __launch_bounds__(64) void file_sums_staged(const uint8_t *__restrict__ arena, uint64_t arena_bytes,
                                                       const FileSpan *__restrict__ files,
                                                       const uint32_t *__restrict__ order, uint32_t nfiles,
                                                       uint32_t seed, uint8_t *__restrict__ out) {
    using Sh = FsShape;
    constexpr uint32_t CH = Sh::kChunks, SEG = Sh::kSeg, NU = Sh::kUnits, PIECE = Sh::kPiece, SLAB = Sh::kSlab,
                       NDMA = Sh::kDma;
    __shared__ __attribute__((aligned(16))) uint8_t slab[2 * SLAB];  // two segments in flight
    const uint32_t lane = threadIdx.x;
    const uint32_t lane_file = blockIdx.x * 64 + lane;
    const bool active = lane_file < nfiles;
    const uint32_t fi = active ? order[lane_file] : order[blockIdx.x * 64];
    const FileSpan F = files[fi];
    const uint64_t pre = SEEDED ? 4u : 0u;
    const uint64_t L = F.len + pre;
    const uint64_t nfull = L >> 6;                 // the tail chunk's index
    const uint64_t nseg64 = nfull / CH + 1;        // segments through the tail chunk
    const uint32_t sh = ALN ? 0u : (uint32_t)(F.offset & 3u);
    const uint64_t fstart = F.offset - sh;         // data read from here (4-byte aligned)
    // staged when every lane's needed bytes [fstart, fstart + SEG nseg (+ 16))
    // lie inside the arena (segment counts kept to 32 bits)
    const bool ok = nseg64 < (1ull << 31) && fstart + SEG * nseg64 + (ALN ? 0 : 16) <= arena_bytes;
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        if (!active) return;
        uint32_t h[4];
        fs_hash_lane(arena, arena_bytes, F, pre, seed, h);
        uint32_t *o = reinterpret_cast<uint32_t *>(out + 16ull * fi);
        o[0] = h[0]; o[1] = h[1]; o[2] = h[2]; o[3] = h[3];
        return;
    }
    const uint32_t nseg = active ? (uint32_t)nseg64 : 0u;
    uint32_t smax = nseg;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) smax = max(smax, (uint32_t)__shfl_xor((int)smax, m, 64));
    const uint32_t S = rfl32(smax);
    // per DMA instruction i: this lane's unit (file j, unit u; ALN: the pad
    // re-reads unit 15), its address at segment 0 and the file's segments
    const uint8_t *ua[NDMA];
    uint32_t un[NDMA];
#pragma unroll
    for (uint32_t i = 0; i < NDMA; i++) {
        const uint32_t idx = 64u * i + lane, j = idx / NU, t = idx - NU * j;
        const uint32_t u = ALN && t == NU - 1 ? t - 1 : t;
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)fstart, (int)j, 64);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(fstart >> 32), (int)j, 64);
        ua[i] = arena + (((uint64_t)hi << 32) | lo) + 16u * u;
        un[i] = max((uint32_t)__shfl((int)nseg, (int)j, 64), 1u) - 1u;  // the file's last segment
    }
#define RSG_FS_DMA(S_, SL_)                                                                                    \
    do {                                                                                                       \
        uint8_t *d_ = slab + (SL_) * SLAB;                                                                     \
        _Pragma("unroll") for (uint32_t i_ = 0; i_ < NDMA; i_++) {                                             \
            const uint8_t *a_ = ua[i_] + (uint64_t)SEG * min((uint32_t)(S_), un[i_]);                         \
            __builtin_amdgcn_global_load_lds((const void *)a_, (__attribute__((address_space(3))) void *)(d_ + 1024u * i_), \
                                             16, 0, AUX);                                                      \
        }                                                                                                      \
    } while (0)
    uint32_t R[4 * NU];
    // volatile: one ds_read_b128 per unit; left to itself the compiler split
    // the reads into ds_read2_b32, whose 32-bank groups conflict
    typedef uint32_t FsVec __attribute__((ext_vector_type(4)));
#define RSG_FS_READ(SL_)                                                                                       \
    do {                                                                                                       \
        const uint8_t *b_ = slab + (SL_) * SLAB + lane * PIECE;                                                \
        _Pragma("unroll") for (uint32_t q_ = 0; q_ < (ALN ? 4 * CH : NU); q_++) {                              \
            const FsVec v_ = *(const volatile __attribute__((address_space(3))) FsVec *)(b_ + 16 * q_);        \
            R[4 * q_ + 0] = v_.x; R[4 * q_ + 1] = v_.y; R[4 * q_ + 2] = v_.z; R[4 * q_ + 3] = v_.w;             \
        }                                                                                                      \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                     \
    } while (0)
    // Two segments in flight per wave: segment s + 2 is issued into the slab
    // segment s was just copied out of
    RSG_FS_DMA(0u, 0u);
    if (S > 1) RSG_FS_DMA(1u, 1u);
    uint32_t h[4];
    md4_init(h);
    uint32_t carry = seed;  // seeded: the message word before the chunk's data words
    uint32_t X[16];
    const uint32_t tail_seg = (uint32_t)(nfull / CH), tail_i = (uint32_t)(nfull % CH);
#pragma unroll 1
    for (uint32_t s = 0; s < S; s++) {
        // segment s has landed once at most the younger segment's NDMA DMAs are pending
        if (s + 1 < S) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        RSG_FS_READ(s & 1u);
        if (s + 2 < S) RSG_FS_DMA(s + 2, s & 1u);  // in flight while segments s and s + 1 hash
        if (s <= tail_seg && s < nseg) {
#pragma unroll
            for (uint32_t i = 0; i < CH; i++) {
                if (s == tail_seg && i > tail_i) break;
                uint32_t D[16];
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    if constexpr (ALN) D[k] = R[16 * i + k];
                    else D[k] = __builtin_amdgcn_alignbyte(R[16 * i + k + 1], R[16 * i + k], sh);
                }
                if (SEEDED) {
                    X[0] = carry;
#pragma unroll
                    for (int k = 1; k < 16; k++) X[k] = D[k - 1];
                    carry = D[15];
                } else {
#pragma unroll
                    for (int k = 0; k < 16; k++) X[k] = D[k];
                }
                if (s == tail_seg && i == tail_i) break;  // the tail chunk's words stay in X
                md4_compress(h, X);
            }
        }
    }
#undef RSG_FS_DMA
#undef RSG_FS_READ
    if (!active) return;
    fs_tail(X, L, h);
    uint32_t *o = reinterpret_cast<uint32_t *>(out + 16ull * fi);
    o[0] = h[0]; o[1] = h[1]; o[2] = h[2]; o[3] = h[3];
}

hipError_t launch_file_sums(const uint8_t *arena, uint64_t arena_bytes, const FileSpan *files, const uint32_t *order,
                            uint32_t nfiles, uint32_t mode, uint32_t seed, uint8_t *out, bool aligned4,
                            hipStream_t stream) {
    if (nfiles == 0) return hipSuccess;
    // one-wave workgroups: the longest-first lane order then gives an LPT
    // schedule over the SIMDs (the second round of waves takes the shorter
    // files); the default cache policy (nt DMA re-read neighbouring units,
    // 1.47x the file bytes, profiles/r03d_filesums_summary.json)
    const dim3 grid((nfiles + 63) / 64), block(64);
    auto kern = mode == 1 ? (aligned4 ? file_sums_staged<true, 0, true> : file_sums_staged<true, 0, false>)
                          : (aligned4 ? file_sums_staged<false, 0, true> : file_sums_staged<false, 0, false>);
    hipLaunchKernelGGL(kern, grid, block, 0, stream, arena, arena_bytes, files, order, nfiles, seed, out);
    return hipGetLastError();
}

}  // namespace rsg
