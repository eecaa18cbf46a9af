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

__global__ __launch_bounds__(64) void file_sums_kernel(const uint8_t *__restrict__ arena, uint64_t arena_bytes,
                                                       const FileSpan *__restrict__ files,
                                                       const uint32_t *__restrict__ order, uint32_t nfiles,
                                                       uint32_t mode, uint32_t seed, uint8_t *__restrict__ out) {
    const uint32_t lane_file = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane_file >= nfiles) return;
    const uint32_t fi = order[lane_file];
    const FileSpan F = files[fi];
    const uint8_t *d = arena + F.offset;
    const uintptr_t end = (uintptr_t)(arena + arena_bytes);
    const uint64_t pre = mode == 1 ? 4u : 0u;  // prefix bytes (the seed)
    const uint64_t L = F.len + pre;             // message length
    const uint64_t nfull = L >> 6;
    uint32_t h[4];
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
    // tail: r = L % 64 message bytes, 0x80, zeros, 64-bit bit length (RFC 1320)
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
    uint32_t *o = reinterpret_cast<uint32_t *>(out + 16ull * fi);
    o[0] = h[0]; o[1] = h[1]; o[2] = h[2]; o[3] = h[3];
}

hipError_t launch_file_sums(const uint8_t *arena, uint64_t arena_bytes, const FileSpan *files, const uint32_t *order,
                            uint32_t nfiles, uint32_t mode, uint32_t seed, uint8_t *out, hipStream_t stream) {
    if (nfiles == 0) return hipSuccess;
    // one-wave workgroups: the longest-first lane order then gives an LPT
    // schedule over the SIMDs (the second round of waves takes the shorter files)
    hipLaunchKernelGGL(file_sums_kernel, dim3((nfiles + 63) / 64), dim3(64), 0, stream, arena, arena_bytes, files,
                       order, nfiles, mode, seed, out);
    return hipGetLastError();
}

}  // namespace rsg
