// rsg_md4.h -- device-side MD4 compression and weak-sum helpers for gfx950.
//
// MD4 is the arithmetic of github.com/mmcloughlin/md4 v0.1.2 (go.mod:11),
// i.e. RFC 1320; the rsync strong block sum is MD4(block || int32_LE(seed))
// (internal/rsyncchecksum/rsyncchecksum.go:53-58).  One lane owns one message:
// MD4 is serial within a message, so the parallelism is across blocks.
//
// Instruction budget per 64-byte chunk (hipcc 7.2, gfx950): round 1 = 16 x
// {v_bitop3_b32, v_add3_u32, v_alignbit_b32}; rounds 2/3 = 16 x {v_bitop3_b32,
// v_add3_u32, v_add_u32 (constant), v_alignbit_b32}; 4 final adds: ~180 VALU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsg {

// Wave-uniform copies in SGPRs.  __builtin_amdgcn_readfirstlane returns int:
// widening that to 64 bits directly sign-extends the low word, so every
// 64-bit value is rebuilt from two uint32_t halves (an offset with bit 31 set
// otherwise came back with its upper word all ones).
__device__ __forceinline__ uint32_t rfl32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl32((uint32_t)(v >> 32)) << 32) | (uint64_t)rfl32((uint32_t)v);
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
    return __builtin_amdgcn_alignbit(x, x, 32 - s);
}

// F = x ? y : z, G = majority, H = parity, each one v_bitop3_b32 (LUT index
// 4*S0 + 2*S1 + S2).  Written as the intrinsic so the compiler cannot split F
// into disjoint AND terms folded into the adds (which costs 2 extra VALU/step).
#define RSG_F(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0xca)
#define RSG_G(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0xe8)
#define RSG_H(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0x96)
#define RSG_R1(a, b, c, d, k, s) a = rotl(a + RSG_F(b, c, d) + X[k], s)
#define RSG_R2(a, b, c, d, k, s) a = rotl(a + RSG_G(b, c, d) + X[k] + 0x5A827999u, s)
#define RSG_R3(a, b, c, d, k, s) a = rotl(a + RSG_H(b, c, d) + X[k] + 0x6ED9EBA1u, s)

// One MD4 compression of the 16 little-endian message words X into h.
__device__ __forceinline__ void md4_compress(uint32_t h[4], const uint32_t X[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    RSG_R1(a, b, c, d, 0, 3);  RSG_R1(d, a, b, c, 1, 7);  RSG_R1(c, d, a, b, 2, 11);  RSG_R1(b, c, d, a, 3, 19);
    RSG_R1(a, b, c, d, 4, 3);  RSG_R1(d, a, b, c, 5, 7);  RSG_R1(c, d, a, b, 6, 11);  RSG_R1(b, c, d, a, 7, 19);
    RSG_R1(a, b, c, d, 8, 3);  RSG_R1(d, a, b, c, 9, 7);  RSG_R1(c, d, a, b, 10, 11); RSG_R1(b, c, d, a, 11, 19);
    RSG_R1(a, b, c, d, 12, 3); RSG_R1(d, a, b, c, 13, 7); RSG_R1(c, d, a, b, 14, 11); RSG_R1(b, c, d, a, 15, 19);

    RSG_R2(a, b, c, d, 0, 3);  RSG_R2(d, a, b, c, 4, 5);  RSG_R2(c, d, a, b, 8, 9);   RSG_R2(b, c, d, a, 12, 13);
    RSG_R2(a, b, c, d, 1, 3);  RSG_R2(d, a, b, c, 5, 5);  RSG_R2(c, d, a, b, 9, 9);   RSG_R2(b, c, d, a, 13, 13);
    RSG_R2(a, b, c, d, 2, 3);  RSG_R2(d, a, b, c, 6, 5);  RSG_R2(c, d, a, b, 10, 9);  RSG_R2(b, c, d, a, 14, 13);
    RSG_R2(a, b, c, d, 3, 3);  RSG_R2(d, a, b, c, 7, 5);  RSG_R2(c, d, a, b, 11, 9);  RSG_R2(b, c, d, a, 15, 13);

    RSG_R3(a, b, c, d, 0, 3);  RSG_R3(d, a, b, c, 8, 9);  RSG_R3(c, d, a, b, 4, 11);  RSG_R3(b, c, d, a, 12, 15);
    RSG_R3(a, b, c, d, 2, 3);  RSG_R3(d, a, b, c, 10, 9); RSG_R3(c, d, a, b, 6, 11);  RSG_R3(b, c, d, a, 14, 15);
    RSG_R3(a, b, c, d, 1, 3);  RSG_R3(d, a, b, c, 9, 9);  RSG_R3(c, d, a, b, 5, 11);  RSG_R3(b, c, d, a, 13, 15);
    RSG_R3(a, b, c, d, 3, 3);  RSG_R3(d, a, b, c, 11, 9); RSG_R3(c, d, a, b, 7, 11);  RSG_R3(b, c, d, a, 15, 15);
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

#undef RSG_R1
#undef RSG_R2
#undef RSG_R3
#undef RSG_F
#undef RSG_G
#undef RSG_H

__device__ __forceinline__ void md4_init(uint32_t h[4]) {
    h[0] = 0x67452301u; h[1] = 0xEFCDAB89u; h[2] = 0x98BADCFEu; h[3] = 0x10325476u;
}

// Weak-sum accumulation over one 64-byte chunk (Checksum1,
// rsyncchecksum.go:29-51).  Bytes are signed (SignExtend, :24-27), which is
// exactly the i8 x i8 product of v_dot4c_i32_i8.  For a block of n bytes
//   s1 = sum x_i,  s2 = sum (n - i) x_i = n*s1 - T,  T = sum i*x_i.
// Per chunk: s1 += dot(x_k, 1), tl += dot(x_k, (4k, 4k+1, 4k+2, 4k+3)); the
// caller adds 64*c*(chunk sum) to T.
__device__ __forceinline__ void weak_chunk(const uint32_t X[16], int32_t &s1, int32_t &tl) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int w = (4 * k) | ((4 * k + 1) << 8) | ((4 * k + 2) << 16) | ((4 * k + 3) << 24);
        s1 = __builtin_amdgcn_sdot4((int)X[k], 0x01010101, s1, false);
        tl = __builtin_amdgcn_sdot4((int)X[k], w, tl, false);
    }
}

}  // namespace rsg
