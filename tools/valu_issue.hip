// VALU issue-rate probe for the instructions of the packed roll
// (rsg_match_kernels.hip roll_packed_kernel): 16 independent chains per lane,
// 1024 threads per workgroup (4 waves per SIMD, the roll's occupancy), one
// workgroup per CU.  Prints cycles per wave-instruction per SIMD at the
// measured clock.  Build: hipcc --offload-arch=gfx950 -O3 -o valu_issue valu_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define STEP8(INS)                                                                         \
    asm volatile(INS : "+v"(a0) : "v"(k0), "v"(k1));                                        \
    if (CH > 8) {                                                                           \
        asm volatile(INS : "+v"(b0) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b1) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b2) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b3) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b4) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b5) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b6) : "v"(k0), "v"(k1));                                    \
        asm volatile(INS : "+v"(b7) : "v"(k0), "v"(k1));                                    \
    }                                                                                       \
    asm volatile(INS : "+v"(a1) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a2) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a3) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a4) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a5) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a6) : "v"(k0), "v"(k1));                                        \
    asm volatile(INS : "+v"(a7) : "v"(k0), "v"(k1));

#define STEP8M(IA, IB)                                                                     \
    asm volatile(IA : "+v"(a0) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(a1) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(a2) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(a3) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(b0) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(b1) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(b2) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(b3) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(a4) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(a5) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(a6) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(a7) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(b4) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(b5) : "v"(k0), "v"(k1));                                         \
    asm volatile(IA : "+v"(b6) : "v"(k0), "v"(k1));                                         \
    asm volatile(IB : "+v"(b7) : "v"(k0), "v"(k1));

template <int OP, int CH>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint64_t *cyc, int iters, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    uint32_t k0 = seed * 3 + threadIdx.x, k1 = seed ^ 0x01020304u;
    uint32_t b0 = a0 * 5, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
        if constexpr (OP == 0) { STEP8("v_xor_b32 %0, %0, %1") }
        if constexpr (OP == 1) { STEP8("v_perm_b32 %0, %0, %1, %2") }
        if constexpr (OP == 2) { STEP8("v_pk_add_u16 %0, %0, %1") }
        if constexpr (OP == 3) { STEP8("v_pk_mad_u16 %0, %0, %1, %2") }
        if constexpr (OP == 4) { STEP8("v_pk_lshrrev_b16 %0, %1, %0") }
        if constexpr (OP == 5) { STEP8("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1") }
        if constexpr (OP == 6) { STEP8("v_add3_u32 %0, %0, %1, %2") }
        if constexpr (OP == 7) { STEP8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80") }
        if constexpr (OP == 8) { STEP8("v_mul_lo_u32 %0, %0, %1") }
        if constexpr (OP == 9) { STEP8("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 10) { STEP8("v_and_b32 %0, %0, %1") }
        if constexpr (OP == 11) { STEP8("v_alignbyte_b32 %0, %0, %1, %2") }
        if constexpr (OP == 12) { STEP8("v_lshl_or_b32 %0, %0, %1, %2") }
        if constexpr (OP == 13) { STEP8("v_dot4_i32_i8 %0, %1, %2, %0") }
        if constexpr (OP == 14) { STEP8("v_pk_sub_u16 %0, %0, %1") }
        if constexpr (OP == 15) { STEP8("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1") }
        if constexpr (OP == 16) { STEP8("v_lshrrev_b32 %0, %1, %0") }
        if constexpr (OP == 17) { STEP8("v_lshlrev_b32 %0, %1, %0") }
        if constexpr (OP == 18) { STEP8("v_and_or_b32 %0, %0, %1, %2") }
        if constexpr (OP == 19) { STEP8("v_bfe_u32 %0, %0, %1, %2") }
        if constexpr (OP == 20) { STEP8("v_bfi_b32 %0, %0, %1, %2") }
        if constexpr (OP == 21) { STEP8("v_lshl_add_u32 %0, %0, %1, %2") }
        if constexpr (OP == 22) { STEP8("v_mad_u32_u16 %0, %0, %1, %2") }
        if constexpr (OP == 23) { STEP8("v_mul_u32_u24 %0, %0, %1") }
        if constexpr (OP == 24) { STEP8("v_pk_lshlrev_b16 %0, %1, %0") }
        if constexpr (OP == 25) { STEP8("v_sub_u32 %0, %0, %1") }
        if constexpr (OP == 26) { STEP8("v_or_b32 %0, %0, %1") }
        if constexpr (OP == 27) { STEP8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") }
        if constexpr (OP == 28) { STEP8("v_cndmask_b32 %0, %0, %1, vcc") }
        if constexpr (OP == 29) { STEP8("v_add_u16 %0, %0, %1") }
        if constexpr (OP == 30) { STEP8("v_lshrrev_b16 %0, %1, %0") }
        if constexpr (OP == 31) { STEP8("v_and_b32_e64 %0, %0, %1") }
        if constexpr (OP == 32) { STEP8("v_xad_u32 %0, %0, %1, %2") }
        if constexpr (OP == 33) { STEP8("v_or3_b32 %0, %0, %1, %2") }
        if constexpr (OP == 34) { STEP8("v_mov_b32 %0, %1") }
        if constexpr (OP == 35) { STEP8("v_pk_max_u16 %0, %0, %1") }
        if constexpr (OP == 36) { STEP8M("v_perm_b32 %0, %0, %1, %2", "v_xor_b32 %0, %0, %1") }
        if constexpr (OP == 37) { STEP8M("v_pk_add_u16 %0, %0, %1", "v_and_b32 %0, %0, %1") }
        if constexpr (OP == 38) { STEP8M("v_pk_add_u16 %0, %0, %1", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x80") }
        if constexpr (OP == 39) { STEP8M("v_xor_b32 %0, %0, %1", "v_and_b32 %0, %0, %1") }
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char *kNames[] = {"v_xor_b32", "v_perm_b32", "v_pk_add_u16", "v_pk_mad_u16", "v_pk_lshrrev_b16", "v_lshlrev_b32_sdwa", "v_add3_u32", "v_bitop3_b32", "v_mul_lo_u32", "v_add_u32", "v_and_b32", "v_alignbyte_b32", "v_lshl_or_b32", "v_dot4_i32_i8", "v_pk_sub_u16", "v_sub_u32_sdwa(byte)", "v_lshrrev_b32", "v_lshlrev_b32", "v_and_or_b32", "v_bfe_u32", "v_bfi_b32", "v_lshl_add_u32", "v_mad_u32_u16", "v_mul_u32_u24", "v_pk_lshlrev_b16", "v_sub_u32", "v_or_b32", "v_bitop3(xor3)", "v_cndmask_b32(vcc)", "v_add_u16", "v_lshrrev_b16", "v_and_b32_e64", "v_xad_u32", "v_or3_b32", "v_mov_b32", "v_pk_max_u16", "mix perm+xor", "mix pk_add+and", "mix pk_add+bitop3", "mix xor+and"};

template <int OP, int CH>
static void run1(uint32_t *out, uint64_t *cyc, uint64_t *hc, int cus, int wps, int iters, double clk_ghz) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int threads = 1024, blocks = cus * wps / 4;  // wps waves per SIMD: wps/4 workgroups of 16 waves per CU
    hipLaunchKernelGGL((probe<OP, CH>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 100, 1u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((probe<OP, CH>), dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const int nw = blocks * 16;
    (void)hipMemcpy(hc, cyc, nw * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < nw; i++) mean += (double)hc[i];
    mean /= nw;
    const double inst = (double)wps * iters * CH;  // wave-instructions per SIMD
    printf("%-22s ch %2d waves/SIMD %d  %8.3f ms  wall %5.2f cyc@%.2fGHz  in-kernel %5.2f cyc/SIMD  (clock %.2f GHz)\n",
           kNames[OP], CH, wps, ms, ms * 1e-3 * clk_ghz * 1e9 / inst, clk_ghz, mean / ((double)iters * CH * wps),
           mean / (ms * 1e-3) / 1e9);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

template <int OP>
static void run(uint32_t *out, uint64_t *cyc, uint64_t *hc, int cus, double clk) {
    run1<OP, 16>(out, cyc, hc, cus, 4, 50000, clk);
    run1<OP, 16>(out, cyc, hc, cus, 8, 50000, clk);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate / 1e6;  // kHz -> GHz
    printf("CUs %d, clock %.3f GHz (peak); in-kernel cycles are per wave-instruction of one wave (issue interval)\n", cus, clk);
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, (size_t)cus * 2048 * 4);
    (void)hipMalloc(&cyc, (size_t)cus * 32 * 8);
    static uint64_t hc[256 * 32];
    run<0>(out, cyc, hc, cus, clk);
    run<1>(out, cyc, hc, cus, clk);
    run<2>(out, cyc, hc, cus, clk);
    run<3>(out, cyc, hc, cus, clk);
    run<4>(out, cyc, hc, cus, clk);
    run<5>(out, cyc, hc, cus, clk);
    run<6>(out, cyc, hc, cus, clk);
    run<7>(out, cyc, hc, cus, clk);
    run<8>(out, cyc, hc, cus, clk);
    run<9>(out, cyc, hc, cus, clk);
    run<10>(out, cyc, hc, cus, clk);
    run<11>(out, cyc, hc, cus, clk);
    run<12>(out, cyc, hc, cus, clk);
    run<13>(out, cyc, hc, cus, clk);
    run<14>(out, cyc, hc, cus, clk);
    run<15>(out, cyc, hc, cus, clk);
    run<16>(out, cyc, hc, cus, clk);
    run<17>(out, cyc, hc, cus, clk);
    run<18>(out, cyc, hc, cus, clk);
    run<19>(out, cyc, hc, cus, clk);
    run<20>(out, cyc, hc, cus, clk);
    run<21>(out, cyc, hc, cus, clk);
    run<22>(out, cyc, hc, cus, clk);
    run<23>(out, cyc, hc, cus, clk);
    run<24>(out, cyc, hc, cus, clk);
    run<25>(out, cyc, hc, cus, clk);
    run<26>(out, cyc, hc, cus, clk);
    run<27>(out, cyc, hc, cus, clk);
    run<28>(out, cyc, hc, cus, clk);
    run<29>(out, cyc, hc, cus, clk);
    run<30>(out, cyc, hc, cus, clk);
    run<31>(out, cyc, hc, cus, clk);
    run<32>(out, cyc, hc, cus, clk);
    run<33>(out, cyc, hc, cus, clk);
    run<34>(out, cyc, hc, cus, clk);
    run<35>(out, cyc, hc, cus, clk);
    run<36>(out, cyc, hc, cus, clk);
    run<37>(out, cyc, hc, cus, clk);
    run<38>(out, cyc, hc, cus, clk);
    run<39>(out, cyc, hc, cus, clk);
    (void)hipFree(out);
    (void)hipFree(cyc);
    return 0;
}
