// rsg_internal.h -- shared declarations between the C-ABI host code and the
// HIP kernels of librsg.so (not part of the public ABI; see include/rsg.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsg {

constexpr uint32_t kRecordBytes = 20;       // int32 sum1 + sum2[16], generator.go:341-346
constexpr uint32_t kBlockSumThreads = 256;  // lanes (= blocks) per workgroup

// Per-file descriptor of a block-sum batch, resident in HBM (32 bytes).
struct DevFile {
    uint64_t offset;       // byte offset of the file in the arena
    uint64_t len;          // file length
    uint64_t first_block;  // global index of the file's first block/record
    uint32_t blen;         // block length B (> 0)
    uint32_t nblocks;      // ceil(len / B)
};
static_assert(sizeof(DevFile) == 32, "DevFile layout");

hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t max_blen, uint32_t seed, uint8_t *out, hipStream_t stream);

// 0 = direct (per-lane loads), 1 = staged (LDS DMA, default for aligned batches).
void set_block_sums_variant(int v);

hipError_t launch_fill_splitmix64(uint8_t *dst, uint64_t n, uint64_t seed, hipStream_t stream);

}  // namespace rsg
