// rsg_internal.h -- shared declarations between the C-ABI host code and the
// HIP kernels of librsg.so (not part of the public ABI; see include/rsg.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsg {

constexpr uint32_t kRecordBytes = 20;       // int32 sum1 + sum2[16], generator.go:341-346
constexpr uint32_t kBlockSumThreads = 256;  // lanes (= blocks) per workgroup
// Unaligned batches of long blocks (>= kLongBlockBytes; the sender's
// confirmation windows) take the deep-prefetch kernel: per-lane loads with
// only one chunk in flight leave HBM latency exposed.
constexpr uint32_t kLongBlockBytes = 8192;

// Per-file descriptor of a block-sum batch, resident in HBM (32 bytes).
struct DevFile {
    uint64_t offset;       // byte offset of the file in the arena
    uint64_t len;          // file length
    uint64_t first_block;  // global index of the file's first block/record
    uint32_t blen;         // block length B (> 0)
    uint32_t nblocks;      // ceil(len / B)
};
static_assert(sizeof(DevFile) == 32, "DevFile layout");

// variant: the calling context's knob (-1 automatic, rsg_set_block_sums_kernel).
hipError_t launch_block_sums(const uint8_t *arena, uint64_t arena_bytes, const DevFile *files,
                             const uint32_t *wg_file, uint64_t total_blocks, uint32_t nwg, bool aligned,
                             uint32_t max_blen, uint32_t seed, uint8_t *out, uint32_t lds_reserve, int variant,
                             hipStream_t stream, bool lines128 = false);
// The variant a launch takes (rsg_blocksums.hip: the automatic rule and the
// fallbacks of variants a batch cannot take); host arithmetic.
// arena_align: 0 = the arena base not 4-byte aligned, 1 = 4-byte, 2 = 128-byte
int block_sums_choice(int variant, bool aligned, bool lines128, int arena_align, uint32_t max_blen);
bool block_sums_variant_valid(int variant);  // -1, 0, 1, 2, 3, 4, 6, 7
// Files packed into an arena by the library start at multiples of this, so
// blocks whose length is a multiple of 128 start on 128-byte lines
constexpr uint64_t kPackAlign = 128;
inline uint64_t pack_round(uint64_t n) { return (n + kPackAlign - 1) & ~(kPackAlign - 1); }

// Device scratch a block-sum launch needs: 4 + 4 * ceil(total_blocks / 64) bytes.
inline uint64_t block_sums_scratch_bytes(uint64_t total_blocks) { return 8 + 4 * ((total_blocks + 63) / 64); }

// RSG_BLOCKSUMS_KERNEL (read once): a context's initial variant.
int block_sums_variant_env();
// Fallback census of the current device: [0] staged waves, [1] park tiles
// (full ones that took per-lane loads); synchronises the device.
hipError_t read_block_sums_fallbacks(uint64_t out[2], bool reset);

// ---- sender search (rsg_match_kernels.hip)
constexpr uint32_t kScanTile = 32768;                          // source bytes per tile
constexpr uint32_t kRollThreads = 1024;                        // lanes per roll workgroup
constexpr uint32_t kRollPerThread = kScanTile / kRollThreads;  // consecutive offsets per lane
constexpr uint32_t kFilterBits = 1u << 20;                     // 128 KiB LDS filter

struct TileAgg {     // per tile: whole tile and its first r = B % kScanTile bytes
    uint32_t a1, a2;  // sum x, sum (i - tile_start) * x
    uint32_t r1, r2;
};
struct TilePrefix {  // at a tile start: P = sum_{i<j} x_i, Q = sum_{i<j} i * x_i (mod 2^32)
    uint32_t p, q;
};

// Blocked Bloom filter of the basis weak sums (low half s1, high half s2):
// every sum sets two bits of ONE 32-bit word, so a probe is one LDS read.
// h = rotl(sum, 13) ^ sum (two VALU: no multiply); word = h[2:16] (the LDS
// byte address is h & 0x1fffc), bits = h[22:26] and h[27:31].  With the
// 32768 sums of a 1 GiB basis at B = 32 KiB, 0.7 % of non-matching offsets
// pass (simulated on uniform sums, as a multiplicative hash; a one-bit 64 KiB
// bitmap passed 6 %).
__host__ __device__ inline uint32_t filter_hash(uint32_t sum) { return ((sum << 13) | (sum >> 19)) ^ sum; }
__host__ __device__ inline uint32_t filter_word(uint32_t h) { return (h >> 2) & 0x7fffu; }  // 2^15 words
__host__ __device__ inline uint32_t filter_mask(uint32_t h) { return (1u << ((h >> 22) & 31u)) | (1u << (h >> 27)); }
// Bit-selection layout (the default): no hash arithmetic.  Word
// sum[2..16] (byte address sum & 0x1fffc), bits sum[24..28] and
// rotr(sum, 29)[0..4] = {sum[29..31], sum[0..1]}: 25 disjoint bits of the sum.
__host__ __device__ inline uint32_t sel_word(uint32_t s) { return (s >> 2) & 0x7fffu; }
__host__ __device__ inline uint32_t sel_mask(uint32_t s) {
    return (1u << ((s >> 24) & 31u)) | (1u << (((s >> 29) | (s << 3)) & 31u));
}

// Exact table of basis weak sums: buckets of kBucketWays u64 entries
// {sum1 << 32 | flags}; a sum lives in bucket hash1 or hash2.
constexpr uint32_t kBucketWays = 4;
__host__ __device__ inline uint32_t bucket_hash1(uint32_t s) { return (s * 0x9E3779B1u) >> 7; }
__host__ __device__ inline uint32_t bucket_hash2(uint32_t s) { return ((s ^ (s >> 15)) * 0x85EBCA77u) >> 9; }

hipError_t launch_tile_agg(const uint8_t *src, uint64_t size, uint32_t r, TileAgg *out, uint32_t ntiles,
                           hipStream_t stream);
hipError_t launch_tile_scan(const TileAgg *agg, uint32_t ntiles, TilePrefix *pre, hipStream_t stream);
// Resolve confirmed windows to blocks (match.go:108-136): window i (record i,
// length files[i].len) -> the first block in targets order with equal Sum1,
// equal length and equal sum2[:s2len], or -1.  groups = (sum1, block) sorted
// by sum1 (stable in targets order), hi16[h] = first group with sum1 >> 16 == h.
hipError_t launch_confirm_plan(const uint64_t *cand, uint32_t n, uint64_t size, uint32_t B, DevFile *files,
                               uint32_t *wg_file, uint32_t nwg, hipStream_t stream);
hipError_t launch_resolve(const uint8_t *records, const DevFile *files, uint64_t n, const uint2 *groups,
                          const uint32_t *hi16, const uint8_t *sum2, int32_t count, int32_t blen, int32_t rem,
                          int32_t s2len, int32_t *res, hipStream_t stream);
// After a roll, on its stream: the candidate count to the pinned host word
// `host` and the device counter back to 0 for the next roll (one launch
// instead of a memset and a 4-byte copy, each with its own dispatch gap).
hipError_t launch_roll_count_out(uint32_t *count, uint32_t *host, hipStream_t stream);
hipError_t launch_roll(const uint8_t *src, uint64_t size, uint32_t B, uint32_t rem, uint64_t end, uint32_t tile_lo,
                       uint32_t tile_hi, const TileAgg *agg, const TilePrefix *pre, uint32_t ntiles,
                       const uint32_t *bitmap, const uint16_t *filter16, const uint64_t *table,
                       const uint32_t *table_keys, uint32_t bmask, uint64_t *cand, uint32_t cap, uint32_t *count,
                       const uint32_t *ovf, uint32_t grid, bool fused, hipStream_t stream);
// The roll's tables (bitmap, filter16 if packed, bucket table of nb buckets
// and its key-only copy) built on the GPU from sum1[0..count), into zeroed
// memory; *ovf = 1 if some key found no slot (rsg_match_kernels.hip).
hipError_t launch_build_tables(const uint32_t *sum1, int32_t count, uint32_t B, uint32_t rem, bool packed,
                               uint32_t *bitmap, uint16_t *filter16, uint64_t *table, uint32_t *keys, uint32_t nb,
                               uint32_t *ovf, bool force_ovf, hipStream_t stream);
// The packed roll's filter (roll_packed_kernel, fused mode, interior tiles):
// 2^16 16-bit words, word ((s1 + 128 B) xor s2) mod 2^16, bits s2[0..3],
// s2[4..7] and s2[8..11] (a third bit: 0.6 % false hits instead of 1.0 %).  s1 of a long window of random bytes is
// a sum of B terms (near-Gaussian mod 2^16): a word indexed by s1 alone passed
// 1.9 % of real window sums with two bits, the xor with s2 ~1.0 %.
constexpr uint32_t kFilter16Words = 1u << 16;
__host__ __device__ inline uint32_t f16_word(uint32_t sum, uint32_t B) {
    return ((sum + 128u * B) ^ (sum >> 16)) & 0xffffu;
}
// The bits sit at 15 - s (s = the nibble): the kernel shifts the word LEFT by
// s (v_pk_lshlrev_b16 masks the count to 4 bits itself), so every tested bit
// lands in bit 15 of its half and the AND of the shifted words is the test,
// read by sign compares with no mask.
__host__ __device__ inline uint32_t f16_mask(uint32_t sum) {
    return (0x8000u >> ((sum >> 16) & 15u)) | (0x8000u >> ((sum >> 20) & 15u)) | (0x8000u >> ((sum >> 24) & 15u));
}
// Block lengths up to which roll derives its window sums itself (no tile_agg
// / tile_scan passes): each workgroup reads B extra bytes once.
constexpr uint32_t kFusedMaxB = 4 * kScanTile;

// ---- small-file sender (rsg_search_small.hip): one wave searches one source
// file end to end (basis sums into LDS, weak sum at every offset, MD4
// confirmation, the greedy walk), so many small files cost one launch.
constexpr uint32_t kSmallMaxSrc = 1u << 20;    // source bytes
constexpr int32_t kSmallMaxCount = 1024;       // basis blocks
constexpr uint32_t kSmallMaxBlock = 8192;      // block length (each lane sums a window of B bytes)
struct SmallJob {        // 40 bytes, one per file of a launch
    uint64_t src;        // device address of the source
    uint64_t sums;       // byte offset in the launch's blob of sum1[count] | targets[count] | sum2[16 count]
    uint32_t size;       // source length, 1..kSmallMaxSrc
    int32_t count;       // 1..kSmallMaxCount
    uint32_t blen;       // SumHead block length (1..kSmallMaxBlock)
    uint32_t rem;        // SumHead remainder (0 = the last block is full)
    uint32_t s2len;      // bytes of sum2 compared (0..16)
    uint32_t pad;
};
static_assert(sizeof(SmallJob) == 40, "SmallJob layout");
struct SmallOut {        // per file: matches at [base, base + n) of the launch's match array
    uint32_t base, n;
    uint32_t status;     // 0 ok, 1 more candidates than the LDS list holds, 2 match array full
    uint32_t ncand;      // weak-sum candidates (filter hits) the roll found
};
// LDS words of one wave for a launch whose counts are <= kc (a power of two):
// filter (reused for the confirmation results) | keys (u64, kc) | candidates (u64, ccap)
inline uint32_t small_ccap(uint32_t kc) { return kc * 2 < 512 ? 512 : kc * 2; }
inline uint32_t small_fwords(uint32_t kc) { return kc * 4 < 512 ? 512 : kc * 4; }
inline uint32_t small_lds_bytes(uint32_t kc) {
    const uint32_t f = small_fwords(kc) > small_ccap(kc) ? small_fwords(kc) : small_ccap(kc);
    return 4 * f + 8 * kc + 8 * small_ccap(kc) + 16;
}
hipError_t launch_search_small(const SmallJob *jobs, const uint32_t *order, uint32_t njobs, const uint8_t *blob,
                               uint32_t seed, uint32_t kc, void *matches, uint32_t match_cap,
                               uint32_t *match_count, SmallOut *outs, hipStream_t stream);

// ---- whole-file sums (rsg_filesums.hip)
struct FileSpan {
    uint64_t offset;  // byte offset of the file in the arena
    uint64_t len;
};
// out[16 * i] = MD4 of file i: mode 0 MD4(file), mode 1 MD4(int32_LE(seed) || file).
// order = a permutation of the files (lane k hashes file order[k]).
// aligned4: every file offset (and the arena) 4-byte aligned -- segments of
// exactly 256 file bytes, no funnel shift.
hipError_t launch_file_sums(const uint8_t *arena, uint64_t arena_bytes, const FileSpan *files, const uint32_t *order,
                            uint32_t nfiles, uint32_t mode, uint32_t seed, uint8_t *out, bool aligned4,
                            hipStream_t stream);

hipError_t launch_fill_splitmix64(uint8_t *dst, uint64_t n, uint64_t seed, hipStream_t stream);

}  // namespace rsg
