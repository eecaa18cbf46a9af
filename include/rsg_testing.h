/*
 * rsg_testing.h -- test hooks of librsg.so.  NOT part of the drop-in
 * boundary (include/rsg.h): no Go binding calls these.  They expose host-only
 * logic of the engine so the CPU test suite can check it without a GPU.
 */
#ifndef RSG_TESTING_H
#define RSG_TESTING_H

#include "rsg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The sender's greedy walk over sorted candidate offsets (the host half of
 * hashSearch, internal/sender/match.go:93-210) with the GPU confirmation
 * replaced by answers: truth[k] = the block candidate k confirms to (>= 0)
 * or -1.  cand must be strictly increasing.  Returns the match list the walk
 * produces and stats[0] = confirmation round trips, stats[1] = windows
 * confirmed, i.e. what the GPU path would have issued.  On input stats[0]
 * picks the sparse batches' selection: 1 = speculative, 0 or 2 = every
 * pending candidate (the default, as the "spec" option of
 * rsg_testing_search_option). */
rsg_status rsg_testing_walk(const uint64_t *cand, uint64_t n, const int32_t *truth, uint64_t size,
                            const rsg_sum_head *head, rsg_match *out, uint64_t cap, uint64_t *n_out,
                            uint64_t stats[2]);

/* The block-sum kernel variant a launch takes (host arithmetic, the rule
 * rsg_set_block_sums_kernel documents): variant (-1 = automatic) for a batch
 * whose blocks are all 4-byte aligned (aligned), all on 128-byte lines
 * (lines128), in an arena whose base is aligned to arena_align (0: less than
 * 4 bytes, 1: 4 bytes, 2: 128 bytes), longest block max_blen.  -2 for a
 * variant rsg_set_block_sums_kernel rejects. */
int32_t rsg_testing_block_sums_choice(int32_t variant, int32_t aligned, int32_t lines128, int32_t arena_align,
                                      uint32_t max_blen);

/* The product's host MD4 (RFC 1320; rsync_amd/csrc/rsg_md4_host.cpp), used
 * for whole-file sums whose bytes stream through host memory: the sender's
 * MD4(int32_LE(seed) || source) in rsg_hash_search_fd and receiveData's
 * check of large files.  seeded != 0 prefixes int32_LE(seed) (match.go:52-53).
 * The data is hashed in `piece`-byte updates (0 = one update) to exercise
 * the streaming path. */
rsg_status rsg_testing_md4(const uint8_t *data, uint64_t n, int32_t seeded, int32_t seed, uint64_t piece,
                           uint8_t out[16]);

/* Per-context options of the sender and receiver, for tests and same-box
 * A/B runs (the defaults are the measured product settings; results are the
 * same under every value):
 *   0 search path: 0 (default) = sources of at most 1 MiB with at most 1024
 *     basis blocks of at most 8 KiB through the one-wave-per-file kernel
 *     (rsync_amd/csrc/rsg_search_small.hip), the rest through the
 *     large-file pipeline; 1 = every source through the pipeline;
 *   1 host-built roll tables (0 default: built on the GPU);
 *   2 report every GPU-built bucket table as overflowed, so the rolls pass
 *     every filter hit on and the confirmation alone decides (0 default);
 *   3 speculative selection of the confirmed windows (0 default);
 *   4 CUs a batch's rolls leave to the previous job's confirmation (default
 *     32; 0 = confirmations serialised behind the rolls);
 *   5 receiveData's whole-file sums: 0 (default) by file size, 1 GPU, 2 host;
 *   6 the whole-file sums' lane order: files sorted longest first in length
 *     buckets of 2^value bytes, 0..40 (default 10; 40 keeps the callers'
 *     order).
 * RSG_ERR_INVALID for an unknown option or value. */
rsg_status rsg_testing_search_option(rsg_ctx *ctx, int32_t option, int32_t value);

/* rsg_generate_files_fd_multi's per-rank record queue: *peak (if not NULL)
 * = the largest number of record bytes any rank had queued during the last
 * call; cap != 0 sets the bound per rank for later calls (default 256 MiB,
 * rsg.h).  Process-wide, not per context. */
rsg_status rsg_testing_multi_queue(uint64_t cap, uint64_t *peak);

#ifdef __cplusplus
}
#endif
#endif /* RSG_TESTING_H */
