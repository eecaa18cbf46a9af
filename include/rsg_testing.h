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
 * confirmed, i.e. what the GPU path would have issued. */
rsg_status rsg_testing_walk(const uint64_t *cand, uint64_t n, const int32_t *truth, uint64_t size,
                            const rsg_sum_head *head, rsg_match *out, uint64_t cap, uint64_t *n_out,
                            uint64_t stats[2]);

#ifdef __cplusplus
}
#endif
#endif /* RSG_TESTING_H */
