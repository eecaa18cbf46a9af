// rsg_match.cpp -- sender hash search (match.go:21-230) orchestration.
#include "rsg_host.h"

using namespace rsgh;

extern "C" {

rsg_status rsg_hash_search_host(rsg_ctx *ctx, const uint8_t *src, uint64_t src_len, const rsg_sum_head *head,
                                const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    (void)src; (void)src_len; (void)head; (void)sum1; (void)sum2; (void)targets; (void)seed;
    (void)matches; (void)match_cap; (void)n_matches;
    return fail(ctx, RSG_ERR_INVALID, "hash search not built yet");
}

rsg_status rsg_hash_search_device(rsg_ctx *ctx, const void *d_src, uint64_t src_len, const rsg_sum_head *head,
                                  const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                  rsg_match *matches, uint64_t match_cap, uint64_t *n_matches) {
    (void)d_src; (void)src_len; (void)head; (void)sum1; (void)sum2; (void)targets; (void)seed;
    (void)matches; (void)match_cap; (void)n_matches;
    return fail(ctx, RSG_ERR_INVALID, "hash search not built yet");
}

}  // extern "C"
