// rsg_receiver.cpp -- the receiver's token application:
// receiveData + recvToken, internal/receiver/receiver.go:98-188 and
// internal/receiver/token.go:6-20.
//
// The token stream (after the SumHead) is: literal runs (int32 LE n > 0, then
// n bytes), block matches (int32 -(i+1): block i of the basis, BlockLength
// bytes at i*BlockLength, RemainderLength for the last block), the int32 0
// terminator, then the sender's 16-byte whole-file sum MD4(int32_LE(seed) ||
// file).  Rebuilding is byte copying (the reference does one ReadAt per
// matched block); the whole-file sum check runs on the GPU through the
// seeded file-sum kernel (rsg_filesums.hip).
#include <string.h>

#include "rsg_host.h"

using namespace rsgh;

namespace {

int32_t rd_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// Walks the stream; copies into out while it fits.  Sets *out_len (the
// rebuilt length) and *sum_at (offset of the 16-byte whole-file sum).
rsg_status apply(rsg_ctx *ctx, const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                 const uint8_t *basis, uint64_t basis_len, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                 uint64_t *sum_at) {
    if (!head || !out_len || (tokens_len && !tokens))
        return fail(ctx, RSG_ERR_INVALID, "NULL argument");
    uint64_t pos = 0, off = 0;
    bool fits = true;
    for (;;) {
        if (pos + 4 > tokens_len) return fail(ctx, RSG_ERR_INVALID, "token stream ends before its terminator");
        const int32_t token = rd_i32(tokens + pos);  // recvToken, token.go:8
        pos += 4;
        if (token == 0) break;  // receiver.go:128-130
        const uint8_t *data;
        uint64_t n;
        if (token > 0) {  // literal: io.ReadFull of token bytes, token.go:15-18
            n = (uint64_t)token;
            if (pos + n > tokens_len)
                return fail(ctx, RSG_ERR_INVALID, "literal of %llu bytes runs past the stream", (unsigned long long)n);
            data = tokens + pos;
            pos += n;
        } else {
            if (!basis)  // receiver.go:143-145 (no local file open)
                return fail(ctx, RSG_ERR_INVALID, "match token without a basis file");
            const int64_t idx = -((int64_t)token + 1);  // receiver.go:146
            const int64_t off2 = idx * (int64_t)head->block_len;
            n = (uint64_t)head->block_len;
            if (idx == head->count - 1 && head->rem != 0) n = (uint64_t)head->rem;  // :148-151
            if ((uint64_t)off2 + n > basis_len)  // ReadAt short read, :155-157
                return fail(ctx, RSG_ERR_INVALID, "block %lld reads past the basis (%llu bytes)", (long long)idx,
                            (unsigned long long)basis_len);
            data = basis + off2;
        }
        if (out && off + n <= out_cap) memcpy(out + off, data, n);
        else if (out) fits = false;
        off += n;
    }
    *out_len = off;
    if (sum_at) *sum_at = pos;
    if (!fits) return fail(ctx, RSG_ERR_TRUNCATED, "rebuilt file needs %llu bytes", (unsigned long long)off);
    return RSG_OK;
}

}  // namespace

extern "C" {

rsg_status rsg_apply_tokens(const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed) {
    uint64_t sum_at = 0;
    rsg_status s = apply(nullptr, tokens, tokens_len, head, basis, basis_len, out, out_cap, out_len, &sum_at);
    if (consumed) *consumed = sum_at;
    return s;
}

rsg_status rsg_receive_data(rsg_ctx *ctx, const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, int32_t seed, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    uint64_t sum_at = 0;
    rsg_status s = apply(ctx, tokens, tokens_len, head, basis, basis_len, out, out_cap, out_len, &sum_at);
    if (s != RSG_OK) return s;
    if (sum_at + 16 > tokens_len)  // io.ReadFull(remoteSum), receiver.go:167-170
        return fail(ctx, RSG_ERR_INVALID, "token stream ends before the whole-file sum");
    if (*out_len && !out) return fail(ctx, RSG_ERR_INVALID, "NULL output");
    // h = MD4(seed_LE || rebuilt file), receiver.go:117-120,166
    rsg_file f;
    memset(&f, 0, sizeof f);
    f.data = out;
    f.len = *out_len;
    uint8_t local[16];
    if ((s = rsg_file_sums_host(ctx, &f, 1, RSG_FILESUM_SEEDED, seed, local)) != RSG_OK) return s;
    if (consumed) *consumed = sum_at + 16;
    if (memcmp(local, tokens + sum_at, 16) != 0)  // receiver.go:171-173
        return fail(ctx, RSG_ERR_CORRUPT, "file corruption: whole-file sum mismatch");
    return RSG_OK;
}

}  // extern "C"
