// rsg_wire.cpp -- the wire formats either side of the checksum path
// (SURVEY.md §8f row 4), as host byte formatting so the GPU's 20-byte
// records leave the engine wire-ready:
//   * the generator's sums stream: int32 idx (generator.go:317), SumHead
//     (types.go:79-86), per block int32 sum1 + sum2[:s2len]
//     (generator.go:341-346), and the two int32 -1 phase markers
//     (generator.go:31,40);
//   * its parser on the sender side: SumHead.ReadFrom with the reference's
//     validation (types.go:38-77) and receiveSums (sender.go:118-151);
//   * MultiplexWriter framing (wire.go:28-36) in <= 256 KiB messages and the
//     MultiplexReader that undoes it (wire.go:46-95);
//   * the int64 escape of Conn.WriteInt64 / ReadInt64 (wire.go:108-117,177-195).
// No GPU work here; every function is re-entrant and allocation-free.
#include <string.h>

#include "rsg_host.h"

using namespace rsgh;

namespace {

constexpr uint32_t kMplexBase = 7;             // wire.go:18
constexpr uint32_t kMaxMessage = 256 * 1024;   // ioBufferSize, wire.go:46-47
constexpr int32_t kMaxBlockLen = 1 << 29;      // types.go:40
constexpr uint8_t kMsgData = 0, kMsgError = 1, kMsgInfo = 2;  // wire.go:12-14

int32_t rd_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// Bounded writer: counts every byte, copies only while it fits.
struct Out {
    uint8_t *p;
    uint64_t cap, pos = 0;
    bool fits = true;
    void put(const void *src, uint64_t n) {
        if (p && pos + n <= cap) memcpy(p + pos, src, n);
        else if (p) fits = false;
        pos += n;
    }
    void i32(int32_t v) {
        const uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
        put(b, 4);
    }
    rsg_status finish(uint64_t *out_len, const char *what) {
        *out_len = pos;
        if (!fits)  // out == NULL is a size query (as rsg_encode_tokens)
            return fail(nullptr, RSG_ERR_TRUNCATED, "%s needs %llu bytes", what, (unsigned long long)pos);
        return RSG_OK;
    }
};

}  // namespace

extern "C" {

rsg_status rsg_check_sum_head(const rsg_sum_head *h) {
    if (!h) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    if (h->count < 0) return fail(nullptr, RSG_ERR_INVALID, "invalid checksum count %d", h->count);
    if (h->block_len < 0 || h->block_len > kMaxBlockLen)
        return fail(nullptr, RSG_ERR_INVALID, "invalid block length %d", h->block_len);
    if (h->s2len < 0 || h->s2len > 16) return fail(nullptr, RSG_ERR_INVALID, "invalid checksum length %d", h->s2len);
    if (h->rem < 0 || h->rem > h->block_len)
        return fail(nullptr, RSG_ERR_INVALID, "invalid remainder length %d", h->rem);
    return RSG_OK;
}

rsg_status rsg_encode_sums(const int32_t *file_idx, const rsg_sum_head *heads, uint64_t nfiles,
                           const uint8_t *records, int32_t terminate, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len) {
    if (!out_len || (nfiles && (!heads || !records))) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    Out o{out, out_cap};
    uint64_t rec = 0;
    for (uint64_t f = 0; f < nfiles; f++) {
        const rsg_sum_head &h = heads[f];
        if (rsg_check_sum_head(&h) != RSG_OK) return RSG_ERR_INVALID;
        if (file_idx) o.i32(file_idx[f]);  // recvGenerator, generator.go:317
        o.i32(h.count);                    // SumHead.WriteTo, types.go:79-86
        o.i32(h.block_len);
        o.i32(h.s2len);
        o.i32(h.rem);
        if (h.s2len == 16) {  // records are already the wire bytes
            o.put(records + rec * RSG_RECORD_BYTES, (uint64_t)h.count * RSG_RECORD_BYTES);
        } else {
            for (int32_t i = 0; i < h.count; i++) o.put(records + (rec + i) * RSG_RECORD_BYTES, 4 + h.s2len);
        }
        rec += (uint64_t)h.count;
    }
    if (terminate) {  // GenerateFiles' phase markers, generator.go:31,40
        o.i32(-1);
        o.i32(-1);
    }
    return o.finish(out_len, "sums stream");
}

rsg_status rsg_decode_sums(const uint8_t *wire, uint64_t wire_len, rsg_sum_head *head, uint32_t *sum1,
                           uint8_t *sum2, uint64_t cap, uint64_t *consumed) {
    if (!head || !consumed || (wire_len && !wire)) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    if (wire_len < 16) return fail(nullptr, RSG_ERR_INVALID, "sum head: unexpected EOF");
    head->count = rd_i32(wire);  // SumHead.ReadFrom, types.go:38-77
    head->block_len = rd_i32(wire + 4);
    head->s2len = rd_i32(wire + 8);
    head->rem = rd_i32(wire + 12);
    if (rsg_check_sum_head(head) != RSG_OK) return RSG_ERR_INVALID;
    const uint64_t n = (uint64_t)head->count, rl = 4 + (uint64_t)head->s2len;
    *consumed = 16 + n * rl;
    if (n && (!sum1 || !sum2 || cap < n))
        return fail(nullptr, RSG_ERR_TRUNCATED, "%llu sums need room", (unsigned long long)n);
    if (wire_len < *consumed) return fail(nullptr, RSG_ERR_INVALID, "sums: unexpected EOF");
    const uint8_t *p = wire + 16;
    for (uint64_t i = 0; i < n; i++, p += rl) {  // receiveSums, sender.go:126-148
        sum1[i] = (uint32_t)rd_i32(p);
        memset(sum2 + i * 16, 0, 16);
        memcpy(sum2 + i * 16, p + 4, head->s2len);
    }
    return RSG_OK;
}

rsg_status rsg_mux_frame(const uint8_t *data, uint64_t len, int32_t tag, uint32_t max_message, uint8_t *out,
                         uint64_t out_cap, uint64_t *out_len) {
    if (!out_len || (len && !data)) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    if (tag < 0 || tag > 255 - (int32_t)kMplexBase) return fail(nullptr, RSG_ERR_INVALID, "invalid tag %d", tag);
    if (max_message == 0 || max_message > kMaxMessage)
        return fail(nullptr, RSG_ERR_INVALID, "message size %u outside (0, %u]", max_message, kMaxMessage);
    Out o{out, out_cap};
    for (uint64_t at = 0; at < len;) {  // WriteMsg, wire.go:28-36
        const uint64_t n = std::min<uint64_t>(max_message, len - at);
        o.i32((int32_t)(((kMplexBase + (uint32_t)tag) << 24) | (uint32_t)n));
        o.put(data + at, n);
        at += n;
    }
    return o.finish(out_len, "mux stream");
}

rsg_status rsg_mux_deframe(const uint8_t *wire, uint64_t wire_len, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len) {
    if (!out_len || (wire_len && !wire)) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    Out o{out, out_cap};
    for (uint64_t at = 0; at < wire_len;) {  // ReadMsg + Read, wire.go:49-95
        if (at + 4 > wire_len) return fail(nullptr, RSG_ERR_INVALID, "mux header: unexpected EOF");
        const uint32_t hdr = (uint32_t)rd_i32(wire + at);
        const uint8_t tag = (uint8_t)((hdr >> 24) - kMplexBase);
        const uint32_t n = hdr & 0x00FFFFFFu;
        if (n > kMaxMessage)
            return fail(nullptr, RSG_ERR_INVALID, "length %u exceeds max message size (%u)", n, kMaxMessage);
        if (at + 4 + n > wire_len) return fail(nullptr, RSG_ERR_INVALID, "mux payload: unexpected EOF");
        const uint8_t *payload = wire + at + 4;
        at += 4 + (uint64_t)n;
        if (tag == kMsgData) o.put(payload, n);
        else if (tag == kMsgInfo) continue;  // logged and skipped
        else if (tag == kMsgError) return fail(nullptr, RSG_ERR_INVALID, "%.*s", (int)n, (const char *)payload);
        else return fail(nullptr, RSG_ERR_INVALID, "unexpected tag: got %u, want %u", tag, kMsgData);
    }
    return o.finish(out_len, "demuxed data");
}

rsg_status rsg_put_int64(int64_t v, uint8_t out[12], uint64_t *out_len) {
    if (!out || !out_len) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    Out o{out, 12};
    if (v >= 0 && v <= 0x7FFFFFFF) {  // WriteInt64, wire.go:108-117
        o.i32((int32_t)v);
    } else {
        o.i32(-1);
        o.i32((int32_t)(uint32_t)(uint64_t)v);
        o.i32((int32_t)(uint32_t)((uint64_t)v >> 32));
    }
    *out_len = o.pos;
    return RSG_OK;
}

rsg_status rsg_get_int64(const uint8_t *in, uint64_t in_len, int64_t *v, uint64_t *consumed) {
    if (!v || !consumed || (in_len && !in)) return fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    if (in_len < 4) return fail(nullptr, RSG_ERR_INVALID, "int64: unexpected EOF");
    const int32_t small = rd_i32(in);  // ReadInt64, wire.go:177-195
    if (small != -1) {
        *v = small;
        *consumed = 4;
        return RSG_OK;
    }
    if (in_len < 12) return fail(nullptr, RSG_ERR_INVALID, "int64: unexpected EOF");
    *v = (int64_t)((uint64_t)(uint32_t)rd_i32(in + 4) | ((uint64_t)(uint32_t)rd_i32(in + 8) << 32));
    *consumed = 12;
    return RSG_OK;
}

}  // extern "C"
