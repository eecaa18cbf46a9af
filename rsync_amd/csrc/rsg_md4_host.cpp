// rsg_md4_host.cpp -- MD4 (RFC 1320) on the host, for the whole-file sums
// whose bytes stream through host memory anyway and whose chain is serial
// (one file = one Merkle-Damgård chain: a GPU gives it one lane).
//
// Used by the product where the reference computes a whole-file MD4 with
// the data in hand:
//   * the sender's file sum h = MD4(int32_LE(seed) || source)
//     (internal/sender/match.go:52-53, fed as the file is read,
//     :262-269, written after the terminator :220-226), by
//     rsg_hash_search_fd while it streams the source to the GPU;
//   * receiveData's check of few, large files (receiver.go:117-120,
//     166-174), where one GPU lane per file is ~10x slower than a host core
//     (DESIGN.md §6.1): rsg_receive_data picks this path by file size.
// The block checksums (the hot path) never come here.
#include <string.h>

#include "../../include/rsg_testing.h"
#include "rsg_host.h"

namespace rsgh {

namespace {

inline uint32_t rl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

// One 64-byte block.  Round functions and constants of RFC 1320 §3.4.
void md4_block(uint32_t st[4], const uint8_t *p) {
    uint32_t x[16];
    for (int i = 0; i < 16; i++)
        x[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
               ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#define RSG_R1(A, B, C, D, K, S) A = rl(A + ((B & C) | (~B & D)) + x[K], S)
#define RSG_R2(A, B, C, D, K, S) A = rl(A + ((B & C) | (B & D) | (C & D)) + x[K] + 0x5A827999u, S)
#define RSG_R3(A, B, C, D, K, S) A = rl(A + (B ^ C ^ D) + x[K] + 0x6ED9EBA1u, S)
    for (int k = 0; k < 16; k += 4) {
        RSG_R1(a, b, c, d, k, 3);
        RSG_R1(d, a, b, c, k + 1, 7);
        RSG_R1(c, d, a, b, k + 2, 11);
        RSG_R1(b, c, d, a, k + 3, 19);
    }
    for (int k = 0; k < 4; k++) {
        RSG_R2(a, b, c, d, k, 3);
        RSG_R2(d, a, b, c, k + 4, 5);
        RSG_R2(c, d, a, b, k + 8, 9);
        RSG_R2(b, c, d, a, k + 12, 13);
    }
    static const int o3[4] = {0, 2, 1, 3};
    for (int k = 0; k < 4; k++) {
        RSG_R3(a, b, c, d, o3[k], 3);
        RSG_R3(d, a, b, c, o3[k] + 8, 9);
        RSG_R3(c, d, a, b, o3[k] + 4, 11);
        RSG_R3(b, c, d, a, o3[k] + 12, 15);
    }
#undef RSG_R1
#undef RSG_R2
#undef RSG_R3
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

}  // namespace

void Md4::init() {
    st[0] = 0x67452301u;
    st[1] = 0xefcdab89u;
    st[2] = 0x98badcfeu;
    st[3] = 0x10325476u;
    total = 0;
    nbuf = 0;
}

void Md4::update(const uint8_t *p, uint64_t n) {
    total += n;
    if (nbuf) {
        const uint64_t k = n < 64 - nbuf ? n : 64 - nbuf;
        memcpy(buf + nbuf, p, (size_t)k);
        nbuf += (uint32_t)k;
        p += k;
        n -= k;
        if (nbuf < 64) return;
        md4_block(st, buf);
        nbuf = 0;
    }
    for (; n >= 64; p += 64, n -= 64) md4_block(st, p);
    if (n) {
        memcpy(buf, p, (size_t)n);
        nbuf = (uint32_t)n;
    }
}

void Md4::final(uint8_t out[16]) {
    const uint64_t bits = total << 3;
    uint8_t pad[72] = {0x80};
    const uint32_t padn = (nbuf < 56 ? 56 : 120) - nbuf;
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (8 * i));
    update(pad, padn);
    update(len, 8);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(st[i] >> (8 * j));
}

}  // namespace rsgh

extern "C" rsg_status rsg_testing_md4(const uint8_t *data, uint64_t n, int32_t seeded, int32_t seed, uint64_t piece,
                                      uint8_t out[16]) {
    if (!out || (n && !data)) return rsgh::fail(nullptr, RSG_ERR_INVALID, "NULL argument");
    rsgh::Md4 h;
    h.init();
    if (seeded) {
        const uint8_t sb[4] = {(uint8_t)seed, (uint8_t)(seed >> 8), (uint8_t)(seed >> 16), (uint8_t)(seed >> 24)};
        h.update(sb, 4);
    }
    const uint64_t step = piece ? piece : (n ? n : 1);
    for (uint64_t o = 0; o < n; o += step) h.update(data + o, n - o < step ? n - o : step);
    h.final(out);
    return RSG_OK;
}
