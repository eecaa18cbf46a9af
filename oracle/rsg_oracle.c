/*
 * rsg_oracle.c -- CPU restatement of the gokrazy/rsync block-checksum hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: it is compiled
 * into oracle/_build/liboracle.so and may be loaded only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * library (rsync_amd/librsg.so) never links, loads or calls it.
 *
 * Every function restates the reference's algorithm (Go, github.com/gokrazy/rsync,
 * read-only at /root/reference) and cites the file:line it follows.  MD4 lives in
 * the third-party module github.com/mmcloughlin/md4 v0.1.2 (go.mod:11, not
 * vendored): it is restated here from its published algorithm, RFC 1320.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - weak sum: the 1780 known-answer values of
 *     internal/rsyncchecksum/checksum_test.go:32-73 (tests/golden/weak_kat.json);
 *   - MD4: RFC 1320 appendix A.5 vectors plus OpenSSL 3 legacy-provider digests
 *     generated in the build container (tests/golden/md4_vectors.json);
 *   - strong block sums: no reference test pins a Checksum2 value; the
 *     fixtures above pin the MD4 arithmetic and the seed-append layout is
 *     restated from rsyncchecksum.go:53-58.
 *   - hash search: no reference test pins token bytes; the serial restatement
 *     below transcribes match.go:21-282 / token.go:4-31 statement by statement
 *     and is cross-checked against an independent pure-Python transcription in
 *     tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Synthetic data: splitmix64 stream, 8 little-endian bytes per output word.  */
/* (SURVEY.md appendix "Synthetic bytes"; not part of the reference.)         */
/* ------------------------------------------------------------------------- */
static inline uint64_t splitmix64_next(uint64_t *state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_fill_splitmix64(uint64_t seed, uint8_t *buf, uint64_t n) {
    uint64_t st = seed;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t z = splitmix64_next(&st);
        memcpy(buf + i, &z, 8); /* host is little-endian (x86-64) */
    }
    if (i < n) {
        uint64_t z = splitmix64_next(&st);
        memcpy(buf + i, &z, (size_t)(n - i));
    }
}

/* ------------------------------------------------------------------------- */
/* Weak checksum.                                                             */
/* ------------------------------------------------------------------------- */

/* rsyncchecksum.SignExtend, internal/rsyncchecksum/rsyncchecksum.go:24-27:
 * bytes are read as signed char (tridge get_checksum1 quirk, :19-23). */
static inline uint32_t sign_extend(uint8_t b) { return (uint32_t)(int32_t)(int8_t)b; }

/* rsyncchecksum.Checksum1, rsyncchecksum.go:29-51.  The reference unrolls by 4
 * (:34-45) then finishes byte by byte (:46-49); both forms compute
 * s1 = sum x_i, s2 = sum (n-i) x_i  (mod 2^32), restated here per byte. */
uint32_t orc_checksum1(const uint8_t *buf, uint64_t n) {
    uint32_t s1 = 0, s2 = 0;
    for (uint64_t i = 0; i < n; i++) {
        s1 += sign_extend(buf[i]);
        s2 += s1;
    }
    return (s1 & 0xffffu) + (s2 << 16); /* :50 */
}

/* rsyncchecksum.Tag2 / Tag, rsyncchecksum.go:11-17. */
static inline uint16_t tag2(uint16_t s1, uint16_t s2) { return (uint16_t)(s1 + s2); }
uint16_t orc_tag(uint32_t sum) { return tag2((uint16_t)(sum & 0xffff), (uint16_t)(sum >> 16)); }

/* ------------------------------------------------------------------------- */
/* MD4 (RFC 1320), the arithmetic of github.com/mmcloughlin/md4 v0.1.2.       */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t h[4];
    uint8_t buf[64];
    uint32_t nbuf;
    uint64_t total;
} md4_ctx;

#define ROTL(x, s) (((x) << (s)) | ((x) >> (32 - (s))))
#define MF(x, y, z) (((x) & (y)) | (~(x) & (z)))
#define MG(x, y, z) (((x) & (y)) | ((x) & (z)) | ((y) & (z)))
#define MH(x, y, z) ((x) ^ (y) ^ (z))

static void md4_compress(uint32_t h[4], const uint8_t blk[64]) {
    uint32_t X[16];
    for (int i = 0; i < 16; i++)
        X[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) |
               ((uint32_t)blk[4 * i + 2] << 16) | ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    static const int r1s[4] = {3, 7, 11, 19};
    static const int r2s[4] = {3, 5, 9, 13};
    static const int r3s[4] = {3, 9, 11, 15};
    static const int r2k[16] = {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
    static const int r3k[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
    for (int i = 0; i < 16; i++) {
        uint32_t t = a + MF(b, c, d) + X[i];
        t = ROTL(t, r1s[i & 3]);
        a = d; d = c; c = b; b = t;
    }
    for (int i = 0; i < 16; i++) {
        uint32_t t = a + MG(b, c, d) + X[r2k[i]] + 0x5A827999u;
        t = ROTL(t, r2s[i & 3]);
        a = d; d = c; c = b; b = t;
    }
    for (int i = 0; i < 16; i++) {
        uint32_t t = a + MH(b, c, d) + X[r3k[i]] + 0x6ED9EBA1u;
        t = ROTL(t, r3s[i & 3]);
        a = d; d = c; c = b; b = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

static void md4_init(md4_ctx *c) {
    c->h[0] = 0x67452301u; c->h[1] = 0xEFCDAB89u; c->h[2] = 0x98BADCFEu; c->h[3] = 0x10325476u;
    c->nbuf = 0; c->total = 0;
}

static void md4_update(md4_ctx *c, const uint8_t *p, uint64_t n) {
    c->total += n;
    if (c->nbuf) {
        uint32_t take = 64 - c->nbuf;
        if (take > n) take = (uint32_t)n;
        memcpy(c->buf + c->nbuf, p, take);
        c->nbuf += take; p += take; n -= take;
        if (c->nbuf == 64) { md4_compress(c->h, c->buf); c->nbuf = 0; }
    }
    while (n >= 64) { md4_compress(c->h, p); p += 64; n -= 64; }
    if (n) { memcpy(c->buf, p, (size_t)n); c->nbuf = (uint32_t)n; }
}

static void md4_final(md4_ctx *c, uint8_t out[16]) {
    uint64_t bits = c->total * 8;
    uint8_t pad[72];
    uint32_t padlen = (c->nbuf < 56) ? (56 - c->nbuf) : (120 - c->nbuf);
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    for (int i = 0; i < 8; i++) pad[padlen + i] = (uint8_t)(bits >> (8 * i));
    uint64_t keep = c->total;
    md4_update(c, pad, padlen + 8);
    c->total = keep;
    for (int i = 0; i < 4; i++) {
        out[4 * i + 0] = (uint8_t)(c->h[i]);
        out[4 * i + 1] = (uint8_t)(c->h[i] >> 8);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 3] = (uint8_t)(c->h[i] >> 24);
    }
}

void orc_md4(const uint8_t *msg, uint64_t n, uint8_t out[16]) {
    md4_ctx c;
    md4_init(&c);
    md4_update(&c, msg, n);
    md4_final(&c, out);
}

/* rsyncchecksum.Checksum2, rsyncchecksum.go:53-58: MD4(buf || int32_LE(seed));
 * the seed is appended, and appended even when it is 0. */
void orc_checksum2(int32_t seed, const uint8_t *buf, uint64_t n, uint8_t out[16]) {
    md4_ctx c;
    uint8_t s[4];
    uint32_t u = (uint32_t)seed;
    s[0] = (uint8_t)u; s[1] = (uint8_t)(u >> 8); s[2] = (uint8_t)(u >> 16); s[3] = (uint8_t)(u >> 24);
    md4_init(&c);
    md4_update(&c, buf, n);
    md4_update(&c, s, 4);
    md4_final(&c, out);
}

/* Whole-file sums.
 * mode 0: MD4(file)                  rsyncchecksum.ReaderChecksum, rsyncchecksum.go:60-66
 *                                    (the --checksum file-list sums, sender/flist.go:276-293,
 *                                    receiver/generator.go:82-88)
 * mode 1: MD4(int32_LE(seed) || file) the transfer's whole-file sum: h = md4.New();
 *                                    binary.Write(h, seed) before any data (match.go:52-53,
 *                                    sender.go:184-206, receiver.go:117-120)
 * The seed is PREPENDED here, unlike Checksum2 where it is appended. */
void orc_file_sum(int32_t mode, int32_t seed, const uint8_t *buf, uint64_t n, uint8_t out[16]) {
    md4_ctx c;
    md4_init(&c);
    if (mode == 1) {
        uint8_t s[4];
        uint32_t u = (uint32_t)seed;
        s[0] = (uint8_t)u; s[1] = (uint8_t)(u >> 8); s[2] = (uint8_t)(u >> 16); s[3] = (uint8_t)(u >> 24);
        md4_update(&c, s, 4);
    }
    md4_update(&c, buf, n);
    md4_final(&c, out);
}

/* ------------------------------------------------------------------------- */
/* Block sizing: rsynccommon.SumSizesSqroot, internal/rsynccommon/rsynccommon.go:14-37 */
/* out = {ChecksumCount, BlockLength, ChecksumLength, RemainderLength}        */
/* (wire order of SumHead.WriteTo, types.go:79-86).                           */
/* ------------------------------------------------------------------------- */
void orc_sum_sizes_sqroot(int64_t len, int32_t out[4]) {
    int32_t blen = (int32_t)sqrt((double)len); /* Go int32(float64) truncates (:22) */
    if (blen < 700) blen = 700;               /* blockSize = 700, :11 */
    out[0] = (int32_t)((len + ((int64_t)blen - 1)) / (int64_t)blen); /* :33 */
    out[1] = blen;
    out[2] = 16;                                /* checksumLength, :31 */
    out[3] = (int32_t)(len % (int64_t)blen);    /* :34 */
}

/* ------------------------------------------------------------------------- */
/* Receiver: generateAndSendSums, internal/receiver/generator.go:325-350.     */
/* Writes count records of 20 bytes: int32 LE sum1 (:341) then sum2[16]       */
/* (:344).  block_len <= 0 selects SumSizesSqroot (:326).  Returns count.     */
/* ------------------------------------------------------------------------- */
int64_t orc_block_sums(const uint8_t *data, uint64_t len, int32_t block_len, int32_t seed,
                       uint8_t *out) {
    int32_t head[4];
    orc_sum_sizes_sqroot((int64_t)len, head);
    if (block_len > 0) {
        head[1] = block_len;
        head[0] = (int32_t)(((int64_t)len + block_len - 1) / block_len);
        head[3] = (int32_t)((int64_t)len % block_len);
    }
    uint64_t remaining = len, off = 0;
    for (int32_t i = 0; i < head[0]; i++) {
        uint64_t n1 = (uint64_t)head[1] < remaining ? (uint64_t)head[1] : remaining; /* :334 */
        uint32_t s1 = orc_checksum1(data + off, n1);
        uint8_t *rec = out + (uint64_t)i * 20;
        rec[0] = (uint8_t)s1; rec[1] = (uint8_t)(s1 >> 8); rec[2] = (uint8_t)(s1 >> 16); rec[3] = (uint8_t)(s1 >> 24);
        orc_checksum2(seed, data + off, n1, rec + 4);
        off += n1;
        remaining -= n1;
    }
    return head[0];
}

/* ------------------------------------------------------------------------- */
/* Sender: hashSearch + matched + simpleSendToken                              */
/* (internal/sender/match.go:21-282, internal/sender/token.go:4-31).          */
/* ------------------------------------------------------------------------- */
#define CHUNK_SIZE (256 * 1024) /* internal/sender/flist.go:52 */

typedef struct {
    const uint8_t *src;
    int64_t size;
    const int64_t *blen_of; /* per block Len (receiveSums, sender.go:135-139) */
    int64_t last_match;     /* st.lastMatch */
    md4_ctx h;
    int64_t *moff; int32_t *midx; int64_t mcap; int64_t nm;
    uint8_t *tok; int64_t tcap; int64_t tlen;
    int overflow;
} hs_state;

static void tok_put(hs_state *s, const void *p, int64_t n) {
    if (s->tlen + n > s->tcap) { s->overflow = 1; s->tlen += n; return; }
    if (s->tok) memcpy(s->tok + s->tlen, p, (size_t)n);
    s->tlen += n;
}

static void tok_i32(hs_state *s, int32_t v) {
    uint8_t b[4];
    uint32_t u = (uint32_t)v;
    b[0] = (uint8_t)u; b[1] = (uint8_t)(u >> 8); b[2] = (uint8_t)(u >> 16); b[3] = (uint8_t)(u >> 24);
    tok_put(s, b, 4);
}

/* simpleSendToken, token.go:4-31 */
static void simple_send_token(hs_state *s, int32_t token, int64_t offset, int64_t n) {
    if (n > 0) {
        for (int64_t l = 0; l < n;) {
            int64_t n1 = n - l < CHUNK_SIZE ? n - l : CHUNK_SIZE;
            tok_i32(s, (int32_t)n1);
            tok_put(s, s->src + offset + l, n1);
            l += n1;
        }
    }
    if (token != -2) tok_i32(s, -(token + 1));
}

/* matched, match.go:233-282 */
static void matched(hs_state *s, int64_t offset, int32_t i) {
    int64_t n = offset - s->last_match;
    int transmit_accumulated = i < 0;
    simple_send_token(s, i, s->last_match, n);
    if (!transmit_accumulated) {
        n += s->blen_of[i];
        if (s->nm < s->mcap) { s->moff[s->nm] = offset; s->midx[s->nm] = i; }
        s->nm++;
    }
    if (n > 0) md4_update(&s->h, s->src + s->last_match, (uint64_t)n); /* :262-269 */
    s->last_match = transmit_accumulated ? offset : offset + s->blen_of[i];
}

/*
 * Returns the number of matches found (may exceed match_cap: then only the
 * first match_cap are stored), or -1 on invalid input.  *tok_len receives the
 * number of token bytes needed (tokens are stored only while they fit in
 * tok_cap): the stream through the terminating int32 0, before the
 * whole-file sum); file_sum receives MD4(int32_LE(seed) || src) (match.go:52-53,
 * 220-226).  targets[] is the Go `targets` order: a permutation of block
 * indices sorted by Tag(sum1) (sender.go:60-83).
 *
 * Deviations, both on inputs where the reference panics: a 0-byte source
 * (update[0] of an empty window) emits just the terminator; a
 * count == 0 head takes the reference's sendFile path (sender.go:86-88), whose
 * token bytes equal an all-literal hash search.
 */
int64_t orc_hash_search(const uint8_t *src, int64_t size,
                        int32_t count, int32_t blen, int32_t s2len, int32_t rem,
                        const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets,
                        int32_t seed,
                        int64_t *match_off, int32_t *match_idx, int64_t match_cap,
                        uint8_t *tokens, int64_t tok_cap, int64_t *tok_len,
                        uint8_t file_sum[16]) {
    if (count < 0 || blen < 0 || s2len < 0 || s2len > 16 || rem < 0 || rem > blen) return -1;
    if (count > 0 && blen == 0) return -1;
    hs_state s;
    memset(&s, 0, sizeof s);
    s.src = src; s.size = size;
    s.moff = match_off; s.midx = match_idx; s.mcap = match_cap;
    s.tok = tokens; s.tcap = tokens ? tok_cap : 0;
    int64_t *lens = (int64_t *)malloc(sizeof(int64_t) * (size_t)(count > 0 ? count : 1));
    for (int32_t i = 0; i < count; i++)
        lens[i] = (i == count - 1 && rem != 0) ? rem : blen; /* sender.go:135-139 */
    s.blen_of = lens;
    md4_init(&s.h);
    {   /* sum_init: h.Write(int32_LE(seed)), match.go:52-53 */
        uint8_t sb[4]; uint32_t u = (uint32_t)seed;
        sb[0] = (uint8_t)u; sb[1] = (uint8_t)(u >> 8); sb[2] = (uint8_t)(u >> 16); sb[3] = (uint8_t)(u >> 24);
        md4_update(&s.h, sb, 4);
    }

    if (count > 0 && size > 0) {
        /* build_hash_table, sender.go:60-83: tagTable[tag] = first k with that tag */
        int32_t *tag_first = (int32_t *)malloc(sizeof(int32_t) * 65536);
        uint16_t *ttag = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)count);
        for (int i = 0; i < 65536; i++) tag_first[i] = -1;
        for (int32_t k = 0; k < count; k++) ttag[k] = orc_tag(sum1[targets[k]]);
        for (int32_t k = count - 1; k >= 0; k--) tag_first[ttag[k]] = k;

        int64_t end = size + 1 - lens[count - 1]; /* match.go:70 */
        int64_t offset = 0;
        int64_t k = 0;
        uint32_t s1 = 0, s2 = 0;
#define READ_CHUNK()                                                  \
    do {                                                              \
        k = blen;                                                     \
        if (size - offset < k) k = size - offset; /* :74-77 */        \
        uint32_t sum_ = orc_checksum1(src + offset, (uint64_t)k);     \
        s1 = sum_ & 0xffff; s2 = sum_ >> 16; /* :83-85 */             \
    } while (0)
        READ_CHUNK();
        for (;;) {
            uint16_t tag = tag2((uint16_t)s1, (uint16_t)s2); /* :95 */
            int32_t j = tag_first[tag];
            int done_outer = 0;
            if (j >= 0) {
                uint32_t sum = (s1 & 0xffff) | (s2 << 16); /* :106 */
                uint8_t local2[16];
                int done2 = 0;
                for (; j < count && ttag[j] == tag; j++) { /* :108 */
                    int32_t i = targets[j];
                    if (sum != sum1[i]) continue;            /* :110 */
                    int64_t l = blen;
                    if (size - offset < l) l = size - offset; /* :114-117 */
                    if (l != lens[i]) continue;              /* :118 */
                    if (!done2) { orc_checksum2(seed, src + offset, (uint64_t)l, local2); done2 = 1; }
                    if (memcmp(local2, sum2 + 16 * (int64_t)i, (size_t)s2len) != 0) continue; /* :133 */
                    matched(&s, offset, i);                  /* :149 */
                    offset += lens[i] - 1;                   /* :158 */
                    READ_CHUNK();
                    if (offset >= end) done_outer = 1;       /* :163-165 */
                    break;
                }
            }
            if (done_outer) break;
            /* rolling update, :171-196 */
            int64_t backup = offset - s.last_match;
            if (backup < 0) backup = 0;
            int more = offset + k < size;
            uint32_t x0 = sign_extend(src[offset]);
            s1 -= x0;
            s2 -= (uint32_t)k * x0;
            if (more) {
                s1 += sign_extend(src[offset + k]);
                s2 += s1;
            } else {
                k--;
            }
            s1 &= 0xffff; s2 &= 0xffff;
            if (backup >= (int64_t)blen + CHUNK_SIZE && end - offset > CHUNK_SIZE) /* :198 */
                matched(&s, offset - blen, -2);
            offset++;
            if (offset >= end) break; /* :206-209 */
        }
#undef READ_CHUNK
        free(tag_first);
        free(ttag);
    }
    matched(&s, size, -1); /* :212 */
    md4_final(&s.h, file_sum);
    if (tok_len) *tok_len = s.tlen;
    free(lens);
    return s.nm; /* callers compare *tok_len with tok_cap to detect truncation */
}

/* ------------------------------------------------------------------------- */
/* Receiver: receiveData + recvToken                                           */
/* (internal/receiver/receiver.go:98-188, internal/receiver/token.go:6-20).   */
/* ------------------------------------------------------------------------- */
static int32_t rd_i32(const uint8_t *p) {
    return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

/*
 * Rebuilds the file from the token stream `tok` (the bytes after the SumHead:
 * tokens, the int32 0 terminator, then the sender's 16-byte whole-file sum)
 * and the basis, and checks MD4(int32_LE(seed) || rebuilt) against that sum.
 * Returns the rebuilt length (stored while it fits in out_cap; out may be
 * NULL to size), or
 *   -1 the stream ends early (recvToken / io.ReadFull errors, token.go:8-18,
 *      receiver.go:167-170),
 *   -2 a match reads outside the basis (localFile.ReadAt error,
 *      receiver.go:155-157) or there is no basis (:143-145),
 *   -3 the whole-file sums differ ("file corruption", receiver.go:171-173).
 * *consumed = stream bytes read through the whole-file sum.
 */
int64_t orc_receive_data(const uint8_t *tok, int64_t tok_len, int32_t count, int32_t blen, int32_t rem,
                         const uint8_t *basis, int64_t basis_len, int32_t seed,
                         uint8_t *out, int64_t out_cap, int64_t *consumed) {
    md4_ctx h;
    md4_init(&h);
    uint8_t sb[4];
    uint32_t us = (uint32_t)seed;
    sb[0] = (uint8_t)us; sb[1] = (uint8_t)(us >> 8); sb[2] = (uint8_t)(us >> 16); sb[3] = (uint8_t)(us >> 24);
    md4_update(&h, sb, 4); /* binary.Write(h, LE, rt.Seed), receiver.go:117-118 */
    int64_t pos = 0, off = 0;
    for (;;) {
        if (pos + 4 > tok_len) return -1;
        int32_t token = rd_i32(tok + pos);
        pos += 4;
        if (token == 0) break; /* receiver.go:128-130 */
        const uint8_t *data;
        int64_t n;
        if (token > 0) { /* literal, token.go:15-19 */
            n = token;
            if (pos + n > tok_len) return -1;
            data = tok + pos;
            pos += n;
        } else {
            if (!basis) return -2;
            int32_t idx = -(token + 1); /* receiver.go:146 */
            int64_t off2 = (int64_t)idx * (int64_t)blen;
            n = blen;
            if (idx == count - 1 && rem != 0) n = rem; /* :148-151 */
            if (off2 + n > basis_len) return -2;
            data = basis + off2;
        }
        if (out && off + n <= out_cap) memcpy(out + off, data, (size_t)n);
        md4_update(&h, data, (uint64_t)n);
        off += n;
    }
    uint8_t local[16];
    md4_final(&h, local);
    if (pos + 16 > tok_len) return -1;
    if (memcmp(local, tok + pos, 16) != 0) return -3;
    pos += 16;
    if (consumed) *consumed = pos;
    return off;
}
