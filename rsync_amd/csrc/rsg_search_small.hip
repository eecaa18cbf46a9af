// rsg_search_small.hip -- the sender's hash search (internal/sender/match.go:21-230)
// for many small source files in one launch.
//
// SendFiles calls hashSearch once per file (internal/sender/sender.go:19-115).
// rsg_match.cpp's pipeline is built for large sources: per file it builds
// tables, rolls, confirms, resolves and walks in separate launches with host
// round trips in between, tens of microseconds of fixed cost -- more than a
// 4-64 KiB file takes to hash.  Here one wave owns one file and does the whole
// search on its own, and a launch covers thousands of files:
//   1. the basis sums: targets[k] and Sum1 of block targets[k] (the Go
//      `targets` order, sender.go:60-83) as (Sum1 << 32 | k) keys, sorted
//      in LDS, and a blocked Bloom filter of the Sum1 values in LDS;
//   2. the weak sum of the window [q, min(q + B, size)) at every visited
//      offset q < end = size + 1 - lastLen (match.go:70), each lane a
//      contiguous range: its first window summed directly, then the
//      reference's rolling update (match.go:171-196); filter hits are
//      appended to an LDS candidate list (offset, sum);
//   3. the candidates sorted by offset (wave bitonic sort in LDS);
//   4. every candidate confirmed: the first key group entry (targets order)
//      with equal Sum1 and Len == window length whose sum2[:s2len] equals
//      MD4(window || int32_LE(seed)) (match.go:108-136), MD4 computed at most
//      once per window;
//   5. the greedy walk (match.go:93-210 restricted to the candidates): a
//      candidate q >= pos with a confirmed block i is a match, pos = q +
//      Len_i (match.go:158); a miss moves pos past q.
// The match list goes to a launch-wide array (one atomic per file).  A file
// whose candidates exceed the LDS list (dense, repetitive data) reports
// status 1 and the host searches it with the large-file pipeline instead, so
// the result is exact either way.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rsg_hash_block.h"
#include "rsg_internal.h"

namespace rsg {

namespace {

constexpr uint32_t kSmallThreads = 64;  // one wave per file

// SignExtend of byte j of w (rsyncchecksum.go:24-27).
__device__ __forceinline__ int32_t sxb(uint32_t w, int j) { return (int32_t)(w << (24 - 8 * j)) >> 24; }

// SignExtend(src[x]) read through the aligned dword that holds it (never
// touches a dword without a byte of the source).
__device__ __forceinline__ int32_t ld_sx(const uint8_t *src, uint32_t x) {
    const uintptr_t a = (uintptr_t)src + x;
    const uint32_t w = *reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    return (int32_t)(w << (24 - 8 * (uint32_t)(a & 3))) >> 24;
}

__device__ __forceinline__ void acc_word(uint32_t w, uint32_t pos, uint32_t &p, uint32_t &q) {
    const int32_t s = __builtin_amdgcn_sdot4((int)w, 0x01010101, 0, false);
    const int32_t t = __builtin_amdgcn_sdot4((int)w, 0x03020100, 0, false);
    p += (uint32_t)s;
    q += (uint32_t)t + (uint32_t)__mul24((int)pos, s);  // |pos| < 2^21, |s| <= 512
}

// p += sum x_i, q += sum i * x_i over the signed bytes [lo, hi) of src (i =
// index in the source, mod 2^32), from aligned loads of dwords that hold at
// least one byte of the range.
__device__ void range_sums(const uint8_t *src, uint32_t lo, uint32_t hi, uint32_t &p, uint32_t &q) {
    if (lo >= hi) return;
    const uintptr_t a0 = (uintptr_t)src + lo, a1 = (uintptr_t)src + hi;
    uintptr_t a = a0 & ~(uintptr_t)3;
    uint32_t pos = lo - (uint32_t)(a0 - a);
    {
        uint32_t w = *reinterpret_cast<const uint32_t *>(a);
        w &= ~0u << (8 * (uint32_t)(a0 - a));
        if (a + 4 > a1) w &= ~0u >> (8 * (uint32_t)(a + 4 - a1));
        acc_word(w, pos, p, q);
        a += 4;
        pos += 4;
    }
#pragma unroll 2
    for (; a + 16 <= a1; a += 16, pos += 16) {
        const u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(a);
        acc_word(v.x, pos, p, q);
        acc_word(v.y, pos + 4, p, q);
        acc_word(v.z, pos + 8, p, q);
        acc_word(v.w, pos + 12, p, q);
    }
    for (; a < a1; a += 4, pos += 4) {
        uint32_t w = *reinterpret_cast<const uint32_t *>(a);
        if (a + 4 > a1) w &= ~0u >> (8 * (uint32_t)(a + 4 - a1));
        acc_word(w, pos, p, q);
    }
}

// 16 source bytes per step from 4-byte aligned vector loads, funnel-shifted
// (v_alignbyte) to the stream's byte offset; the load for the next step is
// issued one step ahead.  A vector that would reach past the source's last
// dword is loaded dword by dword, each clamped to that last dword: what a
// clamped dword returns is only used for offsets past the lane's range.
__device__ __forceinline__ u32x4a4 load4(const uint8_t *v, const uint8_t *lastdw) {
    if (v + 12 <= lastdw) return *reinterpret_cast<const u32x4a4 *>(v);
    u32x4a4 r;
    r.x = *reinterpret_cast<const uint32_t *>(v < lastdw ? v : lastdw);
    r.y = *reinterpret_cast<const uint32_t *>(v + 4 < lastdw ? v + 4 : lastdw);
    r.z = *reinterpret_cast<const uint32_t *>(v + 8 < lastdw ? v + 8 : lastdw);
    r.w = *reinterpret_cast<const uint32_t *>(lastdw);  // v + 12 > lastdw here
    return r;
}

struct Stream16 {
    const uint8_t *a;  // aligned address of c[0]
    uint32_t sh;       // byte offset of the stream in c[0]
    uint32_t c[5];
    u32x4a4 nx;        // dwords a + 20 .. a + 36 (the next step's c[1..4])

    // x <= size - 1: c[0] holds a byte of the source
    __device__ __forceinline__ void init(const uint8_t *src, uint32_t x, const uint8_t *lastdw) {
        const uintptr_t p = (uintptr_t)src + x;
        a = reinterpret_cast<const uint8_t *>(p & ~(uintptr_t)3);
        sh = (uint32_t)(p & 3);
        c[0] = *reinterpret_cast<const uint32_t *>(a);
        const u32x4a4 v = load4(a + 4, lastdw);
        c[1] = v.x; c[2] = v.y; c[3] = v.z; c[4] = v.w;
    }
    __device__ __forceinline__ void prefetch(const uint8_t *lastdw) { nx = load4(a + 20, lastdw); }
    __device__ __forceinline__ uint32_t word(int k) const { return __builtin_amdgcn_alignbyte(c[k + 1], c[k], sh); }
    __device__ __forceinline__ void advance() {
        c[0] = c[4]; c[1] = nx.x; c[2] = nx.y; c[3] = nx.z; c[4] = nx.w;
        a += 16;
    }
};

struct SmallLds {
    uint32_t *filt;  // filter words; after the roll, the confirmation results (int32 per candidate)
    uint64_t *keys;  // kc entries (Sum1 << 32 | k), sorted
    uint64_t *cand;  // ccap entries (offset << 32 | sum)
    uint32_t *cnt;   // candidates appended
    uint32_t wmask, ccap;
};

__device__ __forceinline__ uint32_t pack_sum(uint32_t s1, uint32_t s2) {
    return __builtin_amdgcn_perm(s2, s1, 0x05040100u);  // (s1 & 0xffff) | s2 << 16, match.go:106
}

// The filter: word (sum >> 16) & wmask, bits sum[0..4] and sum[5..9].
__device__ __forceinline__ uint32_t filter_hit(const SmallLds &L, uint32_t sum) {
    const uint32_t w = L.filt[(sum >> 16) & L.wmask];
    return (w >> (sum & 31u)) & (w >> ((sum >> 5) & 31u)) & 1u;
}

__device__ __forceinline__ void append(const SmallLds &L, uint32_t q, uint32_t sum) {
    const uint32_t p = atomicAdd(L.cnt, 1u);
    if (p < L.ccap) L.cand[p] = ((uint64_t)q << 32) | sum;
}

// Offsets [qa, qb) with the general window [q, min(q + B, size)) and the
// reference's general update (match.go:186-196: k-- once the window reaches
// the end), bytes read one at a time.  For the tail (shrinking windows) and
// tiny sources.
__device__ void roll_slow(const SmallLds &L, const uint8_t *src, uint32_t size, uint32_t B, uint32_t qa,
                          uint32_t qb) {
    if (qa >= qb) return;
    uint32_t e = min(qa + B, size);
    uint32_t p = 0, t = 0;
    range_sums(src, qa, e, p, t);
    uint32_t s1 = p, s2 = e * p - t;
    for (uint32_t q = qa;;) {
        const uint32_t sum = pack_sum(s1, s2);
        if (filter_hit(L, sum)) append(L, q, sum);
        if (++q >= qb) break;
        const int32_t xo = ld_sx(src, q - 1);
        const uint32_t k = e - (q - 1);
        s1 -= (uint32_t)xo;
        s2 -= (uint32_t)__mul24((int)k, xo);
        if (e < size) {
            s1 += (uint32_t)ld_sx(src, e);
            s2 += s1;
            e++;
        }
    }
}

// Wave bitonic sort of a[0..n) (n a power of two) in LDS.
__device__ void wave_sort(uint64_t *a, uint32_t n, uint32_t lane) {
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < n; i += kSmallThreads) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t x = a[i], y = a[l];
                    if ((x > y) == ((i & k) == 0)) {
                        a[i] = y;
                        a[l] = x;
                    }
                }
            }
            __syncthreads();  // one-wave workgroup: orders the steps' LDS accesses
        }
    }
}

__device__ __forceinline__ uint32_t len_of(int32_t b, int32_t count, uint32_t blen, uint32_t rem) {
    return (b == count - 1 && rem != 0) ? rem : blen;  // sender.go:135-139
}

__global__ __launch_bounds__(kSmallThreads) void search_small_kernel(
    const SmallJob *__restrict__ jobs, const uint32_t *__restrict__ order, const uint8_t *__restrict__ blob,
    uint32_t seed, uint32_t kc, uint32_t fwords, uint32_t ccap, uint4 *__restrict__ matches, uint32_t match_cap,
    uint32_t *__restrict__ match_count, SmallOut *__restrict__ outs) {
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x;
    const uint32_t jid = order[blockIdx.x];
    const SmallJob J = jobs[jid];
    const uint8_t *src = reinterpret_cast<const uint8_t *>(J.src);
    const uint32_t *sum1 = reinterpret_cast<const uint32_t *>(blob + J.sums);
    const int32_t *targets = reinterpret_cast<const int32_t *>(blob + J.sums + ((4ull * J.count + 15) & ~15ull));
    const uint8_t *sum2 = blob + J.sums + 2 * ((4ull * J.count + 15) & ~15ull);
    const uint32_t size = J.size, B = J.blen;
    const int32_t count = J.count;

    const uint32_t F = fwords > ccap ? fwords : ccap;
    SmallLds L;
    L.filt = lds;
    L.keys = reinterpret_cast<uint64_t *>(lds + F);
    L.cand = reinterpret_cast<uint64_t *>(lds + F + 2 * kc);
    L.cnt = lds + F + 2 * kc + 2 * ccap;
    L.wmask = fwords - 1;
    L.ccap = ccap;

    // 1. keys (Sum1 << 32 | targets position) and the filter
    for (uint32_t i = lane; i < fwords; i += kSmallThreads) L.filt[i] = 0;
    if (lane == 0) *L.cnt = 0;
    __syncthreads();
    for (uint32_t k = lane; k < kc; k += kSmallThreads) {
        uint64_t key = ~0ull;
        if ((int32_t)k < count) {
            const uint32_t s = sum1[targets[k]];
            key = ((uint64_t)s << 32) | k;
            atomicOr(&L.filt[(s >> 16) & L.wmask], (1u << (s & 31u)) | (1u << ((s >> 5) & 31u)));
        }
        L.keys[k] = key;
    }
    __syncthreads();
    wave_sort(L.keys, kc, lane);

    // 2. the roll.  Visited offsets q < end (match.go:70; offset 0 always);
    // [0, ni) have full windows [q, q + B) inside the source, [ni, end) the
    // shrinking tail windows [q, size).
    const uint32_t last_len = J.rem != 0 ? J.rem : B;
    const uint32_t end = size + 1 > last_len ? max(size + 1 - last_len, 1u) : 1u;
    const uint32_t ni = size + 1 > B ? min(size + 1 - B, end) : 0u;
    if (size >= 64 && ni > 0) {
        const uint32_t ms = ((ni + 63) / 64 + 15) & ~15u;  // offsets per lane, whole 16-offset steps
        const uint32_t qa = lane * ms, qb = min(qa + ms, ni);
        const bool live = qa < qb;
        const uint32_t q0 = live ? qa : 0;
        const uint8_t *last = reinterpret_cast<const uint8_t *>(((uintptr_t)src + size - 1) & ~(uintptr_t)3);
        uint32_t p = 0, t = 0;
        if (live) range_sums(src, qa, qa + B, p, t);
        uint32_t s1 = p, s2 = (qa + B) * p - t;
        Stream16 so, si;
        so.init(src, q0, last);
        si.init(src, live ? min(qa + B, size - 1) : 0, last);  // qa + B == size: no byte of it is read
        const uint32_t Bm = B;
        for (uint32_t it = 0, q = q0; it < ms / 16; it++, q += 16) {
            so.prefetch(last);
            si.prefetch(last);
            uint32_t sums[16];
            uint32_t hm = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t wo = so.word(k), wi = si.word(k);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t sum = pack_sum(s1, s2);
                    sums[4 * k + j] = sum;
                    hm |= filter_hit(L, sum) << (4 * k + j);
                    const int32_t xo = sxb(wo, j), xi = sxb(wi, j);
                    s1 += (uint32_t)(xi - xo);
                    s2 += s1 - (uint32_t)__mul24((int)Bm, xo);
                }
            }
            const uint32_t left = live && qb > q ? qb - q : 0u;
            if (left < 16) hm &= (1u << left) - 1u;
            if (__ballot(hm != 0)) {
#pragma unroll
                for (int j = 0; j < 16; j++)
                    if (hm & (1u << j)) append(L, q + j, sums[j]);
            }
            so.advance();
            si.advance();
        }
        if (end > ni) {
            const uint32_t mt = (end - ni + 63) / 64;
            const uint32_t ta = ni + lane * mt;
            roll_slow(L, src, size, B, ta, min(ta + mt, end));
        }
    } else {
        const uint32_t mt = (end + 63) / 64;
        const uint32_t ta = lane * mt;
        roll_slow(L, src, size, B, ta, min(ta + mt, end));
    }
    __syncthreads();
    const uint32_t ncand = *L.cnt;
    SmallOut o{0, 0, 0, ncand};
    if (ncand > ccap) {
        o.status = 1;
        if (lane == 0) outs[jid] = o;
        return;
    }

    // 3. candidates in offset order (offsets are distinct)
    uint32_t n2 = 2;
    while (n2 < ncand) n2 <<= 1;
    for (uint32_t i = ncand + lane; i < n2; i += kSmallThreads) L.cand[i] = ~0ull;
    __syncthreads();
    wave_sort(L.cand, n2, lane);

    // 4. confirmation: res[c] = the block the window at cand[c] matches, or -1
    int32_t *res = reinterpret_cast<int32_t *>(L.filt);
    for (uint32_t c = lane; c < ncand; c += kSmallThreads) {
        const uint64_t e = L.cand[c];
        const uint32_t q = (uint32_t)(e >> 32), sum = (uint32_t)e;
        const uint32_t w = min(B, size - q);  // match.go:114-117
        const uint64_t target = (uint64_t)sum << 32;
        uint32_t i = 0;
        for (uint32_t s = kc; s > 1;) {
            s >>= 1;
            if (L.keys[i + s - 1] < target) i += s;
        }
        if (L.keys[i] < target) i++;
        int32_t found = -1;
        bool hashed = false;
        uint32_t h[4];
        for (; i < kc; i++) {
            const uint64_t key = L.keys[i];
            const uint32_t k = (uint32_t)key;
            if ((uint32_t)(key >> 32) != sum || k >= (uint32_t)count) break;
            const int32_t b = targets[k];
            if (len_of(b, count, B, J.rem) != w) continue;  // match.go:118
            if (!hashed) {
                md4_init(h);
                int32_t ws1 = 0;
                uint32_t wt = 0;
                hash_block_direct<false>(src, (uintptr_t)src + size, q, w, seed, h, ws1, wt);
                hashed = true;
            }
            const u32x4a4 want = *reinterpret_cast<const u32x4a4 *>(sum2 + 16ull * (uint32_t)b);
            const uint32_t wv[4] = {want.x, want.y, want.z, want.w};
            bool eq = true;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int32_t nb = (int32_t)J.s2len - 4 * m;  // match.go:133: sum2[:s2len]
                const uint32_t mask = nb >= 4 ? ~0u : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
                eq = eq && ((h[m] ^ wv[m]) & mask) == 0;
            }
            if (eq) {
                found = b;
                break;
            }
        }
        res[c] = found;
    }
    __syncthreads();

    // 5. the greedy walk, wave-uniform: candidates 64 at a time in lanes,
    // visited in order by a scalar loop; matches compacted into cand[] (entry
    // n <= the candidate's own index, already read)
    uint32_t pos = 0, n = 0;
    for (uint32_t cb = 0; cb < ncand; cb += kSmallThreads) {
        const uint32_t j = cb + lane;
        const uint64_t e = j < ncand ? L.cand[j] : ~0ull;
        const int32_t r = j < ncand ? res[j] : -1;
        const uint32_t qv = (uint32_t)(e >> 32);
        const uint32_t lim = min(ncand - cb, kSmallThreads);
        uint64_t mm = 0;
        for (uint32_t u = 0; u < lim; u++) {
            const uint32_t qu = (uint32_t)__builtin_amdgcn_readlane((int)qv, (int)u);
            const int32_t ru = __builtin_amdgcn_readlane(r, (int)u);
            if (qu >= pos && ru >= 0) {
                mm |= 1ull << u;
                pos = qu + len_of(ru, count, B, J.rem);  // match.go:158 + the roll
            }
        }
        if ((mm >> lane) & 1ull) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
            L.cand[n + rank] = ((uint64_t)qv << 32) | (uint32_t)r;
        }
        n += __builtin_popcountll(mm);
        __syncthreads();
    }

    // 6. the file's matches to the launch's array
    uint32_t base = 0;
    if (lane == 0 && n) base = atomicAdd(match_count, n);
    base = __shfl(base, 0);
    o.n = n;
    o.base = base;
    if ((uint64_t)base + n > match_cap) {
        o.status = 2;
    } else {
        for (uint32_t i = lane; i < n; i += kSmallThreads) {
            const uint64_t e = L.cand[i];
            matches[base + i] = uint4{(uint32_t)(e >> 32), 0u, (uint32_t)e, 0u};  // rsg_match
        }
    }
    if (lane == 0) outs[jid] = o;
}

}  // namespace

hipError_t launch_search_small(const SmallJob *jobs, const uint32_t *order, uint32_t njobs, const uint8_t *blob,
                               uint32_t seed, uint32_t kc, void *matches, uint32_t match_cap,
                               uint32_t *match_count, SmallOut *outs, hipStream_t stream) {
    if (njobs == 0) return hipSuccess;
    hipLaunchKernelGGL(search_small_kernel, dim3(njobs), dim3(kSmallThreads), small_lds_bytes(kc), stream, jobs, order,
                       blob, seed, kc, small_fwords(kc), small_ccap(kc), reinterpret_cast<uint4 *>(matches),
                       match_cap, match_count, outs);
    return hipGetLastError();
}

}  // namespace rsg
