// rsg_host.h -- host-side internals of librsg.so shared by the C-ABI units.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rsg.h"
#include "rsg_internal.h"

// Device buffer that only grows (reused across calls on one context).
struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
};

// Pinned host buffer that only grows.
struct PinBuf {
    void *p = nullptr;
    uint64_t cap = 0;
};

// Sender scratch of one search in flight; a batch rotates three of them so
// later files' tables and kernels overlap file i's walk (rsg_match.cpp).
// Host temporaries of a search's table build (rsg_match.cpp tables()), owned
// by the slot and reused job after job: the ~2.5 MB they span stays faulted
// in (fresh vectors per job page-faulted on the first roll's critical path).
struct TableScratch {
    std::vector<std::pair<uint32_t, int32_t>> pairs, groups;  // (sum1, block), then grouped by sum1
    std::vector<uint32_t> cnt, hi16, bitmap;
    std::vector<std::pair<uint32_t, uint32_t>> keys;  // distinct sum1 -> flags
    std::vector<uint16_t> filter16;
    std::vector<uint64_t> table;
    std::vector<uint32_t> table_keys;  // the table's keys only (empty slots: an existing key)
    std::vector<uint8_t> fill;
};

struct SearchSlot {
    TableScratch hs;                   // host scratch of the table build
    DevBuf agg, prefix, counts;        // tile sums, tile prefixes, candidate count
    PinBuf list;                       // candidate list: pinned host memory the roll writes directly (no
                                       // read-back: a D2H queued beside the next roll waited 0.35-0.6 ms)
    DevBuf blob;                       // basis tables, one upload: groups | hi16 | sum2 | filter | table
    DevBuf src;                        // realigned or uploaded source
    PinBuf stage;                      // pinned staging of the blob
    PinBuf count;                      // candidate count read back
    DevBuf res;                        // confirmation results (block index per window)
    PinBuf hres;                       // ... read back; the job's walk reads them on a worker thread
    PinBuf sel;                        // offsets of the windows a confirm_all batch confirms (the GPU plan reads them)
    // Confirmation scratch of this slot's job (window descriptors, the plan's
    // workgroup table, records, the kernel's fallback words).  Per slot, not
    // per context: two jobs' confirmations run at once on different streams
    // (the last job's beside job n-2's), and a job's later round trips run on
    // a worker thread while the calling thread queues the next job's.
    DevBuf cfiles, cwg, cout, cfb;
    hipEvent_t scanned = nullptr;      // prefix pass done (side stream)
    hipEvent_t tables_b = nullptr;     // the resolve tables' upload done (side stream)
    hipEvent_t rolled = nullptr;       // roll kernel + count read-back done
    void *counts_zeroed = nullptr;     // counts.p once zeroed (every roll_count_out leaves it 0)
    hipEvent_t confirmed = nullptr;    // confirmation batch + result read-back done
};
constexpr int kSearchSlots = 4;  // jobs i-1 (walk on a worker), i (confirming), i+1 (rolling), i+2 (being issued)

// One launch slot of the small-file sender (rsg_sender_small.cpp): pinned
// staging of the launch's descriptors, sums and host sources, its device
// copy, the per-file results and match lists (pinned: the kernel writes them
// straight to host memory) and the launch's match counter.
struct SmallSlot {
    PinBuf stage, outs, matches;
    DevBuf dev, count;
    hipEvent_t up = nullptr, done = nullptr;
};

struct rsg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side[2] = {nullptr, nullptr};  // host-path pipeline streams; sender search slots
    hipEvent_t side_done[2] = {nullptr, nullptr};
    hipStream_t confirm = nullptr;  // sender confirmation batches, beside the next file's roll
    std::recursive_mutex mu;
    std::string err;
    // scratch reused by one-shot calls
    DevBuf d_files, d_wg;
    DevBuf d_in[2], d_out[2], d_desc[2], d_fb[2];
    PinBuf h_in[2], h_out[2], h_desc[2];
    // sender scratch
    SearchSlot search[kSearchSlots];
    SmallSlot small[2];
    // per-context options of the sender and receiver (rsg_testing_search_option;
    // the defaults are the measured product settings)
    struct Options {
        int path = 0;              // 0: small sources through the one-wave-per-file kernel; 1: all through the pipeline
        bool host_tables = false;  // the roll's filters and bucket table built on the host instead of the GPU
        bool force_table_ovf = false;  // report the GPU-built bucket table as overflowed (its fallback's tests)
        bool spec = false;         // speculative selection of the confirmed windows (Walker::spec_batch)
        int confirm_cus = 32;      // CUs a batch's rolls leave to the previous job's confirmation (0: serial)
        int recv_md4 = 0;          // receiveData's whole-file sums: 0 by size, 1 GPU, 2 host
        int fs_key_shift = 10;     // whole-file sums' lane order: length buckets of 2^shift bytes (40: arena order)
    } opts;
    DevBuf d_res;
    // multi-GPU
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // kernel timing (rsg_set_kernel_timing): event pairs bracketing kernels
    // on the streams they run on, kind 0 = roll, 1 = confirmation (block
    // sums of the windows + resolve), 2 = whole-file sums
    struct TimedSpan {
        hipEvent_t a, b;
        int kind;
    };
    bool timing = false;
    std::mutex spans_mu;  // spans and stat_* (a search's tail records them from a worker thread)
    std::vector<TimedSpan> spans;
    // block-sum kernel variant of this context (rsg_set_block_sums_kernel): -1 = automatic
    int bs_variant = -1;
    uint64_t stat_candidates = 0, stat_windows = 0;  // roll candidates read back, windows confirmed
};

// Plan of a block-sum batch (host side + resident device copies).
struct HostPlan {
    std::vector<rsg::DevFile> files;
    std::vector<uint32_t> wg_file;  // nwg + 1 entries
    uint64_t total_blocks = 0;
    uint32_t nwg = 0;
    bool aligned = true;      // every block start is 4-byte aligned (arena base aside)
    bool lines128 = true;     // every block start is 128-byte aligned (arena base aside)
    uint32_t max_blen = 0;    // largest block length (picks blocks per lane)
    uint64_t arena_bytes = 0;
    uint32_t lds_reserve = 0;  // dynamic LDS per workgroup of the long-block kernel (keeps it off CUs
                               // that hold a roll workgroup, rsg_match.cpp)
};

struct rsg_plan {
    rsg_ctx *ctx = nullptr;
    HostPlan host;
    void *d_files = nullptr;
    void *d_wg = nullptr;
    void *d_scratch = nullptr;
};

namespace rsgh {

rsg_status fail(rsg_ctx *ctx, rsg_status code, const char *fmt, ...);
rsg_status hip_fail(rsg_ctx *ctx, hipError_t e, const char *what);
rsg_status ensure_dev(rsg_ctx *ctx, DevBuf &b, uint64_t bytes);
rsg_status ensure_pin(rsg_ctx *ctx, PinBuf &b, uint64_t bytes);

// Head of one file: reference sizing (block_len == 0) or an explicit B.
bool head_for(int64_t len, int32_t block_len, rsg_sum_head *out);

// Fill `plan` from files (device offsets when use_offsets, else packed at
// 16-byte aligned offsets in the order given, which is how the host path lays
// out its staging arena).  `packed_bytes` receives the arena size needed.
rsg_status build_plan(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, uint64_t arena_bytes,
                      bool use_offsets, HostPlan &plan);

// Host memcpy of many (dst, src, n) jobs on a few threads (staging files into
// pinned memory is the host path's limiter on one core).  Jobs are cut into
// pieces of at most 2 MiB and handed out dynamically; small totals stay on
// the calling thread.  Threads: RSG_COPY_THREADS, default 8.
struct CopyJob {
    void *dst;
    const void *src;
    uint64_t n;
};
void parallel_copy(const std::vector<CopyJob> &jobs);

// Whole-file sums (rsg_files.cpp): descriptors through ctx->h_desc[slot] /
// d_desc[slot], kernel on `stream`, asynchronous.
rsg_status launch_file_sums_async(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes,
                                  const std::vector<rsg::FileSpan> &spans, int32_t mode, int32_t seed, void *d_out,
                                  int slot, hipStream_t stream);

// The generator's host loop (rsg_generate.cpp); records_only = only the
// 20-byte records in the stream (the per-rank part of the multi-GPU call).
rsg_status generate_files_fd_impl(rsg_ctx *ctx, const rsg_fd_file *files, uint64_t nfiles, int32_t seed,
                                  int32_t flags, rsg_write_fn write, void *user, rsg_sum_head *heads_out,
                                  uint64_t *bytes_written, bool records_only);

// Ragged RCCL gather of one rank's bytes to the root (rsg_dist.cpp): root
// receives send_bytes[q] from rank q at recv_off[q] (NULL: exclusive prefix).
// Grouped sends/receives; may be nested inside the caller's ncclGroupStart.
// in_place: the root's own bytes already sit at d_recv + recv_off[root].
rsg_status gatherv(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                   const uint64_t *recv_off, int32_t root, hipStream_t st, bool in_place);

// MD4 on the host (rsg_md4_host.cpp): whole-file sums whose serial chain
// streams through host memory (the sender's h, match.go:52-53; receiveData's
// check of large files).  Not used for block checksums.
struct Md4 {
    uint32_t st[4];
    uint64_t total;
    uint8_t buf[64];
    uint32_t nbuf;
    void init();
    void update(const uint8_t *p, uint64_t n);
    void final(uint8_t out[16]);
};

// The small-file sender (rsg_sender_small.cpp): settles every job of a
// search batch that is invalid, empty or eligible for the one-wave-per-file
// kernel; `rest` = the jobs for the large-file pipeline (not eligible, or
// candidates past the kernel's LDS list), in job order; msg[i] = job i's
// error message.  Returns a fatal (HIP / allocation) status or RSG_OK.
bool search_small_eligible(const rsg_ctx *ctx, const rsg_search_job &j);
rsg_status search_small_batch(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed, bool host_src,
                              std::vector<uint64_t> &rest, std::vector<std::string> &msg);

// Kernel timing helpers (no-ops unless ctx->timing): begin records an event
// on `stream` and returns it; end records the closing event.
hipEvent_t timed_begin(rsg_ctx *ctx, hipStream_t stream);
void timed_end(rsg_ctx *ctx, hipEvent_t a, hipStream_t stream, int kind);

// Upload plan descriptors to (grown) device buffers and launch the kernel.
rsg_status launch_plan(rsg_ctx *ctx, const HostPlan &plan, const void *d_files, const void *d_wg,
                       const void *d_arena, int32_t seed, void *d_records, void *d_scratch, hipStream_t stream);

}  // namespace rsgh

#define RSG_HIP(ctx, expr)                                    \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return rsgh::hip_fail((ctx), e_, #expr); \
    } while (0)
