/*
 * rsg.h -- C ABI of the MI355X (gfx950) rsync block-checksum engine.
 *
 * This is the drop-in boundary between the gokrazy/rsync host code and the
 * HIP kernels.  The reference has no FFI of its own (it is pure Go, SURVEY.md
 * F1); every entry point below names the Go function whose work it replaces,
 * and INTEGRATION.md shows the cgo binding a maintainer would add.
 *
 * Conventions
 *  - Plain C types only: pointers + sizes, no torch or HIP types.  `stream`
 *    parameters are a hipStream_t passed as void* (NULL = the context's own
 *    stream).
 *  - Every call returns rsg_status (0 = OK, negative = error) and never
 *    aborts; the message of the last failure on a context is returned by
 *    rsg_last_error(ctx) (Go maps it to `error`, as the reference's functions
 *    return errors and never panic by design).
 *  - The caller owns every buffer.  Nothing retains a caller pointer after
 *    return (cgo pointer rules), except where a *_device call documents that
 *    work is still queued on `stream`.
 *  - Threading: a context serialises its own calls with a mutex; separate
 *    contexts run concurrently (the loopback generator and sender goroutines of
 *    clientmaincmd.go:209-228 use one context each).  Each call selects its
 *    device itself, so Go may migrate OS threads freely.
 *  - All checksum arithmetic runs on the GPU.  There is no CPU fallback: with
 *    no usable gfx950 device, rsg_ctx_create fails with RSG_ERR_NODEV.
 */
#ifndef RSG_H
#define RSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSG_ABI_VERSION 5  /* 2: per-context block-sum kernel knob, multi-GPU calls, rsg_hash_search_fd;
                              3: rsg_hash_search_fd_batch;
                              4: block-sum variants pruned to the shipped set (-1, 0, 1, 2, 3, 4, 6, 14),
                                 small sources searched by the one-wave-per-file kernel;
                              5: variant 7 (line windows) replaces 14 */
/* One wire record: int32 LE sum1 then sum2[16] (generator.go:341-346). */
#define RSG_RECORD_BYTES 20
#define RSG_SUM2_BYTES 16
/* Literal token piece size, internal/sender/flist.go:52. */
#define RSG_CHUNK_SIZE (256 * 1024)
/* SumHead.ReadFrom limit on block_len, types.go:40. */
#define RSG_MAX_BLOCK_LEN (1 << 29)

typedef int32_t rsg_status;
#define RSG_OK 0
#define RSG_ERR_INVALID (-1)   /* bad argument: a Go `error`, nothing ran   */
#define RSG_ERR_NOMEM (-2)     /* device or pinned allocation failed         */
#define RSG_ERR_HIP (-3)       /* HIP runtime error, see rsg_last_error      */
#define RSG_ERR_NODEV (-4)     /* no gfx950 device at that ordinal           */
#define RSG_ERR_TRUNCATED (-5) /* output capacity too small; size reported   */
#define RSG_ERR_CORRUPT (-6)   /* whole-file sum mismatch (receiver.go:171)  */
#define RSG_ERR_IO (-7)        /* file read failed / short, or writer failed */

typedef struct rsg_ctx rsg_ctx;
typedef struct rsg_plan rsg_plan;

/* SumHead, types.go:19-36.  Field order is the wire order of
 * SumHead.WriteTo (types.go:79-86): count, block_len, s2len, rem. */
typedef struct rsg_sum_head {
    int32_t count;
    int32_t block_len;
    int32_t s2len;
    int32_t rem;
} rsg_sum_head;

/* One basis file of a batched block-sum job.
 *  device calls: `offset` is the byte offset of the file in the device arena;
 *  host calls:   `data` points at the file bytes in host memory.
 * block_len = 0 selects the reference sizing SumSizesSqroot
 * (rsynccommon.go:14-37); block_len > 0 is an explicit B. */
typedef struct rsg_file {
    const uint8_t *data;
    uint64_t offset;
    uint64_t len;
    int32_t block_len;
    int32_t reserved;
} rsg_file;

/* One match of the sender search: matched(h, ms, head, offset, i) with i >= 0
 * (match.go:149,233). */
typedef struct rsg_match {
    int64_t offset;
    int32_t index;
    int32_t reserved;
} rsg_match;

/* ------------------------------------------------------------------ misc */
int32_t rsg_abi_version(void);
/* Number of visible gfx950 devices (0 when none). */
int32_t rsg_device_count(void);

/* SumSizesSqroot (rsynccommon.go:14-37) or an explicit block length.
 * Host arithmetic only. */
rsg_status rsg_sum_head_for(int64_t file_len, int32_t block_len, rsg_sum_head *out);

/* ------------------------------------------------------------ context */
rsg_status rsg_ctx_create(int32_t device, rsg_ctx **out);
void rsg_ctx_destroy(rsg_ctx *ctx);
/* Last error message of ctx (or of the calling thread when ctx == NULL). */
const char *rsg_last_error(const rsg_ctx *ctx);
/* Pinned host memory for zero-copy staging of file reads (generator.go:335
 * reads each block into a Go buffer; reading into this memory instead saves
 * one copy on the host path). */
rsg_status rsg_alloc_pinned(rsg_ctx *ctx, uint64_t bytes, void **out);
rsg_status rsg_free_pinned(rsg_ctx *ctx, void *p);
/* Device memory helpers for callers that have no allocator of their own. */
rsg_status rsg_alloc_device(rsg_ctx *ctx, uint64_t bytes, void **out);
rsg_status rsg_free_device(rsg_ctx *ctx, void *p);
rsg_status rsg_memcpy_h2d(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes);
rsg_status rsg_memcpy_d2h(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes);
rsg_status rsg_memcpy_d2d(rsg_ctx *ctx, void *dst, const void *src, uint64_t bytes);
rsg_status rsg_synchronize(rsg_ctx *ctx, void *stream);
/* Synthetic data: dst[0..n) = splitmix64(seed) little-endian byte stream
 * (SURVEY.md appendix), generated on the device. */
rsg_status rsg_fill_splitmix64(rsg_ctx *ctx, void *d_dst, uint64_t n, uint64_t seed, void *stream);

/* ------------------------------------------ receiver: block sums (★ a2,a3,a7)
 * Replaces the per-block loop of (*receiver.Transfer).generateAndSendSums
 * (generator.go:325-350: Checksum1 + Checksum2(seed) per block) for a whole
 * batch of files.  Output: for file i, heads[i] and head.count records of
 * RSG_RECORD_BYTES starting at record first_record[i]; records of consecutive
 * files are contiguous, in file order.  The Go caller writes, per file in
 * file-list order, idx, SumHead, then that file's records (generator.go:317-321),
 * chunked <= 256 KiB per Write on the mux writer (wire.go:46-62). */

/* Host arithmetic: heads, first_record (may be NULL) and the total record count. */
rsg_status rsg_plan_block_sums(const rsg_file *files, uint64_t nfiles, rsg_sum_head *heads,
                               uint64_t *first_record, uint64_t *total_records);

/* Device-resident plan: uploads the per-file descriptors once, for repeated
 * launches over the same file layout in a device arena of arena_bytes. */
rsg_status rsg_plan_create(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles,
                           uint64_t arena_bytes, rsg_plan **out);
void rsg_plan_destroy(rsg_plan *plan);
uint64_t rsg_plan_total_records(const rsg_plan *plan);

/* Launch the block-sum kernel for `plan` over d_arena, writing
 * total_records * 20 bytes at d_records.  Asynchronous on `stream`. */
rsg_status rsg_block_sums_planned(rsg_ctx *ctx, const rsg_plan *plan, const void *d_arena,
                                  int32_t seed, void *d_records, void *stream);

/* Tuning knob of one context: block-sum kernel variant.  Every variant
 * gives identical records; only speed differs.  -1 = automatic (default),
 * 0 = direct per-lane loads, 1 = staged LDS-DMA slabs (256 bytes of every
 * block per segment), 2 = park (three loader waves stream 64-block tiles
 * through LDS, five hasher waves park the blocks in registers; blocks <= 703
 * bytes, otherwise 1 is used), 3 = deep per-lane prefetch for long blocks,
 * 4 = staged with 128-byte segments, 6 = staged for blocks at any byte
 * offset (pieces fetched from the 4-byte aligned address below the block,
 * funnel-shifted in registers; needs a 4-byte aligned arena, else 3 / 0),
 * 7 = line windows: each block's bytes fetched as the 128-byte lines that
 * hold them, each line once, for blocks at any offset (needs a 128-byte
 * aligned arena, else 6 for unaligned blocks and 1 for aligned ones).
 * Automatic, in two lines: unaligned blocks, or blocks of >= 704 bytes off
 * the 128-byte lines -> 7; 512..703 bytes -> park (2); on the 128-byte lines
 * up to 32 KiB -> 4 (the library's own packing keeps file offsets on the
 * lines, so B a multiple of 128 qualifies); otherwise 1.  The LDS-DMA
 * variants fall back to 0 for blocks that are not 4-byte aligned.  The
 * environment variable RSG_BLOCKSUMS_KERNEL sets a new context's initial
 * value.  Returns RSG_ERR_INVALID for any other value (the variants
 * numbered 5, 8..15 in ABI 3 and 4 were measured slower and removed;
 * tools/build_ab.sh rebuilds them from the history). */
rsg_status rsg_set_block_sums_kernel(rsg_ctx *ctx, int32_t variant);

/* Fallback census of ctx's device since the last reset: counts[0] = full
 * 64-block waves of the staged kernels (1, 4, 5, 6), counts[1] = full
 * 64-block tiles of the park kernel (2), that could not be staged through
 * LDS and were hashed with per-lane loads instead (a span past a 31-bit
 * offset, reads that would run past the arena's end).  Records are identical
 * either way; this tells a test or a bench that the fast path was taken.
 * Waits for all work on the device.  reset != 0 zeroes the counters after
 * reading them. */
rsg_status rsg_block_sums_fallbacks(rsg_ctx *ctx, uint64_t counts[2], int32_t reset);

/* One-shot device call: plan + launch + wait. */
rsg_status rsg_block_sums_device(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes,
                                 const rsg_file *files, uint64_t nfiles, int32_t seed,
                                 void *d_records, uint64_t records_cap);

/* Host buffers in (rsg_file.data), host records out: stages through pinned
 * memory, overlapping H2D, kernel and D2H.  Synchronous. */
rsg_status rsg_block_sums_host(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, int32_t seed,
                               uint8_t *records, uint64_t records_cap);

/* ---------------------------------- receiver: the generator's host loop (§8f row 1)
 * Replaces GenerateFiles' per-file work for files that reach
 * generateAndSendSums (generator.go:143-322,325-350): for each file in list
 * order, int32 idx (generator.go:317, with RSG_GEN_IDX), the SumHead
 * (types.go:79-86) and count x (int32 LE sum1, sum2[16]); RSG_GEN_TERMINATE
 * appends the two int32 -1 phase markers (generator.go:31,40).  File bytes
 * are read with pread from `fd` at [offset, offset+len) (io.ReadFull of every
 * block, generator.go:335): a file shorter than len is RSG_ERR_IO "unexpected
 * EOF".  Reading (a few threads, 2 MiB pieces), H2D + kernel + D2H and the
 * writes of consecutive batches (RSG_GEN_BATCH_MB, default 32 MiB) overlap.  The stream goes to
 * write(user, data, len) once per batch (0 = ok; anything else stops the
 * call with RSG_ERR_IO), framed as <= 256 KiB MsgData messages with
 * RSG_GEN_MUX (the server side's MultiplexWriter, wire.go:28-36; the demuxed
 * bytes equal the reference's, message boundaries differ).  heads_out (may be
 * NULL) receives nfiles heads; *bytes_written counts the bytes handed to
 * write.  On failure, the bytes already written are a prefix of the stream.
 * Synchronous; write is called on the calling thread and must not call into
 * the same context (it holds the context's staging buffers). */
typedef struct rsg_fd_file {
    int32_t fd;          /* open for reading (Go: int(f.Fd()))          */
    int32_t idx;         /* file-list index written before the SumHead  */
    int64_t offset;      /* first byte of the file in fd (normally 0)   */
    uint64_t len;        /* fileLen of generateAndSendSums              */
    int32_t block_len;   /* 0 = SumSizesSqroot, else explicit B          */
    int32_t reserved;
} rsg_fd_file;
typedef int32_t (*rsg_write_fn)(void *user, const uint8_t *data, uint64_t len);
#define RSG_GEN_IDX 1
#define RSG_GEN_TERMINATE 2
#define RSG_GEN_MUX 4
rsg_status rsg_generate_files_fd(rsg_ctx *ctx, const rsg_fd_file *files, uint64_t nfiles, int32_t seed,
                                 int32_t flags, rsg_write_fn write, void *user, rsg_sum_head *heads_out,
                                 uint64_t *bytes_written);

/* ---------------------------------------------- sender: hash search (★ a11)
 * Replaces the per-byte search of (*sender.Transfer).hashSearch
 * (match.go:21-230) for one source file against the receiver's sums:
 *   head            SumHead read by receiveSums (sender.go:118-151)
 *   sum1[count]     SumBuf.Sum1 in block-index order
 *   sum2[count*16]  SumBuf.Sum2 (only the first head->s2len bytes compared)
 *   targets[count]  the Go `targets` order: block indices sorted by
 *                   Tag(sum1) (sender.go:60-75); its tie order among equal
 *                   tags decides which duplicate block is reported.
 * Output: the greedy match list in offset order, exactly the (offset, i >= 0)
 * pairs hashSearch passes to matched().  The literal/match token bytes follow
 * from it with rsg_encode_tokens; the whole-file MD4 stays with the caller
 * (match.go:52-53,262-269 feeds it incrementally).
 * *n_matches is always set; RSG_ERR_TRUNCATED when it exceeds match_cap. */
rsg_status rsg_hash_search_host(rsg_ctx *ctx, const uint8_t *src, uint64_t src_len,
                                const rsg_sum_head *head, const uint32_t *sum1, const uint8_t *sum2,
                                const int32_t *targets, int32_t seed, rsg_match *matches,
                                uint64_t match_cap, uint64_t *n_matches);
/* Same with the source already resident at d_src on the device. */
rsg_status rsg_hash_search_device(rsg_ctx *ctx, const void *d_src, uint64_t src_len,
                                  const rsg_sum_head *head, const uint32_t *sum1,
                                  const uint8_t *sum2, const int32_t *targets, int32_t seed,
                                  rsg_match *matches, uint64_t match_cap, uint64_t *n_matches);

/* Same, with the source read from a file by the engine (row a13: the
 * sender's mapFile / ptr window, internal/sender/fileio.go:31-112): bytes
 * [offset, offset + src_len) of fd (src_len = the stat'ed size, as
 * sendFile's fi.Size()) are read with pread in windows of
 * RSG_SEARCH_WINDOW_KB (default 256 MiB; at least 2 B), each uploaded with a
 * B-1 byte halo and searched while the next window is read, so host and HBM
 * use stay bounded by two windows whatever the file size.  A file shorter
 * than src_len (or a read error) is RSG_ERR_IO "file has changed
 * mid-transfer" (fileio.go:99-104).  file_sum != NULL also receives the
 * transfer's whole-file sum MD4(int32_LE(seed) || source) (match.go:52-53,
 * 220-226), computed on a host thread over the same staged bytes (one
 * serial chain per file).  head->count == 0 (sendFile, sender.go:86-88) or
 * an empty source searches nothing and only reads the file for file_sum. */
rsg_status rsg_hash_search_fd(rsg_ctx *ctx, int32_t fd, int64_t offset, uint64_t src_len, const rsg_sum_head *head,
                              const uint32_t *sum1, const uint8_t *sum2, const int32_t *targets, int32_t seed,
                              rsg_match *matches, uint64_t match_cap, uint64_t *n_matches, uint8_t file_sum[16]);

/* rsg_hash_search_fd over the files of a transfer (SendFiles' per-file loop,
 * sender.go:19-115, for sources that are open files): each job is searched
 * as rsg_hash_search_fd would (windows, B-1 halo, "file has changed
 * mid-transfer"), in job order, while the jobs' whole-file sums
 * MD4(int32_LE(seed) || source) (match.go:52-53,220-226) run on
 * RSG_SUM_THREADS host threads (default 10; longest file first, each thread
 * reading its file's bytes itself), so several files' serial MD4 chains
 * proceed side by side instead of one after the other.  file_sum = NULL
 * skips a job's sum; head.count == 0 (sendFile) reads the file only for it.
 * Unlike the reference (match.go:52-53,268) and rsg_hash_search_fd, the sum
 * is computed from a second read of the file, not from the searched bytes: a
 * file rewritten in place at the same length mid-transfer can give a sum
 * that does not match the sent data (the receiver's check then fails; see
 * DESIGN.md 4.2.1).
 * Every job's n_matches and status are set: RSG_OK, RSG_ERR_INVALID (its own
 * arguments), RSG_ERR_TRUNCATED (beyond match_cap; n_matches is the full
 * count), RSG_ERR_IO (short file / read error).  A HIP or allocation failure
 * stops the searches and every unfinished job gets its status.  Returns
 * RSG_OK or the first failing job's status, its message in rsg_last_error. */
typedef struct rsg_fd_search_job {
    int32_t fd;              /* open for reading                              */
    int32_t reserved;
    int64_t offset;          /* first byte of the source in fd                */
    uint64_t src_len;        /* the stat'ed size                              */
    rsg_sum_head head;
    const uint32_t *sum1;    /* as rsg_hash_search_*                          */
    const uint8_t *sum2;
    const int32_t *targets;
    rsg_match *matches;
    uint64_t match_cap;
    uint64_t n_matches;      /* out */
    uint8_t *file_sum;       /* out: 16 bytes, or NULL                        */
    int32_t status;          /* out */
    int32_t reserved2;
} rsg_fd_search_job;
rsg_status rsg_hash_search_fd_batch(rsg_ctx *ctx, rsg_fd_search_job *jobs, uint64_t njobs, int32_t seed);

/* Batched search over the files of a transfer: replaces SendFiles' per-file
 * loop (sender.go:19-115) once their sums have been read, i.e. one
 * hashSearch (sender.go:90) per job, in job order.  Jobs are pipelined: job
 * i+1's basis tables and weak-sum scan run on the GPU while job i is walked
 * and confirmed.  Each job's result equals the single-file call's.
 * Every job's n_matches and status are set: RSG_OK, RSG_ERR_INVALID for its
 * own bad arguments, RSG_ERR_TRUNCATED beyond match_cap (n_matches is the
 * full count).  A HIP or allocation failure stops the batch: that job and
 * the later ones get its status.  The call returns RSG_OK, or the first
 * failing job's status with that job's message in rsg_last_error. */
typedef struct rsg_search_job {
    const void *src;         /* device pointer (_device) or host pointer (_host) */
    uint64_t src_len;
    rsg_sum_head head;
    const uint32_t *sum1;    /* as rsg_hash_search_*                          */
    const uint8_t *sum2;
    const int32_t *targets;
    rsg_match *matches;
    uint64_t match_cap;
    uint64_t n_matches;      /* out */
    int32_t status;          /* out */
    int32_t reserved;
} rsg_search_job;
rsg_status rsg_hash_search_batch_device(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed);
rsg_status rsg_hash_search_batch_host(rsg_ctx *ctx, rsg_search_job *jobs, uint64_t njobs, int32_t seed);

/* Kernel timing for roofline measurements (bench.py): while on, every roll
 * launch and confirmation batch (block sums of the windows + resolve) of the
 * sender and every whole-file-sum launch of ctx is bracketed by HIP events on
 * the stream it runs on.  rsg_kernel_times waits for them and returns
 * out[0] = total roll ms, out[1] = roll launches (a launch of the small-file
 * kernel, which rolls, confirms and walks many files at once, counts as a
 * roll launch), out[2] = total confirmation
 * ms, out[3] = confirmation batches, out[4] = candidate offsets the rolls
 * returned, out[5] = windows confirmed, out[6] = total whole-file-sum kernel
 * ms, out[7] = its launches; reset != 0 drops the recorded events and zeroes
 * the counts. */
rsg_status rsg_set_kernel_timing(rsg_ctx *ctx, int32_t on);
rsg_status rsg_kernel_times(rsg_ctx *ctx, double out[8], int32_t reset);

/* Token stream of simpleSendToken (token.go:4-31) as matched() emits it
 * (match.go:233-282): literal runs in <= 256 KiB pieces (int32 LE n + n bytes),
 * a match as int32 -(i+1), terminated by int32 0 (match.go:212).  Host byte
 * formatting, no checksum work.  out == NULL queries *out_len. */
rsg_status rsg_encode_tokens(const uint8_t *src, uint64_t src_len, const rsg_sum_head *head,
                             const rsg_match *matches, uint64_t n_matches, uint8_t *out,
                             uint64_t out_cap, uint64_t *out_len);

/* ------------------------------------------ receiver token application
 * Replaces (*receiver.Transfer).receiveData's token loop (receiver.go:98-188,
 * recvToken token.go:6-20).  `tokens` = the bytes after the SumHead: literal
 * runs (int32 LE n > 0 + n bytes), matches (int32 -(i+1) = basis block i,
 * head->block_len bytes at i*block_len, head->rem for block count-1), the
 * int32 0 terminator, then the 16-byte whole-file sum.  The file is rebuilt
 * into out (out == NULL or too small: RSG_ERR_TRUNCATED with *out_len set).
 * A stream that ends early, a match past the end of the basis or a match
 * without a basis (basis == NULL) is RSG_ERR_INVALID, as the reference's
 * ReadFull / ReadAt / "local file not open" errors.
 *   rsg_apply_tokens: rebuild only; *consumed = offset of the whole-file sum.
 *   rsg_receive_data: rebuild, then MD4(int32_LE(seed) || file) on the GPU
 *     (seeded file-sum kernel) against the stream's sum: RSG_ERR_CORRUPT on
 *     mismatch ("file corruption", receiver.go:171-173); *consumed includes
 *     the 16 sum bytes. */
rsg_status rsg_apply_tokens(const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed);
rsg_status rsg_receive_data(rsg_ctx *ctx, const uint8_t *tokens, uint64_t tokens_len, const rsg_sum_head *head,
                            const uint8_t *basis, uint64_t basis_len, int32_t seed, uint8_t *out, uint64_t out_cap,
                            uint64_t *out_len, uint64_t *consumed);

/* Batched receiveData for the files of a transfer (RecvFiles' per-file
 * receiveData calls, receiver.go:18-188): every job as rsg_receive_data,
 * with the seeded whole-file sums of many files hashed together (one GPU
 * lane per file; MD4 is serial within a file, so a single large file gains
 * nothing over rsg_receive_data).  Jobs go in batches of <= 256 MiB of
 * rebuilt bytes; batch k is hashed on the GPU while the host applies the
 * tokens of batch k+1.  Per job: out_len, consumed and status (RSG_OK;
 * RSG_ERR_INVALID / RSG_ERR_TRUNCATED for its own stream or capacity, as
 * rsg_receive_data; RSG_ERR_CORRUPT on a whole-file sum mismatch).  A HIP or
 * allocation failure stops the call and is every unfinished job's status.
 * Returns RSG_OK or the first failing job's status. */
typedef struct rsg_recv_job {
    const uint8_t *tokens;   /* bytes after the SumHead: tokens, 0, 16-byte sum */
    uint64_t tokens_len;
    rsg_sum_head head;
    const uint8_t *basis;    /* NULL: no local file                          */
    uint64_t basis_len;
    uint8_t *out;            /* rebuilt file                                 */
    uint64_t out_cap;
    uint64_t out_len;        /* out */
    uint64_t consumed;       /* out: stream bytes used, including the sum     */
    int32_t status;          /* out */
    int32_t reserved;
} rsg_recv_job;
rsg_status rsg_receive_data_batch(rsg_ctx *ctx, rsg_recv_job *jobs, uint64_t njobs, int32_t seed);

/* ------------------------------------------ whole-file sums
 * MD4 of whole files, one GPU lane per file (MD4 is serial within a message,
 * so this pays off for many files per call, e.g. a --checksum file list):
 *   RSG_FILESUM_PLAIN  = MD4(file): rsyncchecksum.ReaderChecksum
 *                        (rsyncchecksum.go:60-66), called per file by the
 *                        sender's file list (sender/flist.go:276-293) and the
 *                        receiver's quick check (receiver/generator.go:82-88);
 *   RSG_FILESUM_SEEDED = MD4(int32_LE(seed) || file): the transfer's whole-file
 *                        sum, seeded before the data (match.go:52-53,
 *                        sender.go:184-206, receiver.go:117-120).
 * out receives nfiles * 16 bytes, digest i at out + 16 i. */
#define RSG_FILESUM_PLAIN 0
#define RSG_FILESUM_SEEDED 1
/* files[i].data / len (offset and block_len ignored). */
rsg_status rsg_file_sums_host(rsg_ctx *ctx, const rsg_file *files, uint64_t nfiles, int32_t mode,
                              int32_t seed, uint8_t *out);
/* files[i].offset / len inside the device arena; d_out on the device. */
rsg_status rsg_file_sums_device(rsg_ctx *ctx, const void *d_arena, uint64_t arena_bytes,
                                const rsg_file *files, uint64_t nfiles, int32_t mode, int32_t seed,
                                void *d_out);

/* ------------------------------------------ multi-GPU sums gather
 * Files shard across the GPUs of one node with no data-path collective; the
 * only exchange is the final gather of each rank's records to the root over
 * RCCL (xGMI).  The caller exchanges the 128-byte unique id out of band (the
 * Go host over its own control channel; bench.py over torch.distributed). */
rsg_status rsg_comm_unique_id(uint8_t id[128]);
rsg_status rsg_comm_init(rsg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]);
/* Ragged gather: rank r sends send_bytes[r] bytes from d_send; the root receives
 * them back to back at d_recv (offsets = exclusive prefix of send_bytes).
 * send_bytes has nranks entries on every rank.  Asynchronous on `stream`. */
rsg_status rsg_gather_bytes(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes,
                            void *d_recv, int32_t root, void *stream);
/* Same with explicit landing offsets: rank q's bytes go to d_recv +
 * recv_offsets[q] on the root (NULL = the exclusive prefix of send_bytes). */
rsg_status rsg_gatherv_bytes(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                             const uint64_t *recv_offsets, int32_t root, void *stream);

/* Pipelined sharded generator step.  A rank's share of the file list
 * (contiguous block ranges, rsync_amd/dist.py) is cut into batches, each
 * with its own plan over the rank's arena.  Batch b's records are written at
 * d_records + 20 * record_offset and, while batch b+1 is hashed (kernel on
 * the context's stream, the transfer on a second one behind an event):
 *   rsg_block_sums_gather: sent to the root over RCCL (xGMI); every rank's
 *     bytes of batch b (send_bytes[q], nranks entries, equal on all ranks)
 *     land at d_recv + recv_offsets[q] on the root, so the root's buffer ends
 *     up in global record order (GenerateFiles' file-list order,
 *     generator.go:20-52).  The root's own kernels write its records
 *     straight to their landing offsets in d_recv (no self copy; its
 *     d_records is not written).  Collective: every rank calls it with the
 *     same nbatch; a rank with no blocks in batch b passes plan = NULL.
 *   rsg_block_sums_d2h: copied to h_records + 20 * record_offset on the
 *     host (ranks do this concurrently over their own PCIe links: the
 *     alternative to gather-then-one-D2H).  Pinned h_records runs at DMA speed.
 * Synchronous: returns after the last transfer. */
typedef struct rsg_shard_batch {
    const rsg_plan *plan;          /* this rank's pieces of batch b (NULL: none) */
    uint64_t record_offset;        /* first record of batch b in d_records       */
    const uint64_t *send_bytes;    /* gather: nranks entries                     */
    const uint64_t *recv_offsets;  /* gather: nranks entries (root byte offsets)  */
} rsg_shard_batch;
rsg_status rsg_block_sums_gather(rsg_ctx *ctx, const rsg_shard_batch *batches, uint64_t nbatch,
                                 const void *d_arena, int32_t seed, void *d_records, void *d_recv,
                                 int32_t root);
rsg_status rsg_block_sums_d2h(rsg_ctx *ctx, const rsg_shard_batch *batches, uint64_t nbatch,
                              const void *d_arena, int32_t seed, void *d_records, uint8_t *h_records);

/* ------------------------------------------ one process, many GPUs
 * gokr-rsync is ONE process whose generator is one goroutine
 * (internal/receiver/do.go:96-98, generator.go:20-52): the drop-in for a node
 * of N GPUs is that process driving N contexts (one per device) from the
 * calling thread.  The file list's global block sequence is cut into N
 * contiguous, byte-balanced ranges on block boundaries (rank q takes range
 * q), each range again into nbatch batches; records of rank q land at
 * rank_offset[q] of the global record stream, so their concatenation is the
 * single-GPU (and the reference's) record order.  The same plan is what the
 * multi-process bench uses (rsync_amd/dist.py restates it for the tests).
 * Multi-context calls report failures in rsg_last_error(ctxs[0]). */

/* One piece of a shard plan: blocks [b0, b1) of file `file` (bytes
 * [offset, offset + length) of it; the last block may be the file's
 * remainder), in rank `rank`'s batch `batch`; `record` = global record index
 * of block b0. */
typedef struct rsg_piece {
    uint64_t file;
    uint64_t b0, b1;
    uint64_t offset, length;
    uint64_t record;
    int32_t block_len;
    int32_t rank;
    int32_t batch;
    int32_t reserved;
} rsg_piece;
/* Host arithmetic.  lengths[nfiles]; block_lens[nfiles] (NULL: every file
 * block_len; 0 = SumSizesSqroot).  Pieces in global order (= rank, batch
 * order); pieces == NULL or cap too small: RSG_ERR_TRUNCATED with *n_pieces
 * set.  records (may be NULL): world * nbatch counts, records[q * nbatch + b]
 * = records of rank q's batch b. */
rsg_status rsg_shard_plan(const uint64_t *lengths, const int32_t *block_lens, uint64_t nfiles, int32_t block_len,
                          int32_t world, int32_t nbatch, rsg_piece *pieces, uint64_t cap, uint64_t *n_pieces,
                          uint64_t *records);

/* RCCL communicator over the devices of n contexts in this process
 * (ncclCommInitAll): ctxs[q] becomes rank q.  Distinct devices only. */
rsg_status rsg_comm_init_all(rsg_ctx *const *ctxs, int32_t n);

/* Device-resident sharded step over n contexts from one thread: rank q's
 * batches (ranks[q].batches, plans of ctxs[q] over ranks[q].d_arena, records
 * into ranks[q].d_records at each batch's record_offset), batch b's kernels on
 * every device, then its records delivered while batch b+1 hashes:
 *   rsg_block_sums_gather_multi: to ranks[root]'s device at d_recv over RCCL
 *     (rsg_comm_init_all first), landing at the batches' recv_offsets;
 *   rsg_block_sums_d2h_multi: every device's records to h_records + 20 *
 *     (rank_record_offset + record_offset) over its own PCIe link.
 * Every rank has the same nbatch.  Synchronous. */
typedef struct rsg_shard_rank {
    rsg_ctx *ctx;
    const void *d_arena;
    void *d_records;
    const rsg_shard_batch *batches;
    uint64_t nbatch;
    uint64_t rank_record_offset;  /* d2h: first global record of this rank */
} rsg_shard_rank;
rsg_status rsg_block_sums_gather_multi(const rsg_shard_rank *ranks, int32_t n, int32_t seed, void *d_recv,
                                       int32_t root);
rsg_status rsg_block_sums_d2h_multi(const rsg_shard_rank *ranks, int32_t n, int32_t seed, uint8_t *h_records);

/* Host buffers in, host records out, over n contexts: rsg_block_sums_host's
 * contract for the whole file list, the global block sequence sharded over
 * the contexts' devices (rsg_shard_plan, one batch per rank), every rank's
 * share staged and hashed on its own device concurrently and its records
 * written straight into `records` at its global offset. */
rsg_status rsg_block_sums_host_multi(rsg_ctx *const *ctxs, int32_t n, const rsg_file *files, uint64_t nfiles,
                                     int32_t seed, uint8_t *records, uint64_t records_cap);

/* rsg_generate_files_fd over n contexts: the same stream (idx, SumHead,
 * records, phase markers; MsgData framing with RSG_GEN_MUX) in file-list
 * order, written on the calling thread, while every rank reads and hashes
 * its contiguous byte-balanced range of the global block sequence (files may
 * be split between ranks on block boundaries) on its own device.  The
 * demuxed bytes equal the single-context call's.  Rank q's records are
 * buffered in host memory until ranks < q have been written, at most 256 MiB
 * per rank (plus one generator batch's records): a rank whose queue is full
 * waits until the writer takes its records, so the call's host memory is
 * bounded whatever the transfer size. */
rsg_status rsg_generate_files_fd_multi(rsg_ctx *const *ctxs, int32_t n, const rsg_fd_file *files, uint64_t nfiles,
                                       int32_t seed, int32_t flags, rsg_write_fn write, void *user,
                                       rsg_sum_head *heads_out, uint64_t *bytes_written);

/* ------------------------------------------ wire formats
 * Host byte formatting around the checksum path, so the engine's records
 * leave wire-ready.  No GPU work; re-entrant.  Outputs follow the
 * rsg_encode_tokens convention: out == NULL queries *out_len; a too-small
 * out is RSG_ERR_TRUNCATED with *out_len set. */

/* SumHead.ReadFrom validation (types.go:38-77): count >= 0,
 * 0 <= block_len <= 1<<29, 0 <= s2len <= 16, 0 <= rem <= block_len. */
rsg_status rsg_check_sum_head(const rsg_sum_head *head);
/* The generator's stream for a batch (replaces the per-block Conn writes of
 * generateAndSendSums, generator.go:325-350): for file f, int32 file_idx[f]
 * (recvGenerator, generator.go:317; omitted when file_idx == NULL), the
 * SumHead (types.go:79-86), then heads[f].count x (int32 LE sum1,
 * sum2[:s2len]) taken from the 20-byte records (files back to back, as
 * rsg_block_sums_* write them).  terminate != 0 appends GenerateFiles'
 * two int32 -1 phase markers (generator.go:31,40). */
rsg_status rsg_encode_sums(const int32_t *file_idx, const rsg_sum_head *heads, uint64_t nfiles,
                           const uint8_t *records, int32_t terminate, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len);
/* Sender side: SumHead.ReadFrom + receiveSums (sender.go:118-151) into the
 * arrays rsg_hash_search_* take: sum1[count], sum2[count*16] (bytes past
 * s2len zeroed).  *consumed = 16 + count*(4+s2len) is set once the head
 * parsed; cap < count is RSG_ERR_TRUNCATED (head filled in), a short stream
 * or an invalid head is RSG_ERR_INVALID with the reference's message. */
rsg_status rsg_decode_sums(const uint8_t *wire, uint64_t wire_len, rsg_sum_head *head, uint32_t *sum1,
                           uint8_t *sum2, uint64_t cap, uint64_t *consumed);
/* MultiplexWriter.WriteMsg (wire.go:28-36): data split into messages of at
 * most max_message (<= 256 KiB, the reader's limit, wire.go:46-62) bytes,
 * each prefixed by int32 LE ((7 + tag) << 24 | len). */
rsg_status rsg_mux_frame(const uint8_t *data, uint64_t len, int32_t tag, uint32_t max_message, uint8_t *out,
                         uint64_t out_cap, uint64_t *out_len);
/* MultiplexReader (wire.go:49-95): concatenated MsgData payloads; MsgInfo is
 * skipped, MsgError or another tag, a length > 256 KiB or a cut message is
 * RSG_ERR_INVALID. */
rsg_status rsg_mux_deframe(const uint8_t *wire, uint64_t wire_len, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len);
/* Conn.WriteInt64 / ReadInt64 (wire.go:108-117,177-195): int32 when
 * 0 <= v <= 0x7fffffff, else int32 -1 then int64 LE. */
rsg_status rsg_put_int64(int64_t v, uint8_t out[12], uint64_t *out_len);
rsg_status rsg_get_int64(const uint8_t *in, uint64_t in_len, int64_t *v, uint64_t *consumed);

#ifdef __cplusplus
}
#endif
#endif /* RSG_H */
