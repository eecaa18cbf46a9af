// rsg_dist.cpp -- multi-GPU exchange of the sharded generator step
// (SURVEY.md §8(e)): RCCL over xGMI for the records gather, and the two
// pipelined delivery modes of a rank's batches (include/rsg.h).
//
// The reference has no distribution of its own: GenerateFiles writes every
// file's sums in file-list order (internal/receiver/generator.go:20-52).
// Here the file list is sharded over the ranks of one node (rsync_amd/dist.py
// plans it); the only exchange is moving each rank's records to where the
// writer is, in global order.  Both modes overlap that movement with the
// hashing of the next batch:
//   kernel(b)  on ctx->stream            kernel(b+1) ...
//   move(b)    on ctx->side[0], after an event recorded behind kernel(b)
// (one batch: the move follows the kernel on ctx->stream; the root of a
// one-rank gather has nothing to move).
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "rsg_host.h"

using namespace rsgh;

namespace rsgh {

// Root receives send_bytes[q] bytes from every rank q at recv_off[q] (or the
// exclusive prefix of send_bytes when recv_off is NULL); grouped
// ncclSend/ncclRecv, since the sizes are ragged (ncclGather is not).
// in_place: the root's own bytes are already at d_recv + recv_off[root] (its
// kernel wrote them there), so there is no self copy.
rsg_status gatherv(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                   const uint64_t *recv_off, int32_t root, hipStream_t st, bool in_place) {
    ncclResult_t r = ncclGroupStart();
    if (ctx->rank == root) {
        uint64_t off = 0;
        for (int q = 0; q < ctx->nranks; q++) {
            uint8_t *dst = (uint8_t *)d_recv + (recv_off ? recv_off[q] : off);
            if (send_bytes[q]) {
                if (q == root && in_place) {
                    // already there
                } else if (q == root) {
                    const hipError_t e = hipMemcpyAsync(dst, d_send, send_bytes[q], hipMemcpyDeviceToDevice, st);
                    if (e != hipSuccess) {
                        ncclGroupEnd();
                        return hip_fail(ctx, e, "gather self copy");
                    }
                } else if (r == ncclSuccess) {
                    r = ncclRecv(dst, send_bytes[q], ncclUint8, q, ctx->comm, st);
                }
            }
            off += send_bytes[q];
        }
    } else if (send_bytes[ctx->rank] && r == ncclSuccess) {
        r = ncclSend(d_send, send_bytes[ctx->rank], ncclUint8, root, ctx->comm, st);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail(ctx, RSG_ERR_HIP, "rccl gather: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    return RSG_OK;
}

}  // namespace rsgh

namespace {

struct Events {  // one per batch, destroyed on every exit
    std::vector<hipEvent_t> ev;
    ~Events() {
        for (hipEvent_t e : ev)
            if (e) hipEventDestroy(e);
    }
};

// Shared driver of the two modes: kernel(b) on ctx->stream, then `move(b, sb,
// stream)`.  With more than one batch the moves run on ctx->side[0] behind an
// event of kernel(b), so batch b moves while batch b + 1 hashes; one batch has
// nothing to overlap and moves on ctx->stream right behind its kernel, and
// moves = false (the root of a one-rank gather: its kernels write the records
// where they land) runs the kernels alone -- no events, no second stream.
// Waits for the streams it used on every exit (nothing outlives the call).
// out(b, sb): where batch b's records are written.
template <class Out, class Move>
rsg_status pipeline(rsg_ctx *ctx, const rsg_shard_batch *batches, uint64_t nbatch, const void *d_arena, int32_t seed,
                    Out out, Move move, bool moves) {
    const bool side = moves && nbatch > 1;
    struct Drain {  // error exits: drain whatever was queued
        rsg_ctx *c;
        bool armed = true;
        ~Drain() {
            if (!armed) return;
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamSynchronize(c->side[0]);
        }
    } drain{ctx};
    Events evs;
    evs.ev.assign(side ? nbatch : 0, nullptr);
    for (uint64_t b = 0; b < nbatch; b++) {
        const rsg_shard_batch &sb = batches[b];
        if (sb.plan) {
            if (sb.plan->ctx != ctx) return fail(ctx, RSG_ERR_INVALID, "batch %llu: plan of another context",
                                                 (unsigned long long)b);
            const rsg_status s = launch_plan(ctx, sb.plan->host, sb.plan->d_files, sb.plan->d_wg, d_arena, seed,
                                             out(b, sb), sb.plan->d_scratch, ctx->stream);
            if (s != RSG_OK) return s;
        }
        if (!moves) continue;
        hipStream_t ms = ctx->stream;
        if (side) {
            RSG_HIP(ctx, hipEventCreateWithFlags(&evs.ev[b], hipEventDisableTiming));
            RSG_HIP(ctx, hipEventRecord(evs.ev[b], ctx->stream));
            RSG_HIP(ctx, hipStreamWaitEvent(ctx->side[0], evs.ev[b], 0));
            ms = ctx->side[0];
        }
        const rsg_status s = move(b, sb, ms);
        if (s != RSG_OK) return s;
    }
    RSG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (side) RSG_HIP(ctx, hipStreamSynchronize(ctx->side[0]));
    drain.armed = false;
    return RSG_OK;
}

uint64_t plan_records(const rsg_shard_batch &sb) { return sb.plan ? sb.plan->host.total_blocks : 0; }

}  // namespace

extern "C" {

rsg_status rsg_comm_unique_id(uint8_t id[128]) {
    if (!id) return fail(nullptr, RSG_ERR_INVALID, "id is NULL");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(nullptr, RSG_ERR_HIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    memcpy(id, u.internal, 128);
    return RSG_OK;
}

rsg_status rsg_comm_init(rsg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(ctx, RSG_ERR_INVALID, "bad rank/nranks");
    if (ctx->comm) {
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    ncclUniqueId u;
    memcpy(u.internal, id, 128);
    const ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) return fail(ctx, RSG_ERR_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return RSG_OK;
}

rsg_status rsg_gather_bytes(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv, int32_t root,
                            void *stream) {
    return rsg_gatherv_bytes(ctx, d_send, send_bytes, d_recv, nullptr, root, stream);
}

rsg_status rsg_gatherv_bytes(rsg_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                             const uint64_t *recv_offsets, int32_t root, void *stream) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (!ctx->comm) return fail(ctx, RSG_ERR_INVALID, "rsg_comm_init not called");
    if (!send_bytes || root < 0 || root >= ctx->nranks) return fail(ctx, RSG_ERR_INVALID, "bad gather arguments");
    return gatherv(ctx, d_send, send_bytes, d_recv, recv_offsets, root, stream ? (hipStream_t)stream : ctx->stream,
                   false);
}

rsg_status rsg_block_sums_gather(rsg_ctx *ctx, const rsg_shard_batch *batches, uint64_t nbatch, const void *d_arena,
                                 int32_t seed, void *d_records, void *d_recv, int32_t root) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if (!ctx->comm) return fail(ctx, RSG_ERR_INVALID, "rsg_comm_init not called");
    if ((nbatch && !batches) || root < 0 || root >= ctx->nranks) return fail(ctx, RSG_ERR_INVALID, "bad arguments");
    for (uint64_t b = 0; b < nbatch; b++) {
        if (!batches[b].send_bytes || !batches[b].recv_offsets)
            return fail(ctx, RSG_ERR_INVALID, "batch %llu: send_bytes / recv_offsets missing", (unsigned long long)b);
        if (batches[b].send_bytes[ctx->rank] != plan_records(batches[b]) * rsg::kRecordBytes)
            return fail(ctx, RSG_ERR_INVALID, "batch %llu: send_bytes[%d] = %llu, the plan has %llu records",
                        (unsigned long long)b, ctx->rank, (unsigned long long)batches[b].send_bytes[ctx->rank],
                        (unsigned long long)plan_records(batches[b]));
    }
    if (ctx->rank == root && !d_recv) return fail(ctx, RSG_ERR_INVALID, "root needs d_recv");
    // the root's kernels write its own records straight to their landing
    // offsets in d_recv: no self copy (at N = 1 nothing moves at all)
    const bool is_root = ctx->rank == root;
    auto out = [&](uint64_t, const rsg_shard_batch &sb) -> uint8_t * {
        return is_root ? (uint8_t *)d_recv + sb.recv_offsets[ctx->rank]
                    : (uint8_t *)d_records + sb.record_offset * rsg::kRecordBytes;
    };
    return pipeline(
        ctx, batches, nbatch, d_arena, seed, out,
        [&](uint64_t, const rsg_shard_batch &sb, hipStream_t st) {
            return gatherv(ctx, (const uint8_t *)d_records + sb.record_offset * rsg::kRecordBytes, sb.send_bytes,
                           d_recv, sb.recv_offsets, root, st, true);
        },
        ctx->nranks > 1);
}

rsg_status rsg_block_sums_d2h(rsg_ctx *ctx, const rsg_shard_batch *batches, uint64_t nbatch, const void *d_arena,
                              int32_t seed, void *d_records, uint8_t *h_records) {
    if (!ctx) return fail(nullptr, RSG_ERR_INVALID, "NULL context");
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    RSG_HIP(ctx, hipSetDevice(ctx->device));
    if ((nbatch && !batches) || !h_records) return fail(ctx, RSG_ERR_INVALID, "bad arguments");
    auto out = [&](uint64_t, const rsg_shard_batch &sb) -> uint8_t * {
        return (uint8_t *)d_records + sb.record_offset * rsg::kRecordBytes;
    };
    return pipeline(ctx, batches, nbatch, d_arena, seed, out,
                    [&](uint64_t, const rsg_shard_batch &sb, hipStream_t st) -> rsg_status {
                        const uint64_t n = plan_records(sb) * rsg::kRecordBytes;
                        if (n)
                            RSG_HIP(ctx, hipMemcpyAsync(h_records + sb.record_offset * rsg::kRecordBytes,
                                                        (const uint8_t *)d_records + sb.record_offset * rsg::kRecordBytes,
                                                        n, hipMemcpyDeviceToHost, st));
                        return RSG_OK;
                    },
                    true);
}

}  // extern "C"
