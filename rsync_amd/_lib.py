"""ctypes binding of librsg.so (include/rsg.h).

Importing this module loads the in-tree HIP library and fails loudly if it is
missing: the package has no CPU fallback for any checksum work.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RSG_LIB_PATH: another in-tree build of the same ABI (same-box A/B of kernel
# revisions, tools/); default the package's own librsg.so
LIB_PATH = os.environ.get("RSG_LIB_PATH") or os.path.join(HERE, "librsg.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "(make -C rsync_amd/csrc). rsync_amd has no CPU fallback.")

lib = ctypes.CDLL(LIB_PATH)

RECORD_BYTES = 20
FILESUM_PLAIN = 0   # MD4(file), rsyncchecksum.go:60-66
FILESUM_SEEDED = 1  # MD4(int32_LE(seed) || file), match.go:52-53
CHUNK_SIZE = 256 * 1024
ABI_VERSION = 5

OK = 0
ERR_INVALID = -1
ERR_NOMEM = -2
ERR_HIP = -3
ERR_NODEV = -4
ERR_TRUNCATED = -5
ERR_CORRUPT = -6
ERR_IO = -7
GEN_IDX = 1        # rsg_generate_files_fd flags
GEN_TERMINATE = 2
GEN_MUX = 4


class SumHead(ctypes.Structure):
    """rsync.SumHead (types.go:19-36), wire field order (types.go:79-86)."""
    _fields_ = [("count", ctypes.c_int32), ("block_len", ctypes.c_int32),
                ("s2len", ctypes.c_int32), ("rem", ctypes.c_int32)]

    def astuple(self):
        return (self.count, self.block_len, self.s2len, self.rem)

    def __repr__(self):
        return f"SumHead(count={self.count}, block_len={self.block_len}, s2len={self.s2len}, rem={self.rem})"


class File(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("offset", ctypes.c_uint64), ("len", ctypes.c_uint64),
                ("block_len", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Match(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("index", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class SearchJob(ctypes.Structure):
    """rsg_search_job: one file of rsg_hash_search_batch_* (n_matches, status out)."""
    _fields_ = [("src", ctypes.c_void_p), ("src_len", ctypes.c_uint64), ("head", SumHead),
                ("sum1", ctypes.c_void_p), ("sum2", ctypes.c_void_p), ("targets", ctypes.c_void_p),
                ("matches", ctypes.POINTER(Match)), ("match_cap", ctypes.c_uint64),
                ("n_matches", ctypes.c_uint64), ("status", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class FdSearchJob(ctypes.Structure):
    """rsg_fd_search_job: one source file of rsg_hash_search_fd_batch (n_matches, file_sum, status out)."""
    _fields_ = [("fd", ctypes.c_int32), ("reserved", ctypes.c_int32), ("offset", ctypes.c_int64),
                ("src_len", ctypes.c_uint64), ("head", SumHead),
                ("sum1", ctypes.c_void_p), ("sum2", ctypes.c_void_p), ("targets", ctypes.c_void_p),
                ("matches", ctypes.POINTER(Match)), ("match_cap", ctypes.c_uint64),
                ("n_matches", ctypes.c_uint64), ("file_sum", ctypes.c_void_p),
                ("status", ctypes.c_int32), ("reserved2", ctypes.c_int32)]


class FdFile(ctypes.Structure):
    """rsg_fd_file: one basis file of rsg_generate_files_fd."""
    _fields_ = [("fd", ctypes.c_int32), ("idx", ctypes.c_int32), ("offset", ctypes.c_int64),
                ("len", ctypes.c_uint64), ("block_len", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class RecvJob(ctypes.Structure):
    """rsg_recv_job: one file of rsg_receive_data_batch (out_len, consumed, status out)."""
    _fields_ = [("tokens", ctypes.c_void_p), ("tokens_len", ctypes.c_uint64), ("head", SumHead),
                ("basis", ctypes.c_void_p), ("basis_len", ctypes.c_uint64), ("out", ctypes.c_void_p),
                ("out_cap", ctypes.c_uint64), ("out_len", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
                ("status", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class ShardBatch(ctypes.Structure):
    """rsg_shard_batch: one batch of a rank's pipelined sharded generator step."""
    _fields_ = [("plan", ctypes.c_void_p), ("record_offset", ctypes.c_uint64),
                ("send_bytes", ctypes.POINTER(ctypes.c_uint64)), ("recv_offsets", ctypes.POINTER(ctypes.c_uint64))]


class Piece(ctypes.Structure):
    """rsg_piece: blocks [b0, b1) of a file in rank `rank`'s batch `batch` (rsg_shard_plan)."""
    _fields_ = [("file", ctypes.c_uint64), ("b0", ctypes.c_uint64), ("b1", ctypes.c_uint64),
                ("offset", ctypes.c_uint64), ("length", ctypes.c_uint64), ("record", ctypes.c_uint64),
                ("block_len", ctypes.c_int32), ("rank", ctypes.c_int32), ("batch", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class ShardRank(ctypes.Structure):
    """rsg_shard_rank: one context's side of rsg_block_sums_{gather,d2h}_multi."""
    _fields_ = [("ctx", ctypes.c_void_p), ("d_arena", ctypes.c_void_p), ("d_records", ctypes.c_void_p),
                ("batches", ctypes.POINTER(ShardBatch)), ("nbatch", ctypes.c_uint64),
                ("rank_record_offset", ctypes.c_uint64)]


# rsg_write_fn: int32 (*)(void *user, const uint8_t *data, uint64_t len)
WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int32
_st = ctypes.c_int32

_PROTOS = {
    "rsg_abi_version": (ctypes.c_int32, []),
    "rsg_device_count": (ctypes.c_int32, []),
    "rsg_sum_head_for": (_st, [ctypes.c_int64, _i32, ctypes.POINTER(SumHead)]),
    "rsg_ctx_create": (_st, [_i32, ctypes.POINTER(_vp)]),
    "rsg_ctx_destroy": (None, [_vp]),
    "rsg_last_error": (ctypes.c_char_p, [_vp]),
    "rsg_alloc_pinned": (_st, [_vp, _u64, ctypes.POINTER(_vp)]),
    "rsg_free_pinned": (_st, [_vp, _vp]),
    "rsg_alloc_device": (_st, [_vp, _u64, ctypes.POINTER(_vp)]),
    "rsg_free_device": (_st, [_vp, _vp]),
    "rsg_memcpy_h2d": (_st, [_vp, _vp, _vp, _u64]),
    "rsg_memcpy_d2h": (_st, [_vp, _vp, _vp, _u64]),
    "rsg_memcpy_d2d": (_st, [_vp, _vp, _vp, _u64]),
    "rsg_synchronize": (_st, [_vp, _vp]),
    "rsg_fill_splitmix64": (_st, [_vp, _vp, _u64, _u64, _vp]),
    "rsg_plan_block_sums": (_st, [ctypes.POINTER(File), _u64, ctypes.POINTER(SumHead),
                                  ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "rsg_plan_create": (_st, [_vp, ctypes.POINTER(File), _u64, _u64, ctypes.POINTER(_vp)]),
    "rsg_plan_destroy": (None, [_vp]),
    "rsg_plan_total_records": (_u64, [_vp]),
    "rsg_block_sums_planned": (_st, [_vp, _vp, _vp, _i32, _vp, _vp]),
    "rsg_set_block_sums_kernel": (_st, [_vp, _i32]),
    "rsg_block_sums_fallbacks": (_st, [_vp, ctypes.POINTER(_u64), _i32]),
    "rsg_block_sums_device": (_st, [_vp, _vp, _u64, ctypes.POINTER(File), _u64, _i32, _vp, _u64]),
    "rsg_block_sums_host": (_st, [_vp, ctypes.POINTER(File), _u64, _i32, _vp, _u64]),
    "rsg_generate_files_fd": (_st, [_vp, ctypes.POINTER(FdFile), _u64, _i32, _i32, WRITE_FN, _vp,
                                    ctypes.POINTER(SumHead), ctypes.POINTER(_u64)]),
    "rsg_hash_search_host": (_st, [_vp, _vp, _u64, ctypes.POINTER(SumHead), _vp, _vp, _vp, _i32,
                                   ctypes.POINTER(Match), _u64, ctypes.POINTER(_u64)]),
    "rsg_hash_search_device": (_st, [_vp, _vp, _u64, ctypes.POINTER(SumHead), _vp, _vp, _vp, _i32,
                                     ctypes.POINTER(Match), _u64, ctypes.POINTER(_u64)]),
    "rsg_hash_search_fd": (_st, [_vp, _i32, ctypes.c_int64, _u64, ctypes.POINTER(SumHead), _vp, _vp, _vp, _i32,
                                 ctypes.POINTER(Match), _u64, ctypes.POINTER(_u64), _vp]),
    "rsg_hash_search_batch_device": (_st, [_vp, ctypes.POINTER(SearchJob), _u64, _i32]),
    "rsg_hash_search_batch_host": (_st, [_vp, ctypes.POINTER(SearchJob), _u64, _i32]),
    "rsg_hash_search_fd_batch": (_st, [_vp, ctypes.POINTER(FdSearchJob), _u64, _i32]),
    "rsg_set_kernel_timing": (_st, [_vp, _i32]),
    "rsg_kernel_times": (_st, [_vp, ctypes.POINTER(ctypes.c_double), _i32]),
    "rsg_encode_tokens": (_st, [_vp, _u64, ctypes.POINTER(SumHead), ctypes.POINTER(Match), _u64,
                                _vp, _u64, ctypes.POINTER(_u64)]),
    "rsg_apply_tokens": (_st, [_vp, _u64, ctypes.POINTER(SumHead), _vp, _u64, _vp, _u64,
                               ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "rsg_receive_data": (_st, [_vp, _vp, _u64, ctypes.POINTER(SumHead), _vp, _u64, _i32, _vp, _u64,
                               ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "rsg_receive_data_batch": (_st, [_vp, ctypes.POINTER(RecvJob), _u64, _i32]),
    "rsg_file_sums_host": (_st, [_vp, ctypes.POINTER(File), _u64, _i32, _i32, _vp]),
    "rsg_file_sums_device": (_st, [_vp, _vp, _u64, ctypes.POINTER(File), _u64, _i32, _i32, _vp]),
    "rsg_comm_unique_id": (_st, [_vp]),
    "rsg_comm_init": (_st, [_vp, _i32, _i32, _vp]),
    "rsg_gather_bytes": (_st, [_vp, _vp, ctypes.POINTER(_u64), _vp, _i32, _vp]),
    "rsg_gatherv_bytes": (_st, [_vp, _vp, ctypes.POINTER(_u64), _vp, ctypes.POINTER(_u64), _i32, _vp]),
    "rsg_block_sums_gather": (_st, [_vp, ctypes.POINTER(ShardBatch), _u64, _vp, _i32, _vp, _vp, _i32]),
    "rsg_block_sums_d2h": (_st, [_vp, ctypes.POINTER(ShardBatch), _u64, _vp, _i32, _vp, _vp]),
    "rsg_shard_plan": (_st, [_vp, _vp, _u64, _i32, _i32, _i32, ctypes.POINTER(Piece), _u64, ctypes.POINTER(_u64),
                             _vp]),
    "rsg_comm_init_all": (_st, [ctypes.POINTER(_vp), _i32]),
    "rsg_block_sums_gather_multi": (_st, [ctypes.POINTER(ShardRank), _i32, _i32, _vp, _i32]),
    "rsg_block_sums_d2h_multi": (_st, [ctypes.POINTER(ShardRank), _i32, _i32, _vp]),
    "rsg_block_sums_host_multi": (_st, [ctypes.POINTER(_vp), _i32, ctypes.POINTER(File), _u64, _i32, _vp, _u64]),
    "rsg_generate_files_fd_multi": (_st, [ctypes.POINTER(_vp), _i32, ctypes.POINTER(FdFile), _u64, _i32, _i32,
                                          WRITE_FN, _vp, ctypes.POINTER(SumHead), ctypes.POINTER(_u64)]),
    "rsg_check_sum_head": (_st, [ctypes.POINTER(SumHead)]),
    "rsg_encode_sums": (_st, [_vp, ctypes.POINTER(SumHead), _u64, _vp, _i32, _vp, _u64, ctypes.POINTER(_u64)]),
    "rsg_decode_sums": (_st, [_vp, _u64, ctypes.POINTER(SumHead), _vp, _vp, _u64, ctypes.POINTER(_u64)]),
    "rsg_mux_frame": (_st, [_vp, _u64, _i32, ctypes.c_uint32, _vp, _u64, ctypes.POINTER(_u64)]),
    "rsg_mux_deframe": (_st, [_vp, _u64, _vp, _u64, ctypes.POINTER(_u64)]),
    "rsg_put_int64": (_st, [ctypes.c_int64, _vp, ctypes.POINTER(_u64)]),
    "rsg_get_int64": (_st, [_vp, _u64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_u64)]),
    # include/rsg_testing.h (test hooks, not part of the drop-in boundary)
    "rsg_testing_walk": (_st, [_vp, _u64, _vp, _u64, ctypes.POINTER(SumHead), ctypes.POINTER(Match), _u64,
                               ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "rsg_testing_md4": (_st, [_vp, _u64, _i32, _i32, _u64, _vp]),
    "rsg_testing_block_sums_choice": (_i32, [_i32, _i32, _i32, _i32, ctypes.c_uint32]),
    "rsg_testing_multi_queue": (_st, [_u64, ctypes.POINTER(_u64)]),
    "rsg_testing_search_option": (_st, [_vp, _i32, _i32]),
}

for _name, (_res, _args) in _PROTOS.items():
    if os.environ.get("RSG_LIB_PATH") and not hasattr(lib, _name):
        continue  # an A/B build of another revision may predate a newer entry point
    _f = getattr(lib, _name)  # AttributeError here = symbol missing from librsg.so
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_PROTOS)


class RsgError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"rsg error {status}: {msg}")
        self.status = status


def check(status: int, ctx=None):
    if status != OK:
        msg = lib.rsg_last_error(ctx)
        raise RsgError(status, msg.decode(errors="replace") if msg else "")
    return status
