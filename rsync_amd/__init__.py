"""rsync_amd -- MI355X-native engine for gokrazy/rsync's block-checksum hot path.

The package is a thin host layer over librsg.so (include/rsg.h): HIP kernels
for gfx950 compute the receiver's weak + seeded-MD4 block sums
(internal/receiver/generator.go:325-350), the sender's byte-rolling match
(internal/sender/match.go:21-230) and whole-file MD4 sums of file batches
(rsyncchecksum.go:60-66, match.go:52-53).  Importing it without the built library
raises ImportError; there is no CPU fallback.
"""
from ._lib import FILESUM_PLAIN, FILESUM_SEEDED, RsgError, SumHead  # noqa: F401  (loads librsg.so, fails loudly)
from .engine import (RECORD_BYTES, Conn, DeviceBuffer, Engine, Plan, checksum1, checksum2,  # noqa: F401
                     apply_tokens, decode_sums, default_engine, device_count, encode_sums, encode_tokens,
                     get_int64, mux_deframe, mux_frame, put_int64, reader_checksum, sum_sizes_sqroot)

__all__ = ["Engine", "Plan", "DeviceBuffer", "Conn", "SumHead", "RsgError", "RECORD_BYTES",
           "FILESUM_PLAIN", "FILESUM_SEEDED", "sum_sizes_sqroot", "checksum1", "checksum2",
           "reader_checksum", "encode_tokens", "apply_tokens", "device_count", "default_engine",
           "encode_sums", "decode_sums", "mux_frame", "mux_deframe", "put_int64", "get_int64"]
