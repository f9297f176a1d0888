"""ctypes binding of the C-ABI in include/hdfs3_crc.h (libhdfs3_amd/lib/libhdfs3_crc.so).

This is exactly the binding a non-C caller of the drop-in boundary would write
(INTEGRATION.md shows the same for C++). There is no fallback: if the HIP
library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_int, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libhdfs3_crc.so")
# measurement library (tools/, the A/B tests, bench.py's read ceiling): the same sources built
# with HDFS3_LAB=1 — the kernel-variant knob and the hdfs3x_* hooks live only there
LAB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libhdfs3_crc_lab.so")


class Hdfs3CrcError(RuntimeError):
    """A C-ABI call returned a negative errno code."""

    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed rc={rc} ({os.strerror(-rc) if rc < 0 else rc}): {msg}")
        self.rc = rc


class PktStream(ctypes.Structure):
    """hdfs3_pkt_stream (include/hdfs3_crc.h)."""

    _fields_ = [("crc_off", c_uint64), ("data_off", c_uint64), ("pitch", c_uint64), ("n", c_uint64),
                ("data_len", c_uint32), ("last_len", c_uint32)]


class PktDesc(ctypes.Structure):
    """hdfs3_pkt_desc (include/hdfs3_crc.h)."""

    _fields_ = [("data_off", c_uint64), ("crc_off", c_uint64), ("data_len", c_uint32),
                ("reserved", c_uint32)]


class DevBlock(ctypes.Structure):
    """hdfs3_dev_block (include/hdfs3_crc.h)."""

    _fields_ = [("data", c_void_p), ("crc_be", c_void_p), ("len", c_uint64)]


# name -> (restype, argtypes); every symbol include/hdfs3_crc.h declares.
PUBLIC_API = {
    "hdfs3_crc_abi_version": (c_int, []),
    "hdfs3_crc_last_error": (ctypes.c_char_p, []),
    "hdfs3_crc_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "hdfs3_crc_ctx_acquire": (c_int, [c_int, POINTER(c_void_p)]),
    "hdfs3_crc_ctx_release": (None, [c_void_p]),
    "hdfs3_crc_pool_stats_get": (c_int, [c_void_p]),
    "hdfs3_crc_pool_trim": (c_int, []),
    "hdfs3_device_numa_node": (c_int, [c_int, POINTER(c_int)]),
    "hdfs3_numa_cpus": (c_int, [ctypes.c_char_p, ctypes.c_char_p, POINTER(c_int), c_int]),
    "hdfs3_crc_ctx_destroy": (None, [c_void_p]),
    "hdfs3_crc_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "hdfs3_crc_ctx_get_stream": (c_void_p, [c_void_p]),
    "hdfs3_crc_ctx_synchronize": (c_int, [c_void_p]),
    "hdfs3_crc_ctx_kernel_launches": (c_uint64, [c_void_p]),
    "hdfs3_crc32c_compute": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p]),
    "hdfs3_crc32c_verify": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p, c_int,
                                    POINTER(c_int64)]),
    "hdfs3_crc32c_compute_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p]),
    "hdfs3_crc32c_compute_dev_async_ex": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p, c_uint32]),
    "hdfs3_crc32c_verify_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p, c_int,
                                        POINTER(c_int64)]),
    "hdfs3_crc32c_verify_dev_async": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p,
                                              c_int, c_void_p]),
    "hdfs3_crc32c_verify_dev_async_ex": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p,
                                                 c_int, c_void_p, c_uint32]),
    "hdfs3_crc_decode_result": (c_int64, [c_uint64]),
    "hdfs3_crc32c_verify_packets": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktDesc),
                                            c_size_t, c_uint32, c_int, POINTER(c_int64),
                                            POINTER(c_int64)]),
    "hdfs3_crc32c_verify_packets_dev": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktDesc),
                                                c_size_t, c_uint32, c_int, POINTER(c_int64),
                                                POINTER(c_int64)]),
    "hdfs3_crc32c_compute_packets_dev": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktDesc),
                                                 c_size_t, c_uint32]),
    "hdfs3_crc32c_verify_packets_dev_async": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktDesc), c_size_t,
                                                      c_uint32, c_int, c_void_p]),
    "hdfs3_crc32c_compute_packets_dev_async": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktDesc), c_size_t,
                                                       c_uint32]),
    "hdfs3_crc32c_verify_packet_stream_dev_async": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktStream),
                                                            c_uint32, c_int, c_void_p, c_uint32]),
    "hdfs3_crc32c_compute_packet_stream_dev_async": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PktStream),
                                                             c_uint32]),
    "hdfs3_crc32c_update_host": (c_uint32, [c_uint32, c_void_p, c_size_t]),
    "hdfs3_dev_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "hdfs3_dev_free": (c_int, [c_void_p]),
    "hdfs3_host_malloc_pinned": (c_int, [POINTER(c_void_p), c_size_t]),
    "hdfs3_host_free_pinned": (c_int, [c_void_p]),
    "hdfs3_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "hdfs3_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "hdfs3_memset_dev": (c_int, [c_void_p, c_void_p, c_int, c_size_t]),
    "hdfs3_device_count": (c_int, [POINTER(c_int)]),
    "hdfs3_crc_ctx_set_checksum_type": (c_int, [c_void_p, c_int]),
    "hdfs3_crc32c_verify_blocks_dev": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32, c_int,
                                               POINTER(c_int64), POINTER(c_int64)]),
    "hdfs3_crc32c_verify_blocks_dev_async": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32, c_int,
                                                     c_void_p]),
    "hdfs3_crc32c_compute_blocks_dev": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32]),
    "hdfs3_crc_ctx_get_checksum_type": (c_int, [c_void_p]),
    "hdfs3_block_checksum_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p, POINTER(c_uint64)]),
    "hdfs3_block_checksum_crcs": (c_int, [c_void_p, c_uint64, c_void_p]),
    "hdfs3_file_checksum_md5md5crc": (c_int, [c_void_p, c_size_t, c_void_p]),
    "hdfs3_multi_create": (c_int, [POINTER(c_int), c_int, POINTER(c_void_p)]),
    "hdfs3_multi_destroy": (None, [c_void_p]),
    "hdfs3_multi_device_count": (c_int, [c_void_p]),
    "hdfs3_crc32c_verify_blocks_multi": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32, c_int,
                                                 POINTER(c_int64)]),
    "hdfs3_crc32c_compute_blocks_multi": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32]),
    "hdfs3_crc32c_verify_host_multi": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32, c_int,
                                               POINTER(c_int64)]),
    "hdfs3_crc32c_compute_host_multi": (c_int, [c_void_p, POINTER(DevBlock), c_size_t, c_uint32]),
}

class BlockId(ctypes.Structure):
    """hdfs3_block_id (include/hdfs3_client.h)."""

    _fields_ = [("pool_id", ctypes.c_char_p), ("block_id", c_uint64), ("generation_stamp", c_uint64),
                ("num_bytes", c_uint64)]


class ReaderOpts(ctypes.Structure):
    """hdfs3_reader_opts (include/hdfs3_client.h)."""

    _fields_ = [("device", c_int), ("verify", c_int), ("batch_packets", c_int), ("timeout_ms", c_int)]


class Datanode(ctypes.Structure):
    """hdfs3_datanode (include/hdfs3_client.h)."""

    _fields_ = [("host", ctypes.c_char_p), ("port", c_int)]


class LocatedBlock(ctypes.Structure):
    """hdfs3_located_block (include/hdfs3_client.h)."""

    _fields_ = [("block", BlockId), ("offset", c_int64), ("replicas", POINTER(Datanode)),
                ("n_replicas", c_int)]


class LocalOpts(ctypes.Structure):
    """hdfs3_local_opts (include/hdfs3_client.h)."""

    _fields_ = [("device", c_int), ("verify", c_int), ("buffer_size", ctypes.c_int32), ("window_buffers", c_int),
                ("flags", c_uint32)]


class PacketInfo(ctypes.Structure):
    """hdfs3_packet_info (include/hdfs3_client.h)."""

    _fields_ = [("seqno", c_int64), ("offset_in_block", c_int64), ("block_index", c_int64),
                ("data_len", ctypes.c_int32), ("num_chunks", ctypes.c_int32),
                ("last_packet_in_block", ctypes.c_int32)]


PACKET_SINK = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, POINTER(PacketInfo))


class WriterOpts(ctypes.Structure):
    """hdfs3_writer_opts (include/hdfs3_client.h)."""

    _fields_ = [("device", c_int), ("bytes_per_checksum", c_uint32), ("packet_size", ctypes.c_int32),
                ("block_size", c_int64), ("batch_packets", c_int)]


class PoolStats(ctypes.Structure):
    """hdfs3_crc_pool_stats (include/hdfs3_crc.h)."""

    _fields_ = [("pooled_contexts", c_uint64), ("pinned_bytes", c_uint64), ("device_bytes", c_uint64),
                ("pinned_cap_bytes", c_uint64)]


class AppendInfo(ctypes.Structure):
    """hdfs3_append_info (include/hdfs3_client.h)."""

    _fields_ = [("file_length", c_int64), ("last_block_bytes", c_int64)]


class PipelineOpts(ctypes.Structure):
    """hdfs3_pipeline_opts (include/hdfs3_client.h)."""

    _fields_ = [("timeout_ms", c_int), ("max_unacked", c_int), ("checksum_type", c_int)]


class BlockChecksumInfo(ctypes.Structure):
    """hdfs3_block_checksum_info (include/hdfs3_client.h)."""

    _fields_ = [("bytes_per_crc", c_uint32), ("crc_per_block", c_uint64), ("md5", ctypes.c_uint8 * 16),
                ("crc_type", c_int)]


# every symbol include/hdfs3_client.h declares
CLIENT_API = {
    "hdfs3_block_checksum_remote": (c_int, [ctypes.c_char_p, c_int, POINTER(BlockId), c_int,
                                            POINTER(BlockChecksumInfo)]),
    "hdfs3_block_reader_open": (c_int, [ctypes.c_char_p, c_int, POINTER(BlockId), c_int64, c_int64,
                                        ctypes.c_char_p, POINTER(ReaderOpts), POINTER(c_void_p)]),
    "hdfs3_block_reader_read": (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32]),
    "hdfs3_block_reader_available": (c_int64, [c_void_p]),
    "hdfs3_block_reader_stats": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint64), POINTER(c_uint64)]),
    "hdfs3_reader_phase_ns": (c_int, [POINTER(c_uint64), c_int, c_int]),
    "hdfs3_block_reader_close": (c_int, [c_void_p]),
    "hdfs3_input_open": (c_int, [POINTER(LocatedBlock), c_int, ctypes.c_char_p, POINTER(ReaderOpts),
                                 POINTER(c_void_p)]),
    "hdfs3_input_read": (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32]),
    "hdfs3_input_pread": (ctypes.c_int32, [c_void_p, c_int64, c_void_p, ctypes.c_int32]),
    "hdfs3_input_seek": (c_int, [c_void_p, c_int64]),
    "hdfs3_input_tell": (c_int64, [c_void_p]),
    "hdfs3_input_available": (c_int, [c_void_p]),
    "hdfs3_input_length": (c_int64, [c_void_p]),
    "hdfs3_input_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "hdfs3_input_close": (c_int, [c_void_p]),
    "hdfs3_input_set_readahead": (c_int, [c_void_p, c_int, c_int64]),
    "hdfs3_input_readahead_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "hdfs3_local_reader_open": (c_int, [ctypes.c_char_p, ctypes.c_char_p, c_int64, c_int64, POINTER(LocalOpts),
                                        POINTER(c_void_p)]),
    "hdfs3_local_reader_read": (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32]),
    "hdfs3_local_reader_available": (c_int64, [c_void_p]),
    "hdfs3_local_reader_stats": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_int), POINTER(c_uint64)]),
    "hdfs3_local_reader_mapped_windows": (c_uint64, [c_void_p]),
    "hdfs3_local_reader_close": (c_int, [c_void_p]),
    "hdfs3_output_open": (c_int, [POINTER(WriterOpts), PACKET_SINK, c_void_p, POINTER(c_void_p)]),
    "hdfs3_output_write": (ctypes.c_int32, [c_void_p, c_void_p, ctypes.c_int32]),
    "hdfs3_output_flush": (c_int, [c_void_p]),
    "hdfs3_output_sync": (c_int, [c_void_p]),
    "hdfs3_output_tell": (c_int64, [c_void_p]),
    "hdfs3_output_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "hdfs3_output_close": (c_int, [c_void_p]),
    "hdfs3_pipeline_open": (c_int, [POINTER(LocatedBlock), c_int, ctypes.c_char_p, c_uint32, POINTER(PipelineOpts),
                                    POINTER(c_void_p)]),
    "hdfs3_pipeline_send": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(PacketInfo)]),
    "hdfs3_pipeline_flush": (c_int, [c_void_p]),
    "hdfs3_pipeline_stats": (c_int, [c_void_p, POINTER(c_int64), c_int, POINTER(c_uint64), POINTER(c_uint64)]),
    "hdfs3_pipeline_error": (ctypes.c_char_p, [c_void_p]),
    "hdfs3_pipeline_close": (c_int, [c_void_p]),
    "hdfs3_output_open_pipeline": (c_int, [POINTER(WriterOpts), c_void_p, POINTER(c_void_p)]),
    "hdfs3_output_open_append": (c_int, [POINTER(WriterOpts), POINTER(AppendInfo), PACKET_SINK, c_void_p,
                                         POINTER(c_void_p)]),
    "hdfs3_output_open_pipeline_append": (c_int, [POINTER(WriterOpts), POINTER(AppendInfo), c_void_p,
                                                  POINTER(c_void_p)]),
    "hdfs3_pipeline_open_append": (c_int, [POINTER(LocatedBlock), c_int, c_uint64, ctypes.c_char_p, c_uint32,
                                           POINTER(PipelineOpts), POINTER(c_void_p)]),
    "hdfs3_pipeline_generation_stamp": (c_int, [c_void_p, c_int, POINTER(c_uint64)]),
}

# every symbol include/hdfs3_hdfs.h declares (hdfs.h prototypes + the namenode stand-in)
HDFS_API = {
    "hdfsGetLastError": (ctypes.c_char_p, []),
    "hdfsFileIsOpenForRead": (c_int, [c_void_p]),
    "hdfsFileIsOpenForWrite": (c_int, [c_void_p]),
    "hdfsDisconnect": (c_int, [c_void_p]),
    "hdfsOpenFile": (c_void_p, [c_void_p, ctypes.c_char_p, c_int, c_int, ctypes.c_short, c_int64]),
    "hdfsCloseFile": (c_int, [c_void_p, c_void_p]),
    "hdfsExists": (c_int, [c_void_p, ctypes.c_char_p]),
    "hdfsSeek": (c_int, [c_void_p, c_void_p, c_int64]),
    "hdfsTell": (c_int64, [c_void_p, c_void_p]),
    "hdfsRead": (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_int32]),
    "hdfsPread": (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_int32, c_int64]),
    "hdfsWrite": (ctypes.c_int32, [c_void_p, c_void_p, c_void_p, ctypes.c_int32]),
    "hdfsFlush": (c_int, [c_void_p, c_void_p]),
    "hdfsHFlush": (c_int, [c_void_p, c_void_p]),
    "hdfsSync": (c_int, [c_void_p, c_void_p]),
    "hdfsAvailable": (c_int, [c_void_p, c_void_p]),
    "hdfs3_fs_new": (c_void_p, [ctypes.c_char_p, c_void_p, c_void_p]),
    "hdfs3_fs_add_file": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_int]),
    "hdfs3_fs_set_sink": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_void_p]),
    "hdfs3_fs_set_pipeline": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_int]),
    "hdfs3_fs_set_readahead": (c_int, [c_void_p, c_int, c_int64]),
    "hdfs3_fs_set_append_stamp": (c_int, [c_void_p, ctypes.c_char_p, c_uint64]),
    "hdfs3_fs_set_block_size": (c_int, [c_void_p, ctypes.c_char_p, ctypes.c_int64]),
}

# measurement hooks (libhdfs3_crc_lab.so only; not in any public header)
BENCH_API = {
    "hdfs3x_stream_read": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "hdfs3x_stream_read_ex": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p, c_uint32]),
    "hdfs3x_lane_read": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, c_void_p]),
    "hdfs3x_grid_cap": (c_int, [c_void_p]),
    "hdfs3x_set_variant": (None, [c_int]),
    "hdfs3x_clock_stamps": (c_int, [c_void_p, ctypes.c_uint]),
    "hdfs3x_wave_stamps": (c_int, [c_void_p, ctypes.c_uint]),
    "hdfs3x_block_reader_timing": (c_int, [c_void_p, POINTER(c_uint64)]),
    "hdfs3x_fail_prefetch_arenas": (None, [c_int]),
}


def load(path: str = LIB_PATH, lab: bool = False) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run `make` (or __graft_entry__.build()) first; "
                          "libhdfs3_amd has no CPU fallback")
    lib = ctypes.CDLL(path, use_errno=True)  # the hdfs.h-style calls report through errno
    for table in (PUBLIC_API, CLIENT_API, HDFS_API) + ((BENCH_API,) if lab else ()):
        for name, (res, args) in table.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    return lib


_LIB: ctypes.CDLL | None = None
_LAB: ctypes.CDLL | None = None


def lib() -> ctypes.CDLL:
    """The product library (libhdfs3_crc.so): what every product caller loads."""
    global _LIB
    if _LIB is None:
        _LIB = load()
    return _LIB


def lab() -> ctypes.CDLL:
    """The measurement library (libhdfs3_crc_lab.so): production code plus the A/B variant
    knob (hdfs3x_set_variant) and measurement kernels. A context belongs to the library that
    created it: never pass a lab ctx to lib() calls or the reverse."""
    global _LAB
    if _LAB is None:
        _LAB = load(LAB_PATH, lab=True)
    return _LAB


LOOPBACK_PATH = os.path.join(os.path.dirname(LIB_PATH), "libhdfs3_loopback.so")
_LOOPBACK: ctypes.CDLL | None = None


def loopback() -> ctypes.CDLL:
    """Test/bench infrastructure: the loopback datanode (tools/loopback)."""
    global _LOOPBACK
    if _LOOPBACK is None:
        if not os.path.exists(LOOPBACK_PATH):
            raise ImportError(f"{LOOPBACK_PATH} is missing: run `make`")
        lb = ctypes.CDLL(LOOPBACK_PATH)
        lb.hdfs3_loopback_start.restype = c_int
        lb.hdfs3_loopback_start.argtypes = [POINTER(c_int)]
        lb.hdfs3_loopback_add_block.restype = c_int
        lb.hdfs3_loopback_add_block.argtypes = [c_int, c_uint64, c_void_p, c_uint64, c_void_p, c_uint32, c_int]
        for fn, args, res in [("clear_blocks", [c_int], c_int), ("set_packet_bytes", [c_int, c_int], c_int),
                              ("set_fail_after", [c_int, c_int64], c_int), ("served_bytes", [c_int], c_uint64),
                              ("requests", [c_int], c_uint64), ("last_status", [c_int], c_int),
                              ("stop", [c_int], c_int), ("set_write_fault", [c_int, c_int, c_int64], c_int),
                              ("set_store_written", [c_int, c_int], c_int),
                              ("write_stats", [c_int] + [POINTER(c_uint64)] * 4, c_int),
                              ("get_block", [c_int, c_uint64, POINTER(c_void_p), POINTER(c_uint64), POINTER(c_void_p),
                                             POINTER(c_uint32)], c_int),
                              ("block_gs", [c_int, c_uint64, POINTER(c_uint64)], c_int)]:
            f = getattr(lb, "hdfs3_loopback_" + fn)
            f.argtypes, f.restype = args, res
        _LOOPBACK = lb
    return _LOOPBACK


def check(fn: str, rc: int, library: ctypes.CDLL | None = None) -> int:
    if rc < 0:
        raise Hdfs3CrcError(fn, rc, (library or lib()).hdfs3_crc_last_error().decode(errors="replace"))
    return rc
