"""Pythonic handle over the C-ABI (include/hdfs3_crc.h), for tests and the bench.

Mirrors the batch semantics of the reference loops it replaces:
  verify(..., check_short_tail=False)  RemoteBlockReader::verifyChecksum
                                       (src/client/RemoteBlockReader.cpp:306-326)
  verify(..., check_short_tail=True)   LocalBlockReader::readAndVerify
                                       (src/client/LocalBlockReader.cpp:138-163)
  compute(...)                         OutputStreamImpl::appendInternal + Packet::addChecksum
                                       (src/client/OutputStreamImpl.cpp:298-359, Packet.cpp:73-81)
Every call runs on the GPU; there is no host fallback.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_int64, c_void_p

import numpy as np

from . import _native
from ._native import Hdfs3CrcError, PktDesc, check  # noqa: F401 (Hdfs3CrcError re-exported)


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def device_count() -> int:
    n = c_int(0)
    check("hdfs3_device_count", _native.lib().hdfs3_device_count(byref(n)))
    return n.value


class DeviceBuffer:
    """Raw HBM allocation owned by Python (hdfs3_dev_malloc/free)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = c_void_p()
        check("hdfs3_dev_malloc", _native.lib().hdfs3_dev_malloc(byref(p), max(self.nbytes, 1)))
        self.ptr = p.value

    def free(self) -> None:
        if self.ptr:
            _native.lib().hdfs3_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class CrcContext:
    """One hdfs3_crc_ctx: like one Checksum instance per reader/writer in the reference."""

    def __init__(self, device: int = 0, lib=None):
        """lib: the product library (default) or _native.lab() for the A/B tools."""
        self._lib = lib if lib is not None else _native.lib()
        p = c_void_p()
        self._check("hdfs3_crc_ctx_create", self._lib.hdfs3_crc_ctx_create(device, byref(p)))
        self.ctx = p.value
        self.device = device

    def _check(self, fn: str, rc: int) -> int:
        return check(fn, rc, self._lib)

    def close(self) -> None:
        if self.ctx:
            self._lib.hdfs3_crc_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing ---------------------------------------------------------------
    @property
    def kernel_launches(self) -> int:
        return int(self._lib.hdfs3_crc_ctx_kernel_launches(self.ctx))

    def set_stream(self, hip_stream: int | None) -> None:
        self._check("hdfs3_crc_ctx_set_stream", self._lib.hdfs3_crc_ctx_set_stream(self.ctx, hip_stream))

    def set_checksum_type(self, ctype: int) -> None:
        """2 = CHECKSUM_CRC32C (default), 1 = CHECKSUM_CRC32 (zlib polynomial)."""
        self._check("hdfs3_crc_ctx_set_checksum_type", self._lib.hdfs3_crc_ctx_set_checksum_type(self.ctx, ctype))

    @property
    def checksum_type(self) -> int:
        return int(self._lib.hdfs3_crc_ctx_get_checksum_type(self.ctx))

    def synchronize(self) -> None:
        self._check("hdfs3_crc_ctx_synchronize", self._lib.hdfs3_crc_ctx_synchronize(self.ctx))

    def upload(self, host: np.ndarray, dev: DeviceBuffer | int | None = None, offset: int = 0):
        """Copy host bytes to a DeviceBuffer (bounds-checked) or a raw device address."""
        host = np.ascontiguousarray(host)
        if dev is None:
            dev = DeviceBuffer(host.nbytes)
        if isinstance(dev, DeviceBuffer):
            assert offset + host.nbytes <= dev.nbytes
            base = dev.ptr
        else:
            base = int(dev)
        self._check("hdfs3_memcpy_h2d", self._lib.hdfs3_memcpy_h2d(self.ctx, base + offset, _ptr(host), host.nbytes))
        return dev

    def download(self, dev: DeviceBuffer | int, nbytes: int, offset: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        base = dev.ptr if isinstance(dev, DeviceBuffer) else int(dev)
        self._check("hdfs3_memcpy_d2h", self._lib.hdfs3_memcpy_d2h(self.ctx, _ptr(out), base + offset, nbytes))
        return out

    def memset(self, dev: DeviceBuffer | int, value: int, nbytes: int, offset: int = 0) -> None:
        base = dev.ptr if isinstance(dev, DeviceBuffer) else int(dev)
        self._check("hdfs3_memset_dev", self._lib.hdfs3_memset_dev(self.ctx, base + offset, value, nbytes))

    # -- host-buffer API ----------------------------------------------------------
    def compute(self, data: np.ndarray, bpc: int) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        n = (data.nbytes + bpc - 1) // bpc
        out = np.zeros(4 * n, dtype=np.uint8)
        self._check("hdfs3_crc32c_compute",
              self._lib.hdfs3_crc32c_compute(self.ctx, _ptr(data), data.nbytes, bpc, _ptr(out)))
        return out

    def verify(self, data: np.ndarray, bpc: int, crc_be: np.ndarray, check_short_tail: bool = False) -> int:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        crc_be = np.ascontiguousarray(crc_be, dtype=np.uint8)
        bad = c_int64(-2)
        self._check("hdfs3_crc32c_verify",
              self._lib.hdfs3_crc32c_verify(self.ctx, _ptr(data), data.nbytes, bpc, _ptr(crc_be),
                                            int(check_short_tail), byref(bad)))
        return bad.value

    # -- device-resident API --------------------------------------------------------
    def compute_dev(self, d_data: int, nbytes: int, bpc: int, d_out: int, overlap_previous: bool = False) -> None:
        """overlap_previous: HDFS3_LAUNCH_OVERLAP_PREVIOUS (hdfs3_crc32c_compute_dev_async_ex; the
        caller's guarantee is in include/hdfs3_crc.h)."""
        if overlap_previous:
            self._check("hdfs3_crc32c_compute_dev_async_ex",
                  self._lib.hdfs3_crc32c_compute_dev_async_ex(self.ctx, d_data, nbytes, bpc, d_out, 1))
            return
        self._check("hdfs3_crc32c_compute_dev",
              self._lib.hdfs3_crc32c_compute_dev(self.ctx, d_data, nbytes, bpc, d_out))

    def verify_dev(self, d_data: int, nbytes: int, bpc: int, d_crc: int, check_short_tail: bool = False) -> int:
        bad = c_int64(-2)
        self._check("hdfs3_crc32c_verify_dev",
              self._lib.hdfs3_crc32c_verify_dev(self.ctx, d_data, nbytes, bpc, d_crc,
                                                int(check_short_tail), byref(bad)))
        return bad.value

    def verify_dev_async(self, d_data: int, nbytes: int, bpc: int, d_crc: int, d_result: int,
                         check_short_tail: bool = False, overlap_previous: bool = False) -> None:
        """overlap_previous: HDFS3_LAUNCH_OVERLAP_PREVIOUS (see include/hdfs3_crc.h for the
        caller's guarantee: the previous op on the stream is a verify and this one's inputs
        were ready before it)."""
        if overlap_previous:
            self._check("hdfs3_crc32c_verify_dev_async_ex",
                  self._lib.hdfs3_crc32c_verify_dev_async_ex(self.ctx, d_data, nbytes, bpc, d_crc,
                                                             int(check_short_tail), d_result, 1))
            return
        self._check("hdfs3_crc32c_verify_dev_async",
              self._lib.hdfs3_crc32c_verify_dev_async(self.ctx, d_data, nbytes, bpc, d_crc,
                                                      int(check_short_tail), d_result))

    def decode_result(self, word: int) -> int:
        return int(self._lib.hdfs3_crc_decode_result(word))

    # -- batch of device-resident blocks ------------------------------------------------
    @staticmethod
    def _blocks(blocks) -> ctypes.Array:
        arr = (_native.DevBlock * max(1, len(blocks)))()
        for i, (d, c, n) in enumerate(blocks):
            arr[i].data, arr[i].crc_be, arr[i].len = d, c, n
        return arr

    def verify_blocks_dev(self, blocks, bpc: int, check_short_tail: bool = False):
        """blocks = [(d_data, d_crc, len)] -> first bad (block, chunk) or (-1, -1)."""
        bb, bc = c_int64(-2), c_int64(-2)
        self._check("hdfs3_crc32c_verify_blocks_dev",
              self._lib.hdfs3_crc32c_verify_blocks_dev(self.ctx, self._blocks(blocks), len(blocks), bpc,
                                                       int(check_short_tail), byref(bb), byref(bc)))
        return bb.value, bc.value

    def verify_blocks_dev_async(self, blocks, bpc: int, d_result: int, check_short_tail: bool = False) -> None:
        self._check("hdfs3_crc32c_verify_blocks_dev_async",
              self._lib.hdfs3_crc32c_verify_blocks_dev_async(self.ctx, self._blocks(blocks), len(blocks), bpc,
                                                             int(check_short_tail), d_result))

    def compute_blocks_dev(self, blocks, bpc: int) -> None:
        self._check("hdfs3_crc32c_compute_blocks_dev",
              self._lib.hdfs3_crc32c_compute_blocks_dev(self.ctx, self._blocks(blocks), len(blocks), bpc))

    # -- block checksum (OP_BLOCK_CHECKSUM's "MD5 of CRC32") ----------------------------
    def block_checksum_dev(self, d_data: int, nbytes: int, bpc: int) -> tuple[bytes, int]:
        """MD5 of the block's BE CRC words (GPU CRCs, host MD5) and crcPerBlock."""
        out = np.zeros(16, dtype=np.uint8)
        n = ctypes.c_uint64(0)
        self._check("hdfs3_block_checksum_dev",
              self._lib.hdfs3_block_checksum_dev(self.ctx, d_data, nbytes, bpc, _ptr(out), byref(n)))
        return out.tobytes(), n.value

    # -- packet-stream API ------------------------------------------------------------
    @staticmethod
    def _descs(pk) -> ctypes.Array:
        if isinstance(pk, ctypes.Array):  # built once by the caller (timed loops)
            return pk
        arr = (PktDesc * len(pk))()
        for i, (data_off, crc_off, data_len) in enumerate(pk):
            arr[i].data_off, arr[i].crc_off, arr[i].data_len, arr[i].reserved = data_off, crc_off, data_len, 0
        return arr

    def verify_packets(self, arena: np.ndarray, pk, bpc: int, check_short_tail: bool = False):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        d = self._descs(pk)
        bp, bc = c_int64(-2), c_int64(-2)
        self._check("hdfs3_crc32c_verify_packets",
              self._lib.hdfs3_crc32c_verify_packets(self.ctx, _ptr(arena), arena.nbytes, d, len(pk), bpc,
                                                    int(check_short_tail), byref(bp), byref(bc)))
        return bp.value, bc.value

    def verify_packets_dev(self, d_arena: int, arena_len: int, pk, bpc: int, check_short_tail: bool = False):
        d = self._descs(pk)
        bp, bc = c_int64(-2), c_int64(-2)
        self._check("hdfs3_crc32c_verify_packets_dev",
              self._lib.hdfs3_crc32c_verify_packets_dev(self.ctx, d_arena, arena_len, d, len(pk), bpc,
                                                        int(check_short_tail), byref(bp), byref(bc)))
        return bp.value, bc.value

    def compute_packets_dev(self, d_arena: int, arena_len: int, pk, bpc: int) -> None:
        d = self._descs(pk)
        self._check("hdfs3_crc32c_compute_packets_dev",
              self._lib.hdfs3_crc32c_compute_packets_dev(self.ctx, d_arena, arena_len, d, len(pk), bpc))

    def verify_packets_dev_async(self, d_arena: int, arena_len: int, pk, bpc: int, d_result: int,
                                 check_short_tail: bool = False) -> None:
        self._check("hdfs3_crc32c_verify_packets_dev_async",
              self._lib.hdfs3_crc32c_verify_packets_dev_async(self.ctx, d_arena, arena_len, self._descs(pk), len(pk),
                                                              bpc, int(check_short_tail), d_result))

    def compute_packets_dev_async(self, d_arena: int, arena_len: int, pk, bpc: int) -> None:
        self._check("hdfs3_crc32c_compute_packets_dev_async",
              self._lib.hdfs3_crc32c_compute_packets_dev_async(self.ctx, d_arena, arena_len, self._descs(pk), len(pk),
                                                               bpc))

    @staticmethod
    def packet_stream(crc_off: int, data_off: int, pitch: int, n: int, data_len: int, last_len: int | None = None):
        """hdfs3_pkt_stream: packet i's words at crc_off + i*pitch, data at data_off + i*pitch."""
        return _native.PktStream(crc_off, data_off, pitch, n, data_len, data_len if last_len is None else last_len)

    def verify_packet_stream_async(self, d_arena: int, arena_len: int, ps, bpc: int, d_result: int,
                                   check_short_tail: bool = False, overlap_previous: bool = False) -> None:
        self._check("hdfs3_crc32c_verify_packet_stream_dev_async",
              self._lib.hdfs3_crc32c_verify_packet_stream_dev_async(self.ctx, d_arena, arena_len, byref(ps), bpc,
                                                                    int(check_short_tail), d_result,
                                                                    1 if overlap_previous else 0))

    def compute_packet_stream_async(self, d_arena: int, arena_len: int, ps, bpc: int) -> None:
        self._check("hdfs3_crc32c_compute_packet_stream_dev_async",
              self._lib.hdfs3_crc32c_compute_packet_stream_dev_async(self.ctx, d_arena, arena_len, byref(ps), bpc))


def block_checksum_crcs(crc_be: bytes | np.ndarray) -> bytes:
    """hdfs3_block_checksum_crcs: MD5 of stored BE CRC words (a .meta file's body)."""
    buf = np.frombuffer(bytes(crc_be), dtype=np.uint8)
    out = np.zeros(16, dtype=np.uint8)
    check("hdfs3_block_checksum_crcs",
          _native.lib().hdfs3_block_checksum_crcs(_ptr(buf) if buf.nbytes else None, buf.nbytes // 4, _ptr(out)))
    return out.tobytes()


def file_checksum_md5md5crc(block_md5s) -> bytes:
    """hdfs3_file_checksum_md5md5crc: MD5 over the blocks' 16-byte digests in order."""
    buf = np.frombuffer(b"".join(block_md5s), dtype=np.uint8)
    out = np.zeros(16, dtype=np.uint8)
    check("hdfs3_file_checksum_md5md5crc",
          _native.lib().hdfs3_file_checksum_md5md5crc(_ptr(buf) if buf.nbytes else None, buf.nbytes // 16,
                                                      _ptr(out)))
    return out.tobytes()


def block_checksum_remote(host: str, port: int, block_id: int, *, pool_id: bytes = b"BP-loopback",
                          generation_stamp: int = 1, num_bytes: int = 0, timeout_ms: int = 60000):
    """hdfs3_block_checksum_remote: (bytes_per_crc, crc_per_block, md5, crc_type) from a datanode."""
    blk = _native.BlockId(pool_id, block_id, generation_stamp, num_bytes)
    info = _native.BlockChecksumInfo()
    check("hdfs3_block_checksum_remote",
          _native.lib().hdfs3_block_checksum_remote(host.encode(), port, byref(blk), timeout_ms, byref(info)))
    return info.bytes_per_crc, info.crc_per_block, bytes(info.md5), info.crc_type


def update_host(state: int, data: bytes | np.ndarray) -> int:
    """Checksum::update on a raw state (sub-chunk streaming shim)."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
    return int(_native.lib().hdfs3_crc32c_update_host(state, _ptr(buf) if buf.nbytes else None, buf.nbytes))


class BlockReader:
    """hdfs3_block_reader (include/hdfs3_client.h): RemoteBlockReader with batched GPU verify."""

    def __init__(self, host: str, port: int, block_id: int, start: int, length: int, *, device: int = 0,
                 verify: bool = True, batch_packets: int = 64, timeout_ms: int = 60000,
                 pool_id: bytes = b"BP-loopback", generation_stamp: int = 1, num_bytes: int = 0):
        self._lib = _native.lib()
        blk = _native.BlockId(pool_id, block_id, generation_stamp, num_bytes)
        opts = _native.ReaderOpts(device, int(verify), batch_packets, timeout_ms)
        p = c_void_p()
        check("hdfs3_block_reader_open",
              self._lib.hdfs3_block_reader_open(host.encode(), port, byref(blk), start, length, b"libhdfs3_amd",
                                                byref(opts), byref(p)))
        self.r = p.value

    def read_into(self, out: np.ndarray, offset: int = 0, n: int | None = None) -> int:
        """RemoteBlockReader::read into out[offset:offset+n]; returns bytes (0 = end of range)."""
        n = out.nbytes - offset if n is None else n
        got = self._lib.hdfs3_block_reader_read(self.r, out.ctypes.data + offset, min(n, 0x7FFFFFFF))
        if got < 0:
            check("hdfs3_block_reader_read", got)
        return got

    def read_all(self, length: int, chunk: int = 1 << 20) -> np.ndarray:
        out = np.empty(length, dtype=np.uint8)
        pos = 0
        while pos < length:
            got = self.read_into(out, pos, min(chunk, length - pos))
            if got == 0:
                break
            pos += got
        return out[:pos]

    def stats(self):
        from ctypes import c_uint32, c_uint64
        bpc, pk, b = c_uint32(), c_uint64(), c_uint64()
        check("hdfs3_block_reader_stats", self._lib.hdfs3_block_reader_stats(self.r, byref(bpc), byref(pk), byref(b)))
        return {"bytes_per_checksum": bpc.value, "packets": pk.value, "gpu_batches": b.value}

    def close(self):
        if self.r:
            self._lib.hdfs3_block_reader_close(self.r)
            self.r = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HdfsIOError(OSError):
    """hdfs.h-style failure (-1 + errno) from an hdfs3_input_* call."""


def _located_blocks(blocks, pool_id: bytes, generation_stamp: int):
    """[(block_id, num_bytes, [(host, port), ...])] -> (LocatedBlock array, objects to keep alive)"""
    arr = (_native.LocatedBlock * len(blocks))()
    keep = [arr]
    off = 0
    for i, (bid, nbytes, reps) in enumerate(blocks):
        dn = (_native.Datanode * max(1, len(reps)))()
        for k, (host, port) in enumerate(reps):
            h = host.encode() if isinstance(host, str) else host
            keep.append(h)
            dn[k].host, dn[k].port = h, port
        keep.append(dn)
        arr[i].block = _native.BlockId(pool_id, bid, generation_stamp, nbytes)
        arr[i].offset = off
        arr[i].replicas = dn
        arr[i].n_replicas = len(reps)
        off += nbytes
    return arr, keep


class Pipeline:
    """hdfs3_pipeline (include/hdfs3_client.h): PipelineImpl for a file's blocks.
    `blocks` = [(block_id, [(host, port), ...])]: what addBlock would return for each block,
    pipeline nodes in order. append=(last_block_bytes, new_generation_stamp): blocks[0] is the
    file's last block, appended to (hdfs3_pipeline_open_append, PIPELINE_SETUP_APPEND)."""

    def __init__(self, blocks, *, bytes_per_checksum: int = 512, timeout_ms: int = 60000, max_unacked: int = 1024,
                 pool_id: bytes = b"BP-loopback", generation_stamp: int = 1, client_name: bytes = b"libhdfs3_amd",
                 append: tuple[int, int] | None = None):
        self._lib = _native.lib()
        self.n_blocks = len(blocks)
        arr, self._keep = _located_blocks([(bid, 0, nodes) for bid, nodes in blocks], pool_id, generation_stamp)
        opts = _native.PipelineOpts(timeout_ms, max_unacked, 0)
        p = c_void_p()
        if append is None:
            check("hdfs3_pipeline_open", self._lib.hdfs3_pipeline_open(arr, len(blocks), client_name,
                                                                       bytes_per_checksum, byref(opts), byref(p)))
        else:
            arr[0].block.num_bytes = append[0]
            check("hdfs3_pipeline_open_append",
                  self._lib.hdfs3_pipeline_open_append(arr, len(blocks), append[1], client_name, bytes_per_checksum,
                                                       byref(opts), byref(p)))
        self.p = p.value

    def generation_stamp(self, block: int) -> int:
        from ctypes import c_uint64
        gs = c_uint64()
        check("hdfs3_pipeline_generation_stamp", self._lib.hdfs3_pipeline_generation_stamp(self.p, block, byref(gs)))
        return gs.value

    @property
    def error(self) -> str:
        return self._lib.hdfs3_pipeline_error(self.p).decode(errors="replace")

    def stats(self):
        from ctypes import c_int64, c_uint64
        acked = (c_int64 * self.n_blocks)()
        pk, ak = c_uint64(), c_uint64()
        check("hdfs3_pipeline_stats", self._lib.hdfs3_pipeline_stats(self.p, acked, self.n_blocks, byref(pk), byref(ak)))
        return {"block_bytes_acked": list(acked), "packets": pk.value, "acks": ak.value}

    def close(self) -> int:
        rc = 0
        if self.p:
            p, self.p = self.p, None
            rc = self._lib.hdfs3_pipeline_close(p)
        return rc

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class InputStream:
    """hdfs3_input_stream (include/hdfs3_client.h): hdfsRead/hdfsPread/hdfsSeek/hdfsTell over
    located blocks with replica failover. `blocks` = [(block_id, num_bytes, [(host, port), ...])]
    in file order."""

    def __init__(self, blocks, *, device: int = 0, verify: bool = True, batch_packets: int = 64,
                 timeout_ms: int = 60000, pool_id: bytes = b"BP-loopback", generation_stamp: int = 1, lib=None):
        """lib: the library to run on (default the product library; tests pass _native.lab() to
        reach its fault-injection hooks)."""
        self._lib = lib or _native.lib()
        arr, self._keep = _located_blocks(blocks, pool_id, generation_stamp)
        opts = _native.ReaderOpts(device, int(verify), batch_packets, timeout_ms)
        p = c_void_p()
        check("hdfs3_input_open", self._lib.hdfs3_input_open(arr, len(blocks), b"libhdfs3_amd", byref(opts), byref(p)))
        self.s = p.value

    def _posix(self, fn: str, rc: int) -> int:
        if rc < 0:
            err = ctypes.get_errno()
            raise HdfsIOError(err, f"{fn}: {self._lib.hdfs3_crc_last_error().decode(errors='replace')}")
        return rc

    def read_into(self, out: np.ndarray, offset: int = 0, n: int | None = None) -> int:
        n = out.nbytes - offset if n is None else n
        return self._posix("hdfsRead", self._lib.hdfs3_input_read(self.s, out.ctypes.data + offset, n))

    def pread_into(self, pos: int, out: np.ndarray, offset: int = 0, n: int | None = None) -> int:
        n = out.nbytes - offset if n is None else n
        return self._posix("hdfsPread", self._lib.hdfs3_input_pread(self.s, pos, out.ctypes.data + offset, n))

    def read_fully(self, length: int, chunk: int = 4 << 20) -> np.ndarray:
        out = np.empty(length, dtype=np.uint8)
        pos = 0
        while pos < length:
            got = self.read_into(out, pos, min(chunk, length - pos))
            if got == 0:
                break
            pos += got
        return out[:pos]

    def seek(self, pos: int) -> None:
        self._posix("hdfsSeek", self._lib.hdfs3_input_seek(self.s, pos))

    def tell(self) -> int:
        return self._posix("hdfsTell", self._lib.hdfs3_input_tell(self.s))

    def available(self) -> int:
        return self._posix("hdfsAvailable", self._lib.hdfs3_input_available(self.s))

    @property
    def length(self) -> int:
        return int(self._lib.hdfs3_input_length(self.s))

    def stats(self):
        from ctypes import c_uint64
        f, o, a, lf = c_uint64(), c_uint64(), c_uint64(), c_uint64()
        check("hdfs3_input_stats", self._lib.hdfs3_input_stats(self.s, byref(f), byref(o)))
        check("hdfs3_input_readahead_stats", self._lib.hdfs3_input_readahead_stats(self.s, byref(a), byref(lf)))
        return {"failovers": f.value, "readers_opened": o.value, "prefetch_readers_opened": a.value,
                "prefetch_local_faults": lf.value}

    def set_readahead(self, blocks: int, max_bytes_per_block: int = 0) -> None:
        """hdfs3_input_set_readahead: blocks i+1 .. i+blocks read by background threads while
        block i is consumed (0 turns it off)."""
        check("hdfs3_input_set_readahead", self._lib.hdfs3_input_set_readahead(self.s, blocks, max_bytes_per_block))

    def close(self):
        if self.s:
            self._lib.hdfs3_input_close(self.s)
            self.s = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OutputStream:
    """hdfs3_output_stream (include/hdfs3_client.h): hdfsWrite/hdfsFlush/hdfsSync/hdfsCloseFile
    with GPU compute-on-write. `sink(packet: bytes, info: dict) -> int` receives every wire
    packet in seqno order (PipelineImpl::send); by default packets are collected in .packets."""

    def __init__(self, *, device: int = 0, bytes_per_checksum: int = 512, packet_size: int = 65536,
                 block_size: int = 64 << 20, batch_packets: int = 64, sink=None, raw_sink=None, raw_user=None,
                 pipeline: "Pipeline | None" = None, append: tuple[int, int] | None = None):
        """pipeline: write to datanodes through hdfs3_output_open_pipeline (flush/sync wait
        for every node's ack) instead of a sink. append = (file_length, last_block_bytes): open
        for append (hdfs3_output_open_append; last_block_bytes -1 = no partial last block)."""
        self._lib = _native.lib()
        self.pipeline = pipeline
        ap = None if append is None else _native.AppendInfo(append[0], append[1])
        if pipeline is not None:
            opts = _native.WriterOpts(device, bytes_per_checksum, packet_size, block_size, batch_packets)
            p = c_void_p()
            check("hdfs3_output_open_pipeline_append",
                  self._lib.hdfs3_output_open_pipeline_append(byref(opts), byref(ap) if ap is not None else None,
                                                              pipeline.p, byref(p)))
            self.s = p.value
            return
        self.packets: list[tuple[bytes, dict]] = []
        user_sink = sink

        def _sink(_user, pkt, n, info):
            i = info.contents
            d = {"seqno": i.seqno, "offset_in_block": i.offset_in_block, "block_index": i.block_index,
                 "data_len": i.data_len, "num_chunks": i.num_chunks, "last": bool(i.last_packet_in_block)}
            b = ctypes.string_at(pkt, n)
            if user_sink is not None:
                return int(user_sink(b, d))
            self.packets.append((b, d))
            return 0

        # a C sink (raw_sink: ctypes function pointer, raw_user: void*) skips the Python callback
        self._cb = _native.PACKET_SINK(_sink) if raw_sink is None else ctypes.cast(raw_sink, _native.PACKET_SINK)
        opts = _native.WriterOpts(device, bytes_per_checksum, packet_size, block_size, batch_packets)
        p = c_void_p()
        check("hdfs3_output_open_append",
              self._lib.hdfs3_output_open_append(byref(opts), byref(ap) if ap is not None else None, self._cb,
                                                 raw_user, byref(p)))
        self.s = p.value

    def _posix(self, fn: str, rc: int) -> int:
        if rc < 0:
            raise HdfsIOError(ctypes.get_errno(), f"{fn}: {self._lib.hdfs3_crc_last_error().decode(errors='replace')}")
        return rc

    def write(self, data) -> int:
        buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
        return self._posix("hdfsWrite", self._lib.hdfs3_output_write(self.s, buf.ctypes.data, buf.nbytes))

    def flush(self) -> None:
        self._posix("hdfsFlush", self._lib.hdfs3_output_flush(self.s))

    def sync(self) -> None:
        self._posix("hdfsSync", self._lib.hdfs3_output_sync(self.s))

    def tell(self) -> int:
        return self._posix("hdfsTell", self._lib.hdfs3_output_tell(self.s))

    def stats(self):
        from ctypes import c_uint64
        pk, b = c_uint64(), c_uint64()
        check("hdfs3_output_stats", self._lib.hdfs3_output_stats(self.s, byref(pk), byref(b)))
        return {"packets": pk.value, "gpu_batches": b.value}

    def close(self) -> None:
        if self.s:
            s, self.s = self.s, None
            self._posix("hdfsCloseFile", self._lib.hdfs3_output_close(s))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if self.s:
            self.close()

    def __del__(self):
        try:
            if self.s:
                self._lib.hdfs3_output_close(self.s)
        except Exception:
            pass


class LocalBlockReader:
    """hdfs3_local_reader (include/hdfs3_client.h): short-circuit read of a block file and
    its .meta file with GPU verification of every chunk."""

    def __init__(self, data_path: str, meta_path: str, *, num_bytes: int = 0, offset: int = 0, device: int = 0,
                 verify: bool = True, buffer_size: int = 1 << 20, window_buffers: int = 4,
                 crc32_as_zlib: bool = False):
        """crc32_as_zlib: HDFS3_LOCAL_CRC32_AS_ZLIB (verify CHECKSUM_CRC32 meta with the zlib
        polynomial; the default is the reference's CRC32C)."""
        self._lib = _native.lib()
        opts = _native.LocalOpts(device, int(verify), buffer_size, window_buffers, 1 if crc32_as_zlib else 0)
        p = c_void_p()
        check("hdfs3_local_reader_open",
              self._lib.hdfs3_local_reader_open(str(data_path).encode(), str(meta_path).encode(), num_bytes, offset,
                                                byref(opts), byref(p)))
        self.r = p.value

    def read_into(self, out: np.ndarray, offset: int = 0, n: int | None = None) -> int:
        n = out.nbytes - offset if n is None else n
        got = self._lib.hdfs3_local_reader_read(self.r, out.ctypes.data + offset, min(n, 0x7FFFFFFF))
        return check("hdfs3_local_reader_read", got)

    def read_all(self, length: int, chunk: int = 4 << 20) -> np.ndarray:
        out = np.empty(length, dtype=np.uint8)
        pos = 0
        while pos < length:
            got = self.read_into(out, pos, min(chunk, length - pos))
            if got == 0:
                break
            pos += got
        return out[:pos]

    def stats(self):
        from ctypes import c_uint32, c_uint64
        bpc, t, b = c_uint32(), c_int(), c_uint64()
        check("hdfs3_local_reader_stats", self._lib.hdfs3_local_reader_stats(self.r, byref(bpc), byref(t), byref(b)))
        return {"bytes_per_checksum": bpc.value, "checksum_type": t.value, "gpu_batches": b.value,
                "mapped_windows": int(self._lib.hdfs3_local_reader_mapped_windows(self.r))}

    def close(self):
        if self.r:
            self._lib.hdfs3_local_reader_close(self.r)
            self.r = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
