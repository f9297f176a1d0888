"""Test/bench infrastructure: a Python handle on one loopback datanode
(tools/loopback/loopback_datanode.cpp). Several instances act as the replicas of a block."""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np

CHECKSUM_NULL, CHECKSUM_CRC32, CHECKSUM_CRC32C = 0, 1, 2


class LoopbackDatanode:
    def __init__(self, packet_bytes: int | None = None):
        from libhdfs3_amd import _native

        self.lb = _native.loopback()
        port = ctypes.c_int(0)
        rc = self.lb.hdfs3_loopback_start(ctypes.byref(port))
        assert rc == 0, rc
        self.port = port.value
        self._keep = []
        if packet_bytes:
            self.set_packet_bytes(packet_bytes)

    def add_block(self, block_id: int, data: np.ndarray, crc: np.ndarray | None, bpc: int,
                  ctype: int = CHECKSUM_CRC32C) -> None:
        """Serve block_id; data/crc stay referenced (kept alive here)."""
        crc = np.zeros(4, np.uint8) if crc is None else crc
        self._keep.append((data, crc))
        rc = self.lb.hdfs3_loopback_add_block(self.port, block_id, data.ctypes.data, data.nbytes,
                                              crc.ctypes.data, bpc, ctype)
        assert rc == 0, rc

    def set_packet_bytes(self, n: int) -> None:
        assert self.lb.hdfs3_loopback_set_packet_bytes(self.port, n) == 0

    def set_fail_after(self, nbytes: int) -> None:
        assert self.lb.hdfs3_loopback_set_fail_after(self.port, nbytes) == 0

    @property
    def served_bytes(self) -> int:
        return int(self.lb.hdfs3_loopback_served_bytes(self.port))

    @property
    def requests(self) -> int:
        return int(self.lb.hdfs3_loopback_requests(self.port))

    def last_status(self, wait_for: int | None = None, timeout: float = 2.0) -> int:
        deadline = time.time() + timeout
        st = self.lb.hdfs3_loopback_last_status(self.port)
        while wait_for is not None and st != wait_for and time.time() < deadline:
            time.sleep(0.01)
            st = self.lb.hdfs3_loopback_last_status(self.port)
        return st

    # write side (OP_WRITE_BLOCK)
    FAULT_NONE, FAULT_REFUSE_SETUP, FAULT_ACK_ERROR, FAULT_CORRUPT_IN_TRANSIT, FAULT_DROP_AT = range(5)

    def set_write_fault(self, mode: int, seqno: int = -1) -> None:
        assert self.lb.hdfs3_loopback_set_write_fault(self.port, mode, seqno) == 0

    def set_store_written(self, store: bool) -> None:
        assert self.lb.hdfs3_loopback_set_store_written(self.port, int(store)) == 0

    def write_stats(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(4)]
        assert self.lb.hdfs3_loopback_write_stats(self.port, *[ctypes.byref(x) for x in v]) == 0
        return dict(zip(("packets", "bytes", "checksum_errors", "finalized"), (x.value for x in v)))

    def wait_finalized(self, n: int, timeout: float = 10.0) -> int:
        deadline = time.time() + timeout
        while self.write_stats()["finalized"] < n and time.time() < deadline:
            time.sleep(0.005)
        return self.write_stats()["finalized"]

    def get_block(self, block_id: int):
        """(data, crc_be, bpc) of a block this node holds (copies), or None"""
        d, c = ctypes.c_void_p(), ctypes.c_void_p()
        n, bpc = ctypes.c_uint64(), ctypes.c_uint32()
        rc = self.lb.hdfs3_loopback_get_block(self.port, block_id, ctypes.byref(d), ctypes.byref(n), ctypes.byref(c),
                                              ctypes.byref(bpc))
        if rc != 0:
            return None
        nch = (n.value + bpc.value - 1) // bpc.value
        data = np.frombuffer(ctypes.string_at(d, n.value), np.uint8).copy() if n.value else np.zeros(0, np.uint8)
        crc = np.frombuffer(ctypes.string_at(c, 4 * nch), np.uint8).copy() if nch else np.zeros(0, np.uint8)
        return data, crc, bpc.value

    def block_gs(self, block_id: int) -> int | None:
        """the generation stamp a written block was finalized with (0: added to serve)"""
        gs = ctypes.c_uint64()
        rc = self.lb.hdfs3_loopback_block_gs(self.port, block_id, ctypes.byref(gs))
        return None if rc != 0 else gs.value

    def stop(self) -> None:
        if self.port:
            self.lb.hdfs3_loopback_stop(self.port)
            self.port = 0


class ChildDatanode:
    """The loopback datanode in a child process (tools/loopback/serve.py; bench.py config 5, round 6).
    Start it before this process touches a GPU (a plain child: nothing is exec'd from a GPU process).
    Blocks are served from files both processes map (share_blocks: one file in /dev/shm for the data,
    one for the words), and cpu_seconds() is the child's own CPU time, so a pass can charge the
    datanode's sender threads apart from the client's."""

    SERVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools", "loopback", "serve.py")

    def __init__(self, packet_bytes: int | None = None):
        import subprocess
        import sys

        self.p = subprocess.Popen([sys.executable, "-u", self.SERVE], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  text=True, bufsize=1)
        reply = self._reply()
        if not reply.startswith("port "):
            raise OSError(f"loopback child: {reply}")
        self.port = int(reply.split()[1])
        self.pid = self.p.pid
        self._files = []
        if packet_bytes:
            self._cmd(f"packet_bytes {packet_bytes}")

    def _reply(self) -> str:
        line = self.p.stdout.readline()
        if not line:
            raise OSError(f"loopback child exited ({self.p.poll()})")
        return line.strip()

    def _cmd(self, line: str) -> str:
        self.p.stdin.write(line + "\n")
        self.p.stdin.flush()
        reply = self._reply()
        if reply.startswith("error"):
            raise OSError(f"loopback child: {line!r}: {reply}")
        return reply

    def share_blocks(self, data: np.ndarray, crc: np.ndarray, blocks, bpc: int, tag: str = "blk"):
        """Serve blocks = [(block_id, data_offset, length)] of `data` (words at 4 * offset / bpc of
        `crc`). Returns the shared read-only view of the data (the bytes the child serves)."""
        base = f"/dev/shm/hdfs3_{tag}_{os.getpid()}_{len(self._files)}"
        paths = (base + "_data", base + "_crc")
        arrs = []
        for path, a in zip(paths, (data, crc)):
            m = np.memmap(path, dtype=np.uint8, mode="w+", shape=(max(1, a.nbytes),))
            m[:a.nbytes] = a.reshape(-1)
            m.flush()
            arrs.append(m)
        try:
            for bid, off, n in blocks:
                self._cmd(f"add {bid} {paths[0]} {off} {n} {paths[1]} {4 * (off // bpc)} {bpc}")
        finally:
            for path in paths:  # both processes keep their mappings; the names go now
                os.unlink(path)
        self._files.append(arrs)
        return arrs[0][:data.nbytes]

    def cpu_seconds(self) -> float:
        return float(self._cmd("cpu").split()[1])

    def stop(self) -> None:
        if self.p.poll() is None:
            try:
                self.p.stdin.write("quit\n")
                self.p.stdin.flush()
                self.p.wait(timeout=10)
            except Exception:  # noqa: BLE001 - a child that does not quit is killed
                self.p.kill()
                self.p.wait()
        self._files.clear()


def reference_read_block(port: int, block_id: int, nbytes: int, out: np.ndarray, offset: int = 0, *,
                         verify: bool = True, engine: str = "reference") -> int:
    """Test/bench infrastructure (bench.py's config-5 CPU baseline): one block read the way the
    reference's RemoteBlockReader reads it — OP_READ_BLOCK, the BlockOpResponseProto check, then
    every packet received, verified by the CPU engine on this thread and copied to `out`
    (RemoteBlockReader.cpp:112-357, oracle/remote_loop.h), then the ClientReadStatusProto.
    engine: "reference" = oracle/_ref's HWCrc32c (the reference source), "hw" / "pcl" = the
    oracle's restatements. Returns the bytes delivered; raises on a checksum mismatch."""
    import dtp
    from util import HW, PCL, oracle, ref_lib

    conn = dtp.Conn(port)
    try:
        conn.s.settimeout(None)
        conn.s.sendall(dtp.read_block_request(block_id, 0, nbytes, pool=b"BP-loopback"))
        resp = dtp.parse(conn.recv_delimited())
        if resp[1][0] != 0:
            raise OSError(f"datanode refused block {block_id}: status {resp[1][0]}")
        bpc = dtp.parse(dtp.parse(resp[4][0])[1][0])[2][0]
        bad = ctypes.c_int64(-1)
        view = out[offset:offset + nbytes]
        if engine == "reference":
            lib = ref_lib()
            fn = lib.ref_remote_read_block
            fn.restype, fn.argtypes = ctypes.c_int64, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                                       ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
            got = fn(conn.s.fileno(), view.ctypes.data, nbytes, bpc, int(verify), ctypes.byref(bad))
        else:
            fn = oracle().oracle_remote_read_block
            fn.restype, fn.argtypes = ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                                       ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
            got = fn(conn.s.fileno(), {"hw": HW, "pcl": PCL}[engine], view.ctypes.data, nbytes, bpc, int(verify),
                     ctypes.byref(bad))
        if got < 0:
            raise OSError(f"block {block_id}: the reference read loop failed")
        if bad.value >= 0:
            raise OSError(f"ChecksumException: block {block_id} packet {bad.value}")
        conn.send_status(6 if verify else 0)  # CHECKSUM_OK / SUCCESS (RemoteBlockReader.cpp:289-304)
        return got
    finally:
        conn.close()
