"""Test/bench infrastructure: a Python handle on one loopback datanode
(tools/loopback/loopback_datanode.cpp). Several instances act as the replicas of a block."""
from __future__ import annotations

import ctypes
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

    def stop(self) -> None:
        if self.port:
            self.lb.hdfs3_loopback_stop(self.port)
            self.port = 0
