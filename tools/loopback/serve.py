#!/usr/bin/env python3
"""Test/bench infrastructure: the loopback datanode (loopback_datanode.cpp) in a process of its own
(bench.py config 5, round 6). The parent starts it before it touches a GPU and talks to it over
stdin/stdout, one line per command and one reply line each:

  (start)                                   -> "port <n>"
  packet_bytes <n>                          -> "ok"
  add <block> <data_path> <data_off> <len> <crc_path> <crc_off> <bpc>
                                            -> "ok"   (both files mapped read-only: no copy)
  cpu                                       -> "cpu <user+system seconds of this process>"
  quit / EOF                                -> the datanode stops, the process exits

So the datanode's sender threads are neither charged to the client's CPU time nor compete inside the
client's process unseen; the parent reads their CPU time with `cpu`."""
import ctypes
import os
import resource
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main() -> int:
    import numpy as np

    from libhdfs3_amd import _native

    lb = _native.loopback()
    port = ctypes.c_int(0)
    if lb.hdfs3_loopback_start(ctypes.byref(port)) != 0:
        print("error start", flush=True)
        return 1
    print(f"port {port.value}", flush=True)
    keep = []
    try:
        for line in sys.stdin:
            cmd = line.split()
            if not cmd:
                continue
            if cmd[0] == "quit":
                break
            if cmd[0] == "packet_bytes":
                rc = lb.hdfs3_loopback_set_packet_bytes(port.value, int(cmd[1]))
                print("ok" if rc == 0 else f"error {rc}", flush=True)
            elif cmd[0] == "add":
                bid, dpath, doff, n, cpath, coff, bpc = cmd[1:8]
                n, bpc = int(n), int(bpc)
                nw = 4 * ((n + bpc - 1) // bpc)
                data = np.memmap(dpath, dtype=np.uint8, mode="r", offset=int(doff), shape=(n,))
                crc = np.memmap(cpath, dtype=np.uint8, mode="r", offset=int(coff), shape=(nw,))
                keep.append((data, crc))
                rc = lb.hdfs3_loopback_add_block(port.value, int(bid), data.ctypes.data, n, crc.ctypes.data, bpc, 2)
                print("ok" if rc == 0 else f"error {rc}", flush=True)
            elif cmd[0] == "cpu":  # every thread of this process, microsecond resolution
                ru = resource.getrusage(resource.RUSAGE_SELF)
                print(f"cpu {ru.ru_utime + ru.ru_stime:.6f}", flush=True)
            else:
                print(f"error unknown {cmd[0]}", flush=True)
    finally:
        lb.hdfs3_loopback_stop(port.value)
    return 0


if __name__ == "__main__":
    sys.exit(main())
