#!/usr/bin/env python3
"""Host issue timeline of short timed regions (the driver's K=20 form): after the warmup, K
launches of verify or compute (overlapped or barriered) between two HIP events, with the start of
the region prepared three ways:
  sync   torch.cuda.synchronize(), then the start event and the launches (bench.py until r3v);
  spin   poll an event recorded after the warmup until it completes (the host thread stays on its
         core), then torch.cuda.synchronize() (returns at once), the start event, the launches;
  gate   the stream waits on a host-memory flag (hipStreamWaitValue32) queued before the start
         event; the launches are all queued, then the host opens the gate: no host issue inside the
         timed region at all.
Prints per case the GPU time per launch and the host issue times (perf_counter after each call)."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0)
    ctx.set_stream(st.cuda_stream)
    blocks, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((blocks, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(blocks):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    out = torch.full_like(crc, 0xA5)
    res = torch.zeros(4096, dtype=torch.int64, device=dev)
    dp = [data[b].data_ptr() for b in range(blocks)]
    cp = [crc[b].data_ptr() for b in range(blocks)]
    op = [out[b].data_ptr() for b in range(blocks)]
    rp = res.data_ptr()

    hip = ctypes.CDLL("libamdhip64.so")
    flag_h = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(flag_h), ctypes.c_size_t(64), ctypes.c_uint(0x2)) == 0  # mapped
    flag_d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(flag_d), flag_h, ctypes.c_uint(0)) == 0
    flag = ctypes.cast(flag_h, ctypes.POINTER(ctypes.c_uint32))
    hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint,
                                         ctypes.c_uint32]

    def v_pre(i, ov):
        ctx.verify_dev_async(dp[i % 8], bb, bpc, cp[i % 8], rp + 8 * i, overlap_previous=ov and i > 0)

    def c_pre(i, ov):
        ctx.compute_dev(dp[i % 8], bb, bpc, op[i % 8], overlap_previous=ov and i > 0)

    K = int(os.environ.get("K", "20"))
    for rep in range(5):
        for name, fn in (("verify", v_pre), ("compute", c_pre)):
            for ov in (True, False):
                for mode in ("sync", "spin", "gate"):
                    for i in range(200):
                        fn(i % 4096, ov)
                    done = torch.cuda.Event()
                    done.record(st)
                    if mode == "spin":
                        while not done.query():
                            pass
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    if mode == "gate":
                        flag[0] = 0
                        # wait until *flag >= 1 (hipStreamWaitValueGte = 0)
                        assert hip.hipStreamWaitValue32(ctypes.c_void_p(st.cuda_stream), flag_d, 1, 0, 0xFFFFFFFF) == 0
                    t0 = time.perf_counter()
                    e0.record(st)
                    ts = []
                    for i in range(K):
                        fn(i, ov)
                        ts.append(time.perf_counter() - t0)
                    e1.record(st)
                    if mode == "gate":
                        flag[0] = 1
                    torch.cuda.synchronize()
                    gpu = e0.elapsed_time(e1) * 1e3 / K
                    print(json.dumps({"case": name, "overlap": ov, "mode": mode, "rep": rep, "K": K,
                                      "gpu_us_per_launch": round(gpu, 2),
                                      "issue_us": [round(t * 1e6, 1) for t in ts]}), flush=True)
    assert int(res.abs().sum()) == 0


if __name__ == "__main__":
    main()
