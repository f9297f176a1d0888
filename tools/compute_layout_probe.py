#!/usr/bin/env python3
"""Where compute mode loses time on packet streams (docs/DESIGN_HISTORY.md §4.3): 1 GiB of 64 KiB packets at
bpc 512, CRC words written (a) into one contiguous array, (b) into each packet's own 512 B region
of the wire layout. The data layout (contiguous vs 66,048 B pitch) and the word layout are varied
independently through the multi-block API (constant strides -> the wave kernel's pitch mode), so
the two effects separate. The product path writes in-packet words densely into the ctx's
scratch and scatters them with a copy kernel; variant 55 writes them in place (the A/B). All
cases in one process, interleaved rounds, medians."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    bpc, pkt = 512, 65536
    n = (1 << 30) // pkt
    wpp = pkt // bpc * 4  # word bytes per packet
    pitch = pkt + wpp     # wire-dense [words][data]
    arena = torch.randint(0, 256, (n * pitch,), dtype=torch.uint8, device="cuda")
    block = torch.randint(0, 256, (n * pkt,), dtype=torch.uint8, device="cuda")
    words = torch.zeros(n * wpp, dtype=torch.uint8, device="cuda")
    scattered = torch.zeros(n * pitch, dtype=torch.uint8, device="cuda")  # words at the wire pitch, no data
    ps = CrcContext.packet_stream(0, wpp, pitch, n, pkt)
    a0, b0, w0, s0 = arena.data_ptr(), block.data_ptr(), words.data_ptr(), scattered.data_ptr()
    import ctypes
    ps_ref = ctypes.byref(ps)
    # block lists (data, words, len) packed once: the sync blocks API's own host pass over them is
    # in every blocks-API case alike
    descs = {
        "pitch_data/in_packet_words (blocks API)": [(a0 + i * pitch + wpp, a0 + i * pitch, pkt) for i in range(n)],
        "pitch_data/contiguous_words (blocks API)": [(a0 + i * pitch + wpp, w0 + i * wpp, pkt) for i in range(n)],
        "contiguous_data/scattered_words (blocks API)": [(b0 + i * pkt, s0 + i * pitch, pkt) for i in range(n)],
        "contiguous_data/contiguous_words (blocks API)": [(b0 + i * pkt, w0 + i * wpp, pkt) for i in range(n)],
    }
    cases = {
        "contiguous_data/contiguous_words (compute_dev)":
            lambda: _native.check("compute", lib.hdfs3_crc32c_compute_dev(ctx.ctx, b0, n * pkt, bpc, w0)),
        "pitch_data/in_packet_words (packet stream)":
            lambda: lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, a0, arena.numel(), ps_ref, bpc),
    }
    for k, v in descs.items():
        pk = ctx._blocks(v)
        cases[k] = (lambda pk=pk: _native.check("compute_blocks", lib.hdfs3_crc32c_compute_blocks_dev(ctx.ctx, pk, n,
                                                                                                    bpc)))
    dst_view, src_view = arena.view(n, pitch)[:, :wpp], words.view(n, wpp)
    pk_dense = ctx._blocks(descs["pitch_data/contiguous_words (blocks API)"])

    def dense_then_scatter():
        _native.check("compute_blocks", lib.hdfs3_crc32c_compute_blocks_dev(ctx.ctx, pk_dense, n, bpc))
        dst_view.copy_(src_view)  # torch strided copy on the same stream: the words' scatter alone
    cases["pitch_data/contiguous_words + torch scatter into the packets"] = dense_then_scatter
    cases["torch scatter alone (8 MiB -> 16384 x 512 B at the wire pitch)"] = lambda: dst_view.copy_(src_view)

    def in_place_stream():  # A/B variant 55: the words written into the packets by the kernel itself
        lib.hdfs3x_set_variant(55)
        lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, a0, arena.numel(), ps_ref, bpc)
        lib.hdfs3x_set_variant(0)
    cases["pitch_data/in_packet_words (packet stream, in place: variant 55)"] = in_place_stream
    # writer-shaped wire packets (127 chunks = 65,024 B of data, not whole 4 KiB rounds): the
    # segmented kernel, words in each packet vs in one array
    wl = 127 * bpc
    wn = (1 << 30) // wl
    wwords = 127 * 4
    wpitch = 32 + wwords + wl
    wpitch += (-wpitch) % 16
    warena = torch.randint(0, 256, (wn * wpitch,), dtype=torch.uint8, device="cuda")
    wdense = torch.zeros(wn * wwords, dtype=torch.uint8, device="cuda")
    wa0, wd0 = warena.data_ptr(), wdense.data_ptr()
    wdata_off = wpitch - wl
    wps = CrcContext.packet_stream(wdata_off - wwords, wdata_off, wpitch, wn, wl)
    wps_ref = ctypes.byref(wps)
    cases["wire 65,024 B packets: in_packet_words (packet stream -> segmented kernel)"] = \
        lambda: lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, wa0, warena.numel(), wps_ref, bpc)
    pk_w_in = ctx._blocks([(wa0 + i * wpitch + wdata_off, wa0 + i * wpitch + wdata_off - wwords, wl) for i in range(wn)])
    pk_w_dense = ctx._blocks([(wa0 + i * wpitch + wdata_off, wd0 + i * wwords, wl) for i in range(wn)])
    cases["wire 65,024 B packets: in_packet_words (blocks API, segmented)"] = \
        lambda: _native.check("compute_blocks", lib.hdfs3_crc32c_compute_blocks_dev(ctx.ctx, pk_w_in, wn, bpc))
    cases["wire 65,024 B packets: contiguous_words (blocks API, segmented)"] = \
        lambda: _native.check("compute_blocks", lib.hdfs3_crc32c_compute_blocks_dev(ctx.ctx, pk_w_dense, wn, bpc))
    torch.cuda.synchronize()

    def timed(fn, reps=10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    for _ in range(200):
        lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, a0, arena.numel(), ps_ref, bpc)
    torch.cuda.synchronize()
    samples = {k: [] for k in cases}
    for _ in range(5):
        for k, f in cases.items():
            samples[k].append(timed(f))
    # kernel-only figure for the async packet stream (HIP events on the launch stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        cases["pitch_data/in_packet_words (packet stream)"]()
    e1.record(stream)
    torch.cuda.synchronize()
    ev_stream = e0.elapsed_time(e1) * 1e3 / 20
    # parity of the layouts against each other: in-arena words == contiguous words
    got = arena.view(n, pitch)[:, :wpp].contiguous().view(-1)
    cases["pitch_data/contiguous_words (blocks API)"]()
    torch.cuda.synchronize()
    same = bool(torch.equal(got, words))
    for k, v in samples.items():
        v.sort()
        print(json.dumps({"bench": "compute_layout", "case": k, "us_med_wall": round(v[len(v) // 2], 1),
                          "us_min_wall": round(v[0], 1)}), flush=True)
    print(json.dumps({"bench": "compute_layout", "case": "packet stream, HIP events", "us": round(ev_stream, 1),
                      "words_equal_across_layouts": same}), flush=True)


if __name__ == "__main__":
    main()
