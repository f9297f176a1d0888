"""GPU parity of PARTIAL rounds (round 6): packets whose whole chunks end inside a 4 KiB round, and
packets of a number of rounds that is not a power of two, on the round kernel instead of the
one-chunk-per-lane passes.

* The output stream's own batches (OutputStreamImpl.cpp:161-170 computePacketChunkSize; Packet.cpp:73-92):
  at the default 64 KiB packet size a packet carries 127 chunks at bpc 512 (65,024 B = 15 rounds +
  3,584 B), 63 at 1024, 31 at 2048 and 15 at 4096 (15 whole rounds: not a power of two). Laid out as
  output_stream.cpp lays a batch: packet slots [lead][data] at one stride, the words compact after
  the slots.
* Chunks of R x 4096 whose packets hold a number of rounds that is not a power of two (12 KiB and 20 KiB
  chunks: 5 and 3 per 60 KiB packet, 15 rounds; RemoteBlockReader.cpp:150-156 takes any bpc).
* Ragged descriptor lists (no constant pitch): the segmented kernel's partial last unit per packet.

Every verify key (packet, chunk) and every computed word is compared with the oracle; flips sit in
the partial round's first and last whole chunk and in the short tail."""
import numpy as np
import pytest

from util import oracle_compute, oracle_verify, splitmix_bytes

pytestmark = pytest.mark.gpu

HEADER = 31  # PacketHeader::GetPkHeaderLen (PacketHeader.cpp:38)


def writer_geometry(bpc, packet_size=65536):
    """output_stream.cpp init(): chunks per packet, slot lead and stride."""
    with_sum = bpc + 4
    cpp = max(1, (packet_size - HEADER + with_sum - 1) // with_sum)
    lead = (HEADER + 4 * cpp + 15) // 16 * 16
    stride = lead + (cpp * bpc + 15) // 16 * 16
    return cpp, lead, stride


def writer_batch(bpc, n, last_len=None, seed=1):
    """One output-stream batch: n packet slots, the last holding last_len bytes, words compact."""
    cpp, lead, stride = writer_geometry(bpc)
    plen = cpp * bpc
    last_len = plen if last_len is None else last_len
    crc_region = stride * n
    nch = [(plen if i + 1 < n else last_len + bpc - 1) // bpc for i in range(n)]
    arena = np.zeros(crc_region + 4 * sum(nch) + 64, np.uint8)
    pk, datas, w = [], [], crc_region
    for i in range(n):
        dl = plen if i + 1 < n else last_len
        d = splitmix_bytes(dl, seed * 1000 + i)
        off = lead + stride * i
        arena[off:off + dl] = d
        words = oracle_compute(d, bpc)
        arena[w:w + words.nbytes] = words
        pk.append((off, w, dl))
        datas.append(d)
        w += words.nbytes
    return arena, pk, datas


def first_bad(arena, pk, bpc, local):
    for i, (off, w, dl) in enumerate(pk):
        c = oracle_verify(arena[off:off + dl], bpc, arena[w:w + 4 * (-(-dl // bpc))], local)
        if c >= 0:
            return i, c
    return -1, -1


def check_batch(ctx, arena, pk, bpc, flips):
    dev = ctx.upload(arena)
    for local in (False, True):
        assert ctx.verify_packets_dev(dev.ptr, arena.nbytes, pk, bpc, local) == (-1, -1)
    for p, q in flips:
        bad = arena.copy()
        bad[pk[p][0] + q] ^= 0x02
        ctx.upload(bad, dev)
        for local in (False, True):
            want = first_bad(bad, pk, bpc, local)
            assert ctx.verify_packets_dev(dev.ptr, arena.nbytes, pk, bpc, local) == want, (p, q, local)
    blank = arena.copy()
    for off, w, dl in pk:
        blank[w:w + 4 * (-(-dl // bpc))] = 0xA5
    ctx.upload(blank, dev)
    ctx.compute_packets_dev(dev.ptr, arena.nbytes, pk, bpc)
    assert np.array_equal(ctx.download(dev, arena.nbytes), arena)


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096])
@pytest.mark.parametrize("last", ["full", "partial_round", "short_tail", "tiny"])
def test_writer_batch_layout(gpu_ctx, bpc, last):
    cpp, _, _ = writer_geometry(bpc)
    plen = cpp * bpc
    last_len = {"full": plen, "partial_round": plen - bpc, "short_tail": plen - bpc - 77, "tiny": 300}[last]
    n = 64
    arena, pk, datas = writer_batch(bpc, n, last_len, seed=bpc + len(last))
    whole = plen // 4096 * 4096  # the first byte of a packet's partial round (== plen when none)
    flips = [(0, 0), (5, min(whole, plen - 1)), (33, plen - 1), (n - 1, last_len - 1), (n - 1, 0)]
    check_batch(gpu_ctx, arena, pk, bpc, flips)


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096])
@pytest.mark.parametrize("rounds_x", [(3, 0), (5, 1536), (15, 0), (15, 3584), (17, 512), (1, 512), (0, 1024)])
def test_non_power_of_two_streams(gpu_ctx, bpc, rounds_x):
    """hdfs3_pkt_stream (wire layout: words in the packet) over packets of r whole rounds + x bytes of
    whole chunks: the pitch walk's multiply-shift packet index and its partial last round."""
    from libhdfs3_amd.engine import CrcContext

    r, x = rounds_x
    plen = r * 4096 + x // bpc * bpc
    if plen == 0:
        pytest.skip("no whole chunk at this bpc")
    n = 300
    wb = 4 * (plen // bpc)
    crc_off = 32
    data_off = (crc_off + wb + 15) // 16 * 16
    pitch = (data_off + plen + 15) // 16 * 16
    last = plen - 1
    arena = np.zeros(n * pitch + 64, np.uint8)
    datas = []
    for i in range(n):
        dl = plen if i + 1 < n else last
        d = splitmix_bytes(dl, 77 + i + plen)
        arena[i * pitch + data_off:i * pitch + data_off + dl] = d
        w = oracle_compute(d, bpc)
        arena[i * pitch + crc_off:i * pitch + crc_off + w.nbytes] = w
        datas.append(d)
    pk = [(i * pitch + data_off, i * pitch + crc_off, datas[i].size) for i in range(n)]
    dev = gpu_ctx.upload(arena)
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last)
    from test_gpu_packet_stream import run_stream

    for local in (False, True):
        assert run_stream(gpu_ctx, dev, arena.nbytes, ps, bpc, local) == (-1, -1)
    for p, q in [(0, plen - 1), (n // 2, plen // 2), (n - 2, 0), (n - 1, last - 1)]:
        bad = arena.copy()
        bad[p * pitch + data_off + q] ^= 0x40
        gpu_ctx.upload(bad, dev)
        for local in (False, True):
            want = first_bad(bad, pk, bpc, local)
            assert run_stream(gpu_ctx, dev, arena.nbytes, ps, bpc, local) == want, (p, q, local)
            assert gpu_ctx.verify_packets_dev(dev.ptr, arena.nbytes, pk, bpc, local) == want, (p, q, local)
    blank = arena.copy()
    for i in range(n):
        blank[i * pitch + crc_off:i * pitch + data_off] = 0
    gpu_ctx.upload(blank, dev)
    gpu_ctx.compute_packet_stream_async(dev.ptr, arena.nbytes, ps, bpc)
    assert np.array_equal(gpu_ctx.download(dev, arena.nbytes), arena)


@pytest.mark.parametrize("bpc", [12288, 20480])
@pytest.mark.parametrize("last", ["full", "one_chunk_short", "short_tail"])
def test_chunks_of_three_and_five_rounds(gpu_ctx, bpc, last):
    """bpc 12288 / 20480 (3 and 5 rounds per chunk): the writer's batch at its own geometry (6 / 4
    chunks = 18 / 20 rounds per 64 KiB packet, words compact) and a wire stream of 60 KiB packets (5 / 3
    chunks, 15 rounds): the pitch walk's pieces + the combine, the short chunk on one lane."""
    from libhdfs3_amd.engine import CrcContext

    def last_of(plen):
        return {"full": plen, "one_chunk_short": plen - bpc, "short_tail": plen - bpc - 999}[last]

    n = 40
    cpp, _, _ = writer_geometry(bpc)
    plen = cpp * bpc
    arena, pk, _ = writer_batch(bpc, n, last_of(plen), seed=bpc // 4096)
    check_batch(gpu_ctx, arena, pk, bpc, [(0, bpc), (7, plen - 1), (n - 1, last_of(plen) - 1)])
    # the wire layout: [words][data] per packet at one pitch, 60 KiB packets
    cpp = 61440 // bpc
    plen = cpp * bpc
    last_len = last_of(plen)
    wb = 4 * cpp
    pitch = 64 + plen
    wire = np.zeros(n * pitch + 64, np.uint8)
    wpk = []
    for i in range(n):
        d = splitmix_bytes(plen if i + 1 < n else last_len, 40 * bpc + i)
        w = oracle_compute(d, bpc)
        wire[i * pitch + 64 - wb:i * pitch + 64 - wb + w.nbytes] = w
        wire[i * pitch + 64:i * pitch + 64 + d.size] = d
        wpk.append((i * pitch + 64, i * pitch + 64 - wb, d.size))
    dev = gpu_ctx.upload(wire)
    ps = CrcContext.packet_stream(64 - wb, 64, pitch, n, plen, last_len)
    from test_gpu_packet_stream import run_stream

    for p, q in [(None, None), (3, 5), (n - 1, last_len - 1)]:
        bad = wire.copy()
        if p is not None:
            bad[wpk[p][0] + q] ^= 0x01
        gpu_ctx.upload(bad, dev)
        for local in (False, True):
            want = first_bad(bad, wpk, bpc, local)
            assert run_stream(gpu_ctx, dev, wire.nbytes, ps, bpc, local) == want, (p, q, local)
    blank = wire.copy()
    for off, w, dl in wpk:
        blank[w:off] = 0
    gpu_ctx.upload(blank, dev)
    gpu_ctx.compute_packet_stream_async(dev.ptr, wire.nbytes, ps, bpc)
    assert np.array_equal(gpu_ctx.download(dev, wire.nbytes), wire)


@pytest.mark.parametrize("bpc", [512, 2048])
def test_ragged_descriptor_list_partial_units(gpu_ctx, bpc):
    """A descriptor list with no constant pitch and lengths that end inside rounds (whole chunks,
    a short chunk, under one chunk): the segmented kernel's partial last unit per segment."""
    rng = np.random.default_rng(bpc)
    sizes = [65024, 300, 4096 * 3 + bpc, 4096 * 7 + 2 * bpc + 5, bpc, 4096, 65536, 3 * bpc + 1]
    sizes += [int(s) // bpc * bpc + int(rng.integers(0, 2)) * int(rng.integers(1, bpc)) for s in
              rng.integers(1, 100000, size=40)]
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 64 for s in sizes) + 64, np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        d = splitmix_bytes(s, 5000 + i)
        w = oracle_compute(d, bpc)
        arena[off:off + w.nbytes] = w
        doff = off + w.nbytes
        doff += (-doff) % 16
        arena[doff:doff + s] = d
        pk.append((doff, off, s))
        off = doff + s + 16 * int(rng.integers(0, 3))
    flips = [(0, 65023), (0, 61440), (3, 4096 * 7 + bpc + 1), (7, 3 * bpc), (len(sizes) - 1, sizes[-1] - 1)]
    check_batch(gpu_ctx, arena, pk, bpc, flips)


def test_segments_variant_1024_threads_same_keys(lab_ctx):
    """Lab variant 161 runs the segmented kernel at 1024 threads per workgroup at every size (production
    before round 6): same keys and words as production on a ragged list."""
    from libhdfs3_amd import _native

    lib = _native.lab()
    bpc = 512
    sizes = [65024] * 9 + [1000, 4096 * 2 + 512 * 5]
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 48 for s in sizes), np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        d = splitmix_bytes(s, 70 + i)
        w = oracle_compute(d, bpc)
        arena[off:off + w.nbytes] = w
        doff = off + w.nbytes + (-(off + w.nbytes)) % 16
        arena[doff:doff + s] = d
        pk.append((doff, off, s))
        off = doff + s + 32
    try:
        for v in (0, 161):
            lib.hdfs3x_set_variant(v)
            check_batch(lab_ctx, arena, pk, bpc, [(4, 61440 + 3583), (10, 4096 * 2 + 512 * 4)])
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.parametrize("bpc", [8192, 12288, 20480, 65536])
def test_ragged_descriptor_list_chunks_above_4k(gpu_ctx, bpc):
    """Round 6: a descriptor list at bpc = R x 4096 that is not one constant-pitch stream (ragged lengths,
    gaps between packets) takes the segmented kernel's 4096-byte piece CRCs and a per-segment combine,
    the short last chunks one lane each (before: the chunk-per-lane packet kernel). Keys and every
    computed word against the oracle, remote and local tail semantics, flips in whole chunks and in
    short tails; packets shorter than one chunk, and of exactly one chunk."""
    rng = np.random.default_rng(bpc + 1)
    sizes = [3 * bpc, bpc + 777, 61440 // bpc * bpc or bpc, 500, bpc, 2 * bpc + 4096, 7 * bpc - 1]
    sizes += [int(x) for x in rng.integers(1, 6 * bpc, size=12)]
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 96 for s in sizes) + 64, np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        d = splitmix_bytes(s, 9000 + i + bpc)
        w = oracle_compute(d, bpc)
        arena[off:off + w.nbytes] = w
        doff = off + w.nbytes
        doff += (-doff) % 16
        arena[doff:doff + s] = d
        pk.append((doff, off, s))
        off = doff + s + 16 * int(rng.integers(1, 4))
    flips = [(0, 2 * bpc + 5), (1, bpc + 700), (3, 499), (5, 2 * bpc + 4000), (6, 7 * bpc - 2),
             (len(sizes) - 1, sizes[-1] - 1)]
    check_batch(gpu_ctx, arena, pk, bpc, flips)


@pytest.mark.parametrize("bpc", [512, 4096, 12288])
def test_long_ragged_descriptor_list_unit_map(gpu_ctx, bpc):
    """Round 6: descriptor lists of more than 256 packets that are not one constant-pitch stream take a
    unit -> segment map built on the device (one scalar load per round in place of a binary search):
    700 packets of ragged lengths (under one chunk, whole chunks, short tails, several rounds), every
    word and the first bad (packet, chunk) against the oracle, flips early, in the middle and last."""
    rng = np.random.default_rng(bpc + 7)
    sizes = [int(x) for x in rng.integers(1, 12 * max(bpc, 4096) // 4, size=700)]
    sizes[5] = bpc - 1
    sizes[6] = bpc
    sizes[400] = 8 * 4096
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 64 for s in sizes) + 64, np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        d = splitmix_bytes(s, 13000 + i + bpc)
        w = oracle_compute(d, bpc)
        arena[off:off + w.nbytes] = w
        doff = off + w.nbytes
        doff += (-doff) % 16
        arena[doff:doff + s] = d
        pk.append((doff, off, s))
        off = doff + s + 16 * int(rng.integers(0, 3))
    flips = [(2, sizes[2] // 2), (400, 5 * 4096 + 3), (699, sizes[699] - 1)]
    check_batch(gpu_ctx, arena, pk, bpc, flips)


@pytest.mark.parametrize("bpc", [512, 4096, 8192])
@pytest.mark.parametrize("shape", ["tails_only", "one_long_among_tails", "long_last"])
def test_long_list_zero_unit_segments(gpu_ctx, bpc, shape):
    """Lists of more than 256 packets whose packets mostly hold no whole round (shorter than one chunk):
    the unit map has entries only for the packets that do (none, one in the middle, the last), and the
    segments' short chunks go one lane each. Every word and the first bad (packet, chunk)."""
    n = 300
    sizes = [100 + (i * 37) % (bpc - 100) for i in range(n)]
    if shape == "one_long_among_tails":
        sizes[150] = 16 * 4096 + bpc // 2
    elif shape == "long_last":
        sizes[-1] = 9 * 4096
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 48 for s in sizes) + 64, np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        d = splitmix_bytes(s, 17000 + i + bpc)
        w = oracle_compute(d, bpc)
        arena[off:off + w.nbytes] = w
        doff = off + w.nbytes
        doff += (-doff) % 16
        arena[doff:doff + s] = d
        pk.append((doff, off, s))
        off = doff + s + 16 * (i % 3)
    flips = [(0, 5), (n - 1, sizes[-1] - 1)]
    if shape == "one_long_among_tails":
        flips.append((150, 4096 * 8 + 1))
    check_batch(gpu_ctx, arena, pk, bpc, flips)
