"""GPU parity of packet streams at a constant pitch (hdfs3_pkt_stream, the asynchronous packet
APIs, and the wave kernel's pitch mode that serves them): every (packet, chunk) result key and
every computed word must equal the oracle's, for whole-round packets (pitch mode), packets the
pitch mode does not take (65024-byte writer packets, other bpc: descriptor fallback), short
last packets with remote/local tail semantics, and chained overlapped launches."""
import numpy as np
import pytest

from util import oracle_compute, oracle_verify, splitmix_bytes

pytestmark = pytest.mark.gpu


def build_arena(n, plen, last_len, bpc, seed, gap=32):
    """[gap][words][data] per packet at one pitch (data 16 B aligned when gap + words is)."""
    crc_bytes = 4 * (-(-plen // bpc))
    pitch = gap + crc_bytes + plen
    pitch += (-pitch) % 16
    arena = np.zeros(n * pitch + 64, np.uint8)
    datas = []
    for i in range(n):
        dl = plen if i + 1 < n else last_len
        data = splitmix_bytes(dl, seed + i)
        crc = oracle_compute(data, bpc)
        crc_off = i * pitch + gap
        arena[crc_off:crc_off + crc.nbytes] = crc
        arena[crc_off + crc_bytes:crc_off + crc_bytes + dl] = data
        datas.append(data)
    return arena, pitch, gap, gap + crc_bytes, datas


def oracle_key(datas, arena, pitch, crc_off, bpc, local):
    for i, d in enumerate(datas):
        words = arena[i * pitch + crc_off:i * pitch + crc_off + 4 * (-(-d.size // bpc))]
        c = oracle_verify(d, bpc, words, local)
        if c >= 0:
            return i, c
    return -1, -1


def run_stream(ctx, d, nbytes, ps, bpc, local):
    from libhdfs3_amd.engine import DeviceBuffer

    res = DeviceBuffer(8)
    ctx.memset(res, 0, 8)
    ctx.verify_packet_stream_async(d.ptr, nbytes, ps, bpc, res.ptr, local)
    w = int(ctx.download(res, 8).view(np.uint64)[0])
    if w == 0:
        return -1, -1
    key = ctx.decode_result(w)
    return key >> 32, key & 0xFFFFFFFF


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096])
@pytest.mark.parametrize("plen,last", [(65536, 65536), (65536, 65536 - 300), (65536, 4096 * 3 + 1), (65536, 100),
                                       (131072, 131072 - 7), (4096, 4096), (65024, 65024 - 11), (65536 + 512, 700)])
def test_packet_stream_matches_oracle(gpu_ctx, bpc, plen, last):
    from libhdfs3_amd.engine import CrcContext

    n = 24
    arena, pitch, crc_off, data_off, datas = build_arena(n, plen, last, bpc, 100 + bpc + plen % 997)
    d = gpu_ctx.upload(arena)
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last)
    for local in (False, True):
        assert run_stream(gpu_ctx, d, arena.nbytes, ps, bpc, local) == (-1, -1)
    rng = np.random.default_rng(bpc * 7 + plen)
    for p, q in [(0, 0), (n - 1, last - 1), (int(rng.integers(0, n)), None)]:
        q = int(rng.integers(0, datas[p].size)) if q is None else q
        bad = arena.copy()
        bad[p * pitch + data_off + q] ^= 0x04
        gpu_ctx.upload(bad, d)
        for local in (False, True):
            want = oracle_key([np.frombuffer(bad[i * pitch + data_off:i * pitch + data_off + datas[i].size], np.uint8)
                               for i in range(n)], bad, pitch, crc_off, bpc, local)
            assert run_stream(gpu_ctx, d, arena.nbytes, ps, bpc, local) == want, (p, q, local)
    # compute: every region rewritten with the oracle's words
    blank = arena.copy()
    for i in range(n):
        blank[i * pitch + crc_off:i * pitch + data_off] = 0
    gpu_ctx.upload(blank, d)
    gpu_ctx.compute_packet_stream_async(d.ptr, arena.nbytes, ps, bpc)
    assert np.array_equal(gpu_ctx.download(d, arena.nbytes), arena)


def test_descriptor_async_equals_sync(gpu_ctx):
    """hdfs3_crc32c_{verify,compute}_packets_dev_async: same keys and words as the sync calls,
    for a ragged (non-constant-pitch) descriptor list."""
    from libhdfs3_amd.engine import DeviceBuffer

    bpc = 512
    sizes = [65536, 300, 65536 * 2, 4096 * 5 + 17, 512, 65536]
    arena = np.zeros(sum(s + 4 * (-(-s // bpc)) + 48 for s in sizes), np.uint8)
    pk, off = [], 16
    for i, s in enumerate(sizes):
        data = splitmix_bytes(s, 900 + i)
        crc = oracle_compute(data, bpc)
        arena[off:off + crc.nbytes] = crc
        doff = off + crc.nbytes
        doff += (-doff) % 16
        arena[doff:doff + s] = data
        pk.append((doff, off, s))
        off = doff + s + 16
    d = gpu_ctx.upload(arena)
    res = DeviceBuffer(8)
    for flip in (None, (3, 4096 * 2 + 5), (5, 65535)):
        a = arena.copy()
        if flip:
            a[pk[flip[0]][0] + flip[1]] ^= 1
        gpu_ctx.upload(a, d)
        sync = gpu_ctx.verify_packets_dev(d.ptr, a.nbytes, pk, bpc, True)
        gpu_ctx.memset(res, 0, 8)
        gpu_ctx.verify_packets_dev_async(d.ptr, a.nbytes, pk, bpc, res.ptr, True)
        w = int(gpu_ctx.download(res, 8).view(np.uint64)[0])
        key = gpu_ctx.decode_result(w) if w else -1
        got = (key >> 32, key & 0xFFFFFFFF) if w else (-1, -1)
        assert got == sync == ((flip[0], flip[1] // bpc) if flip else (-1, -1))
    blank = arena.copy()
    for doff, coff, s in pk:
        blank[coff:coff + 4 * (-(-s // bpc))] = 0
    gpu_ctx.upload(blank, d)
    gpu_ctx.compute_packets_dev_async(d.ptr, arena.nbytes, pk, bpc)
    assert np.array_equal(gpu_ctx.download(d, arena.nbytes), arena)


def test_stream_bounds_rejected(gpu_ctx):
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer, Hdfs3CrcError

    arena, pitch, crc_off, data_off, _ = build_arena(4, 65536, 65536, 512, 5)
    d = gpu_ctx.upload(arena)
    res = DeviceBuffer(8)
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, 5, 65536, 65536)  # one packet too many
    with pytest.raises(Hdfs3CrcError):
        gpu_ctx.verify_packet_stream_async(d.ptr, arena.nbytes, ps, 512, res.ptr)
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, 4, 65536, 70000)  # last above data_len
    with pytest.raises(Hdfs3CrcError):
        gpu_ctx.verify_packet_stream_async(d.ptr, arena.nbytes, ps, 512, res.ptr)


def test_overlapped_stream_chain_and_large_stream(gpu_ctx):
    """256 MiB of 64 KiB packets: compute -> verify round trip, then 24 chained overlapped
    verifies (HDFS3_LAUNCH_OVERLAP_PREVIOUS) over four resident arenas, one corrupted, each
    into its own result word: every word reports exactly its arena's first bad key.
    (No torch here: this process initialised HIP through the library first.)"""
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer

    n, plen, bpc = 4096, 65536, 512
    pitch = 512 + plen + 16
    crc_off, data_off = 16, 16 + 512
    host = np.random.default_rng(77).integers(0, 256, size=n * pitch, dtype=np.uint8)
    arenas = [DeviceBuffer(n * pitch) for _ in range(4)]
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen)
    for a in arenas:
        gpu_ctx.upload(host, a)
        gpu_ctx.compute_packet_stream_async(a.ptr, n * pitch, ps, bpc)
    gpu_ctx.synchronize()
    got = gpu_ctx.download(arenas[0], n * pitch)
    for p in (0, n // 2, n - 1):
        blob = got[p * pitch:(p + 1) * pitch]
        assert np.array_equal(blob[crc_off:crc_off + 512], oracle_compute(blob[data_off:data_off + plen], bpc))
    p_bad, q_bad = 3001, 40000
    flipped = got[p_bad * pitch + data_off + q_bad:p_bad * pitch + data_off + q_bad + 1] ^ np.uint8(0x10)
    gpu_ctx.upload(flipped, arenas[2], offset=p_bad * pitch + data_off + q_bad)
    res = DeviceBuffer(24 * 8)
    gpu_ctx.memset(res, 0, 24 * 8)
    for i in range(24):
        a = arenas[i % 4]
        gpu_ctx.verify_packet_stream_async(a.ptr, n * pitch, ps, bpc, res.ptr + 8 * i, overlap_previous=i > 0)
    gpu_ctx.synchronize()
    words = gpu_ctx.download(res, 24 * 8).view(np.uint64).tolist()
    for i, w in enumerate(words):
        if i % 4 == 2:
            key = gpu_ctx.decode_result(int(w))
            assert (key >> 32, key & 0xFFFFFFFF) == (p_bad, q_bad // bpc), i
        else:
            assert w == 0, i


@pytest.mark.parametrize("aligned", [True, False])
@pytest.mark.parametrize("bpc", [8192, 65536])
def test_overlapped_chain_chunks_above_4k_pieces(gpu_ctx, bpc, aligned):
    """an overlapped verify at bpc = R x 4096 runs the piece compute of the pitch walk
    (crc32c_wave_kernel<4096, compute, PITCH, SOLO>) without the AQL barrier, then the combine. 30
    chained launches over 5 resident arenas of 64 KiB packets (one arena corrupted, one with a short
    last packet), each into its own result word, alternating the two piece buffers: every word
    reports exactly its arena's first bad (packet, chunk), and a compute -> verify round trip in
    the same overlapped form writes the oracle's words. aligned=False puts the data 4 bytes off a
    16-byte boundary at bpc 65536 (4-byte word regions): the stream falls back to descriptors and the
    chunk-per-lane kernel, queued 30 deep without a sync — the case that found the descriptor staging
    ring being rewritten under a queued copy (round 5, packets_async)."""
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer

    n, plen = 96, 65536
    arenas, streams, hosts = [], [], []
    for a in range(5):
        last = plen if a != 3 else (bpc * 2 + 300 if bpc * 2 + 300 < plen else plen - 300)
        words = 4 * (-(-plen // bpc))
        gap = 32 + ((-(32 + words)) % 16 if aligned else 0)
        host, pitch, crc_off, data_off, datas = build_arena(n, plen, last, bpc, 7000 + 131 * a + bpc % 1013, gap)
        hosts.append((host, pitch, crc_off, data_off, datas))
        arenas.append(gpu_ctx.upload(host))
        streams.append(CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last))
    p_bad, q_bad = 61, 40000
    host, pitch, crc_off, data_off, datas = hosts[2]
    bad = host.copy()
    bad[p_bad * pitch + data_off + q_bad] ^= 0x20
    gpu_ctx.upload(bad, arenas[2])
    want2 = oracle_key([np.frombuffer(bad[i * pitch + data_off:i * pitch + data_off + datas[i].size], np.uint8)
                        for i in range(n)], bad, pitch, crc_off, bpc, False)
    assert want2 == (p_bad, q_bad // bpc)
    res = DeviceBuffer(30 * 8)
    gpu_ctx.memset(res, 0, 30 * 8)
    for i in range(30):
        a = i % 5
        gpu_ctx.verify_packet_stream_async(arenas[a].ptr, hosts[a][0].nbytes, streams[a], bpc, res.ptr + 8 * i,
                                           overlap_previous=i > 0)
    gpu_ctx.synchronize()
    words = gpu_ctx.download(res, 30 * 8).view(np.uint64).tolist()
    for i, w in enumerate(words):
        if i % 5 == 2:
            key = gpu_ctx.decode_result(int(w))
            assert (key >> 32, key & 0xFFFFFFFF) == want2, i
        else:
            assert w == 0, i
    # compute (barriered, its scratch alternating with the verifies') then overlapped verifies of it
    host, pitch, crc_off, data_off, datas = hosts[3]
    blank = host.copy()
    for i in range(n):
        blank[i * pitch + crc_off:i * pitch + data_off] = 0
    gpu_ctx.upload(blank, arenas[3])
    gpu_ctx.compute_packet_stream_async(arenas[3].ptr, host.nbytes, streams[3], bpc)
    gpu_ctx.memset(res, 0, 30 * 8)
    for i in range(6):
        gpu_ctx.verify_packet_stream_async(arenas[3].ptr, host.nbytes, streams[3], bpc, res.ptr + 8 * i,
                                           overlap_previous=i > 0)
    assert np.array_equal(gpu_ctx.download(arenas[3], host.nbytes), host)
    assert not gpu_ctx.download(res, 6 * 8).view(np.uint64).any()


def test_compute_word_scratch_grows_across_calls(gpu_ctx):
    """Compute over in-packet words goes through the ctx's dense word scratch and a scatter
    kernel. Streams of growing length on one ctx (the scratch is reallocated between them, after
    the previous use completed), each with a short last packet: every packet's words equal the
    oracle's and no other byte of the arena changes."""
    from libhdfs3_amd.engine import CrcContext

    bpc, plen = 512, 16384
    for n, last in [(3, plen), (40, plen - 700), (300, 1), (40, 4096)]:
        arena, pitch, crc_off, data_off, datas = build_arena(n, plen, last, bpc, 4000 + n)
        blank = arena.copy()
        for i in range(n):
            blank[i * pitch + crc_off:i * pitch + data_off] = 0xA5
        d = gpu_ctx.upload(blank)
        ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last)
        gpu_ctx.compute_packet_stream_async(d.ptr, arena.nbytes, ps, bpc)
        got = gpu_ctx.download(d, arena.nbytes)
        # the words of a short last packet end before its region does: the rest keeps 0xA5
        want = arena.copy()
        lw = 4 * (-(-last // bpc))
        want[(n - 1) * pitch + crc_off + lw:(n - 1) * pitch + data_off] = 0xA5
        assert np.array_equal(got, want), (n, last)



@pytest.mark.parametrize("variant", [0, 124])
def test_packet_stream_solo_variant_overlapped_chain(lab_ctx, variant):
    """The pitch walk with the solo last step (production since round 4 for overlapped launches up to
    256 MiB; lab variant 124 runs it without, as before) as the bench's packets block runs it: 128 MiB of 64 KiB packets at the block reader's 66,048-byte
    pitch, and a 37-packet stream with a short last packet (slow region), chained overlapped
    verifies each into its own result word, one arena corrupted: every word its first bad key."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer

    lib = _native.lab()
    bpc, plen = 512, 65536
    pitch, crc_off, data_off = 512 + plen, 0, 512
    try:
        lib.hdfs3x_set_variant(variant)
        # the 37-packet stream's last packet: 5 whole rounds, 3 whole chunks in the slow region and a
        # short tail (which remote semantics do not check, RemoteBlockReader.cpp:319); the flip sits
        # in the slow region's second chunk
        for n, last in ((2048, plen), (37, 4096 * 5 + 512 * 3 + 300)):
            host = np.random.default_rng(n + variant).integers(0, 256, size=n * pitch, dtype=np.uint8)
            for i in range(n):
                dl = plen if i + 1 < n else last
                host[i * pitch + crc_off:i * pitch + crc_off + 4 * (-(-dl // bpc))] = \
                    oracle_compute(host[i * pitch + data_off:i * pitch + data_off + dl], bpc)
            ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last)
            arenas = [lab_ctx.upload(host) for _ in range(3)]
            p_bad = n - 1 if n < 100 else 1500
            q_bad = 4096 * 5 + 512 + 100 if n < 100 else 33333
            lab_ctx.upload(np.array([host[p_bad * pitch + data_off + q_bad] ^ 0x40], np.uint8), arenas[1],
                           offset=p_bad * pitch + data_off + q_bad)
            res = DeviceBuffer(12 * 8)
            lab_ctx.memset(res, 0, 12 * 8)
            for i in range(12):
                lab_ctx.verify_packet_stream_async(arenas[i % 3].ptr, n * pitch, ps, bpc, res.ptr + 8 * i,
                                                   overlap_previous=i > 0)
            lab_ctx.synchronize()
            for i, w in enumerate(lab_ctx.download(res, 12 * 8).view(np.uint64).tolist()):
                if i % 3 == 1:
                    key = lab_ctx.decode_result(int(w))
                    assert (key >> 32, key & 0xFFFFFFFF) == (p_bad, q_bad // bpc), (variant, n, i)
                else:
                    assert w == 0, (variant, n, i)
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.parametrize("bpc", [8192, 16384, 32768, 65536])
@pytest.mark.parametrize("last", [65536, 65536 - 300, 8192 * 3 + 100, 100])
def test_packet_stream_chunks_above_4k_pieces(gpu_ctx, bpc, last):
    """Packet streams at bpc = R * 4096 (64 KiB datanode packets at 8 / 16 / 32 / 64 KiB chunks; round
    4): the pitch walk's 4096-byte piece CRCs, the combine into each packet's own CRC region, the last
    packet's short chunk on the byte-exact kernel. Keys (packet, chunk) and every computed word against
    the oracle, remote and local tail semantics, flips in the first, a middle and the last packet, and
    the descriptor form of the same stream (packets API) gives the same keys."""
    from libhdfs3_amd.engine import CrcContext

    n, plen = 24, 65536
    arena, pitch, crc_off, data_off, datas = build_arena(n, plen, last, bpc, 300 + bpc % 977 + last % 13)
    d = gpu_ctx.upload(arena)
    ps = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last)
    for local in (False, True):
        assert run_stream(gpu_ctx, d, arena.nbytes, ps, bpc, local) == (-1, -1)
    rng = np.random.default_rng(bpc + last)
    for p, q in [(0, 5), (n // 2, int(rng.integers(0, plen))), (n - 1, last - 1), (n - 1, 0)]:
        bad = arena.copy()
        bad[p * pitch + data_off + q] ^= 0x08
        gpu_ctx.upload(bad, d)
        for local in (False, True):
            want = oracle_key([np.frombuffer(bad[i * pitch + data_off:i * pitch + data_off + datas[i].size], np.uint8)
                               for i in range(n)], bad, pitch, crc_off, bpc, local)
            assert run_stream(gpu_ctx, d, arena.nbytes, ps, bpc, local) == want, (p, q, local)
            pk = [(i * pitch + data_off, i * pitch + crc_off, datas[i].size) for i in range(n)]
            assert gpu_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc, local) == want, (p, q, local)
    blank = arena.copy()
    for i in range(n):
        blank[i * pitch + crc_off:i * pitch + data_off] = 0
    gpu_ctx.upload(blank, d)
    gpu_ctx.compute_packet_stream_async(d.ptr, arena.nbytes, ps, bpc)
    assert np.array_equal(gpu_ctx.download(d, arena.nbytes), arena)


@pytest.mark.parametrize("bpc", [1024, 4096, 8192, 65536])
@pytest.mark.parametrize("last", [65536, 65536 - 4096 * 3, 4096 * 2 + 77])
def test_descriptors_with_words_at_their_own_pitch(gpu_ctx, bpc, last):
    """Round 5: a descriptor list whose packets sit at one data pitch and whose words are dense (the
    output stream's batches) takes the pitch walk with its own word pitch (and at R x 4096 its pieces +
    the packet-mode combine). Verify keys and computed words against the oracle, with a flip in the
    first and the last packet; remote and local tail semantics."""
    n, plen, pitch = 20, 65536, 65536 + 4096
    wpp = 4 * (plen // bpc)
    arena = np.zeros(n * pitch + n * wpp + 4096, np.uint8)
    wbase = n * pitch
    datas, pk = [], []
    for i in range(n):
        dl = plen if i + 1 < n else last
        d = splitmix_bytes(dl, 600 + i + bpc)
        arena[i * pitch:i * pitch + dl] = d
        w = oracle_compute(d, bpc)
        arena[wbase + i * wpp:wbase + i * wpp + w.nbytes] = w
        datas.append(d)
        pk.append((i * pitch, wbase + i * wpp, dl))
    dev = gpu_ctx.upload(arena)
    for local in (False, True):
        assert gpu_ctx.verify_packets_dev(dev.ptr, arena.nbytes, pk, bpc, local) == (-1, -1)
    for p, q in [(0, 7), (n - 1, last - 1)]:
        bad = arena.copy()
        bad[p * pitch + q] ^= 0x01
        gpu_ctx.upload(bad, dev)
        for local in (False, True):
            want = (-1, -1)
            for i in range(n):
                c = oracle_verify(bad[i * pitch:i * pitch + datas[i].size], bpc,
                                  bad[wbase + i * wpp:wbase + i * wpp + 4 * (-(-datas[i].size // bpc))], local)
                if c >= 0:
                    want = (i, c)
                    break
            assert gpu_ctx.verify_packets_dev(dev.ptr, arena.nbytes, pk, bpc, local) == want, (p, q, local)
    blank = arena.copy()
    blank[wbase:] = 0xA5
    gpu_ctx.upload(blank, dev)
    gpu_ctx.compute_packets_dev(dev.ptr, arena.nbytes, pk, bpc)
    got = gpu_ctx.download(dev, arena.nbytes)
    for i in range(n):
        nw = 4 * (-(-datas[i].size // bpc))
        assert np.array_equal(got[wbase + i * wpp:wbase + i * wpp + nw], oracle_compute(datas[i], bpc)), i
    assert np.array_equal(got[:wbase], arena[:wbase])
