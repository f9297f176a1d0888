"""GPU parity tests: the HIP path (through the C-ABI) vs the oracle and the reference's fixtures.

Bar: bit-exact CRC32C words and identical first-bad-chunk indices. Small cases are
compared word for word with the oracle; BASELINE.json's full sizes (128 MiB block,
1 GiB stream, bpc 512/2048/4096) are compared word for word as well (the C oracle
is fast enough) plus compute->verify round trips and single-bit corruption.
"""
import json
import os

import numpy as np
import pytest

from util import (GOLDEN, oracle, oracle_compute, oracle_verify, ptr, read_checksum1, read_checksum2,
                  splitmix_bytes)

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(GOLDEN, "ref_hwcrc32c.npz"))
META = json.load(open(os.path.join(GOLDEN, "ref_hwcrc32c.json")))


def test_reference_kats_checksum1_on_gpu(gpu_ctx):
    from libhdfs3_amd.engine import DeviceBuffer

    cases = read_checksum1()
    dbuf = DeviceBuffer(4096 + 64)
    dout = DeviceBuffer(64)
    for want, s in cases:
        a = np.frombuffer(s, dtype=np.uint8)
        # host API: one short chunk
        assert gpu_ctx.compute(a, 4096).view(">u4")[0] == want
        # device API at the 8 alignments of TestChecksum.cpp:92-99 (generic kernel)
        for j in range(8):
            gpu_ctx.upload(a, dbuf, offset=j)
            gpu_ctx.compute_dev(dbuf.ptr + j, len(s), 4096, dout.ptr)
            assert gpu_ctx.download(dout, 4).view(">u4")[0] == want, (len(s), j)


def test_reference_checksum2_streamed_total_on_gpu(gpu_ctx):
    # the streamed total is one CRC over the concatenation of every line
    result, lines = read_checksum2()
    blob = np.frombuffer(b"".join(lines), dtype=np.uint8)
    assert gpu_ctx.compute(blob, (blob.nbytes + 3) // 4 * 4).view(">u4")[0] == result


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_bpc_fixture_host_and_device(gpu_ctx, bpc):
    from libhdfs3_amd.engine import DeviceBuffer

    big = splitmix_bytes(1 << 20, META["seeds"]["bpc"])
    want = GOLD[f"bpc{bpc}"]
    assert np.array_equal(gpu_ctx.compute(big, bpc), want)
    d = gpu_ctx.upload(big)
    dc = DeviceBuffer(want.nbytes)
    gpu_ctx.compute_dev(d.ptr, big.nbytes, bpc, dc.ptr)
    assert np.array_equal(gpu_ctx.download(dc, want.nbytes), want)
    assert gpu_ctx.verify(big, bpc, want, False) == -1
    assert gpu_ctx.verify_dev(d.ptr, big.nbytes, bpc, dc.ptr, True) == -1


def test_packet_fixture_verify_semantics(gpu_ctx):
    pkt = splitmix_bytes(65536, META["seeds"]["packet"])
    crc = GOLD["pkt_crc"]
    v = META["verify"]
    assert gpu_ctx.verify(pkt, 512, crc, False) == v["clean_remote"]
    bad = pkt.copy()
    bad[META["packet"]["flip_byte"]] ^= META["packet"]["flip_mask"]
    assert gpu_ctx.verify(bad, 512, crc, False) == v["flip77_remote"]
    assert gpu_ctx.verify(bad, 512, crc, True) == v["flip77_local"]
    n = META["packet"]["tail_len"]
    tail = GOLD["tail_crc"]
    corrupt = tail.copy()
    corrupt[4 * 127] ^= 0xFF
    assert np.array_equal(gpu_ctx.compute(pkt[:n], 512), tail)
    assert gpu_ctx.verify(pkt[:n], 512, tail, True) == v["tail_clean_local"]
    assert gpu_ctx.verify(pkt[:n], 512, corrupt, False) == v["tail_corrupt_remote"]
    assert gpu_ctx.verify(pkt[:n], 512, corrupt, True) == v["tail_corrupt_local"]


# bpc 1, 3, 513, 517: readers accept any bytesPerChecksum > 0 (RemoteBlockReader.cpp:150-156,
# LocalBlockReader.cpp:110-115); the byte-granular kernel verifies them
@pytest.mark.parametrize("bpc", [1, 3, 4, 12, 64, 500, 512, 513, 516, 517, 1024, 2048, 4096, 65536])
def test_ragged_lengths_vs_oracle(gpu_ctx, bpc):
    rng = np.random.default_rng(bpc)
    for n in [0, 1, 3, bpc - 1, bpc, bpc + 1, 3 * bpc + 7] + [int(x) for x in rng.integers(0, 300_000, 6)]:
        if n < 0:
            continue
        data = splitmix_bytes(n, 1000 + n)
        want = oracle_compute(data, bpc)
        got = gpu_ctx.compute(data, bpc)
        assert np.array_equal(got, want), (bpc, n)
        assert gpu_ctx.verify(data, bpc, want, True) == -1
        if n:
            k = int(rng.integers(0, n))
            bad = data.copy()
            bad[k] ^= 0x40
            for tail in (False, True):
                assert gpu_ctx.verify(bad, bpc, want, tail) == oracle_verify(bad, bpc, want, tail), (bpc, n, k, tail)


@pytest.mark.parametrize("offset", [1, 2, 3, 4, 8, 12])
def test_unaligned_device_pointers(gpu_ctx, offset):
    from libhdfs3_amd.engine import DeviceBuffer

    data = splitmix_bytes(513 * 97 + 5, offset)
    d = DeviceBuffer(data.nbytes + 64)
    gpu_ctx.upload(data, d, offset=offset)
    for bpc in (512, 2048, 516, 517, 3):
        want = oracle_compute(data, bpc)
        dc = DeviceBuffer(want.nbytes + 8)
        gpu_ctx.compute_dev(d.ptr + offset, data.nbytes, bpc, dc.ptr + 1)  # unaligned CRC array too
        assert np.array_equal(gpu_ctx.download(dc, want.nbytes, offset=1), want), (offset, bpc)
        assert gpu_ctx.verify_dev(d.ptr + offset, data.nbytes, bpc, dc.ptr + 1, True) == -1


def _wire_arena(n_pkts, bpc, rng, short_last=True):
    """Build an arena of HDFS data packets in wire order: [31 B header][BE CRCs][data]
    (RemoteBlockReader.cpp:240-245); descriptors point at the CRC and data regions."""
    parts, descs, off = [], [], 0
    for p in range(n_pkts):
        data_len = 65536 if not (short_last and p == n_pkts - 1) else int(rng.integers(1, 65536))
        data = splitmix_bytes(data_len, 77 + p)
        crc = oracle_compute(data, bpc)
        hdr = np.zeros(31, np.uint8)
        crc_off = off + 31
        data_off = crc_off + crc.nbytes
        parts += [hdr, crc, data]
        descs.append((data_off, crc_off, data_len))
        off = data_off + data_len
    return np.concatenate(parts), descs


@pytest.mark.parametrize("bpc", [3, 512, 513, 4096])
def test_packets_api(gpu_ctx, bpc):
    from libhdfs3_amd.engine import DeviceBuffer

    rng = np.random.default_rng(bpc)
    arena, pk = _wire_arena(17, bpc, rng)
    assert gpu_ctx.verify_packets(arena, pk, bpc) == (-1, -1)
    bad = arena.copy()
    d_off, _, _ = pk[5]
    bad[d_off + 3 * bpc + 11] ^= 1
    bad[pk[9][0] + 2] ^= 1
    assert gpu_ctx.verify_packets(bad, pk, bpc) == (5, (3 * bpc + 11) // bpc)
    # corrupt the short tail chunk's CRC of the last packet: remote ignores, local flags
    last = len(pk) - 1
    data_off, crc_off, data_len = pk[last]
    nchunks = (data_len + bpc - 1) // bpc
    if data_len % bpc:
        t = arena.copy()
        t[crc_off + 4 * (nchunks - 1)] ^= 0x10
        assert gpu_ctx.verify_packets(t, pk, bpc, False) == (-1, -1)
        assert gpu_ctx.verify_packets(t, pk, bpc, True) == (last, nchunks - 1)
    # device-resident arena + compute in place (write path)
    d = gpu_ctx.upload(arena)
    assert gpu_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc) == (-1, -1)
    wiped = arena.copy()
    for data_off, crc_off, data_len in pk:
        wiped[crc_off:data_off] = 0
    d2 = gpu_ctx.upload(wiped)
    gpu_ctx.compute_packets_dev(d2.ptr, wiped.nbytes, pk, bpc)
    assert np.array_equal(gpu_ctx.download(d2, arena.nbytes), arena)


@pytest.mark.parametrize("n_pkts", [33, 70])
def test_packets_api_large_host_arena(gpu_ctx, n_pkts):
    """A host packet arena of MiBs (odd length: a short last packet) is staged through the host
    copy pool: a flip in the arena's very last byte must still be found, in the last packet's
    last chunk (local semantics check the short tail)."""
    rng = np.random.default_rng(n_pkts)
    arena, pk = _wire_arena(n_pkts, 512, rng)
    assert arena.nbytes > (2 << 20)
    assert gpu_ctx.verify_packets(arena, pk, 512, True) == (-1, -1)
    bad = arena.copy()
    bad[-1] ^= 0x01
    data_off, crc_off, data_len = pk[-1]
    assert data_off + data_len == arena.nbytes
    assert gpu_ctx.verify_packets(bad, pk, 512, True) == (n_pkts - 1, (data_len - 1) // 512)


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_full_size_stream_1gib_roundtrip(gpu_ctx, bpc):
    """Config 3: 1 GiB stream, compute (write) then verify (read); every CRC word checked."""
    from libhdfs3_amd.engine import DeviceBuffer

    n = 1 << 30
    data = splitmix_bytes(n, 0xB10C + bpc)
    d = gpu_ctx.upload(data)
    nc = n // bpc
    dc = DeviceBuffer(4 * nc)
    gpu_ctx.compute_dev(d.ptr, n, bpc, dc.ptr)
    got = gpu_ctx.download(dc, 4 * nc)
    assert np.array_equal(got, oracle_compute(data, bpc))
    assert gpu_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, False) == -1
    for k in (0, nc // 2 + 3, nc - 1):
        pos = k * bpc + (k % bpc)
        flipped = np.array([data[pos] ^ 0x80], dtype=np.uint8)
        gpu_ctx.upload(flipped, d, offset=pos)
        assert gpu_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, False) == k
        gpu_ctx.upload(data[pos:pos + 1], d, offset=pos)
    assert gpu_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, True) == -1


@pytest.mark.parametrize("n", [(1 << 30) + (3 << 20) + 4096 * 5 + 300, (2 << 30) + 4096 * 13 + 4096 - 1])
def test_compute_held_stores_past_64_rounds_per_wave(gpu_ctx, n):
    """Compute at bpc 512 holds each wave's CRC words in VGPRs (up to 64 rounds) and stores
    them in bursts (kOptHoldStore). Sizes where waves run past one full hold (flush mid-stream),
    end on a partial 8-round group, and leave a slow region and a short tail: every word
    against the oracle."""
    from libhdfs3_amd.engine import DeviceBuffer

    bpc = 512
    data = splitmix_bytes(n, 0x5704E + n)
    d = gpu_ctx.upload(data)
    nc = (n + bpc - 1) // bpc
    dc = DeviceBuffer(4 * nc)
    gpu_ctx.compute_dev(d.ptr, n, bpc, dc.ptr)
    assert np.array_equal(gpu_ctx.download(dc, 4 * nc), oracle_compute(data, bpc))


@pytest.mark.parametrize("bpc,n", [(512, 128 << 20), (512, 512 << 20), (512, (512 << 20) + 4096),
                                   (512, (128 << 20) + 4096 * 3 + 517), (512, 4096 * 4096 * 7 + 4096 * 5),
                                   (512, 4096 * 33 + 100), (1024, 1 << 30), (1024, (1 << 30) + 4096),
                                   (1024, (128 << 20) + 4096 * 3 + 517), (1024, 4096 * 33 + 100),
                                   (2048, 2 << 30), (2048, (2 << 30) + 4096), (2048, (512 << 20) + 4096 * 5 + 1000),
                                   (2048, 4096 * 33 + 100),
                                   # bpc 4096 holds one word per round in lane k % 64 of one VGPR and
                                   # stores a line per 64 rounds (crc32c_wave.h:341-357): exactly
                                   # 64 / 128 rounds per wave, waves of 65 (kr > 0, a partial second
                                   # line) and 129 rounds with a slow region and a short tail
                                   (4096, 1 << 30), (4096, (1 << 30) + 4096 * 5 + 300), (4096, 2 << 30),
                                   (4096, (2 << 30) + 4096 * 13), (4096, 4096 * 33 + 100)])
@pytest.mark.parametrize("overlap", [False, True])
def test_compute_staged_words_boundaries(gpu_ctx, bpc, n, overlap):
    """Compute at bpc 512 / 1024 / 2048 over a contiguous block whose waves have at most bpc / 16
    rounds (32 / 64 / 128) stages every word in LDS and writes them as whole runs when the workgroup
    ends (kStageWords, crc32c_wave.h). Sizes at exactly the limit (512 MiB / 1 GiB / 2 GiB), one round
    past it (held stores at 512; at 1024 / 2048 a second window, written out after a workgroup barrier), waves with unequal round counts, a slow
    region and short tail, and a small grid: every word against the oracle, words poisoned first,
    barriered and overlapped (the solo last step)."""
    from libhdfs3_amd.engine import DeviceBuffer

    data = splitmix_bytes(n, 0x57A6E + n)
    d = gpu_ctx.upload(data)
    nc = (n + bpc - 1) // bpc
    dc = gpu_ctx.upload(np.full(4 * nc + 64, 0xA5, dtype=np.uint8))
    if overlap:  # the previous op on the stream is a compute whose inputs were ready (the ABI contract)
        other = DeviceBuffer(4 * nc)
        gpu_ctx.compute_dev(d.ptr, n, bpc, other.ptr)
    gpu_ctx.compute_dev(d.ptr, n, bpc, dc.ptr, overlap_previous=overlap)
    got = gpu_ctx.download(dc, 4 * nc + 64)
    assert np.array_equal(got[:4 * nc], oracle_compute(data, bpc))
    assert np.all(got[4 * nc:] == 0xA5)


@pytest.mark.parametrize("bpc", [8192, 12288, 32768, 65536])
def test_chunks_above_4k_pieces_and_combine(gpu_ctx, bpc):
    """bpc a multiple of 4096 above 4096: the round kernel's 4096-byte piece CRCs into the ctx
    scratch, then the combine kernel (launch_pieces). Whole chunks, a short tail (verified only with
    local semantics), a flipped bit in the first / middle / last chunk, and overlapped back-to-back
    computes of different blocks (the scratch alternates between two buffers): every word against
    the oracle."""
    from libhdfs3_amd.engine import DeviceBuffer

    # 8 / 16 / 64 KiB chunks take the pieces from 256 MiB per launch (kPiecesMinBytes), other
    # multiples of 4096 at every length
    for n in (bpc * 37, bpc * 37 + 4096 * 2 + 300, bpc * 2, bpc * 5 + 1, (64 << 20) + 5 * bpc + 77,
              (256 << 20) + 3 * bpc + 100):
        data = splitmix_bytes(n, 0xC0B1 + bpc + n)
        want = oracle_compute(data, bpc)
        d = gpu_ctx.upload(data)
        dc = gpu_ctx.upload(np.full(want.nbytes, 0xA5, dtype=np.uint8))
        gpu_ctx.compute_dev(d.ptr, n, bpc, dc.ptr)
        assert np.array_equal(gpu_ctx.download(dc, want.nbytes), want), (bpc, n)
        assert gpu_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, True) == -1
        nfull = n // bpc
        for k in (0, nfull // 2, nfull - 1):
            pos = k * bpc + (k * 977) % bpc
            gpu_ctx.upload(np.array([data[pos] ^ 0x10], dtype=np.uint8), d, offset=pos)
            assert gpu_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, False) == k, (bpc, n, k)
            gpu_ctx.upload(data[pos:pos + 1], d, offset=pos)
    # overlapped computes of 4 different blocks back to back, then every word
    blocks = [splitmix_bytes(bpc * 300 + 4096, 0xD0B1 + bpc + i) for i in range(4)]
    ds = [gpu_ctx.upload(b) for b in blocks]
    wants = [oracle_compute(b, bpc) for b in blocks]
    outs = [gpu_ctx.upload(np.full(w.nbytes, 0xA5, dtype=np.uint8)) for w in wants]
    for rep in range(3):
        for i in range(4):
            gpu_ctx.compute_dev(ds[i].ptr, blocks[i].nbytes, bpc, outs[i].ptr, overlap_previous=i > 0)
    for i in range(4):
        assert np.array_equal(gpu_ctx.download(outs[i], wants[i].nbytes), wants[i]), (bpc, i)


def test_block_128mib_async_result_and_launch_count(gpu_ctx):
    """Config 2: one 128 MiB block, 512 B chunks, device-resident async verify."""
    from libhdfs3_amd.engine import DeviceBuffer

    n = 128 << 20
    data = splitmix_bytes(n, 0x128)
    crc = oracle_compute(data, 512)
    d = gpu_ctx.upload(data)
    dc = gpu_ctx.upload(crc)
    res = DeviceBuffer(8 * 4)
    gpu_ctx.memset(res, 0, 32)
    before = gpu_ctx.kernel_launches
    gpu_ctx.verify_dev_async(d.ptr, n, 512, dc.ptr, res.ptr)
    bad = crc.copy()
    bad[4 * 1000 + 2] ^= 4
    bad[4 * 200000] ^= 4
    dbad = gpu_ctx.upload(bad)
    gpu_ctx.verify_dev_async(d.ptr, n, 512, dbad.ptr, res.ptr + 8)
    gpu_ctx.synchronize()
    words = gpu_ctx.download(res, 32).view(np.uint64)
    assert gpu_ctx.decode_result(int(words[0])) == -1 and words[0] == 0
    assert gpu_ctx.decode_result(int(words[1])) == 1000
    assert gpu_ctx.kernel_launches == before + 2


def test_bit_flip_every_position_in_one_chunk(gpu_ctx):
    """CRC32C detects every single-bit error: flip each of the 4096 bits of chunk 3."""
    data = splitmix_bytes(8 * 512, 5)
    crc = oracle_compute(data, 512)
    for byte in range(0, 512, 7):
        for bit in (0, 3, 7):
            bad = data.copy()
            bad[3 * 512 + byte] ^= 1 << bit
            assert gpu_ctx.verify(bad, 512, crc, True) == 3


@pytest.mark.parametrize("bpc,n", [(512, (512 << 20) + 4096 * 3 + 100), (512, 768 << 20), (512, 1 << 30),
                                   (512, (1 << 30) + 4096 * 4097 + 517), (1024, (1 << 30) + 4096 * 5),
                                   (1024, 1536 << 20), (2048, (2 << 30) + 4096)])
def test_compute_staged_windows_lab(lab_ctx, bpc, n):
    """Lab 130 (kLabStageWin): compute words staged in LDS past kStageMaxRounds too, each window of
    bpc / 16 rounds written out after the step that finishes it (two workgroup barriers), the last
    window at the workgroup's end. Launches one round past the limit, whole windows, partial last
    windows, unequal round counts and a short tail: every word against the oracle, poison kept."""
    from libhdfs3_amd import _native

    lib = _native.lab()
    try:
        lib.hdfs3x_set_variant(130)
        data = splitmix_bytes(n, 0x3A17 + bpc + n)
        d = lab_ctx.upload(data)
        nc = (n + bpc - 1) // bpc
        dc = lab_ctx.upload(np.full(4 * nc + 64, 0xA5, dtype=np.uint8))
        lab_ctx.compute_dev(d.ptr, n, bpc, dc.ptr)
        got = lab_ctx.download(dc, 4 * nc + 64)
        assert np.array_equal(got[:4 * nc], oracle_compute(data, bpc)), (bpc, n)
        assert np.all(got[4 * nc:] == 0xA5)
    finally:
        lib.hdfs3x_set_variant(0)


# every bit-exact variant (the diagnostic variant 77 gives wrong results on purpose); the lab
# variants exist for the round kernel's chunk sizes only
@pytest.mark.parametrize("variant,bpc", [(0, b) for b in (512, 1024, 2048, 4096, 8192)] +
                         [(v, b) for v in (92, 93, 94, 95, 115, 117) for b in (512, 1024, 2048, 4096)] +
                         [(115, 8192), (122, 512), (122, 2048)] +
                         [(157, b) for b in (512, 1024, 2048, 4096)])
def test_every_kernel_variant_matches_oracle(lab_ctx, variant, bpc):
    """All kernel designs kept for A/B (hdfs3x_set_variant) are parity-checked too:
    whole rounds, the slow region (len not a multiple of the 4 KiB round) and the tail."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import DeviceBuffer

    lib = _native.lab()
    try:
        lib.hdfs3x_set_variant(variant)
        for n in (4096 * 37, 4096 * 64 * 17 + 3 * bpc, 4096 * 300 + bpc * 2 + 77, bpc * 65 + 5):
            data = splitmix_bytes(n, variant * 1000 + bpc + n)
            want = oracle_compute(data, bpc)
            d = lab_ctx.upload(data)
            dc = DeviceBuffer(want.nbytes)
            lab_ctx.compute_dev(d.ptr, n, bpc, dc.ptr)
            assert np.array_equal(lab_ctx.download(dc, want.nbytes), want), (variant, bpc, n)
            assert lab_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, True) == -1
            nc = (n + bpc - 1) // bpc
            for k in (0, nc // 2, nc - 2):
                pos = k * bpc + 1
                lab_ctx.upload(np.array([data[pos] ^ 4], np.uint8), d, offset=pos)
                assert lab_ctx.verify_dev(d.ptr, n, bpc, dc.ptr, False) == k, (variant, bpc, n, k)
                lab_ctx.upload(data[pos:pos + 1], d, offset=pos)
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.parametrize("variant", [0, 92, 93, 94, 115, 117, 125, 132, 134, 137, 146, 157])
@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_round_kernel_variants_overlapped_match_oracle(lab_ctx, variant, bpc):
    """The round kernel's prefetch/last-step variants as they run in the bench: overlapped
    launches (the solo last step only runs there), sizes giving 1 to 9 rounds per wave so both
    loop copies of the solo form (an even and an odd number of full steps) run, a bad chunk
    located. 146: the per-wave stamps of tools/wave_spread.py leave the results alone."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import DeviceBuffer

    lib = _native.lab()
    sizes = [(8 << 20) + 4099, (48 << 20) + 3 * 4096, 64 << 20, (100 << 20) + 777, (132 << 20) + bpc]
    try:
        lib.hdfs3x_set_variant(variant)
        res = DeviceBuffer(8 * 2 * len(sizes))
        lab_ctx.memset(res, 0, 8 * 2 * len(sizes))
        blocks, bads = [], []
        for i, n in enumerate(sizes):
            data = splitmix_bytes(n, 7000 + variant * 10 + i + bpc)
            blocks.append((lab_ctx.upload(data), lab_ctx.upload(oracle_compute(data, bpc)), n, data))
            nc = n // bpc
            bads.append((nc - 1) if i % 2 else (nc // 3 + i))
        lab_ctx.synchronize()
        for i, (d, c, n, _) in enumerate(blocks):  # one overlapped chain over clean blocks
            lab_ctx.verify_dev_async(d.ptr, n, bpc, c.ptr, res.ptr + 16 * i, overlap_previous=i > 0)
        lab_ctx.synchronize()
        for (d, _, _, data), bad in zip(blocks, bads):
            pos = bad * bpc + 7
            lab_ctx.upload(np.array([data[pos] ^ 0x10], np.uint8), d, offset=pos)
        lab_ctx.synchronize()
        for i, (d, c, n, _) in enumerate(blocks):  # and over the corrupted ones
            lab_ctx.verify_dev_async(d.ptr, n, bpc, c.ptr, res.ptr + 16 * i + 8, overlap_previous=i > 0)
        lab_ctx.synchronize()
        words = lab_ctx.download(res, 16 * len(sizes)).view(np.uint64)
        for i in range(len(sizes)):
            assert lab_ctx.decode_result(int(words[2 * i])) == -1, (variant, bpc, i)
            assert lab_ctx.decode_result(int(words[2 * i + 1])) == bads[i], (variant, bpc, i)
    finally:
        lib.hdfs3x_set_variant(0)


def test_beyond_4gib_single_call_64bit_addressing(gpu_ctx):
    """Maximum sizes: one verify over 4.5 GiB (the reference's Checksum::update takes an int,
    so its callers never exceed 2 GiB per call; the batch API takes size_t). Distinct data
    everywhere (aliasing past 4 GiB would read different bytes); words around the 4 GiB mark
    are checked against the oracle and bit flips past it are located exactly. Uses only the
    C-ABI: torch bundles its own HIP runtime, so it is not mixed in after ours."""
    from libhdfs3_amd.engine import DeviceBuffer

    bpc, piece = 512, 256 << 20
    n = (9 << 29) + 3 * bpc + 100  # 4.5 GiB + ragged tail
    dbuf = DeviceBuffer(n)
    host = {}
    for i, off in enumerate(range(0, n, piece)):
        part = splitmix_bytes(min(piece, n - off), 0xB16B00B5 + i)
        gpu_ctx.upload(part, dbuf, offset=off)
        host[off] = part

    def host_bytes(start, length):
        out = np.empty(length, np.uint8)
        pos = 0
        while pos < length:
            off = (start + pos) // piece * piece
            k = start + pos - off
            take = min(length - pos, host[off].nbytes - k)
            out[pos:pos + take] = host[off][k:k + take]
            pos += take
        return out

    nch = (n + bpc - 1) // bpc
    crc = DeviceBuffer(4 * nch)
    gpu_ctx.compute_dev(dbuf.ptr, n, bpc, crc.ptr)
    assert gpu_ctx.verify_dev(dbuf.ptr, n, bpc, crc.ptr, True) == -1
    for start in (0, (1 << 32) - 8192, (1 << 32) + 4096 * 7, n - n % bpc - 8 * bpc):
        start -= start % bpc
        length = min(20 * bpc, n - start)
        want = oracle_compute(host_bytes(start, length), bpc)
        got = gpu_ctx.download(crc, want.nbytes, offset=4 * (start // bpc))
        assert np.array_equal(got, want), start
    for pos in ((1 << 32) + 12345, n - 50):
        orig = host_bytes(pos, 1)
        gpu_ctx.upload(orig ^ 1, dbuf, offset=pos)
        assert gpu_ctx.verify_dev(dbuf.ptr, n, bpc, crc.ptr, True) == pos // bpc
        gpu_ctx.upload(orig, dbuf, offset=pos)
    dbuf.free()


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_overlapped_verify_chain_matches_oracle(gpu_ctx, bpc):
    """HDFS3_LAUNCH_OVERLAP_PREVIOUS: a chain of verifies whose launches overlap (AQL packets
    without the barrier bit) gives every block exactly its own result: clean blocks 0, the
    corrupted block its first bad chunk, over many launches and ragged block lengths."""
    from libhdfs3_amd.engine import DeviceBuffer

    nblk, reps = 6, 8
    lens = [(8 << 20) + (i * 4099 if i % 2 else 0) for i in range(nblk)]
    blocks = []
    for i, n in enumerate(lens):
        data = splitmix_bytes(n, 0xC4A1 + i + bpc)
        want = oracle_compute(data, bpc)
        blocks.append((gpu_ctx.upload(data), gpu_ctx.upload(want), n, data))
    bad_blk, bad_chunk = 3, (lens[3] // bpc) // 2 + 5
    pos = bad_chunk * bpc + 11
    gpu_ctx.upload(np.array([blocks[bad_blk][3][pos] ^ 0x40], np.uint8), blocks[bad_blk][0], offset=pos)
    res = DeviceBuffer(8 * nblk * reps)
    gpu_ctx.memset(res, 0, 8 * nblk * reps)
    gpu_ctx.synchronize()
    for r in range(reps):
        for i, (d, c, n, _) in enumerate(blocks):
            gpu_ctx.verify_dev_async(d.ptr, n, bpc, c.ptr, res.ptr + 8 * (r * nblk + i), check_short_tail=True,
                                     overlap_previous=(r, i) != (0, 0))
    gpu_ctx.synchronize()
    words = gpu_ctx.download(res, 8 * nblk * reps).view(np.uint64)
    for r in range(reps):
        for i in range(nblk):
            got = gpu_ctx.decode_result(int(words[r * nblk + i]))
            assert got == (bad_chunk if i == bad_blk else -1), (r, i, got)


@pytest.mark.parametrize("bpc", [512, 2048, 4096, 516, 8192])
def test_overlapped_compute_chain_matches_oracle(gpu_ctx, bpc):
    """hdfs3_crc32c_compute_dev_async_ex with HDFS3_LAUNCH_OVERLAP_PREVIOUS: a chain of compute
    launches over resident blocks (ragged lengths, each writing its own CRC array, then the
    chain once more into fresh arrays) gives every block exactly the oracle's words. Chunk sizes
    the wave kernel does not take (516, 8192) accept the flag and launch barriered."""
    from libhdfs3_amd.engine import DeviceBuffer

    nblk = 6
    lens = [(8 << 20) + (i * 4099 if i % 2 else 0) for i in range(nblk)]
    blocks = []
    for i, n in enumerate(lens):
        data = splitmix_bytes(n, 0xC0DE + i + bpc)
        want = oracle_compute(data, bpc)
        outs = [DeviceBuffer(want.nbytes) for _ in range(2)]
        for o in outs:
            gpu_ctx.memset(o, 0xA5, want.nbytes)
        blocks.append((gpu_ctx.upload(data), outs, n, want))
    gpu_ctx.synchronize()
    for r in range(2):
        for i, (d, outs, n, _) in enumerate(blocks):
            gpu_ctx.compute_dev(d.ptr, n, bpc, outs[r].ptr, overlap_previous=(r, i) != (0, 0))
    gpu_ctx.synchronize()
    for i, (_, outs, _, want) in enumerate(blocks):
        for r in range(2):
            assert np.array_equal(gpu_ctx.download(outs[r], want.nbytes), want), (i, r)


def test_overlapped_chain_at_bench_size(gpu_ctx):
    """BASELINE configs[1] size through the bench's launch mode: 8 x 128 MiB blocks verified by
    overlapped single-block launches, three passes; a flipped bit in the LAST chunk of block 5
    is reported in every pass, every other block is clean."""
    from libhdfs3_amd.engine import DeviceBuffer

    n, nblk, passes = 128 << 20, 8, 3
    blocks = []
    for i in range(nblk):
        data = splitmix_bytes(n, 0xB16 + i)
        blocks.append((gpu_ctx.upload(data), gpu_ctx.upload(oracle_compute(data, 512)), data))
    last = n // 512 - 1
    pos = last * 512 + 500
    gpu_ctx.upload(np.array([blocks[5][2][pos] ^ 1], np.uint8), blocks[5][0], offset=pos)
    res = DeviceBuffer(8 * nblk * passes)
    gpu_ctx.memset(res, 0, 8 * nblk * passes)
    k = 0
    for p in range(passes):
        for i, (d, c, _) in enumerate(blocks):
            gpu_ctx.verify_dev_async(d.ptr, n, 512, c.ptr, res.ptr + 8 * k, overlap_previous=k > 0)
            k += 1
    gpu_ctx.synchronize()
    words = gpu_ctx.download(res, 8 * nblk * passes).view(np.uint64)
    got = [gpu_ctx.decode_result(int(w)) for w in words]
    assert got == [last if i % nblk == 5 else -1 for i in range(nblk * passes)]


@pytest.mark.parametrize("n", [(2 << 20) + 1, (4 << 20) + 3, (16 << 20) + (4 << 20) + 2])
def test_host_api_pageable_staging_every_byte(gpu_ctx, n):
    """The host-buffer API stages pageable buffers through the host copy pool (split for copies
    of 2 MiB or more): lengths that split unevenly must compute and verify every chunk,
    including the last, exactly as the oracle does."""
    data = splitmix_bytes(n, n)
    for bpc in (512, 4096):
        want = oracle_compute(data, bpc)
        assert np.array_equal(gpu_ctx.compute(data, bpc), want), (n, bpc)
        assert gpu_ctx.verify(data, bpc, want, True) == -1
        bad = data.copy()
        bad[-1] ^= 0x80  # the very last byte lives in the piece that used to be dropped
        assert gpu_ctx.verify(bad, bpc, want, True) == oracle_verify(bad, bpc, want, True) == (n - 1) // bpc


def test_host_api_random_sizes_and_offsets(gpu_ctx):
    """Host-buffer API over random lengths (1-40 MiB: one to three 16 MiB staging segments,
    copies split over the copy pool) at random offsets into pageable numpy buffers, random
    chunk sizes: every word the oracle's, and a flip at a random position found at its chunk."""
    rng = np.random.default_rng(20261017)
    base = splitmix_bytes((41 << 20) + 64, 0x5151)
    for _ in range(12):
        n = int(rng.integers(1 << 20, 40 << 20))
        off = int(rng.integers(0, 64))
        bpc = int(rng.choice([512, 1024, 2048, 4096, 516]))
        data = base[off:off + n]
        want = oracle_compute(data, bpc)
        assert np.array_equal(gpu_ctx.compute(data, bpc), want), (n, off, bpc)
        pos = int(rng.integers(0, n))
        bad = data.copy()
        bad[pos] ^= 0x02
        assert gpu_ctx.verify(bad, bpc, want, True) == pos // bpc, (n, off, bpc, pos)


@pytest.mark.parametrize("variant", [0, 92, 93, 94, 95, 122, 128, 157])
@pytest.mark.parametrize("bpc", [512, 1024, 4096])
def test_round_kernel_variants_overlapped_compute_match_oracle(lab_ctx, variant, bpc):
    """Compute-mode variants of the round kernel (held stores or not, solo last step or not) as
    overlapped chains: sizes giving 1 to 9 rounds per wave (both loop copies of the solo form, a
    partial octet of held words), arrays poisoned with 0xA5 first, every word against the oracle."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import DeviceBuffer

    lib = _native.lab()
    sizes = [(8 << 20) + 4099, (48 << 20) + 3 * 4096, 64 << 20, (100 << 20) + 777, (132 << 20) + bpc]
    try:
        lib.hdfs3x_set_variant(variant)
        blocks = []
        for i, n in enumerate(sizes):
            data = splitmix_bytes(n, 8100 + variant * 10 + i + bpc)
            want = oracle_compute(data, bpc)
            out = DeviceBuffer(want.nbytes)
            lab_ctx.memset(out, 0xA5, want.nbytes)
            blocks.append((lab_ctx.upload(data), out, n, want))
        lab_ctx.synchronize()
        for i, (d, out, n, _) in enumerate(blocks):
            lab_ctx.compute_dev(d.ptr, n, bpc, out.ptr, overlap_previous=i > 0)
        lab_ctx.synchronize()
        for i, (_, out, _, want) in enumerate(blocks):
            assert np.array_equal(lab_ctx.download(out, want.nbytes), want), (variant, bpc, i)
    finally:
        lib.hdfs3x_set_variant(0)
