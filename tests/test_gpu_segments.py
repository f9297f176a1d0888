"""GPU parity of the segmented wave kernel: the multi-block batch API
(hdfs3_crc32c_{verify,compute}_blocks_dev*) and the packet API's fast path. Every block of
a batch must get exactly the words and first-bad chunk it gets alone (oracle per block);
the packet path must agree with the chunk-per-lane packet kernel (variant 17) and the
oracle, including short tails (remote vs local semantics) and odd sizes."""
import numpy as np
import pytest

from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu


def make_blocks(ctx, sizes, bpc, seed, pad=0):
    from libhdfs3_amd.engine import DeviceBuffer

    blocks, keep, datas = [], [], []
    for i, n in enumerate(sizes):
        d = splitmix_bytes(n, seed + i)
        db = DeviceBuffer(n + pad + 16)
        if n:
            ctx.upload(d, db, offset=pad)
        cb = DeviceBuffer(4 * ((n + bpc - 1) // bpc) + 8)
        blocks.append((db.ptr + pad, cb.ptr, n))
        keep += [db, cb]
        datas.append(d)
    return blocks, keep, datas


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096])
@pytest.mark.parametrize("sizes", [
    [1 << 20] * 8,                                     # uniform: direct unit -> segment map
    [4096 * 5 + 700, 0, 300, 1 << 20, 4096, 8192 + 1],  # ragged: binary search, slow pass, empty
    [65536] * 37 + [1000],                              # packet-like
    [1 << 20] * 5 + [(1 << 20) - 4096 * 3 - 300],       # equal blocks + shorter last: wave kernel table mode
    [1 << 18] * 16,                                     # the table mode's 16-block limit
])
def test_blocks_batch_matches_per_block_oracle(gpu_ctx, bpc, sizes):
    blocks, keep, datas = make_blocks(gpu_ctx, sizes, bpc, bpc * 13 + len(sizes))
    gpu_ctx.compute_blocks_dev(blocks, bpc)
    for (d, c, n), data in zip(blocks, datas):
        want = oracle_compute(data, bpc)
        assert np.array_equal(gpu_ctx.download(c, want.nbytes), want), (bpc, n)
    assert gpu_ctx.verify_blocks_dev(blocks, bpc, True) == (-1, -1)
    # corrupt two blocks: the lexicographically first (block, chunk) is reported
    nz = [i for i, n in enumerate(sizes) if n >= bpc]
    hit = [nz[-1], nz[len(nz) // 2]]
    for bi in hit:
        d, c, n = blocks[bi]
        pos = (n // bpc - 1) * bpc + 5
        gpu_ctx.upload(np.array([datas[bi][pos] ^ 1], np.uint8), d, offset=pos)
    first = min(hit)
    assert gpu_ctx.verify_blocks_dev(blocks, bpc) == (first, sizes[first] // bpc - 1)


def test_short_tail_semantics_and_async(gpu_ctx):
    import ctypes

    from libhdfs3_amd.engine import DeviceBuffer

    bpc = 512
    sizes = [4096 * 3 + 100, 8192, 4096 * 2 + 512 + 33]
    blocks, keep, datas = make_blocks(gpu_ctx, sizes, bpc, 77)
    gpu_ctx.compute_blocks_dev(blocks, bpc)
    d, c, n = blocks[2]
    tail = n - 10  # inside block 2's short tail
    gpu_ctx.upload(np.array([datas[2][tail] ^ 1], np.uint8), d, offset=tail)
    assert gpu_ctx.verify_blocks_dev(blocks, bpc, check_short_tail=False) == (-1, -1)
    assert gpu_ctx.verify_blocks_dev(blocks, bpc, check_short_tail=True) == (2, n // bpc)
    res = DeviceBuffer(8)
    gpu_ctx.memset(res, 0, 8)
    gpu_ctx.verify_blocks_dev_async(blocks, bpc, res.ptr, check_short_tail=True)
    gpu_ctx.synchronize()
    word = int(gpu_ctx.download(res, 8).view(np.uint64)[0])
    key = gpu_ctx.decode_result(word)
    assert (key >> 32, key & 0xFFFFFFFF) == (2, n // bpc)


def test_unaligned_and_odd_bpc_fall_back_with_same_keys(gpu_ctx):
    for bpc, pad in [(512, 3), (100, 0)]:
        sizes = [5000, 64 * 1024 + 7, 1234]
        blocks, keep, datas = make_blocks(gpu_ctx, sizes, bpc, 900 + bpc, pad=pad)
        gpu_ctx.compute_blocks_dev(blocks, bpc)
        for (d, c, n), data in zip(blocks, datas):
            want = oracle_compute(data, bpc)
            assert np.array_equal(gpu_ctx.download(c, want.nbytes), want), (bpc, pad, n)
        d, c, n = blocks[1]
        gpu_ctx.upload(np.array([datas[1][777] ^ 4], np.uint8), d, offset=777)
        assert gpu_ctx.verify_blocks_dev(blocks, bpc) == (1, 777 // bpc)


def test_many_small_blocks_binary_search(gpu_ctx):
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(0, 40000, size=300)]
    blocks, keep, datas = make_blocks(gpu_ctx, sizes, 512, 4242)
    gpu_ctx.compute_blocks_dev(blocks, 512)
    for (d, c, n), data in zip(blocks[::17], datas[::17]):
        want = oracle_compute(data, 512)
        assert np.array_equal(gpu_ctx.download(c, want.nbytes), want)
    assert gpu_ctx.verify_blocks_dev(blocks, 512, True) == (-1, -1)


@pytest.mark.parametrize("bpc", [512, 4096])
def test_packet_fast_path_agrees_with_packet_kernel(lab_ctx, bpc):
    from libhdfs3_amd import _native

    lib = _native.lab()
    rng = np.random.default_rng(bpc)
    pk, parts, off = [], [], 0
    lens = [65536] * 40 + [65536 - 100, 777, 4096, 20000, 65536]
    for i, n in enumerate(lens):
        data = splitmix_bytes(n, 3000 + i)
        crc = oracle_compute(data, bpc)
        pad = (-(off + crc.nbytes)) % 16
        parts += [np.zeros(pad, np.uint8), crc, data]
        pk.append((off + pad + crc.nbytes, off + pad, n))
        off += pad + crc.nbytes + n
    arena = np.concatenate(parts)
    d = lab_ctx.upload(arena)
    try:
        for v in (0, 17):
            lib.hdfs3x_set_variant(v)
            assert lab_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc) == (-1, -1)
        for trial in range(4):
            bad = arena.copy()
            p = int(rng.integers(0, len(pk)))
            q = int(rng.integers(0, pk[p][2]))
            bad[pk[p][0] + q] ^= 0x80
            lab_ctx.upload(bad, d)
            got = []
            for v in (0, 17):
                lib.hdfs3x_set_variant(v)
                got.append((lab_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc),
                            lab_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc, True)))
            assert got[0] == got[1], (p, q, got)
            chunk = q // bpc
            short = pk[p][2] % bpc and chunk == pk[p][2] // bpc
            assert got[0][1] == (p, chunk)
            assert got[0][0] == ((-1, -1) if short else (p, chunk))
        # compute through the fast path writes the same words
        lib.hdfs3x_set_variant(0)
        blank = arena.copy()
        for data_off, crc_off, n in pk:
            blank[crc_off:crc_off + 4 * ((n + bpc - 1) // bpc)] = 0
        lab_ctx.upload(blank, d)
        lab_ctx.compute_packets_dev(d.ptr, arena.nbytes, pk, bpc)
        assert np.array_equal(lab_ctx.download(d, arena.nbytes), arena)
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_single_segment_batch(lab_ctx, bpc):
    """One block through the batch API (segmented kernel with one segment). Words and first
    bad chunk."""
    from libhdfs3_amd import _native

    lib = _native.lab()
    n = 4096 * 1000 + 3 * bpc + 77
    try:
        lib.hdfs3x_set_variant(0)
        blocks, keep, datas = make_blocks(lab_ctx, [n], bpc, 4900 + bpc)
        lab_ctx.compute_blocks_dev(blocks, bpc)
        d, c, _ = blocks[0]
        want = oracle_compute(datas[0], bpc)
        assert np.array_equal(lab_ctx.download(c, want.nbytes), want)
        assert lab_ctx.verify_blocks_dev(blocks, bpc, True) == (-1, -1)
        k = (n // bpc) // 2
        pos = k * bpc + 5
        lab_ctx.upload(np.array([datas[0][pos] ^ 8], np.uint8), keep[0], offset=pos)
        assert lab_ctx.verify_blocks_dev(blocks, bpc, False) == (0, k)
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.gpu
@pytest.mark.parametrize("bpc", [512, 4096])
@pytest.mark.parametrize("last_len", [65536, 65536 - 300, 100])
def test_constant_pitch_packets_without_descriptors(lab_ctx, bpc, last_len):
    """Packets at one pitch in one arena (the reader's and writer's layout) go to the wave
    kernel's pitch mode (variant 0) with no descriptor array. Same keys and words as the
    segmented kernel's strided launch (A/B variant 53), with descriptors (variant 52) and as
    the packet kernel (variant 17)."""
    from libhdfs3_amd import _native

    lib = _native.lab()
    rng = np.random.default_rng(bpc + last_len)
    n, plen = 40, 65536
    crc_bytes = 4 * (plen // bpc)
    pitch = 31 + 1 + crc_bytes + plen  # header-sized gap keeps data 16 B aligned below
    pitch += (-pitch) % 16
    arena = np.zeros(n * pitch, np.uint8)
    pk = []
    for i in range(n):
        dl = plen if i + 1 < n else last_len
        data = splitmix_bytes(dl, 7000 + i)
        crc = oracle_compute(data, bpc)
        crc_off = i * pitch + 32
        data_off = crc_off + crc_bytes
        arena[crc_off:crc_off + crc.nbytes] = crc
        arena[data_off:data_off + dl] = data
        pk.append((data_off, crc_off, dl))
    d = lab_ctx.upload(arena)
    try:
        for v in (0, 53, 52, 17):
            lib.hdfs3x_set_variant(v)
            assert lab_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc, True) == (-1, -1), v
        for _ in range(3):
            p = int(rng.integers(0, n))
            q = int(rng.integers(0, pk[p][2]))
            bad = arena.copy()
            bad[pk[p][0] + q] ^= 0x20
            lab_ctx.upload(bad, d)
            got = set()
            for v in (0, 53, 52, 17):
                lib.hdfs3x_set_variant(v)
                got.add(lab_ctx.verify_packets_dev(d.ptr, arena.nbytes, pk, bpc, True))
            assert got == {(p, q // bpc)}, (p, q, got)
        blank = arena.copy()
        for data_off, crc_off, dl in pk:
            blank[crc_off:data_off] = 0
        for v in (0, 53, 52):
            lib.hdfs3x_set_variant(v)
            lab_ctx.upload(blank, d)
            lab_ctx.compute_packets_dev(d.ptr, arena.nbytes, pk, bpc)
            assert np.array_equal(lab_ctx.download(d, arena.nbytes), arena), v
    finally:
        lib.hdfs3x_set_variant(0)


@pytest.mark.gpu
@pytest.mark.parametrize("bpc", [512, 2048])
@pytest.mark.parametrize("last", [1 << 20, (1 << 20) - 4096 * 7 - 100, 300])
def test_strided_blocks_take_the_wave_kernel(lab_ctx, bpc, last):
    """Blocks of one 2-D arrangement (data at a constant stride, words at another; the bench's
    [blocks, bytes] tensor) go to the wave kernel's pitch mode with its own word pitch (variant
    0); the segmented kernel (variant 54) and the oracle must agree on every word and key. Compute
    writes the words densely into the ctx's scratch and scatters them (variant 55: in place); no
    byte between the word regions may change."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import DeviceBuffer

    lib = _native.lab()
    n, L = 6, 1 << 20
    dstride, wstride = L + 4096, 4 * (L // bpc) + 64  # both padded: strides differ from sizes
    datas = [splitmix_bytes(L if i + 1 < n else last, 300 + i + bpc) for i in range(n)]
    dbuf, wbuf = DeviceBuffer(n * dstride), DeviceBuffer(n * wstride)
    for i, d in enumerate(datas):
        lab_ctx.upload(d, dbuf, offset=i * dstride)
    blocks = [(dbuf.ptr + i * dstride, wbuf.ptr + i * wstride, d.size) for i, d in enumerate(datas)]
    try:
        for v in (0, 54, 55):
            lib.hdfs3x_set_variant(v)
            lab_ctx.memset(wbuf, 0xA5, n * wstride)
            lab_ctx.compute_blocks_dev(blocks, bpc)
            got = lab_ctx.download(wbuf, n * wstride)
            for i, d in enumerate(datas):
                want = oracle_compute(d, bpc)
                assert np.array_equal(got[i * wstride:i * wstride + want.nbytes], want), (v, i)
                end = (i + 1) * wstride if i + 1 < n else n * wstride
                assert (got[i * wstride + want.nbytes:end] == 0xA5).all(), (v, i)
            assert lab_ctx.verify_blocks_dev(blocks, bpc, True) == (-1, -1), v
        for bi, pos in [(n - 1, last - 1), (2, 4096 * 9 + 3), (0, 0)]:
            lab_ctx.upload(np.array([datas[bi][pos] ^ 0x80], np.uint8), dbuf, offset=bi * dstride + pos)
            got = set()
            for v in (0, 54, 55):
                lib.hdfs3x_set_variant(v)
                got.add(lab_ctx.verify_blocks_dev(blocks, bpc, True))
            assert got == {(bi, pos // bpc)}, (bi, pos, got)
    finally:
        lib.hdfs3x_set_variant(0)
