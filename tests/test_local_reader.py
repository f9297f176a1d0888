"""GPU tests of the short-circuit reader (hdfs3_local_reader) against .meta files written
here in the datanode layout (BE16 version 1 | u8 type | BE32 bpc | BE32 CRC per chunk,
LocalBlockReader.cpp:40-121). Reference semantics checked (LocalBlockReader.cpp):
every chunk including the short tail is verified (:149-161, unlike the remote reader);
nothing of the input.localread.default.buffersize buffer holding a bad chunk is
returned (readAndVerify verifies the whole buffer first, :138-163, :197-214); an offset
skips to the chunk boundary and re-verifies that chunk (:232-263); NULL type reads
without verification; a version other than 1 is an error (:70-76)."""
import errno
import struct

import numpy as np
import pytest

from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["default", "mmap", "pread"])
def staging(request, monkeypatch):
    """Every staging of the short-circuit reader must deliver identical results: default
    (verified windows pread in parallel into pinned arenas; unverified reads copied straight
    out of the mmap'd file), HDFS3_LOCAL_MMAP=1 (verified windows registered and DMA'd from the
    mapping) and HDFS3_LOCAL_MMAP=0 (no mapping at all)."""
    if request.param == "default":
        monkeypatch.delenv("HDFS3_LOCAL_MMAP", raising=False)
    else:
        monkeypatch.setenv("HDFS3_LOCAL_MMAP", "1" if request.param == "mmap" else "0")
    return request.param


def write_block(tmp_path, name, data, bpc=512, ctype=2, version=1, crc=None):
    d, m = tmp_path / f"{name}", tmp_path / f"{name}.meta"
    d.write_bytes(data.tobytes())
    words = b"" if ctype == 0 else (oracle_compute(data, bpc) if crc is None else crc).tobytes()
    m.write_bytes(struct.pack(">hBI", version, ctype, bpc) + words)
    return str(d), str(m)


def read(d, m, **kw):
    from libhdfs3_amd.engine import LocalBlockReader

    with LocalBlockReader(d, m, **kw) as r:
        out = r.read_all(1 << 30)
        return out, r.stats()


@pytest.mark.parametrize("bpc", [512, 4096])
def test_full_and_offset_reads(tmp_path, bpc, staging):
    data = splitmix_bytes(3 * (1 << 20) + 777, bpc)
    d, m = write_block(tmp_path, f"blk_{bpc}", data, bpc)
    out, st = read(d, m, buffer_size=1 << 18, window_buffers=3)
    assert np.array_equal(out, data)
    assert st["bytes_per_checksum"] == bpc and st["checksum_type"] == 2 and st["gpu_batches"] >= 4
    assert (st["mapped_windows"] == st["gpu_batches"]) if staging == "mmap" else st["mapped_windows"] == 0
    for off in [1, bpc - 1, bpc + 5, 1 << 20, data.nbytes - 10, data.nbytes]:
        out, _ = read(d, m, offset=off)
        assert np.array_equal(out, data[off:]), off
    out, _ = read(d, m, num_bytes=245 * 4096)  # a chunk-aligned prefix of the block
    assert np.array_equal(out, data[:245 * 4096])
    # a length that cuts a chunk short makes the last chunk's stored word (over the whole
    # on-disk chunk) mismatch — readAndVerify checks bufferSize % chunkSize bytes (:145-151)
    from libhdfs3_amd._native import Hdfs3CrcError
    with pytest.raises(Hdfs3CrcError):
        read(d, m, num_bytes=245 * 4096 + 100)


@pytest.mark.parametrize("where", [0, 300_000, (1 << 20) + 5, 3 * (1 << 20) + 700])
def test_corruption_withholds_the_whole_local_buffer(tmp_path, where, staging):
    from libhdfs3_amd.engine import LocalBlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    bpc, buf = 512, 1 << 18
    data = splitmix_bytes(3 * (1 << 20) + 777, 9)
    crc = oracle_compute(data, bpc)
    bad = data.copy()
    bad[where] ^= 0x20  # the last position is inside the short tail chunk: checked locally
    d, m = write_block(tmp_path, "blk_bad", bad, bpc, crc=crc)
    with LocalBlockReader(d, m, buffer_size=buf, window_buffers=2) as r:
        out = np.zeros(data.nbytes, np.uint8)
        pos = 0
        with pytest.raises(Hdfs3CrcError) as ei:
            while True:
                n = r.read_into(out, pos, 100_000)
                assert n > 0
                pos += n
        assert ei.value.rc == -errno.EIO and "ChecksumException" in str(ei.value)
    assert pos == where // buf * buf
    assert np.array_equal(out[:pos], data[:pos])


def test_corrupt_meta_word_and_offset_recheck(tmp_path, staging):
    from libhdfs3_amd.engine import LocalBlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    data = splitmix_bytes(1 << 20, 10)
    crc = oracle_compute(data, 512).copy()
    crc[4 * 100] ^= 1  # chunk 100 = bytes [51200, 51712)
    d, m = write_block(tmp_path, "blk_meta", data, crc=crc)
    with pytest.raises(Hdfs3CrcError):
        read(d, m)
    # a read starting inside chunk 100 still verifies that whole chunk (skip aligns down)
    with pytest.raises(Hdfs3CrcError):
        read(d, m, offset=51300)
    out, _ = read(d, m, offset=51712)  # past it: fine
    assert np.array_equal(out, data[51712:])


def test_null_type_and_verify_off_read_without_checking(tmp_path, staging):
    data = splitmix_bytes(500_000, 11)
    bad = data.copy()
    bad[1234] ^= 1
    d, m = write_block(tmp_path, "blk_null", bad, ctype=0)
    out, st = read(d, m)
    assert np.array_equal(out, bad) and st["checksum_type"] == 0
    d, m = write_block(tmp_path, "blk_off", bad, crc=oracle_compute(data, 512))
    out, _ = read(d, m, verify=False)
    assert np.array_equal(out, bad)


def test_bad_version_is_an_error(tmp_path):
    from libhdfs3_amd._native import Hdfs3CrcError

    data = splitmix_bytes(4096, 12)
    d, m = write_block(tmp_path, "blk_v2", data, version=2)
    with pytest.raises(Hdfs3CrcError) as ei:
        read(d, m)
    assert ei.value.rc == -errno.EIO and "version" in str(ei.value)


def test_crc32_meta_is_verified_with_crc32c_like_the_reference(tmp_path):
    """LocalBlockReader.cpp:85-98: CHECKSUM_CRC32 and CHECKSUM_CRC32C both select the CRC32C
    engine. A block whose meta declares type 1 with zlib words therefore fails at its first
    chunk (ChecksumException -> EIO, nothing delivered) exactly where the oracle's CRC32C
    verify of those words fails; type-1 meta holding CRC32C words reads clean."""
    from libhdfs3_amd._native import Hdfs3CrcError
    from libhdfs3_amd.engine import LocalBlockReader
    from util import oracle_compute_crc32, oracle_verify

    data = splitmix_bytes(1_000_003, 13)
    zwords = oracle_compute_crc32(data, 512)
    assert oracle_verify(data, 512, zwords, True) == 0  # the reference's verdict: chunk 0
    d, m = write_block(tmp_path, "blk_crc32", data, ctype=1, crc=zwords)
    with LocalBlockReader(d, m, buffer_size=1 << 18) as r:
        out = np.zeros(data.nbytes, np.uint8)
        with pytest.raises(Hdfs3CrcError) as ei:
            r.read_into(out)
        assert ei.value.rc == -errno.EIO and "ChecksumException" in str(ei.value)
        assert r.stats()["checksum_type"] == 1
    d, m = write_block(tmp_path, "blk_crc32_c", data, ctype=1)  # CRC32C words, type byte 1
    out, st = read(d, m)
    assert np.array_equal(out, data) and st["checksum_type"] == 1


def test_crc32_meta_zlib_opt_in(tmp_path):
    """HDFS3_LOCAL_CRC32_AS_ZLIB (opt-in departure from the reference): type-1 meta verified
    with the zlib polynomial it declares."""
    from libhdfs3_amd._native import Hdfs3CrcError
    from util import oracle_compute_crc32

    data = splitmix_bytes(1_000_003, 13)
    d, m = write_block(tmp_path, "blk_crc32", data, ctype=1, crc=oracle_compute_crc32(data, 512))
    out, st = read(d, m, crc32_as_zlib=True)
    assert np.array_equal(out, data) and st["checksum_type"] == 1
    bad = data.copy()
    bad[-1] ^= 1  # short tail: checked locally
    d, m = write_block(tmp_path, "blk_crc32_bad", bad, ctype=1, crc=oracle_compute_crc32(data, 512))
    with pytest.raises(Hdfs3CrcError):
        read(d, m, crc32_as_zlib=True)


@pytest.mark.parametrize("bpc", [1, 3, 513, 517])
def test_any_positive_bytes_per_checksum(tmp_path, bpc):
    """The reference accepts any bytesPerChecksum > 0 from the meta header (:110-115): chunk
    sizes that are not a multiple of 4 verify, and a flipped bit is caught at the chunk the
    oracle names (the whole local buffer holding it withheld)."""
    from libhdfs3_amd._native import Hdfs3CrcError
    from libhdfs3_amd.engine import LocalBlockReader
    from util import oracle_verify

    n = 200_000 + bpc * 7 + 5
    data = splitmix_bytes(n, 100 + bpc)
    d, m = write_block(tmp_path, f"blk_{bpc}", data, bpc)
    out, st = read(d, m, buffer_size=1 << 16)
    assert np.array_equal(out, data) and st["bytes_per_checksum"] == bpc
    out, _ = read(d, m, offset=12345)
    assert np.array_equal(out, data[12345:])
    crc = oracle_compute(data, bpc)
    bad = data.copy()
    where = 150_001
    bad[where] ^= 4
    k = oracle_verify(bad, bpc, crc, True)
    assert k == where // bpc
    d, m = write_block(tmp_path, f"blk_{bpc}_bad", bad, bpc, crc=crc)
    buf = (65536 + bpc - 1) // bpc * bpc  # chunk-rounded local buffer (:112-116)
    with LocalBlockReader(d, m, buffer_size=1 << 16) as r:
        got = np.zeros(n, np.uint8)
        pos = 0
        with pytest.raises(Hdfs3CrcError):
            while True:
                pos += r.read_into(got, pos, 50_000)
    assert pos == (k * bpc) // buf * buf and np.array_equal(got[:pos], data[:pos])


def test_local_buffer_above_1gib_is_rejected(tmp_path):
    from libhdfs3_amd._native import Hdfs3CrcError
    data = splitmix_bytes(8192, 14)
    d, m = write_block(tmp_path, "blk_big", data)
    with pytest.raises(Hdfs3CrcError) as ei:
        read(d, m, buffer_size=(1 << 30) + 1)
    assert ei.value.rc == -errno.EINVAL


@pytest.mark.parametrize("piece", [(2 << 20) + 1, (2 << 20) + 3, (4 << 20) + 2, (3 << 20) + 5])
def test_read_sizes_that_split_unevenly(tmp_path, piece, staging):
    """Copies of 2 MiB or more are split over the host copy pool (csrc/copy_pool.h). Sizes whose
    quarter is a whole number of 4 KiB pages plus 1-3 bytes once lost their last bytes (the
    pieces were sized from the floor); every byte of every read must be the file's."""
    from libhdfs3_amd.engine import LocalBlockReader

    data = splitmix_bytes(9 * (1 << 20) + 17, piece)
    d, m = write_block(tmp_path, "blk_uneven", data)
    for verify in (True, False):
        with LocalBlockReader(d, m, verify=verify, buffer_size=1 << 20, window_buffers=8) as r:
            out = np.full(data.nbytes, 0xEE, np.uint8)
            pos = 0
            while pos < data.nbytes:
                got = r.read_into(out, pos, min(piece, data.nbytes - pos))
                assert got > 0
                pos += got
            assert pos == data.nbytes and np.array_equal(out, data), verify


def test_random_offsets_and_read_sizes(tmp_path):
    """Short-circuit reads with random block sizes, start offsets and read sizes (1 KiB to
    6 MiB, so copies both below and above the copy pool's 2 MiB split): every byte returned is
    the file's, verification on and off."""
    from libhdfs3_amd.engine import LocalBlockReader

    rng = np.random.default_rng(1017)
    for case in range(6):
        n = int(rng.integers(1 << 20, 12 << 20))
        data = splitmix_bytes(n, 4000 + case)
        d, m = write_block(tmp_path, f"blk_rand{case}", data)
        start = int(rng.integers(0, n // 2))
        for verify in (True, False):
            with LocalBlockReader(d, m, offset=start, verify=verify) as r:
                out = np.full(n - start, 0xEE, np.uint8)
                pos = 0
                while pos < out.nbytes:
                    want = int(rng.integers(1 << 10, 6 << 20))
                    got = r.read_into(out, pos, min(want, out.nbytes - pos))
                    assert got > 0
                    pos += got
                assert np.array_equal(out, data[start:]), (case, verify, start)


_POOL_CHILD = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from libhdfs3_amd import _native
from libhdfs3_amd.engine import LocalBlockReader
lib = _native.lib()
st = _native.PoolStats()
files = sys.argv[2:]
readers = [LocalBlockReader(files[i], files[i + 1]) for i in range(0, len(files), 2)]
for r in readers:
    r.read_all(1 << 30)
for r in readers:
    r.close()
assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
print(st.pinned_bytes, st.pinned_cap_bytes, st.pooled_contexts)
n = lib.hdfs3_crc_pool_trim()
assert n == st.pooled_contexts, (n, st.pooled_contexts)
assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
print(st.pinned_bytes, st.pinned_cap_bytes, st.pooled_contexts)
"""


@pytest.mark.parametrize("cap_mib", [24, 1024])
def test_pooled_readers_count_against_the_pinned_cap(tmp_path, cap_mib):
    """Closed short-circuit readers keep their ctx and windows in the library's pool; those bytes
    are reported by hdfs3_crc_pool_stats_get, kept under HDFS3_POOL_PINNED_MAX together with the
    contexts' pool (24 MiB: two readers' 3 x 4 MiB windows do not fit, so one reader's stay), and
    freed by hdfs3_crc_pool_trim. The cap is read once per process: a child process per cap."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = []
    for i in range(6):
        args += write_block(tmp_path, f"blk{i}", splitmix_bytes((9 << 20) + 300 * i, 900 + i))
    env = dict(os.environ, HDFS3_POOL_PINNED_MAX=f"{cap_mib}M")
    out = subprocess.run([sys.executable, "-c", _POOL_CHILD, repo] + args, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    (pinned, cap, pooled), (p2, _, n2) = [tuple(int(x) for x in ln.split()) for ln in out.stdout.split("\n")[:2]]
    assert cap == cap_mib << 20
    assert pinned <= cap, (pinned, cap)
    # a reader's windows: 3 x (4 MiB + its CRC words); one reader's worth fits 24 MiB, six fit 1 GiB
    windows = 3 * ((4 << 20) + 4 * ((4 << 20) // 512))
    assert pinned >= (windows if cap_mib == 24 else 6 * windows), (pinned, windows)
    assert pooled >= 1
    assert p2 == 0 and n2 == 0


_CONCURRENT_POOL_CHILD = r"""
import ctypes, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
from libhdfs3_amd import _native
from libhdfs3_amd.engine import CrcContext, LocalBlockReader
lib = _native.lib()
files = sys.argv[2:]
pairs = [(files[i], files[i + 1]) for i in range(0, len(files), 2)]
over, errors = [], []
mu = threading.Lock()

def sample(where):
    st = _native.PoolStats()
    assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
    if st.pinned_bytes > st.pinned_cap_bytes:
        with mu:
            over.append((where, st.pinned_bytes, st.pinned_cap_bytes))

def local_worker(t):
    try:
        for k in range(2):  # 8 threads x 2 readers = the 16 block files, closed concurrently
            d, m = pairs[2 * t + k]
            r = LocalBlockReader(d, m)
            out = r.read_all(1 << 30)
            assert out.nbytes == np.fromfile(d, dtype=np.uint8).nbytes
            r.close()
            sample(f"local {t}.{k}")
    except Exception as e:
        errors.append(repr(e))

def ctx_worker(t):
    # contexts released into the ctx pool at the same time, each holding host-API staging
    try:
        data = np.random.default_rng(t).integers(0, 256, (3 << 20) + 512 * t, dtype=np.uint8)
        for k in range(3):
            p = ctypes.c_void_p()
            assert lib.hdfs3_crc_ctx_acquire(0, ctypes.byref(p)) == 0
            words = np.zeros(4 * ((data.nbytes + 511) // 512), np.uint8)
            assert lib.hdfs3_crc32c_compute(p, data.ctypes.data, data.nbytes, 512, words.ctypes.data) == 0
            lib.hdfs3_crc_ctx_release(p)
            sample(f"ctx {t}.{k}")
    except Exception as e:
        errors.append(repr(e))

th = [threading.Thread(target=local_worker, args=(t,)) for t in range(8)]
th += [threading.Thread(target=ctx_worker, args=(t,)) for t in range(4)]
for x in th:
    x.start()
for x in th:
    x.join()
sample("end")
st = _native.PoolStats()
assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
print("over", len(over), over[:3])
print("errors", len(errors), errors[:3])
print("final", st.pinned_bytes, st.pinned_cap_bytes, st.pooled_contexts)
"""


def test_concurrent_closes_keep_the_pinned_cap(tmp_path):
    """ADVICE/VERDICT r4: admissions into the two pools used to be check-then-act across two mutexes, so
    readers closing at once could each take the same headroom. 16 short-circuit readers closed from 8
    threads while 4 more threads release host-API contexts into the ctx pool, at a 24 MiB cap: after
    every close and release, hdfs3_crc_pool_stats_get reports pinned_bytes <= cap."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = []
    for i in range(16):
        args += write_block(tmp_path, f"cblk{i}", splitmix_bytes((5 << 20) + 4096 * i + 77, 1300 + i))
    env = dict(os.environ, HDFS3_POOL_PINNED_MAX="24M")
    out = subprocess.run([sys.executable, "-c", _CONCURRENT_POOL_CHILD, repo] + args, env=env, capture_output=True,
                         text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = {ln.split()[0]: ln for ln in out.stdout.splitlines() if ln.strip()}
    assert lines["errors"].startswith("errors 0"), lines["errors"]
    assert lines["over"].startswith("over 0 "), lines["over"]
    pinned, cap, pooled = (int(x) for x in lines["final"].split()[1:])
    assert cap == 24 << 20 and pinned <= cap and pooled >= 1


_KNOB_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from libhdfs3_amd.engine import LocalBlockReader
d, m, n, bad = sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
ref = np.fromfile(d, dtype=np.uint8)
with LocalBlockReader(d, m) as r:
    out = np.zeros(n, dtype=np.uint8)
    pos = 0
    try:
        while pos < n:
            got = r.read_into(out, pos, min((2 << 20) + 3, n - pos))
            if got <= 0:
                break
            pos += got
    except Exception as e:
        print("error", pos, type(e).__name__)
    assert np.array_equal(out[:pos], ref[:pos])
    print("read", pos)
"""


@pytest.mark.parametrize("knobs", [{"HDFS3_COPY_NT": "1"}, {"HDFS3_LOCAL_BLOCKING_SYNC": "1"},
                                   {"HDFS3_COPY_NT": "1", "HDFS3_LOCAL_BLOCKING_SYNC": "1", "HDFS3_COPY_HELPERS": "8"}])
@pytest.mark.parametrize("corrupt", [False, True])
def test_host_side_knobs_keep_the_bytes_and_the_checks(tmp_path, knobs, corrupt):
    """The short-circuit reader's host-side knobs (streaming-store copies, blocking window events, the
    copy pool's helper count; read once per process, so a child per setting): every delivered byte
    equals the file's, reads of 2 MiB + 3 bytes split unevenly over the pool, and a corrupt chunk
    still withholds its whole 1 MiB local buffer (LocalBlockReader.cpp:138-163)."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = (13 << 20) + 777
    data = splitmix_bytes(n, 4242)
    crc = oracle_compute(data, 512)
    bad = (9 << 20) + 12345
    if corrupt:
        data = data.copy()
        data[bad] ^= 0x40
    d, m = write_block(tmp_path, "knob", data, crc=crc)
    env = dict(os.environ, **knobs)
    out = subprocess.run([sys.executable, "-c", _KNOB_CHILD, repo, d, m, str(n), str(bad)], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.split()
    got = int(lines[lines.index("read") + 1])
    if corrupt:
        assert "error" in lines and got == (bad >> 20) << 20, out.stdout  # up to the bad chunk's 1 MiB buffer
    else:
        assert "error" not in lines and got == n, out.stdout
