#!/usr/bin/env python3
"""Device-resident CRC32C throughput over 512 B HDFS chunks (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): one 128 MiB HDFS block, 512 B chunks, verify on
one MI355X. A *step* = one hdfs3_crc32c_verify_dev_async launch over one whole block
(262,144 chunks, data + BE CRC array resident in HBM). Each rank rotates over
`--blocks` distinct blocks (default 8 = 1 GiB + CRCs) so the 256 MiB Infinity Cache
cannot serve repeats. Multi-GPU (config 4): independent blocks shard one set per
GPU, no collectives on the data path (weak scaling); value = all ranks' payload
bytes / max-over-ranks time.

Also reported, in the same run:
  roofline      alg bytes per launch (N*(C+4)) / average launch time
                from HIP events on the launch stream, vs the 8.0 TB/s HBM peak;
                `traffic` = DRAM bytes per launch from rocprofv3 PMC passes
                (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, separate passes);
  cpu_baseline  the reference CPU path (oracle/_ref HWCrc32c built from the
                reference sources, else the oracle's crc_pcl restatement) timed on
                this host on a bounded sample (rank 0, N=1 only).

    python bench.py [--gpus N --steps K --warmup W --bpc 512 --mode verify]

--gpus N > 1 without a launcher (no WORLD_SIZE in the environment) starts N rank processes
itself, before anything touches a GPU, exactly as `torch.distributed.run --nproc-per-node N`
would: rank r drives cuda:r (r mod the visible GPUs), the ranks meet over RCCL (or gloo with
HDFS3_BENCH_BACKEND=gloo) and rank 0 prints the one JSON line.

Clock: `value`, `ms_per_step` and `roofline.achieved` all come from ONE clock, HIP events on
the launch stream around the K timed steps (max over ranks); the host wall clock of the same
barrier + synchronize bracket is reported beside it (`host_ms_per_step`).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "device-resident CRC32C GiB/s over 512 B HDFS chunks; % of HBM roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 1000 warmup launches (~25 ms): the GPU needs ~25 ms of sustained load to leave its
    # idle power state; with 10 warmup launches the first ~1000 timed launches run ~15 %
    # slower (docs/DESIGN_HISTORY.md §5: W=10 27.0 us/launch, W=100 24.2, W>=1000 23.3, same box)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=1000)
    p.add_argument("--bpc", type=int, default=512)
    p.add_argument("--mode", choices=["verify", "compute"], default="verify")
    p.add_argument("--block-mib", type=int, default=128)
    p.add_argument("--blocks", type=int, default=8)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--no-compute", action="store_true", help="skip the compute-on-write block of the line")
    p.add_argument("--no-packets", action="store_true", help="skip the packet-stream block of the line")
    p.add_argument("--no-configs2", action="store_true",
                   help="skip BASELINE.json configs[2] (1 GiB compute + verify, bpc 512/2048/4096)")
    p.add_argument("--no-config5", action="store_true",
                   help="skip BASELINE.json configs[4] (loopback hdfsRead of 1 GiB, PCIe-inclusive, CPU reference)")
    p.add_argument("--sweep", action="store_true", help="extra diagnostics on stderr")
    p.add_argument("--graph", action="store_true",
                   help="replay the K steps from captured HIP graphs instead of launching them eagerly "
                        "(no consistent gain measured: docs/DESIGN_HISTORY.md §5)")
    p.add_argument("--no-overlap", action="store_true",
                   help="barrier every timed launch (no HDFS3_LAUNCH_OVERLAP_PREVIOUS); the overlapped "
                        "run is the default and the barriered one is reported beside it")
    p.add_argument("--out-json", default=None, help="also write the JSON line to this file (rank 0)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--plumbing-check", action="store_true",
                   help="CPU-only rehearsal of the N-rank entry (tests/test_multigpu.py): rank spawn, "
                        "rendezvous, per-rank block sets, barrier and max-over-ranks; no GPU work")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---- multi-GPU plumbing (config 4: independent blocks, one set per GPU, no collective
# on the data path). Kept free of GPU calls so tests/test_multigpu.py can run it on
# CPU ranks with the gloo backend.

def rank_seed(rank: int) -> int:
    """Each rank verifies its own distinct synthetic blocks."""
    return 1234 + 7919 * rank


def max_over_ranks(dist, value: float, device) -> float:
    """Whole-job time = the slowest rank's time (barrier-bracketed region)."""
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(bytes_per_rank: int, world: int, elapsed_max: float) -> float:
    """value = all ranks' payload bytes / max-over-ranks time, in GiB/s (weak scaling)."""
    return bytes_per_rank * world / elapsed_max / 2**30


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """--gpus N outside a launcher: N rank processes of this same command, started before any
    GPU call in this process (the parent only waits), with the environment torch.distributed.run
    would give them. If a rank fails the others are stopped (their exact PIDs); the exit code is
    the first failure's."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def check_distinct_devices(rows, world, ndev):
    """rows: gather_per_rank rows [rank, current_device, seed, elapsed, host_elapsed, rate, pci...].
    With world > 1 and at least `world` visible GPUs, every rank must report its own device (ordinal
    and, where torch exposes it, PCI address); otherwise SystemExit. Returns what was checked."""
    if world <= 1:
        return {"checked": False, "why": "one rank"}
    if ndev < world:
        return {"checked": False, "why": f"{ndev} visible GPU(s) for {world} ranks (a rehearsal sharing devices)"}
    ords = [int(r[1]) for r in rows]
    pcis = [tuple(int(x) for x in r[6:9]) for r in rows]
    if len(set(ords)) != world or (all(p[1] >= 0 for p in pcis) and len(set(pcis)) != world):
        raise SystemExit(f"MULTI-GPU FAILURE: {world} ranks on {ndev} visible GPUs but devices {ords} / pci {pcis} "
                         "are not distinct")
    return {"checked": True, "devices": ords}


def gather_per_rank(dist, world, rank, row, device):
    """Every rank's row of floats, on rank 0 (all ranks take part)."""
    import torch
    t = torch.zeros((world, len(row)), dtype=torch.float64, device=device)
    t[rank] = torch.tensor(row, dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().tolist()


def rank_host_placement(device_index=None):
    """[effective cores, NUMA node] of this rank: the cores a CPU baseline here may use (min of the
    affinity and the cgroup quota, as cpu_baseline counts them) and the node of its GPU's PCI function
    (hdfs3_device_numa_node; -1 when unknown or without a GPU)."""
    affinity = max(1, len(os.sched_getaffinity(0)))
    quota = cpu_quota_cores()
    cores = max(1, min(affinity, int(quota))) if quota else affinity
    node = -1
    if device_index is not None:
        try:
            import ctypes
            from libhdfs3_amd import _native
            n = ctypes.c_int(-1)
            if _native.lib().hdfs3_device_numa_node(int(device_index), ctypes.byref(n)) == 0:
                node = n.value
        except Exception:  # noqa: BLE001 - placement is reported, not required
            node = -1
    return [cores, node]


def plumbing_check(args):
    """The N-rank entry without GPU work (CPU, gloo): every rank derives its own block set,
    then barrier -> a rank-dependent elapsed -> max over ranks -> per-rank rows on rank 0."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    dist_ok = world > 1
    if dist_ok:
        dist.barrier()
    elapsed = 1e-3 * (1 + rank)
    emax = max_over_ranks(dist, elapsed, torch.device("cpu")) if dist_ok else elapsed
    rows = gather_per_rank(dist, world, rank, [rank, int(os.environ.get("LOCAL_RANK", "0")), rank_seed(rank),
                                               elapsed, os.getpid()] + rank_host_placement(), torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"plumbing_check": True, "n_gpus": world, "requested_gpus": args.gpus,
                          "elapsed_max": emax,
                          "per_rank": [{"rank": int(r[0]), "local_rank": int(r[1]), "seed": int(r[2]),
                                        "elapsed": r[3], "pid": int(r[4]), "cpu_cores": int(r[5]),
                                        "numa_node": int(r[6])} for r in rows]}), flush=True)
    if dist_ok:
        dist.barrier()
        dist.destroy_process_group()


class Workload:
    """Per-rank device arena: `blocks` blocks of data + their BE CRC arrays, in HBM."""

    def __init__(self, torch, ctx, device, block_bytes, blocks, bpc, seed):
        self.torch, self.ctx = torch, ctx
        self.block_bytes, self.blocks, self.bpc = block_bytes, blocks, bpc
        self.nchunks = block_bytes // bpc
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        self.data = torch.randint(0, 256, (blocks, block_bytes), dtype=torch.uint8, device=device, generator=g)
        self.crc = torch.empty((blocks, 4 * self.nchunks), dtype=torch.uint8, device=device)
        # device pointers resolved once: the timed loops index plain lists, not tensors (a tensor
        # index costs the box's host several us per launch, docs/DESIGN_HISTORY.md §5 "short timed regions")
        self._dp = [self.data[b].data_ptr() for b in range(blocks)]
        self._cp = [self.crc[b].data_ptr() for b in range(blocks)]
        for b in range(blocks):  # stored CRCs written by the GPU compute path, checked below
            ctx.compute_dev(self.data_ptr(b), block_bytes, bpc, self.crc_ptr(b))
        ctx.synchronize()

    def data_ptr(self, b):
        return self._dp[b]

    def crc_ptr(self, b):
        return self._cp[b]


def settle(torch, stream):
    """Wait for everything queued so far with the host thread polling (it stays on its core), then
    torch.cuda.synchronize(), which returns at once. A thread that sleeps in the synchronize wakes
    up late on some boxes: the first launch of a 20-launch timed region then went out up to 180 us
    after the start event (tools/launch_host_probe.py, profiles/r03/reentry/)."""
    done = torch.cuda.Event()
    done.record(stream)
    while not done.query():
        pass
    torch.cuda.synchronize()


def check_against_oracle(work, ctx):
    """Block 0's device-computed CRC array must equal the oracle's, word for word, and a
    single flipped bit must be reported at its chunk (parity gate before timing)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from util import oracle_compute  # test infrastructure: used as the checker only

    data = work.data[0].cpu().numpy()
    got = work.crc[0].cpu().numpy()
    want = oracle_compute(data, work.bpc)
    if not np.array_equal(got, want):
        bad = int(np.nonzero(got != want)[0][0]) // 4
        raise SystemExit(f"PARITY FAILURE: device CRC of chunk {bad} differs from the oracle")
    k = work.nchunks // 3
    pos = k * work.bpc + 17
    orig = work.data[0, pos].item()
    work.data[0, pos] = orig ^ 0x20
    work.torch.cuda.synchronize()
    first = ctx.verify_dev(work.data_ptr(0), work.block_bytes, work.bpc, work.crc_ptr(0))
    work.data[0, pos] = orig
    work.torch.cuda.synchronize()
    if first != k:
        raise SystemExit(f"PARITY FAILURE: flipped bit in chunk {k} reported as {first}")
    if ctx.verify_dev(work.data_ptr(0), work.block_bytes, work.bpc, work.crc_ptr(0)) != -1:
        raise SystemExit("PARITY FAILURE: clean block reported bad")


def run_steps(work, ctx, mode, n, result, events=None, base=0, overlap=False):
    """n steps, one launch each. overlap: every launch after the first of this run goes out
    with HDFS3_LAUNCH_OVERLAP_PREVIOUS (include/hdfs3_crc.h) — its predecessor on the stream
    is a verify of this run and all blocks, CRC arrays and zeroed result words were ready
    before the run started; the first launch of a run stays barriered behind whatever the
    stream held before (the result memset, events)."""
    rp, rn = result.data_ptr(), result.numel()
    dp, cp, nb, bb, bpc = work._dp, work._cp, work.blocks, work.block_bytes, work.bpc
    for i in range(n):
        s = base + i
        b = s % nb
        if events is not None:
            events[2 * i].record()
        if mode == "verify":
            ctx.verify_dev_async(dp[b], bb, bpc, cp[b], rp + 8 * (s % rn),
                                 overlap_previous=overlap and i > 0 and events is None)
        else:
            ctx.compute_dev(dp[b], bb, bpc, cp[b], overlap_previous=overlap and i > 0 and events is None)
        if events is not None:
            events[2 * i + 1].record()


def batched_rate(torch, work, ctx, mode, reps=100, warm=300):
    """Secondary measurement (never `value`): the same `blocks` blocks per call through the
    multi-block batch API (hdfs3_crc32c_{verify,compute}_blocks_dev*, one launch of the
    segmented wave kernel; each block keeps its own data, CRC array and (block, chunk)
    result key). Amortises the per-launch head and dispatch gap (docs/DESIGN_HISTORY.md §5)."""
    blocks = [(work.data_ptr(b), work.crc_ptr(b), work.block_bytes) for b in range(work.blocks)]
    nbytes = work.block_bytes * work.blocks
    res = torch.zeros(reps, dtype=torch.int64, device=work.data.device)

    def one(i):
        if mode == "verify":
            ctx.verify_blocks_dev_async(blocks, work.bpc, res.data_ptr() + 8 * i)
        else:
            ctx.compute_blocks_dev(blocks, work.bpc)

    # its own sustained state: `warm` calls (~50 ms) before the timed ones, so the mode measured
    # just before (the compute block writes every word of 8 blocks) does not carry over
    for i in range(warm):
        one(0)
    torch.cuda.synchronize()
    res.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        one(i)
    e1.record()
    torch.cuda.synchronize()
    if mode == "verify" and bool((res != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean blocks reported a bad chunk in the batched pass")
    t = e0.elapsed_time(e1) * 1e-3 / reps
    alg = work.blocks * work.nchunks * (work.bpc + 4)
    return {"api": "hdfs3_crc32c_verify_blocks_dev_async" if mode == "verify" else "hdfs3_crc32c_compute_blocks_dev",
            "blocks_per_launch": work.blocks, "value": round(nbytes / t / 2**30, 2), "unit": "GiB/s",
            "avg_launch_us": round(t * 1e6, 2), "achieved_GBps": round(alg / t / 1e9, 1),
            "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)}


class StepGraphs:
    """The timed K steps as replays of captured HIP graphs (torch.cuda.graph on the launch
    stream; the library shares torch's HIP runtime). Graph i holds `per` consecutive steps
    with exactly the eager loop's block rotation and result slots; a shorter graph covers
    K % per. Each step is still one launch verifying one whole block — the graph only
    removes per-launch CPU submission and shrinks the dispatch gap (docs/DESIGN_HISTORY.md §5)."""

    def __init__(self, torch, work, ctx, mode, K, result, stream, per=64):
        self.torch = torch
        self.per = min(per, K)
        self.full, rem = divmod(K, self.per)
        self.graphs = []
        for n, base in [(self.per, 0)] + ([(rem, self.full * self.per)] if rem else []):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                run_steps(work, ctx, mode, n, result, base=base)
            self.graphs.append(g)
        for g in self.graphs:  # first replay uploads/instantiates the graph: keep it untimed
            g.replay()
        torch.cuda.synchronize()

    def run(self):
        for _ in range(self.full):
            self.graphs[0].replay()
        if len(self.graphs) > 1:
            self.graphs[1].replay()


PRE_PASS = 2000  # launches of `value`'s pre-passes before its warmup (the diagnostic pass, then the barriered one)


def compute_block(torch, work, ctx, K, W, stream, read_ceilings):
    """Compute-on-write at the bench's shape (BASELINE.json configs[2]'s write half at configs[1]'s
    block): `hdfs3_crc32c_compute_dev` over the same rotated blocks, one 128 MiB block per launch,
    on the same clock as `value` (HIP events on the launch stream around K launches), overlapped
    (HDFS3_LAUNCH_OVERLAP_PREVIOUS after the first) and barriered, each in `value`'s own form:
    PRE_PASS barriered launches, W warmup launches, settle, K timed launches (round 4; until then
    500 warmup launches and no pre-pass, so the compute region started from a different power state
    than the verify region it is compared with). The words go to fresh arrays (poisoned before the
    pre-pass) and every word of every block is checked against the oracle after the timed region.
    read_ceilings: (overlapped, barriered) same-shape plain-read GB/s."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from util import oracle_compute  # test infrastructure: the checker only, after timing

    out = torch.full_like(work.crc, 0xA5)
    scratch = torch.empty_like(work.crc)  # the warmup launches' words
    alg = work.nchunks * (work.bpc + 4)  # reads C, writes 4 per chunk

    op = [out[b].data_ptr() for b in range(work.blocks)]
    sp = [scratch[b].data_ptr() for b in range(work.blocks)]
    dp, nb, bb, bpc = work._dp, work.blocks, work.block_bytes, work.bpc

    def launches(n, overlap, dst):
        for i in range(n):
            b = i % nb
            ctx.compute_dev(dp[b], bb, bpc, dst[b], overlap_previous=overlap and i > 0)

    res = {"api": "hdfs3_crc32c_compute_dev", "alg_bytes_per_launch": alg,
           "timing": "HIP events on the launch stream around K launches (the clock of value)"}
    for name, overlap in (("overlapped", True), ("barriered", False)):
        # poison first, then the pre-pass and warmup (into scratch): the poison's 8 MiB of dirty lines
        # leave the caches before the timed region (a fill right before it cost the driver's K = 20
        # form ~2.5 us per launch, profiles/r03/reentry/r3zc_bench_k20.json)
        out.fill_(0xA5)
        launches(PRE_PASS, False, sp)
        launches(W, overlap, sp)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launches(K, overlap, op)
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3 / K
        r = {"value": round(work.block_bytes / t / 2**30, 2), "unit": "GiB/s", "avg_launch_us": round(t * 1e6, 2),
             "achieved_GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)}
        ceil = read_ceilings[0 if overlap else 1] if read_ceilings else None
        if ceil:
            r["frac_of_achievable_per_block"] = round(alg / t / 1e9 / (ceil * alg / work.block_bytes), 4)
        r["paired"] = paired_regions(torch, work, ctx, stream, max(K, 200), overlap, sp)
        res[name] = r
    # every word the timed launches wrote (the last K launches covered all blocks when K >= blocks)
    host = out.cpu().numpy()
    for b in range(min(K, work.blocks)):
        want = oracle_compute(work.data[b].cpu().numpy(), work.bpc)
        if not np.array_equal(host[b], want):
            bad = int(np.nonzero(host[b] != want)[0][0]) // 4
            raise SystemExit(f"PARITY FAILURE: compute block {b} chunk {bad} differs from the oracle")
    res["checked"] = f"every CRC word of {min(K, work.blocks)} blocks against the oracle after the timed region"
    return res


def packets_block(torch, work, ctx, K, W, stream, reps=3):
    """Verify-on-read over synthetic DATA-TRANSFER PACKET STREAMS (north_star: "device-resident
    throughput on synthetic packet streams"; RemoteBlockReader.cpp:240-245, 306-326). The same 1 GiB
    payload as `value`, laid out as the block reader lays packets into its device arenas
    (block_reader.cpp: the 31-byte header is parsed on the host, each packet's 128 BE32 words then
    its 64 KiB of data, 16 B aligned): 16,384 packets at a 66,048-byte pitch. One launch verifies
    2,048 packets = 128 MiB of payload (one block's worth, the unit of `value`) through
    hdfs3_crc32c_verify_packet_stream_dev_async, rotating over the 8 streams of the arena. Timed in
    `value`'s form (PRE_PASS barriered launches, W warmup, settle, K launches between HIP events, the
    first barriered, the rest overlapped; and all barriered), and paired with contiguous-block verifies in identical regions
    (`reps` x (packets, contiguous); medians), so frac_vs_contiguous carries no box drift. Every
    launch's result slot is checked after timing; before it, one flipped bit must come back as its
    (packet, chunk)."""
    npk, pitch, cpp, bpc = 2048, 512 + 65536, 128, work.bpc
    if bpc != 512 or work.block_bytes != npk * 65536:
        return None
    nstreams = work.blocks
    arena = torch.empty((nstreams * npk, pitch), dtype=torch.uint8, device=work.data.device)
    arena[:, 512:] = work.data.view(-1, 65536)
    arena[:, :512] = work.crc.view(-1, 4 * cpp)
    torch.cuda.synchronize()
    base = arena.data_ptr()
    span = npk * pitch
    ps = ctx.packet_stream(0, 512, pitch, npk, 65536)
    res = torch.zeros(max(K, 256), dtype=torch.int64, device=work.data.device)
    rp = res.data_ptr()
    # the gate: a flipped bit in packet 777 chunk 45 of stream 3
    pk_, ch_ = 777, 45
    pos = (3 * npk + pk_, 512 + ch_ * 512 + 100)
    orig = int(arena[pos].item())
    arena[pos] = orig ^ 0x10
    torch.cuda.synchronize()
    ctx.verify_packet_stream_async(base + 3 * span, span, ps, bpc, rp)
    torch.cuda.synchronize()
    got = int(res[0].item())
    arena[pos] = orig
    res.zero_()
    torch.cuda.synchronize()
    if got == 0 or ((~got) & (2**64 - 1)) != (pk_ << 32) | ch_:
        raise SystemExit(f"PARITY FAILURE: packet stream reported {got:#x} for a flip in packet {pk_} chunk {ch_}")
    dp, cp, nb, bb = work._dp, work._cp, work.blocks, work.block_bytes
    alg = work.nchunks * (bpc + 4)

    def pk_launch(i, slot, overlap):
        ctx.verify_packet_stream_async(base + (i % nstreams) * span, span, ps, bpc, rp + 8 * slot,
                                       overlap_previous=overlap and i > 0)

    def blk_launch(i, slot, overlap):
        ctx.verify_dev_async(dp[i % nb], bb, bpc, cp[i % nb], rp + 8 * slot, overlap_previous=overlap and i > 0)

    def region(fn, n, warm, overlap):
        for i in range(warm):
            fn(i, i % res.numel(), overlap)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(n):
            fn(i, i % res.numel(), overlap)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / n

    out = {"api": "hdfs3_crc32c_verify_packet_stream_dev_async",
           "layout": f"{nstreams * npk} packets of 64 KiB, [128 BE32 words][64 KiB data] at a {pitch}-byte pitch "
                     f"(the block reader's device arena), {npk} packets (128 MiB payload) per launch",
           "alg_bytes_per_launch": alg,
           "timing": "HIP events on the launch stream around K launches (the clock of value)"}
    for name, overlap in (("overlapped", True), ("barriered", False)):
        for i in range(PRE_PASS):  # `value`'s form: its pre-pass, W warmup, settle, K timed
            pk_launch(i, i % res.numel(), False)
        t = region(pk_launch, K, W, overlap)
        r = {"value": round(bb / t / 2**30, 2), "unit": "GiB/s", "avg_launch_us": round(t * 1e6, 2),
             "achieved_GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)}
        n = max(K, 200)
        pk, bl = [], []
        for _ in range(reps):
            pk.append(region(pk_launch, n, 50, overlap))
            bl.append(region(blk_launch, n, 50, overlap))
        pm, bm = sorted(pk)[reps // 2], sorted(bl)[reps // 2]
        r["paired"] = {"launches": n, "packets_us": round(pm * 1e6, 2), "contiguous_us": round(bm * 1e6, 2),
                       "how": f"{reps} x (packet region, contiguous region), 50 warmup + settle + {n} timed each; medians"}
        r["frac_vs_contiguous"] = round(bm / pm, 4)
        out[name] = r
    if bool((res != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean packets reported a bad chunk in the packet-stream regions")
    out["checked"] = "every launch's result slot after the timed regions; a flipped bit located before them"
    del arena
    out["reader_batch"] = reader_batch_layouts(torch, work, ctx, stream)
    out["writer_batch"] = writer_batch_layout(torch, work, ctx, stream)
    return out


def reader_batch_layouts(torch, work, ctx, stream, npk=64, nbat=16, reps=5, n=200):
    """The block reader's own GPU unit: one batch of 64 datanode packets (64 KiB data, 512 B chunks),
    verified by one barriered launch, in the two device layouts the reader can land a batch in
    (block_reader.cpp): `wire` = [128 BE32 words][64 KiB data] per packet at a 66,048-byte pitch (the
    pitch walk; rounds 1-4), `dense` = the 64 packets' words back to back, then their data back to back
    from a 4 KiB boundary (one contiguous 4 MiB block and its word array: the block walk; round 5
    default). `nbat` batches rotate (64 MiB, as the reader's just-copied arenas, cache-resident); per
    layout `reps` regions of `n` barriered launches (HIP events), median. Results checked."""
    plen, bpc = 65536, 512
    dev = work.data.device
    src = work.data[0, :nbat * npk * plen].view(nbat, npk, plen)
    words = work.crc[0, :nbat * npk * 512].view(nbat, npk, 512)
    pitch = 512 + plen
    wire = torch.empty((nbat, npk, pitch), dtype=torch.uint8, device=dev)
    wire[:, :, :512] = words
    wire[:, :, 512:] = src
    d0 = npk * 512  # 32 KiB of words, already 4 KiB aligned
    dense = torch.empty((nbat, d0 + npk * plen), dtype=torch.uint8, device=dev)
    dense[:, :d0] = words.reshape(nbat, -1)
    dense[:, d0:] = src.reshape(nbat, -1)
    torch.cuda.synchronize()
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    rp = res.data_ptr()
    ps = ctx.packet_stream(0, 512, pitch, npk, plen)
    wb, db, wspan, dspan = wire.data_ptr(), dense.data_ptr(), npk * pitch, d0 + npk * plen

    def w_launch(i):
        ctx.verify_packet_stream_async(wb + (i % nbat) * wspan, wspan, ps, bpc, rp + 8 * (i % 256))

    def d_launch(i):
        b = db + (i % nbat) * dspan
        ctx.verify_dev_async(b + d0, npk * plen, bpc, b, rp + 8 * (i % 256))

    def region(fn):
        for i in range(50):
            fn(i)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(n):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    w, d = [], []
    for _ in range(reps):
        w.append(region(w_launch))
        d.append(region(d_launch))
    if bool((res != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean reader batches reported a bad chunk")
    wm, dm = sorted(w)[reps // 2], sorted(d)[reps // 2]
    alg = npk * (plen // bpc) * (bpc + 4)
    del wire, dense
    return {"packets_per_batch": npk, "batch_payload_bytes": npk * plen, "launch": "barriered, one per batch",
            "wire_us": round(wm, 2), "dense_us": round(dm, 2), "dense_speedup": round(wm / dm, 4),
            "wire_frac": round(alg / (wm * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "dense_frac": round(alg / (dm * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "how": f"{nbat} resident batches rotating, {reps} x (wire region, dense region) of 50 warmup + {n} "
                   "timed barriered launches; medians; every result slot checked"}


WRITER_HEADER = 31  # PacketHeader::GetPkHeaderLen (PacketHeader.cpp:38)


def writer_batch_layout(torch, work, ctx, stream, npk=64, nbat=16, reps=5, n=200):
    """The output stream's own GPU unit (output_stream.cpp dispatch): one batch of 64 packets of 127
    chunks at bpc 512 (computePacketChunkSize at the default 64 KiB packet, OutputStreamImpl.cpp:161-170;
    65,024 B = 15 whole rounds + 3,584 B), compute-on-write by one barriered launch of
    hdfs3_crc32c_compute_packets_dev_async over the batch's descriptors, in the writer's device layout:
    packet slots [lead: header + words room][data] at one stride, the batch's words compact after the
    slots. `nbat` batches rotate (device-resident). Paired, region by region, with the reader's dense
    4 MiB batch verify (`reps` x (writer region, reader region) of `n` barriered launches; medians), and
    the same batches verified (verify_packets_dev_async) for the symmetric read-side number. The words
    are checked against block 0's (the packets are its consecutive chunk-aligned slices)."""
    bpc, plen0 = 512, 65536
    with_sum = bpc + 4
    cpp = max(1, (plen0 - WRITER_HEADER + with_sum - 1) // with_sum)
    plen = cpp * bpc
    lead = (WRITER_HEADER + 4 * cpp + 15) // 16 * 16
    stride = lead + (plen + 15) // 16 * 16
    crc_region = stride * npk
    span = crc_region + 4 * cpp * npk
    span += (-span) % 4096
    dev = work.data.device
    if nbat * npk * plen > work.block_bytes:
        return None
    src = work.data[0, :nbat * npk * plen].view(nbat, npk, plen)
    want = work.crc[0, :nbat * npk * cpp * 4].view(nbat, npk * cpp * 4)
    arena = torch.zeros((nbat, span), dtype=torch.uint8, device=dev)
    arena[:, :crc_region].view(nbat, npk, stride)[:, :, lead:lead + plen] = src
    arena[:, crc_region:crc_region + 4 * cpp * npk] = want  # stored words for the verify leg
    # the reader's dense batch (64 x 64 KiB + its words), as reader_batch_layouts lays it
    rsrc = work.data[0, :nbat * 64 * plen0].view(nbat, -1)
    rwords = work.crc[0, :nbat * 64 * 512].view(nbat, -1)
    d0 = 64 * 512
    dense = torch.empty((nbat, d0 + 64 * plen0), dtype=torch.uint8, device=dev)
    dense[:, :d0] = rwords
    dense[:, d0:] = rsrc
    torch.cuda.synchronize()
    from libhdfs3_amd.engine import CrcContext
    descs = CrcContext._descs([(lead + stride * p, crc_region + 4 * cpp * p, plen) for p in range(npk)])
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    rp, ab, db, dspan = res.data_ptr(), arena.data_ptr(), dense.data_ptr(), d0 + 64 * plen0

    def w_compute(i):
        ctx.compute_packets_dev_async(ab + (i % nbat) * span, span, descs, bpc)

    def w_verify(i):
        ctx.verify_packets_dev_async(ab + (i % nbat) * span, span, descs, bpc, rp + 8 * (i % 256))

    def r_launch(i):
        b = db + (i % nbat) * dspan
        ctx.verify_dev_async(b + d0, 64 * plen0, bpc, b, rp + 8 * (i % 256))

    def region(fn):
        for i in range(50):
            fn(i)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(n):
            fn(i)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    # the gate: a flipped bit in the partial round of packet 9 of batch 3 comes back as its key
    q = 61440 + 3 * bpc + 17
    pos = (3, lead + stride * 9 + q)
    orig = int(arena[pos].item())
    arena[pos] = orig ^ 0x08
    torch.cuda.synchronize()
    w_verify(3)
    torch.cuda.synchronize()
    got = int(res[3].item())
    arena[pos] = orig
    res.zero_()
    torch.cuda.synchronize()
    if got == 0 or ((~got) & (2**64 - 1)) != (9 << 32) | (q // bpc):
        raise SystemExit(f"PARITY FAILURE: writer batch reported {got:#x} for a flip in packet 9 chunk {q // bpc}")
    arena[:, crc_region:crc_region + 4 * cpp * npk] = 0
    c, rv, wv = [], [], []
    for _ in range(reps):
        c.append(region(w_compute))
        rv.append(region(r_launch))
        wv.append(region(w_verify))
    if not bool(torch.equal(arena[:, crc_region:crc_region + 4 * cpp * npk], want)):
        raise SystemExit("PARITY FAILURE: the writer batches' computed words differ from the block's")
    if bool((res != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean writer / reader batches reported a bad chunk")
    cm, rm, vm = (sorted(x)[reps // 2] for x in (c, rv, wv))
    alg = npk * cpp * (bpc + 4)
    ralg = 64 * (plen0 // bpc) * (bpc + 4)
    del arena, dense
    return {"packets_per_batch": npk, "chunks_per_packet": cpp, "packet_data_bytes": plen,
            "slot_stride": stride, "batch_payload_bytes": npk * plen, "alg_bytes": alg,
            "api": "hdfs3_crc32c_compute_packets_dev_async (descriptors; the output stream's launch_packet_batch)",
            "launch": "barriered, one per batch",
            "compute_us": round(cm, 2), "verify_us": round(vm, 2), "reader_dense_us": round(rm, 2),
            "compute_frac": round(alg / (cm * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "verify_frac": round(alg / (vm * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "compute_vs_reader_dense": round(cm / rm, 4),
            "compute_vs_reader_dense_per_byte": round((cm / alg) / (rm / ralg), 4),
            "how": f"{nbat} resident batches rotating, {reps} x (writer compute, reader dense verify, writer "
                   f"verify) regions of 50 warmup + {n} timed barriered launches; medians; words and result "
                   "slots checked"}


def paired_regions(torch, work, ctx, stream, n, overlap, dst, reps=3):
    """Compute against verify in identical timed regions: per rep, a verify region then a compute
    region, each 50 warmup launches, settle, n timed launches (first barriered, the rest overlapped
    when `overlap`); medians of the per-launch times. Two 20-launch regions timed minutes apart on
    a box differ by up to 12 % (docs/DESIGN_HISTORY.md §5, the driver's form); a ratio of paired regions does not
    carry that."""
    res = torch.zeros(256, dtype=torch.int64, device=work.data.device)
    rp, dp, cp, nb, bb, bpc = res.data_ptr(), work._dp, work._cp, work.blocks, work.block_bytes, work.bpc

    def region(fn):
        for i in range(50):
            fn(i, i % 256)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(n):
            fn(i, i % 256)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    ver = lambda i, s: ctx.verify_dev_async(dp[i % nb], bb, bpc, cp[i % nb], rp + 8 * s,
                                            overlap_previous=overlap and i > 0)
    cmp_ = lambda i, s: ctx.compute_dev(dp[i % nb], bb, bpc, dst[i % nb], overlap_previous=overlap and i > 0)
    v, c = [], []
    for _ in range(reps):
        v.append(region(ver))
        c.append(region(cmp_))
    if bool((res != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean blocks reported a bad chunk in the paired verify regions")
    vm, cm = sorted(v)[reps // 2], sorted(c)[reps // 2]
    return {"launches": n, "verify_us": round(vm, 2), "compute_us": round(cm, 2),
            "compute_vs_verify": round(vm / cm, 4),
            "how": f"{reps} x (verify region, compute region), 50 warmup + settle + {n} timed launches each; medians"}


def configs2_block(torch, work, ctx, stream, K, host_data, reps=3, warm=120, bpcs=(512, 2048, 4096)):
    """BASELINE.json configs[2]: a 1 GiB synthetic stream per launch (the rank's 8 blocks as ONE
    contiguous 1 GiB buffer, which they are in HBM), compute-on-write (`hdfs3_crc32c_compute_dev`,
    OutputStreamImpl.cpp:298-359 / Packet.cpp:73-81) and verify-on-read (`hdfs3_crc32c_verify_dev_async`,
    RemoteBlockReader.cpp:306-326) at bytes-per-checksum 512 / 2048 / 4096. Per bpc and launch form
    (overlapped: HDFS3_LAUNCH_OVERLAP_PREVIOUS after each region's first launch; barriered: every
    launch), `reps` x (verify region, compute region), each `warm` untimed launches (~20 ms of
    sustained load), settle, then n = max(K, 20) timed launches between HIP events on the launch
    stream; medians. Checked: the words the first compute wrote equal the oracle's for every chunk
    of the GiB (before timing), a flipped bit comes back as its chunk, every verify result slot of
    the timed regions is clean, and the timed compute launches' words equal those words (after)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from util import oracle_compute  # test infrastructure: the checker only, outside the timed regions

    dev = work.data.device
    flat = work.data.view(-1)
    n_bytes = flat.numel()
    dptr = flat.data_ptr()
    n = max(K, 20)
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    rp = res.data_ptr()
    out = {"workload": f"{n_bytes >> 20} MiB contiguous stream per launch (the rank's {work.blocks} blocks), "
                       "compute and verify, device-resident",
           "bytes_per_launch": n_bytes, "timed_launches_per_region": n, "warmup_launches_per_region": warm,
           "how": f"{reps} x (verify region, compute region) per launch form; medians",
           "timing": "HIP events on the launch stream around each region's n launches (the clock of value)",
           "bpc": {}}
    for bpc in bpcs:
        nch = (n_bytes + bpc - 1) // bpc
        words = torch.full((4 * nch,), 0xA5, dtype=torch.uint8, device=dev)
        dst = torch.full_like(words, 0x5A)
        wp, op = words.data_ptr(), dst.data_ptr()
        ctx.compute_dev(dptr, n_bytes, bpc, wp)
        ctx.synchronize()
        want = oracle_compute(host_data, bpc)
        got = words.cpu().numpy()
        if not np.array_equal(got, want):
            bad = int(np.nonzero(got != want)[0][0]) // 4
            raise SystemExit(f"PARITY FAILURE: configs2 bpc {bpc}: compute word {bad} differs from the oracle")
        k = (nch * 5) // 7
        pos = k * bpc + bpc // 3
        orig = int(flat[pos].item())
        flat[pos] = orig ^ 0x02
        torch.cuda.synchronize()
        first = ctx.verify_dev(dptr, n_bytes, bpc, wp)
        flat[pos] = orig
        torch.cuda.synchronize()
        if first != k or ctx.verify_dev(dptr, n_bytes, bpc, wp) != -1:
            raise SystemExit(f"PARITY FAILURE: configs2 bpc {bpc}: flip in chunk {k} reported as {first}")
        alg = nch * (bpc + 4)  # verify reads C + 4 per chunk; compute reads C, writes 4

        def ver(i, overlap):
            ctx.verify_dev_async(dptr, n_bytes, bpc, wp, rp + 8 * (i % 256), overlap_previous=overlap and i > 0)

        def cmp_(i, overlap):
            ctx.compute_dev(dptr, n_bytes, bpc, op, overlap_previous=overlap and i > 0)

        def region(fn, overlap):
            for i in range(warm):
                fn(i, overlap)
            settle(torch, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(n):
                fn(i, overlap)
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e-3 / n

        row = {}
        for form, overlap in (("overlapped", True), ("barriered", False)):
            v, c = [], []
            for _ in range(reps):
                v.append(region(ver, overlap))
                c.append(region(cmp_, overlap))
            for mode, ts in (("verify", v), ("compute", c)):
                t = sorted(ts)[reps // 2]
                row.setdefault(mode, {})[form] = {
                    "avg_launch_us": round(t * 1e6, 2), "value": round(n_bytes / t / 2**30, 1), "unit": "GiB/s",
                    "achieved_GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4),
                    "regions_us": [round(x * 1e6, 2) for x in ts]}
            row.setdefault("compute_vs_verify", {})[form] = round(sorted(v)[reps // 2] / sorted(c)[reps // 2], 4)
        if bool((res != 0).any().item()):
            raise SystemExit(f"PARITY FAILURE: configs2 bpc {bpc}: a clean stream reported a bad chunk")
        if not torch.equal(dst, words):
            raise SystemExit(f"PARITY FAILURE: configs2 bpc {bpc}: the timed compute launches wrote other words")
        row["alg_bytes_per_launch"] = alg
        row["checked"] = (f"all {nch} words of the first compute against the oracle, a flipped bit in chunk {k}, "
                          "every timed verify's result slot, the timed computes' words against those")
        out["bpc"][str(bpc)] = row
        del words, dst
    return out


def config5_block(torch, device, host_data, bpc, block_bytes, reps=3, read_mib=4, dn=None, reads_only=False):
    """BASELINE.json configs[4]: a 1 GiB file of 128 MiB blocks served by the loopback datanode over
    127.0.0.1 TCP (64 KiB packets, test infrastructure), read end to end through the product's hdfsRead
    (hdfs3_input_read, 4 MiB reads: InputStreamImpl's block walk -> the block reader's receiver ->
    pinned arena -> H2D -> GPU verify -> caller buffer), i.e. PCIe-inclusive: verify on, verify off,
    and block read-ahead 2 (hdfs3_input_set_readahead); 8 concurrent hdfsPreads of one block each (8
    streams, one thread and one InputStream each); the host API on the same GiB (hdfs3_crc32c_verify:
    pinned and pageable host buffers, H2D-inclusive). Beside them, the reference CPU path on the same
    packet stream: RemoteBlockReader's receive -> verifyChecksum -> copy loop on the reading thread with
    the reference's own HWCrc32c (oracle/_ref; test infrastructure, this baseline leg only;
    RemoteBlockReader.cpp:226-357), verify on and off, on 1 and on 8 threads. The write direction
    (compute-on-write: H2D of the data, D2H of the words): hdfsWrite of the GiB into a sink, beside the
    reference's write loop (OutputStreamImpl::appendInternal + Packet, its HWCrc32c) into the same sink.

    Round 6: the datanode runs in its own process (`dn`, tools/loopback/serve.py, started before this
    process touched the GPU), so its sender threads are not charged to the client, and every read line
    carries CPU-seconds per GiB: the client's (this process: time.process_time over the pass, every
    thread) and the datanode's (the child's getrusage). Every line: one untimed first pass (cold), then
    `reps` timed passes (median and all); every pass's output buffer is compared with the file, byte
    for byte. GPU and reference lines of one shape are timed pass by pass alternately (paired)."""
    import ctypes
    import threading
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from loopback import LoopbackDatanode, reference_read_block
    from util import ref_lib
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext, InputStream

    total = host_data.nbytes
    nblk = total // block_bytes
    crc_host = None
    own_dn = dn is None
    if own_dn:
        dn = LoopbackDatanode(packet_bytes=65536)
    outbuf = np.empty(total, dtype=np.uint8)
    lines = {}
    dev = device.index or 0
    try:
        hctx = CrcContext(dev)  # the host API's own ctx (its pinned staging ring)
        crc_host = hctx.compute(host_data, bpc)  # the .meta words the datanode serves (GPU compute)
        blocks = [(100 + i, block_bytes) for i in range(nblk)]
        if own_dn:
            for i in range(nblk):
                dn.add_block(100 + i, host_data[i * block_bytes:(i + 1) * block_bytes],
                             crc_host[4 * (i * block_bytes // bpc):4 * ((i + 1) * block_bytes // bpc)], bpc)
        else:
            dn.share_blocks(host_data, crc_host, [(100 + i, i * block_bytes, block_bytes) for i in range(nblk)], bpc,
                            tag="c5")
        located = [(b, nb, [("127.0.0.1", dn.port)]) for b, nb in blocks]
        dn_cpu = (lambda: dn.cpu_seconds()) if not own_dn else (lambda: 0.0)

        def hdfs_read(verify, ahead):
            with InputStream(located, device=dev, verify=verify, batch_packets=64) as s:
                if ahead:
                    s.set_readahead(ahead)
                pos = 0
                while pos < total:
                    got = s.read_into(outbuf, pos, min(read_mib << 20, total - pos))
                    if got <= 0:
                        raise SystemExit(f"config5: hdfsRead returned {got} at {pos}")
                    pos += got

        caller_cpu = [0.0]  # CPU seconds of the threads that called the read API in the current pass

        def threads(fn):
            errs = []

            def one(i):
                t0 = time.thread_time()
                try:
                    fn(i)
                except Exception as e:  # noqa: BLE001 - reported below
                    errs.append(f"block {i}: {e}")
                caller_cpu[0] += time.thread_time() - t0  # (+= of floats under the GIL)
            th = [threading.Thread(target=one, args=(i,)) for i in range(nblk)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errs:
                raise SystemExit("config5: " + "; ".join(errs))

        def hdfs_pread8(verify):
            def one(i):
                with InputStream(located, device=dev, verify=verify, batch_packets=64) as s:
                    got = s.pread_into(i * block_bytes, outbuf, i * block_bytes, block_bytes)
                    if got != block_bytes:
                        raise OSError(f"short pread {got}")
            threads(one)

        def ref_read(verify):
            for i, (b, nb) in enumerate(blocks):
                reference_read_block(dn.port, b, nb, outbuf, i * block_bytes, verify=verify)

        def ref_read8(verify):
            threads(lambda i: reference_read_block(dn.port, blocks[i][0], block_bytes, outbuf, i * block_bytes,
                                                   verify=verify))

        def host_api(buf):
            bad = hctx.verify(buf, bpc, crc_host)
            if bad != -1:
                raise SystemExit(f"PARITY FAILURE: config5 host API reported chunk {bad} on a clean GiB")

        phase_buf = (ctypes.c_uint64 * 8)()

        def reader_phases():  # the block readers closed since the last call (hdfs3_reader_phase_ns)
            _native.check("hdfs3_reader_phase_ns", _native.lib().hdfs3_reader_phase_ns(phase_buf, 8, 1))
            return [int(x) for x in phase_buf]

        def one_pass(fn, check_out=True):
            if check_out:
                outbuf[::4096] = ~host_data[::4096]  # poison: every pass must rewrite the buffer
            reader_phases()
            caller_cpu[0] = 0.0
            c0, d0, q0 = time.process_time(), dn_cpu(), cgroup_throttled_s()
            m0 = time.thread_time()
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            m1 = time.thread_time()
            c1, d1, q1 = time.process_time(), dn_cpu(), cgroup_throttled_s()
            ph = reader_phases()
            throttled = (q1 - q0) / dt if q0 is not None and q1 is not None else 0.0
            if check_out and not np.array_equal(outbuf, host_data):
                bad = int(np.nonzero(outbuf != host_data)[0][0])
                raise SystemExit(f"PARITY FAILURE: config5 delivered a wrong byte at {bad}")
            gib = total / 2**30
            # the calling threads' own CPU: the pass's worker threads, or this thread for a one-stream pass
            callers = caller_cpu[0] + (m1 - m0)
            return ((total / dt / 2**30, (c1 - c0) / gib, (d1 - d0) / gib) + tuple(x * 1e-9 / gib for x in ph) +
                    (throttled, callers / gib))

        phase_names = ("recv", "arena", "launch", "gpu_wait", "copy_out", "rx_wait_free_slot",
                       "caller_wait_batch", "receiver_cpu")

        def summary(passes):
            timed = passes[1:]
            med = lambda k: sorted(x[k] for x in timed)[len(timed) // 2]
            out = {"gib_s": round(med(0), 2), "gib_s_all": [round(x[0], 2) for x in timed],
                   "cold_gib_s": round(passes[0][0], 2), "unit": "GiB/s",
                   "client_cpu_s_per_gib": round(med(1), 4)}
            if not own_dn:
                out["datanode_cpu_s_per_gib"] = round(med(2), 4)
            # the quota's throttling over the pass (cgroup cpu.stat), seconds per second of wall: > 0 means
            # the box's CPU share, not the datanode or the GPU, held the pass back at times
            out["cgroup_throttled_s_per_s"] = round(med(11), 4)
            # of client_cpu_s_per_gib: the threads that called the read API (hdfsRead / hdfsPread, or the
            # reference loop's own), the rest being the library's receivers and the HIP runtime's threads
            out["caller_threads_cpu_s_per_gib"] = round(med(12), 4)
            if any(x[3 + i] for x in timed for i in range(8)):
                # summed over the pass's block readers (threads): seconds per GiB delivered
                out["reader_phase_s_per_gib"] = {n: round(med(3 + i), 4) for i, n in enumerate(phase_names)}
            return out

        def measure(fn, check_out=True):
            return summary([one_pass(fn, check_out) for _ in range(1 + reps)])

        def measure_paired(fa, fb):
            # the GPU path and the reference loop pass by pass (A B A B ...), so that drift of the box
            # (page cache, clocks, other tenants' load) falls on both alike; each with its untimed first pass
            pa, pb = [], []
            for rep in range(1 + reps):
                pa.append(one_pass(fa))
                pb.append(one_pass(fb))
            ratios = sorted(a[0] / b[0] for a, b in zip(pa[1:], pb[1:]))
            cpu_ratios = sorted(a[1] / b[1] for a, b in zip(pa[1:], pb[1:]) if b[1] > 0)
            return summary(pa), summary(pb), {"rate": round(ratios[len(ratios) // 2], 3),
                                              "client_cpu": round(cpu_ratios[len(cpu_ratios) // 2], 3)
                                              if cpu_ratios else None}

        paired = {}
        if ref_lib() is not None:
            for verify, gk, rk in ((True, "hdfsRead_verify", "reference_cpu_verify"),
                                   (False, "hdfsRead_no_verify", "reference_cpu_no_verify")):
                g, r, paired[("1", verify)] = measure_paired(lambda v=verify: hdfs_read(v, 0),
                                                             lambda v=verify: ref_read(v))
                lines[gk] = dict(g, readahead_blocks=0, verify=verify, streams=1)
                lines[rk] = dict(r, verify=verify, streams=1, cores=1, kind="reference")
            for verify, gk, rk in ((True, "hdfsPread8_verify", "reference_cpu8_verify"),
                                   (False, "hdfsPread8_no_verify", "reference_cpu8_no_verify")):
                g, r, paired[("8", verify)] = measure_paired(lambda v=verify: hdfs_pread8(v),
                                                             lambda v=verify: ref_read8(v))
                lines[gk] = dict(g, verify=verify, streams=nblk, api="hdfs3_input_pread of one whole block per "
                                                                     "thread, one InputStream each")
                lines[rk] = dict(r, verify=verify, streams=nblk, cores=nblk, kind="reference")
        else:
            lines["hdfsRead_verify"] = dict(measure(lambda: hdfs_read(True, 0)), readahead_blocks=0, verify=True)
            lines["hdfsRead_no_verify"] = dict(measure(lambda: hdfs_read(False, 0)), readahead_blocks=0,
                                               verify=False)
            lines["hdfsPread8_verify"] = dict(measure(lambda: hdfs_pread8(True)), verify=True, streams=nblk)
        lines["hdfsRead_verify_readahead2"] = dict(measure(lambda: hdfs_read(True, 2)), readahead_blocks=2,
                                                   verify=True)
        if reads_only:  # tools/config5_ab.py: the read lines only
            return {"lines": lines, "paired": {f"{k[0]}_{'verify' if k[1] else 'no_verify'}": v
                                               for k, v in paired.items()}}
        hp = ctypes.c_void_p()
        _native.check("hdfs3_host_malloc_pinned", _native.lib().hdfs3_host_malloc_pinned(ctypes.byref(hp), total))
        try:
            pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
            pinned[:] = host_data
            lines["host_api_pinned"] = dict(measure(lambda: host_api(pinned), check_out=False),
                                            api="hdfs3_crc32c_verify on a pinned 1 GiB host buffer (H2D + verify)")
            del pinned
        finally:
            _native.lib().hdfs3_host_free_pinned(hp)
        lines["host_api_pageable"] = dict(measure(lambda: host_api(host_data), check_out=False),
                                          api="hdfs3_crc32c_verify on a pageable 1 GiB host buffer "
                                              "(staging copy + H2D + verify)")
        # the write direction (compute-on-write, H2D of the data + D2H of the words): hdfsWrite of the same
        # GiB in 1 MiB writes into a sink that reads the packets (tools/loopback's count sink), beside the
        # reference's write loop with its HWCrc32c on the writing thread (oracle/ref_driver.cpp
        # ref_write_packets); both sinks must see the same packets and wire bytes
        lines.update(write_lines(host_data, bpc, block_bytes, dev, reps))
        hctx.close()
    finally:
        if own_dn:
            dn.stop()
    out = {"workload": f"{total >> 20} MiB file = {nblk} x {block_bytes >> 20} MiB blocks, {bpc} B chunks, "
                       f"64 KiB packets from a loopback datanode on 127.0.0.1 (test infrastructure), "
                       f"{read_mib} MiB hdfsRead calls (1 stream) or {nblk} concurrent whole-block hdfsPreads",
           "datanode": ("a child process (tools/loopback/serve.py), started before the bench touched the GPU; "
                        "its CPU time is datanode_cpu_s_per_gib" if not own_dn else
                        "in this process (its threads are charged to client_cpu_s_per_gib)"),
           "cpu_quota_cores": cpu_quota_cores(),
           "lines": lines,
           "reference_cpu": ("RemoteBlockReader's loop on the reading thread (receive a packet, verifyChecksum "
                             "with the reference HWCrc32c built from src/common/HWCrc32c.cpp, copy to the caller; "
                             "RemoteBlockReader.cpp:226-357) over the same loopback packet stream"),
           "checked": "every pass's 1 GiB output buffer byte for byte against the file (poisoned before each "
                      "pass); host API passes must report the GiB clean"}
    if "reference_cpu_verify" in lines:
        out["gpu_over_reference_cpu"] = round(lines["hdfsRead_verify"]["gib_s"] / lines["reference_cpu_verify"]["gib_s"], 2)
        out["gpu8_over_reference_cpu8"] = round(lines["hdfsPread8_verify"]["gib_s"] /
                                                lines["reference_cpu8_verify"]["gib_s"], 2)
        # median over the timed passes of (GPU pass rate / the reference pass run right after it), and of
        # (GPU pass client CPU per GiB / the reference pass's)
        out["paired_gpu_over_reference_cpu"] = {
            "verify": paired[("1", True)], "no_verify": paired[("1", False)],
            "verify_8_streams": paired[("8", True)], "no_verify_8_streams": paired[("8", False)],
            "how": "GPU and reference passes alternated; medians of the per-pair ratios (rate: higher is "
                   "better for the GPU path; client_cpu: CPU-seconds per GiB, lower is better)"}
        out["readahead2_over_reference_cpu"] = round(
            lines["hdfsRead_verify_readahead2"]["gib_s"] / lines["reference_cpu_verify"]["gib_s"], 2)
    return out


def write_lines(host_data, bpc, block_bytes, dev, reps):
    """config5's write lines (see config5_block): GPU compute-on-write through hdfs3_output_* into a C sink,
    and the reference's loop. Rates are GiB/s of user data; 1 untimed + `reps` timed passes each."""
    import ctypes
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from util import ref_lib
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import OutputStream

    total = host_data.nbytes
    sink = ctypes.cast(_native.loopback().hdfs3_loopback_count_sink, ctypes.c_void_p).value
    seen = {}

    def gpu_write():
        counts = (ctypes.c_uint64 * 3)()
        with OutputStream(device=dev, bytes_per_checksum=bpc, block_size=block_bytes, batch_packets=64,
                          raw_sink=sink, raw_user=ctypes.addressof(counts)) as s:
            for off in range(0, total, 1 << 20):
                s.write(host_data[off:off + (1 << 20)])
            s.close()
        seen["gpu"] = (int(counts[0]), int(counts[1]))

    def rates(fn):
        r = []
        for _ in range(1 + reps):
            t0 = time.perf_counter()
            fn()
            r.append(total / (time.perf_counter() - t0) / 2**30)
        t = r[1:]
        return {"gib_s": round(sorted(t)[len(t) // 2], 2), "gib_s_all": [round(x, 2) for x in t],
                "cold_gib_s": round(r[0], 2), "unit": "GiB/s"}

    out = {"hdfsWrite_sink": dict(rates(gpu_write), api="hdfs3_output_write, 1 MiB writes, 64-packet GPU batches "
                                                       "(H2D data, compute, D2H words) into a C sink")}
    ref = ref_lib()
    if ref is not None:
        f = ref.ref_write_packets
        f.restype = ctypes.c_double
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        pk, wb = ctypes.c_uint64(), ctypes.c_uint64()

        def ref_write():
            if f(host_data.ctypes.data, total, bpc, 65536, block_bytes, ctypes.byref(pk), ctypes.byref(wb)) < 0:
                raise SystemExit("config5: the reference write loop failed")
            seen["ref"] = (pk.value, wb.value)

        out["reference_cpu_write_sink"] = dict(rates(ref_write), cores=1, kind="reference",
                                               api="OutputStreamImpl::appendInternal + Packet::addChecksum/addData "
                                                   "with the reference HWCrc32c, the same sink")
        if seen["gpu"] != seen["ref"]:
            raise SystemExit(f"PARITY FAILURE: config5 write: GPU path sent {seen['gpu']} (packets, bytes), "
                             f"the reference loop {seen['ref']}")
        out["hdfsWrite_sink"]["checked"] = (f"{seen['gpu'][0]} packets / {seen['gpu'][1]} wire bytes, equal to the "
                                            "reference loop's (every packet's bytes: tests/test_output_stream.py)")
    return out


def lab_context(work, stream):
    """A context of the measurement library (libhdfs3_crc_lab.so) on the bench's device and
    stream: the plain-read ceiling kernels live there, not in the product library."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext
    lab = CrcContext(work.data.device.index or 0, lib=_native.lab())
    lab.set_stream(stream.cuda_stream)
    return lab


def stream_read_ceiling(torch, work, lab, reps=10, overlap=False):
    """Achievable HBM read on the same arena with a plain coalesced 16 B/lane read kernel
    (no CRC): best of grid 256/512 x default/non-temporal loads.
    Returns (1 GiB-per-launch GB/s, per-launch GB/s at the bench's own shape: one block per
    launch rotating over the blocks, back to back, i.e. including the per-launch head and
    dependent-launch overhead the CRC launches pay too)."""
    from libhdfs3_amd import _native
    lib = _native.lab()
    sink = torch.zeros(4, dtype=torch.int32, device=work.data.device)
    total = work.blocks * work.block_bytes

    def rate(grid, nbytes, n, ptr_of, overlap=False):
        for i in range(3):
            lib.hdfs3x_stream_read(lab.ctx, ptr_of(i), nbytes, grid, sink.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            lib.hdfs3x_stream_read_ex(lab.ctx, ptr_of(i), nbytes, grid, sink.data_ptr(), int(overlap and i > 0))
        e1.record()
        torch.cuda.synchronize()
        return nbytes * n / (e0.elapsed_time(e1) * 1e-3) / 1e9

    best, best_grid = 0.0, 256
    for grid in (256, 512, -256, -512):  # negative: non-temporal loads
        r = rate(grid, total, reps, lambda i: work.data.data_ptr())
        if r > best:
            best, best_grid = r, grid
    per_block = rate(best_grid, work.block_bytes, 400, lambda i: work.data_ptr(i % work.blocks), overlap)
    return best, per_block, best_grid


def same_form_read(torch, work, lab, stream, grid, K, W, overlap, reps=5):
    """The plain read in exactly the timed region's form: W warmup launches, settle (the
    synchronize), then K launches of one block each between two HIP events, the first barriered
    and the rest overlapped when `overlap`. Median per-launch GB/s over `reps` such regions. A short
    region pays the start of a run from an idle GPU (a barriered first launch, the ramp of the
    first few; profiles/r02/bench_k20_trace.jsonl) and the steady-state ceiling above does not."""
    from libhdfs3_amd import _native
    lib = _native.lab()
    sink = torch.zeros(4, dtype=torch.int32, device=work.data.device)
    dp, nb, bb = work._dp, work.blocks, work.block_bytes
    sp = sink.data_ptr()

    def launches(n):
        for i in range(n):
            lib.hdfs3x_stream_read_ex(lab.ctx, dp[i % nb], bb, grid, sp, int(overlap and i > 0))

    rates = []
    for _ in range(reps):
        launches(W)
        settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launches(K)
        e1.record(stream)
        torch.cuda.synchronize()
        rates.append(bb * K / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    return sorted(rates)[len(rates) // 2]


def lane_read_rate(torch, work, lab, reps=10):
    from libhdfs3_amd import _native
    lib = _native.lab()
    sink = torch.zeros(4, dtype=torch.int32, device=work.data.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        b = r % work.blocks
        lib.hdfs3x_lane_read(lab.ctx, work.data_ptr(b), work.block_bytes, work.bpc, sink.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    return work.block_bytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def cpu_quota_cores():
    """cgroup v2 CPU quota of this process in cores (None when unlimited or unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        return None


def cgroup_throttled_s():
    """CPU time this cgroup's tasks were throttled by its quota, in seconds (cpu.stat: cgroup v2
    throttled_usec, v1 throttled_time in ns), or None when unknown."""
    for path, key, scale in (("/sys/fs/cgroup/cpu.stat", "throttled_usec", 1e-6),
                             ("/sys/fs/cgroup/cpu/cpu.stat", "throttled_time", 1e-9)):
        try:
            for line in open(path):
                k, v = line.split()
                if k == key:
                    return int(v) * scale
        except Exception:
            continue
    return None


def cpu_baseline(work, seconds, bpc, data=None, crc=None):
    """Reference CPU path on this host, a bounded streaming sample of the same workload: the
    rank's whole block set (8 x 128 MiB = 1 GiB, host copies of the blocks and their CRC arrays),
    each thread verifying its own contiguous part, so every rep streams ~1 GiB from DRAM (more
    than the host's last-level caches) instead of re-reading a cache-resident slice. Threads = the
    cores this process may actually use (min of os.sched_getaffinity and the cgroup CPU quota),
    and one core; each leg is sized from a two-rep pilot to run >= seconds / 3, and reports the
    process CPU seconds it consumed (getrusage) beside its thread count."""
    import ctypes
    import resource
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from util import PCL, oracle, ref_lib  # test infrastructure: baseline leg only

    if data is None:
        data = np.ascontiguousarray(work.data.cpu().numpy()).reshape(-1)  # [blocks, bytes] -> one stream
    if crc is None:
        crc = np.ascontiguousarray(work.crc.cpu().numpy()).reshape(-1)    # the blocks' CRC arrays, in order
    affinity = max(1, len(os.sched_getaffinity(0)))
    quota = cpu_quota_cores()
    threads = max(1, min(affinity, int(quota))) if quota else affinity
    ref = ref_lib()
    bad = ctypes.c_int64(0)
    if ref is not None and ref.ref_hw_available():
        kind, engine = "reference", "HWCrc32c (reference src/common/HWCrc32c.cpp, built by oracle/Makefile)"
        run = lambda nthreads, reps: ref.ref_hw_bench_verify(data.ctypes.data, data.nbytes, bpc, crc.ctypes.data,
                                                            nthreads, reps, ctypes.byref(bad))
    else:
        kind, engine = "port", "oracle crc_pcl restatement (3-way crc32q + pclmul, IntelAsmCrc32c behaviour)"
        run = lambda nthreads, reps: oracle().oracle_bench_verify(PCL, data.ctypes.data, data.nbytes, bpc,
                                                                 crc.ctypes.data, nthreads, reps, ctypes.byref(bad))

    def cpu_s():
        u = resource.getrusage(resource.RUSAGE_SELF)
        return u.ru_utime + u.ru_stime

    def timed(fn, nthreads, budget):
        t2 = fn(nthreads, 2)  # pilot: two reps, so thread start-up does not size the sample
        reps = max(2, int(budget * 2 / max(t2, 1e-6)))
        for _ in range(3):  # the pilot ran cold: resize until the sample fills its budget
            c0 = cpu_s()
            t = fn(nthreads, reps)
            used = cpu_s() - c0
            if t >= 0.8 * budget:
                break
            reps = max(reps + 1, int(reps * budget / max(t, 1e-6) * 1.1))
        if bad.value != -1:
            raise SystemExit(f"cpu baseline reported a bad chunk {bad.value} on a clean block set")
        return {"value": round(data.nbytes * reps / t / 2**30, 3), "unit": "GiB/s", "cores": nthreads,
                "wall_s": round(t, 2), "cpu_s": round(used, 2), "reps": reps}

    budget = seconds / 3
    allc = timed(run, threads, budget)
    out = dict(allc, kind=kind,
               sample=(f"{allc['reps']} x verify of the rank's {data.nbytes >> 20} MiB block set ({bpc} B chunks, "
                       f"RemoteBlockReader::verifyChecksum loop), one contiguous part per thread, {threads} threads, "
                       f"{allc['wall_s']} s wall, {allc['cpu_s']} CPU s; engine: {engine}"),
               nproc=os.cpu_count(), affinity_cpus=affinity, cgroup_cpu_quota_cores=quota,
               effective_cores=threads)
    one = timed(run, 1, budget)
    out["one_core"] = dict(one, kind=kind, sample=f"{one['reps']} x the same block set on 1 thread, {one['wall_s']} s")
    # the reference's production x86 engine is IntelAsmCrc32c (crc_pcl, 3-way crc32q + pclmul;
    # needs yasm, not buildable here): time its restatement too, the stronger CPU baseline
    if kind == "reference":
        fp = lambda n, reps: oracle().oracle_bench_verify(PCL, data.ctypes.data, data.nbytes, bpc, crc.ctypes.data,
                                                          n, reps, ctypes.byref(bad))
        out["pcl_port"] = {"all_cores": timed(fp, threads, budget / 2), "one_core": timed(fp, 1, budget / 2),
                           "kind": "port",
                           "engine": "oracle crc_pcl restatement (IntelAsmCrc32c behaviour, "
                                     "src/common/crc_iscsi_v_pcl.asm:93-340)"}
    # BASELINE.json configs[0]: one 64 KiB packet (128 x 512 B chunks) through the reference
    # CPU path on one core, 10^4 repetitions timed inside the C loop
    if ref is not None and ref.ref_hw_available():
        pkt = 65536
        tp = ref.ref_hw_bench_verify(data.ctypes.data, pkt, bpc, crc.ctypes.data, 1, 10000, ctypes.byref(bad))
        if bad.value == -1:
            out["config0_packet_us"] = round(tp / 10000 * 1e6, 3)
            out["config0_packet_GiBps_1core"] = round(pkt * 10000 / tp / 2**30, 3)
    return out


def pmc_traffic(args):
    """DRAM bytes per verify launch: two rocprofv3 passes (FETCH_SIZE, WRITE_SIZE) over a
    short child run; FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 counts wide
    streaming reads at half their bytes)."""
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not on PATH"
    out_root = os.path.join(REPO, "gpurun_out", "bench_pmc")
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out_root, counter)
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--bpc", str(args.bpc),
               "--mode", args.mode, "--block-mib", str(args.block_mib), "--blocks", str(args.blocks)]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        except Exception as e:  # profiling is best effort; the value line does not depend on it
            return None, f"rocprofv3 {counter} pass failed: {e}"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            return None, f"no counter csv for {counter}"
        per = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                # the timed kernel: crc32c_*_kernel<bpc, VERIFY,...>; setup launches are compute
                is_mode = ("true" in name or "Lb1E" in name) if args.mode == "verify" else ("false" in name or "Lb0E" in name)
                if "crc32c_" in name and is_mode and row.get("Counter_Name") == counter:
                    per.append(float(row["Counter_Value"]))
        if not per:
            return None, f"no crc32c kernel rows for {counter}"
        per = per[len(per) // 2:]  # steady state (skip the CRC-setup launches)
        vals[counter] = sum(per) / len(per)
    # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    return fetch + write, f"FETCH_SIZE {vals['FETCH_SIZE']:.0f} KiB x2 + WRITE_SIZE {vals['WRITE_SIZE']:.0f} KiB per launch"


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(spawn_ranks(args.gpus))  # nothing in this process has touched a GPU
    if args.plumbing_check:
        return plumbing_check(args)
    # config 5's loopback datanode in a process of its own, started before anything here touches a GPU
    # (round 6): its sender threads are then neither charged to the client's CPU time nor competing
    # inside the client's process unseen
    dn_child = None
    if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.mode == "verify" and not args.no_config5 and
            args.bpc == 512 and not args.pmc_child):
        import atexit
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from loopback import ChildDatanode
        dn_child = ChildDatanode(packet_bytes=65536)
        atexit.register(dn_child.stop)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and rank == 0:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; the launcher's world size is used")
    # RCCL for the timing barrier/all-reduce on a GPU node; HDFS3_BENCH_BACKEND=gloo lets
    # a 1-GPU box rehearse N ranks (device = LOCAL_RANK mod visible GPUs, identity on 8)
    backend = os.environ.get("HDFS3_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local % ndev)
    device = torch.device("cuda", local % ndev)
    if world > 1:
        dist.init_process_group(backend, init_method="env://")
    coll_device = device if backend == "nccl" else torch.device("cpu")

    from libhdfs3_amd.engine import CrcContext
    ctx = CrcContext(local % ndev)
    # One explicit stream for the kernels and the HIP events that time them (the
    # default stream's handle is 0, which the C-ABI reads as "use the ctx stream").
    stream = torch.cuda.Stream(device=device)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    block_bytes = args.block_mib << 20
    work = Workload(torch, ctx, device, block_bytes, args.blocks, args.bpc, seed=rank_seed(rank))

    if args.pmc_child:
        res = torch.zeros(64, dtype=torch.int64, device=device)
        run_steps(work, ctx, args.mode, 16, res)
        torch.cuda.synchronize()
        return

    check_against_oracle(work, ctx)

    K, W = args.steps, args.warmup
    result = torch.zeros(max(K, W, 1), dtype=torch.int64, device=device)
    # (0) diagnostic pass, before the warmup: max(K, 2000) launches eagerly, each bracketed
    # by HIP events on the launch stream (per-launch duration including dispatch, averaged
    # over the last K). Running it first also takes the GPU out of its idle power state
    # (docs/DESIGN_HISTORY.md §5: ~25 ms of load), so short --warmup values still time a steady GPU
    D = max(K, 2000)
    events = [torch.cuda.Event(enable_timing=True) for _ in range(2 * D)]
    run_steps(work, ctx, args.mode, D, result, events)
    torch.cuda.synchronize()
    if args.mode == "verify" and bool((result != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean blocks reported a bad chunk in the roofline pass")
    overlap = not args.no_overlap
    alg_bytes = work.nchunks * (args.bpc + 4)  # verify reads data + CRC; compute reads data, writes CRC
    # (0b) barriered pass (reported beside the overlapped `value`, first-class: it is what a
    # caller issuing one plain hdfs3_crc32c_verify_dev_async per block gets): max(D - K, 1000)
    # untimed then K timed launches, every one with the AQL barrier bit. It runs before the
    # warmup: together with (0) it keeps the GPU under sustained load for ~100 ms before the
    # timed region, whatever W is
    barriered = None
    if overlap:
        result.zero_()
        run_steps(work, ctx, args.mode, max(D - K, 1000), result)  # its own untimed warmup
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b0.record(stream)
        run_steps(work, ctx, args.mode, K, result)
        b1.record(stream)
        torch.cuda.synchronize()
        if bool((result != 0).any().item()):
            raise SystemExit("PARITY FAILURE: clean blocks reported a bad chunk in the barriered pass")
        bl = b0.elapsed_time(b1) * 1e-3 / K
        barriered = {"api": "hdfs3_crc32c_verify_dev_async (AQL barrier bit on every launch)",
                     "value": round(block_bytes / bl / 2**30, 2), "unit": "GiB/s", "ms_per_step": round(bl * 1e3, 4),
                     "avg_launch_us": round(bl * 1e6, 2), "achieved_GBps": round(alg_bytes / bl / 1e9, 1),
                     "frac": round(alg_bytes / bl / 1e9 / HBM_PEAK_GBPS, 4),
                     "timing": "HIP events on the launch stream around K barriered launches"}
    result.zero_()
    run_steps(work, ctx, args.mode, W, result, overlap=overlap)
    graphs = StepGraphs(torch, work, ctx, args.mode, K, result, stream) if args.graph else None
    result.zero_()
    # (1) timed region: W warmup steps done, now exactly K steps (graph replays, or K eager
    # launches), nothing else on the stream, bracketed by barrier + synchronize on both sides.
    # The clock of `value`: HIP events on the launch stream around the K steps (max over ranks).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        settle(torch, stream)
        dist.barrier()
    settle(torch, stream)  # ends in torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    if graphs is not None:
        graphs.run()
    else:
        run_steps(work, ctx, args.mode, K, result, overlap=overlap)
    ev1.record(stream)
    torch.cuda.synchronize()
    host_elapsed = time.perf_counter() - t0
    elapsed = ev0.elapsed_time(ev1) * 1e-3
    if world > 1:
        dist.barrier()
    if args.mode == "verify" and bool((result != 0).any().item()):
        raise SystemExit("PARITY FAILURE: clean blocks reported a bad chunk in the timed region")
    my_rate = block_bytes * K / elapsed / 2**30
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    pci = [getattr(props, "pci_domain_id", -1), getattr(props, "pci_bus_id", -1), getattr(props, "pci_device_id", -1)]
    rows = gather_per_rank(dist, world, rank, [rank, torch.cuda.current_device(), rank_seed(rank), elapsed,
                                               host_elapsed, my_rate] + pci +
                           rank_host_placement(torch.cuda.current_device()), coll_device)
    dist_world = dist.get_world_size() if dist.is_initialized() else 1
    elapsed_max = max(r[3] for r in rows)
    host_max = max(r[4] for r in rows)
    value = aggregate_rate(block_bytes * K, world, elapsed_max)
    # N > 1 on a node with >= N visible GPUs: every rank must have driven its own device (config 4 is
    # one block set PER GPU); a launcher that mapped two ranks onto one device fails loudly here
    distinct = check_distinct_devices(rows, world, ndev)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    pre_pass = {"diagnostic_event_bracketed": D, "barriered": (max(D - K, 1000) + K) if overlap else 0,
                "warmup": W}
    pre_pass["total_before_timed_region"] = sum(pre_pass.values())
    launch_ms = [events[2 * s].elapsed_time(events[2 * s + 1]) for s in range(D)]
    eager_launch_s = sum(launch_ms[-K:]) / K * 1e-3  # the last K of the diagnostic pass
    avg_launch_s = elapsed / K  # rank 0's own launches, same clock as value
    achieved = alg_bytes / avg_launch_s / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                "alg_bytes_per_launch": alg_bytes, "avg_launch_us": round(avg_launch_s * 1e6, 2),
                "timing": "HIP events on the launch stream around the K timed steps / K (the clock of value)",
                "eager_per_launch_us": round(eager_launch_s * 1e6, 2)}
    if world > 1:
        # the whole job against the whole node's HBM: N x alg bytes x K / max elapsed / (N x 8 TB/s)
        roofline["aggregate_frac"] = round(world * alg_bytes * K / elapsed_max / 1e9 / (world * HBM_PEAK_GBPS), 4)
        roofline["aggregate_achieved"] = round(world * alg_bytes * K / elapsed_max / 1e9, 1)
        roofline["aggregate_peak"] = world * HBM_PEAK_GBPS
        roofline["frac_note"] = "frac/achieved: rank 0's own launches; aggregate_*: all ranks over the slowest rank's time"
    extra = {}
    lab = None
    ceilings = None
    if world == 1:
        try:
            lab = lab_context(work, stream)
            whole, per_block, best_grid = stream_read_ceiling(torch, work, lab, overlap=overlap)
            roofline["achievable_read_GBps"] = round(whole, 1)
            # the same shape as the timed steps: a plain read of one block per launch, with
            # the same launch mode (overlapped or barriered)
            roofline["achievable_read_per_block_launch_GBps"] = round(per_block, 1)
            roofline["frac_of_achievable_per_block"] = round(achieved / (per_block * alg_bytes / block_bytes), 4)
            # the same plain read in the timed region's own form (W warmup, synchronize, K launches):
            # a short region (the driver's K = 20) starts from an idle GPU, the 400-launch ceiling
            # above does not; both are reported, the ceiling above stays the conservative one
            same = same_form_read(torch, work, lab, stream, best_grid, K, W, overlap)
            roofline["achievable_read_same_form_GBps"] = round(same, 1)
            roofline["frac_of_achievable_same_form"] = round(achieved / (same * alg_bytes / block_bytes), 4)
            roofline["same_form"] = (f"plain read of one block per launch in the timed region's form: {W} warmup "
                                     f"launches, synchronize, {K} timed launches (median of 5 regions)")
            ceilings = [per_block, None]
            if barriered is not None:
                _, per_block_b, _ = stream_read_ceiling(torch, work, lab, overlap=False)
                ceilings[1] = per_block_b
                barriered["achievable_read_per_block_launch_GBps"] = round(per_block_b, 1)
                barriered["frac_of_achievable_per_block"] = round(
                    barriered["achieved_GBps"] / (per_block_b * alg_bytes / block_bytes), 4)
        except Exception as e:
            log("stream ceiling failed:", e)
        if barriered is not None:
            extra["barriered"] = barriered
        if args.mode == "verify" and not args.no_compute:
            extra["compute"] = compute_block(torch, work, ctx, K, W, stream, ceilings)
            for m in ("overlapped", "barriered"):
                v = roofline["frac"] if m == "overlapped" else (barriered or {}).get("frac")
                if v:
                    extra["compute"][m]["frac_vs_verify"] = round(extra["compute"][m]["frac"] / v, 4)
        host_data = None
        if args.mode == "verify" and (not args.no_configs2 or not args.no_config5):
            # a numpy-owned copy (numpy asks for transparent huge pages on large arrays; torch's CPU tensors,
            # by default, do not): config5's loopback datanode serves the file from this buffer, and served
            # from the torch tensor one hdfsRead stream ran at 5.8-5.9 GiB/s against 7.8-7.9 in
            # tools/e2e_read.py's numpy buffer on the same box (profiles/r05/r5n, r5o)
            host_data = np.empty(work.data.numel(), dtype=np.uint8)
            host_data[:] = work.data.view(-1).cpu().numpy()
        if args.mode == "verify" and not args.no_configs2:
            extra["configs2"] = configs2_block(torch, work, ctx, stream, K, host_data)
        if args.mode == "verify" and not args.no_packets:
            pk = packets_block(torch, work, ctx, K, W, stream)
            if pk:
                pk["overlapped"]["frac_vs_value"] = round(pk["overlapped"]["frac"] / roofline["frac"], 4)
                extra["packets"] = pk
        try:
            extra["batched"] = batched_rate(torch, work, ctx, args.mode)
        except SystemExit:
            raise
        except Exception as e:
            log("batched pass failed:", e)
    if world == 1 and args.mode == "verify" and not args.no_config5 and args.bpc == 512:
        extra["config5"] = config5_block(torch, device, host_data, args.bpc, block_bytes, reps=5, dn=dn_child)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(work, args.cpu_seconds, args.bpc, data=host_data)
    if args.sweep and world == 1 and lab is not None:
        log(json.dumps({"lane_read_GBps": round(lane_read_rate(torch, work, lab), 1)}))
    if world == 1 and not args.no_pmc:
        traffic, note = pmc_traffic(args)
        roofline["traffic"] = int(traffic) if traffic else None
        roofline["traffic_note"] = note

    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": K,
        "warmup": W, "pre_pass_launches": pre_pass, "ms_per_step": round(elapsed_max / K * 1e3, 4),
        "higher_is_better": True,
        "host_ms_per_step": round(host_max / K * 1e3, 4),
        "clock": "value, ms_per_step and roofline: HIP events on each rank's launch stream around its K timed "
                 "steps (max over ranks); host_ms_per_step: host wall clock of the same barrier+synchronize bracket",
        "launch": (f"HIP graph replay, {graphs.per} single-block launches per graph" if graphs is not None
                   else "eager, one launch per step; launches after the first overlap their predecessor "
                        "(HDFS3_LAUNCH_OVERLAP_PREVIOUS)" if overlap else "eager, one barriered launch per step"),
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (torch.randint bytes)",
        "config": {"workload": f"{args.mode} of one {args.block_mib} MiB HDFS block per step, "
                               f"{args.bpc} B chunks, device-resident (BASELINE.json configs[1]"
                               f"{'; configs[3] sharding: one block set per GPU' if world > 1 else ''})",
                   "bpc": args.bpc, "block_bytes": block_bytes, "chunks_per_block": work.nchunks,
                   "blocks_rotated_per_gpu": args.blocks, "mode": args.mode,
                   "parallelism": f"{world} GPU(s), independent blocks one set per GPU, no collectives"},
        "world_size": dist_world, "backend": backend if world > 1 else None,
        "roofline": roofline, "cpu_baseline": cpu,
        "per_rank": [{"rank": int(r[0]), "current_device": int(r[1]), "pci": [int(x) for x in r[6:9]],
                      "seed": int(r[2]), "ms_per_step": round(r[3] / K * 1e3, 4), "value": round(r[5], 2),
                      "frac": round(alg_bytes * K / r[3] / 1e9 / HBM_PEAK_GBPS, 4),
                      # the cores a CPU baseline on this rank's host share may use, and its GPU's NUMA node
                      "cpu_cores": int(r[9]), "numa_node": int(r[10])} for r in rows],
        "distinct_devices": distinct,
    }
    if "barriered" in extra:
        line["barriered"] = extra["barriered"]
    if "batched" in extra:
        line["batched"] = extra["batched"]
    if "packets" in extra:
        line["packets"] = extra["packets"]
    if "compute" in extra:
        line["compute"] = extra["compute"]
    if "configs2" in extra:
        line["configs2"] = extra["configs2"]
    if "config5" in extra:
        line["config5"] = extra["config5"]
    if cpu:
        line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        line["gpu_over_cpu_note"] = (f"against the reference engine on {cpu['cores']} threads = the effective cores "
                                     f"(affinity {cpu['affinity_cpus']} CPUs, cgroup quota "
                                     f"{cpu['cgroup_cpu_quota_cores']}), streaming the 1 GiB block set")
        if "pcl_port" in cpu and "all_cores" in cpu["pcl_port"]:
            line["gpu_over_cpu_pcl"] = round(value / cpu["pcl_port"]["all_cores"]["value"], 1)
    print(json.dumps(line), flush=True)
    if args.out_json:
        with open(args.out_json, "w") as f:
            f.write(json.dumps(line) + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
