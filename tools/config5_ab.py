#!/usr/bin/env python3
"""A/B of the read drop-in's reader knobs on config 5's read lines (bench.config5_block, reads only):
the loopback datanode in its own process (started before this process touches the GPU), 1 GiB of
128 MiB blocks, hdfsRead on 1 stream and 8 concurrent whole-block hdfsPreads, each paired pass by pass
with the reference loop, with CPU-seconds per GiB for the client and the datanode. Each variant sets
environment variables the reader reads when it opens (e.g. HDFS3_READER_WAIT=spin); variants
alternate, `--rounds` times.

  python tools/config5_ab.py --variant spin:HDFS3_READER_WAIT=spin --variant poll:HDFS3_READER_WAIT=poll"""
import argparse
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", required=True, help="name:VAR=value[,VAR=value]")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from loopback import ChildDatanode

    dn = ChildDatanode(packet_bytes=65536)  # before anything touches the GPU
    try:
        import numpy as np
        import torch

        import bench

        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        host = np.random.default_rng(5).integers(0, 256, size=1 << 30, dtype=np.uint8)
        variants = []
        for v in args.variant:
            name, _, kv = v.partition(":")
            env = dict(x.split("=", 1) for x in kv.split(",") if x)
            variants.append((name, env))
        for rnd in range(args.rounds):
            for name, env in variants:
                saved = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                try:
                    out = bench.config5_block(torch, device, host, 512, 128 << 20, reps=args.reps, dn=dn,
                                              reads_only=True)
                finally:
                    for k, old in saved.items():
                        if old is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = old
                print(json.dumps({"tool": "config5_ab", "variant": name, "env": env, "round": rnd, **out}),
                      flush=True)
    finally:
        dn.stop()


if __name__ == "__main__":
    main()
