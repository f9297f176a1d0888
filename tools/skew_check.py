#!/usr/bin/env python3
"""Coverage check of the lab skew variants (126/127, crc32c_experiments.hip): every unit of a few
workgroups corrupted in turn (one CRC word flipped) must be reported as the first bad chunk."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    ctx = CrcContext(0, lib=lib)
    dev = torch.device("cuda", 0)
    bb, bpc = 128 << 20, 512
    data = torch.randint(0, 256, (bb,), dtype=torch.uint8, device=dev)
    crc = torch.empty(4 * (bb // bpc), dtype=torch.uint8, device=dev)
    res = torch.zeros(1, dtype=torch.int64, device=dev)
    lib.hdfs3x_set_variant(0)
    ctx.compute_dev(data.data_ptr(), bb, bpc, crc.data_ptr())
    torch.cuda.synchronize()
    units, nwaves = bb // 4096, 256 * 16
    kq = units // nwaves
    bad = 0
    for v in (126, 127):
        lib.hdfs3x_set_variant(v)
        checked = 0
        for g in (0, 5, 255):
            for s in range(16):
                for col in range(kq):
                    u = col * nwaves + g * 16 + s
                    c = u * 8 + (s % 8)  # one chunk of the unit
                    crc[4 * c] ^= 1
                    res.zero_()
                    ctx.verify_dev_async(data.data_ptr(), bb, bpc, crc.data_ptr(), res.data_ptr())
                    torch.cuda.synchronize()
                    got = ~int(res.item()) if int(res.item()) != 0 else None
                    crc[4 * c] ^= 1
                    checked += 1
                    if got != c:
                        bad += 1
                        if bad < 10:
                            print(f"v{v}: unit {u} (wg {g} slot {s} col {col}) chunk {c}: got {got}")
        res.zero_()
        ctx.verify_dev_async(data.data_ptr(), bb, bpc, crc.data_ptr(), res.data_ptr())
        torch.cuda.synchronize()
        print(f"v{v}: {checked} single-unit flips checked, clean run result {int(res.item())}")
    lib.hdfs3x_set_variant(0)
    print("skew coverage", "OK" if bad == 0 else f"FAILED ({bad})")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
