"""Standalone CRC pass over a repair tasklet's rebuilt rows (256 rows of 262,144 B at non-uniform
addresses, as cfsec_ec_reconstruct_batch_crc hands them over) and over 128 rows of 5,592,406 B, vs
the workgroup count (CFSEC_CRC32_GROUPS_PROBE, re-read per launch); words checked against zlib."""
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import reedsolomon  # noqa: E402


def case(name, n, S, spread):
    buf = torch.randint(0, 256, (n * spread, (S + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
    rows = [buf[i * spread] for i in range(n)]
    ptrs = [r.data_ptr() for r in rows]
    want = [zlib.crc32(rows[i][:S].cpu().numpy().tobytes()) & 0xFFFFFFFF for i in (0, n - 1)]
    for g in (512, 1024, 2048, 4096, 8192):
        os.environ["CFSEC_CRC32_GROUPS_PROBE"] = str(g)
        got = reedsolomon.crc32_ieee_batch(ptrs, S, device=0)
        assert [got[0], got[-1]] == want, name
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            reedsolomon.crc32_ieee_batch(ptrs, S, device=0)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(f"{name:34s} groups {g:5d}  {us:8.1f} us/call (incl. sync)  {n * S / us / 1e3:7.1f} GB/s", flush=True)


case("C5 rebuilt rows 256 x 262144", 256, 262144, 2)
case("EC12P4 8 stripes 128 x 5592406", 128, 5592406, 1)
