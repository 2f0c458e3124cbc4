#!/usr/bin/env python3
"""Library ceiling for the contraction shapes: torch._int_mm (hipBLASLt int8 GEMM, int32 out) on
the implicit-GEMM shapes of the bench layers, with the im2col matrix already materialised (so
this times the GEMM alone, no quantize / epilogue / im2col).  A reference point for what a tuned
library int8 GEMM reaches on MI355X at these M x N x K, not part of the product.

    python tools/int_mm_ref.py [--reps 20]
"""
import argparse
import json

import torch

SHAPES = {  # name: (M, N, K) = (pixels, cout, kh*kw*cin)
    "r50_headline_256@14x14_3x3_b256": (50176, 256, 2304),
    "r50_512@7x7_3x3_b256": (12544, 512, 4608),
    "r18_64@56x56_3x3_b128": (401408, 64, 576),
    "r18_256@14x14_3x3_b128": (25088, 256, 2304),
    "r50_expand_64->256@56_b256": (802816, 256, 64),
    "square_8192": (8192, 8192, 8192),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for name, (M, N, K) in SHAPES.items():
        x = torch.randint(-128, 127, (M, K), dtype=torch.int8, device=dev)
        w = torch.randint(-128, 127, (N, K), dtype=torch.int8, device=dev)
        res = {"shape": name, "M": M, "N": N, "K": K}
        for lay, wt in (("NT", w.t()), ("NN", w.t().contiguous())):
            try:
                for _ in range(3):
                    torch._int_mm(x, wt)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    torch._int_mm(x, wt)
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) / a.reps * 1e3
                tops = 2 * M * N * K / us / 1e6
                res[lay] = {"us": round(us, 2), "tops": round(tops, 1), "frac": round(tops / 5000.0, 4)}
            except Exception as ex:  # noqa: BLE001 - report what the library refuses
                res[lay] = {"error": str(ex)[:160]}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
