"""Vendor-library reference points on this MI355X (context for the roofline, never the product
path): torch.linalg.cholesky (ROCm solver library) fp64 at the BASELINE sizes, and a sustained fp64
DGEMM (rocBLAS via torch.matmul) -- the practical MFMA ceiling under the chip's power limit.

    python scripts/vendor_ref.py  ->  one JSON line
"""
import json
import time

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    out = {"device": torch.cuda.get_device_name(0), "potrf": {}, "dgemm": {}}
    g = torch.Generator(device="cuda").manual_seed(0)
    for n in (2048, 4096, 8192):
        M = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
        A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
        ms = timed(lambda: torch.linalg.cholesky(A), 5)
        out["potrf"][n] = {"ms": ms, "tflops": n ** 3 / 3 / ms / 1e9}
        print(f"torch.linalg.cholesky n={n}: {ms:.3f} ms", flush=True)
        del M, A
    for n in (8192,):
        X = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g)
        Y = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g)
        ms = timed(lambda: X @ Y, 10)
        out["dgemm"][n] = {"ms": ms, "tflops": 2 * n ** 3 / ms / 1e9}
        print(f"dgemm n={n}: {ms:.3f} ms", flush=True)
    # the Newton path's GEMM shapes: the KKT product C^T W C (n x m times m x n, full) and the
    # Cholesky's K = 256 trailing update
    for (mm, nn, kk) in ((8192, 8192, 2048), (7680, 7680, 256), (2048, 2048, 512)):
        X = torch.rand((mm, kk), dtype=torch.float64, device="cuda", generator=g)
        Y = torch.rand((kk, nn), dtype=torch.float64, device="cuda", generator=g)
        ms = timed(lambda: X @ Y, 10)
        out["dgemm"][f"{mm}x{nn}x{kk}"] = {"ms": ms, "tflops": 2 * mm * nn * kk / ms / 1e9}
        print(f"dgemm {mm}x{nn}x{kk}: {ms:.3f} ms {2 * mm * nn * kk / ms / 1e9:.1f} TF/s", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
