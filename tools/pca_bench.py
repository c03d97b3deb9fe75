"""Time the GPU PCA training path (csrc/pca.hip): the f64-MFMA SYRK of c3h_pca_add_data
on device rows and the solve (unpack / rotations / projection / dsyevd / sort).

Usage: python tools/pca_bench.py [rows] [F]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mapping-private_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import c3hlac  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 981
    dev = torch.device("cuda", 0)
    X = torch.rand((n, F), device=dev, dtype=torch.float32)
    torch.cuda.synchronize()
    nb = (F + 1 + 127) // 128
    flops = nb * (nb + 1) // 2 * 128 * 128 * 2 * n  # tile pairs actually computed
    for rot in (False, True):
        pca = c3hlac.PCA(mean_flg=False)
        pca.add_data(X[:4096], rotate24=rot)  # warm up (allocations, code objects)
        pca.solve()
        reps = 5
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            pca.add_data(X, rotate24=rot)
        torch.cuda.synchronize()
        t_add = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        pca.solve()
        t_solve = time.perf_counter() - t0
        print("rows %d F %d rotate24 %d: add_data %.3f ms (%.1f TFLOP/s f64 MFMA incl. reduce, %.1f GB/s rows)  "
              "solve %.1f ms" % (n, F, rot, t_add * 1e3, flops / t_add / 1e12, n * F * 4 / t_add / 1e9,
                                 t_solve * 1e3), flush=True)
        pca.close()


if __name__ == "__main__":
    main()
