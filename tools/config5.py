"""BASELINE configs[4] on one GPU (a parity case, not the bench line): 512^3 dense grid
(100 % occupancy, colour = hash(voxel index)), C3-HLAC-981 at S=10, compress 981->100,
10 models x r=20, box 2x2x2, rank 1.  Prints per-stage kernel times (HIP events) and the
SURVEY 8(d) compute-bound accounting: 1,224 algorithmic flop per occupied voxel for
C3-HLAC-981 (fp32 formulation; the kernel computes it exactly in u8 x u8 -> u32 dot4)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mapping-private_amd")]
import numpy as np  # noqa: E402
import c3hlac  # noqa: E402
from c3hlac import synth  # noqa: E402

G, S, THR = 512, 10, (147, 146, 148)
M, D, R = 10, 100, 20


def _arg(name, dflt):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else dflt


M, R = _arg("--models", M), _arg("--r", R)  # the stress case: --models 63 --r 70
ENGINE = _arg("--engine", 0)  # c3h_set_score_engine: 0 auto, 1 VALU, 2 matrix cores
t0 = time.time()
words = synth.dense_words(G, seed=synth.BASE_SEED + 5).reshape(-1)
print("grid generated in %.1f s" % (time.time() - t0), flush=True)
with c3hlac.Context(0) as ctx:
    ctx.set_grid(words, (G, G, G))
    del words
    axis_t, var, axis_q = synth.random_bases(981, D, M, R, seed=synth.BASE_SEED)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    if "--fp16" in sys.argv:
        ctx.set_search_precision(True)
    ctx.set_score_engine(ENGINE)
    print("models %d x r=%d, D=%d, score engine %d" % (M, R, D, ENGINE), flush=True)
    res = []
    for rep in range(4):
        ctx.timing(True)
        ctx.kernel_times(reset=True)
        t0 = time.perf_counter()
        sb, hn = ctx.extract(981, THR, S)
        lists, nm = ctx.search((2, 2, 2), 100)
        wall = time.perf_counter() - t0
        kt = ctx.kernel_times(reset=True)
        ctx.timing(False)
        res.append((wall, kt))
        print("rep %d wall %.2f ms  c3hlac %.3f ms  compress %.3f ms  score %.3f ms  replay %.3f ms" %
              (rep, wall * 1e3, kt["c3hlac"][0], kt["compress"][0], kt["score"][0], kt["replay"][0]), flush=True)
    wall, kt = min(res[1:], key=lambda r: r[0])
    nvox = G ** 3
    c3_ms = kt["c3hlac"][0]
    flop = 1224.0 * nvox
    P = (sb[0] - 1) * (sb[1] - 1) * (sb[2] - 1)
    print("config5: subdivisions %s  C3 %.3f ms = %.0f Mvoxels/s = %.1f TFLOP/s algorithmic (%.1f %% of "
          "157.3 TF fp32 VALU)" % (sb, c3_ms, nvox / c3_ms / 1e3, flop / c3_ms / 1e9,
                                   100 * flop / c3_ms / 1e9 / 157.3))
    s_ms = kt["compress"][0] + kt["score"][0] + kt["replay"][0]
    print("config5: search (compress + score + replay) %.3f ms = %.3g detections/s (%d positions x %d models)"
          % (s_ms, P * M / s_ms * 1e3, P, M))
    pf = 2.0 * P * M * R * D
    print("config5: projection GEMM %.1f GFLOP; score stage (box sums + projection + argmax) %.3f ms = %.1f TFLOP/s"
          % (pf / 1e9, kt["score"][0], pf / kt["score"][0] / 1e9))
    print("config5: end to end (extract + search, host wall) %.2f ms = %.0f Mvoxels/s" % (wall * 1e3, nvox / wall / 1e6))
