"""The per-callback loop driven from C++ on the C-ABI alone (tools/single_frame_native.cpp,
bench.py's single_frame.native) returns the same detection lists as the same calls through
the ctypes binding: 1M-point Kinect scenes at configs[2]'s shape (256^3, C3-HLAC-117 S = 10,
117 -> 100, 10 models x r = 20, box 2^3, rank 1), bit-identical records, and each scene's
records are the oracle's (its float64 maximum or an exact tie within 2e-5, score within 1e-5): the
lists are reset per frame (c3h_clean_max = the callback's cleanData), so no frame inherits
the previous scene's maxima."""
import sys

import numpy as np
import pytest

import c3hlac
import pyoracle as po
from c3hlac import synth
from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


@pytest.mark.gpu
def test_native_loop_lists_match_ctypes(tmp_path):
    exe = ROOT / "mapping-private_amd" / "lib" / "single_frame_native"
    assert exe.exists(), "make -C mapping-private_amd builds lib/single_frame_native"
    scenes = [bench.scene_points(synth, 0, s) for s in range(2)]
    axis_t, var, axis_q = synth.random_bases(bench.VARIANT, bench.D, bench.M, bench.R, seed=synth.BASE_SEED)
    ctx = c3hlac.Context(0)
    try:
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(bench.RANK)
        want = []
        for sc in scenes:  # both scenes on one context: cleanData between them
            ctx.voxelize(sc, bench.LEAF)
            ctx.clean_max()
            ctx.extract(bench.VARIANT, bench.THR, bench.SUBDIV)
            lists, _ = ctx.search(bench.BOX, bench.EXIST_THR)
            want.append(lists[:, 0].copy())
    finally:
        ctx.close()
    out = tmp_path / "lists.bin"
    res = bench.native_single_frame(scenes, axis_t, var, axis_q, 4, lists_out=out)
    got = np.fromfile(out, dtype=c3hlac.DET_DTYPE).reshape(len(scenes), bench.M)
    for s in range(len(scenes)):
        assert float(want[s][0]["score"]) > 0
        assert got[s].tobytes() == want[s].tobytes(), "scene %d" % s
    # the oracle on each scene (voxelize -> C3-HLAC-117 -> exist -> float64 search)
    ap = synth.whiten(axis_t, var)
    for s, sc in enumerate(scenes):
        g, layout, cloud = po.voxelize(sc, bench.LEAF)
        f, sb, _ = po.c3hlac(g, layout, cloud, 117, bench.THR, bench.LEAF, bench.SUBDIV)
        _, _, scores = po.search(sb, f, po.exist(f), ap, axis_q, bench.BOX, bench.RANK, bench.EXIST_THR, dbl=True,
                                 want_scores=True)
        scores = scores.reshape(bench.M, -1)
        px, py = sb[0] - bench.BOX[0] + 1, sb[1] - bench.BOX[1] + 1
        for m in range(bench.M):  # bench.py cpu_baseline's frame check
            r = want[s][m]
            p = (int(r["z"]) * py + int(r["y"])) * px + int(r["x"])
            best = int(np.argmax(scores[m]))
            assert int(r["mode"]) == 0 and abs(float(r["score"]) - scores[m, p]) <= 1e-5 * scores[m, p], (s, m)
            assert p == best or scores[m, p] >= scores[m, best] * (1 - 2e-5), (s, m, p, best)
    assert res["frames_with_detection"] == 4 and res["ms_per_frame_end_to_end"] > 0
