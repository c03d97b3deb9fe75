"""Debug: ragged last subdivision on dense random grids (GPU vs crop oracle vs full oracle)."""
import sys
sys.path[:0] = ["mapping-private_amd", "oracle", "tests"]
import numpy as np
import c3hlac
import pyoracle as po
from test_gpu_config5_nonperiodic import _crop_row

THR = (147, 146, 148)
ctx = c3hlac.Context(0)
for G in (22, 42, 52, 102, 130, 256, 512):
    S = 10
    rng = np.random.default_rng(G)
    w = (rng.integers(0, 1 << 24, size=G ** 3, dtype=np.uint32) | np.uint32(1 << 24)).reshape(G, G, G)
    ctx.set_grid(w.reshape(-1), (G,) * 3, leaf=0.01)
    for variant in (981, 117):
        sb, H = ctx.extract(variant, THR, S)
        n = sb[0]
        f = ctx.features().reshape(n, n, n, variant)
        bad = []
        subs = [(n - 1, n - 1, n - 1), (n - 1, 0, 0), (0, n - 1, 0), (0, 0, n - 1), (n - 2, n - 2, n - 2), (1, 1, 1)]
        for s in subs:
            ref = _crop_row(w, s, S, variant)
            nb = int((f[s[2], s[1], s[0]] != ref).sum())
            if nb:
                bad.append((s, nb))
        full = ""
        if G <= 52:
            g, layout, cloud = po.grid_inputs(w.reshape(-1), (G,) * 3, 0.01)
            fe, _, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.01, S, exact=True)
            fe = fe.reshape(n, n, n, variant)
            rows = np.argwhere((fe != f).any(-1))
            full = "full-oracle bad rows %d %s" % (len(rows), rows[:6].tolist())
            crop_ok = all(np.array_equal(_crop_row(w, s, S, variant), fe[s[2], s[1], s[0]]) for s in subs)
            full += " crop==full %s" % crop_ok
        print(G, variant, "bad", bad, full, flush=True)
