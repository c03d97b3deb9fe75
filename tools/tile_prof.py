"""The dot4 C3 tile body on a points-in frame (configs[3]'s per-frame shape: a 1M-point
Kinect frame at leaf 0.02 -> 128^3, C3-HLAC-981 S = 10): c3h_voxelize + c3h_extract, the
extract timed with HIP events (median of reps).  With a diagnostics build (C3HLAC_LIB=
lib/variants/diag*.so) and C3H_PROF=<file>, each extract appends the tile kernel's per-block
phase timestamps (capi.hip prof_dump: p1 tables, p3 halo staged, p4 centres compacted, p2
first chunk's operands, p5 dot4 done, p6 first tile's epilogue, p7 block end).
usage: python tools/tile_prof.py [reps] [variant] [S]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mapping-private_amd")]


def main():
    import c3hlac
    from c3hlac import synth
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    variant = int(sys.argv[2]) if len(sys.argv) > 2 else 981
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    pts = synth.kinect_scene(1_000_000, grid=128, leaf=0.02, seed=synth.BASE_SEED + 7000)
    thr = (147, 146, 148)
    with c3hlac.Context(0) as ctx:
        gi = ctx.voxelize(pts, 0.02)
        ctx.extract(variant, thr, S)
        ms = []
        for _ in range(reps):
            ctx.timing(c3hlac.timing_mask("c3hlac"))
            ctx.kernel_times(reset=True)
            ctx.extract(variant, thr, S)
            ctx.synchronize()
            kt = ctx.kernel_times(reset=True)
            ms.append(kt["c3hlac"][0])
        ctx.timing(False)
        ex = ctx.exist()
        print(json.dumps({"div_b": list(gi.div_b), "n_occ": int(gi.n_occ), "variant": variant, "S": S,
                          "nonempty_subdivisions": int((ex > 0).sum()), "subdivisions": int(ex.size),
                          "extract_ms_median": float(np.median(ms)), "extract_ms_min": float(np.min(ms))}))


if __name__ == "__main__":
    main()
