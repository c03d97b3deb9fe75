"""ctypes wrapper of oracle/lib/libc3hlac_oracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this: it is
the checker and the timed CPU baseline, never part of the product path.
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "lib" / "libc3hlac_oracle.so"
_lib = None


class OrcGrid(C.Structure):
    _fields_ = [("div_b", C.c_int32 * 3), ("min_b", C.c_int32 * 3), ("max_b", C.c_int32 * 3),
                ("n_valid", C.c_int64), ("n_occ", C.c_int64), ("leaf", C.c_float),
                ("inv_leaf", C.c_float)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = C.CDLL(str(LIB))
        P = C.c_void_p
        lib.orc_lut.argtypes = [C.c_int, P]
        lib.orc_voxel_bounds.argtypes = [P, C.c_int64, C.c_float, C.c_float, C.POINTER(OrcGrid)]
        lib.orc_voxel_fill.argtypes = [P, C.c_int64, C.c_float, C.POINTER(OrcGrid), P, P]
        lib.orc_c3hlac.restype = C.c_int64
        lib.orc_c3hlac.argtypes = [C.POINTER(OrcGrid), P, P, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   P, P]
        lib.orc_exist.argtypes = [P, C.c_int64, C.c_int, P]
        lib.orc_search.argtypes = [C.c_int, C.c_int, C.c_int, P, C.c_int, P, P, C.c_int, P, C.c_int,
                                   P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_int, P, P, P, P, P, P]
        lib.orc_remove_overlap.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P]
        lib.orc_set_voxel_semantics.argtypes = [C.c_int]
        lib.orc_pca_read.argtypes = [C.c_char_p, C.c_int, P, P, P, C.POINTER(C.c_int), C.c_int]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


COLOR_C3_FLOAT, COLOR_C3_DOUBLE, COLOR_CHLAC = 0, 1, 2  # c3hlac_oracle.h ORC_COLOR_*


def lut(color_mode=COLOR_C3_DOUBLE):
    out = np.zeros(512, np.int32)
    load().orc_lut(int(color_mode), _p(out))
    return out.reshape(256, 2)


def set_voxel_semantics(pcl_era=True):
    """True (default): the reference's PCL 1.0 / Eigen 3.0 voxel-grid arithmetic (centroid =
    sum * (1/n), neighbour base floor(c / leaf)); False: later PCL (true division, base
    floor(c * (1/leaf))).  Process-wide; the fixture test switches it to show the difference."""
    load().orc_set_voxel_semantics(int(bool(pcl_era)))


def voxelize(pts, leaf, z_limit=float("inf")):
    """-> (grid dict, leaf_layout (div product,), cloud (n_occ,4) float32)."""
    pts = np.ascontiguousarray(pts, dtype=np.float32)
    lib = load()
    g = OrcGrid()
    rc = lib.orc_voxel_bounds(_p(pts), pts.shape[0], float(leaf), float(z_limit), C.byref(g))
    if rc != 0:
        raise RuntimeError("orc_voxel_bounds failed: %d" % rc)
    nvox = int(g.div_b[0]) * int(g.div_b[1]) * int(g.div_b[2]) if g.n_valid else 0
    layout = np.full(max(nvox, 1), -1, np.int32)
    cloud = np.zeros((max(int(g.n_valid), 1), 4), np.float32)
    if g.n_valid:
        rc = lib.orc_voxel_fill(_p(pts), pts.shape[0], float(z_limit), C.byref(g), _p(layout), _p(cloud))
        if rc != 0:
            raise RuntimeError("orc_voxel_fill failed: %d" % rc)
    return g, layout[:nvox], cloud[: int(g.n_occ)].copy()


def c3hlac(g, layout, cloud, variant, thr, voxel_size, subdiv=0, offset=(0, 0, 0),
           color_mode=COLOR_C3_DOUBLE, exact=False):
    lib = load()
    layout = np.ascontiguousarray(layout, np.int32)
    cloud = np.ascontiguousarray(cloud, np.float32)
    sb = np.zeros(3, np.int32)
    args = (C.byref(g), _p(layout), _p(cloud), int(variant), int(thr[0]), int(thr[1]), int(thr[2]),
            float(voxel_size), int(subdiv), int(offset[0]), int(offset[1]), int(offset[2]),
            int(color_mode), int(exact))
    hn = lib.orc_c3hlac(*args, None, _p(sb))
    if hn < 0:
        return np.zeros((0, variant), np.float32), tuple(int(x) for x in sb), int(hn)
    feat = np.zeros((max(hn, 1), variant), np.float32)
    hn2 = lib.orc_c3hlac(*args, _p(feat), _p(sb))
    if hn2 < 0:  # -5: a centroid's subdivision past the last one (out of bounds in the reference)
        return np.zeros((0, variant), np.float32), tuple(int(x) for x in sb), int(hn2)
    assert hn2 == hn
    return feat[:hn], tuple(int(x) for x in sb), int(hn)


def exist(feat):
    feat = np.ascontiguousarray(feat, np.float32)
    out = np.zeros(feat.shape[0], np.int32)
    if feat.shape[0]:
        load().orc_exist(_p(feat), feat.shape[0], feat.shape[1], _p(out))
    return out


class Lists:
    """SearchObjMulti list state (M x rank): score, x, y, z, mode."""

    def __init__(self, M, rank):
        self.M, self.rank = M, rank
        self.score = np.zeros(M * rank, np.float64)
        self.x = np.zeros(M * rank, np.int32)
        self.y = np.zeros(M * rank, np.int32)
        self.z = np.zeros(M * rank, np.int32)
        self.mode = np.zeros(M * rank, np.int32)

    def clean(self):
        self.score[:] = 0
        self.x[:] = 0
        self.y[:] = 0
        self.z[:] = 0

    def records(self):
        return [[(float(self.score[m * self.rank + i]), int(self.x[m * self.rank + i]),
                  int(self.y[m * self.rank + i]), int(self.z[m * self.rank + i]),
                  int(self.mode[m * self.rank + i])) for i in range(self.rank)] for m in range(self.M)]


def search(subdiv, feat, exist_, axis_p, axis_q, ranges, rank_or_lists, thr, rotate=True,
           dbl=False, fmax=None, want_scores=False):
    """Run setData + search (SearchObjMulti semantics).  axis_p (D,F) whitened or None."""
    lib = load()
    feat = np.ascontiguousarray(feat, np.float32)
    exist_ = np.ascontiguousarray(exist_, np.int32)
    axis_q = np.ascontiguousarray(axis_q, np.float32)
    M, r, D = axis_q.shape
    F = feat.shape[1]
    if axis_p is not None:
        axis_p = np.ascontiguousarray(axis_p, np.float32)
    L = rank_or_lists if isinstance(rank_or_lists, Lists) else Lists(M, int(rank_or_lists))
    fm = None if fmax is None else np.ascontiguousarray(fmax, np.float32)
    scores = None
    if want_scores:
        xn, yn, zn = subdiv
        tot = 0
        for (xr, yr, zr) in _mode_ranges(ranges, rotate):
            xe, ye, ze = xn - xr + 1, yn - yr + 1, zn - zr + 1
            if xe > 0 and ye > 0 and ze > 0:
                tot += xe * ye * ze * M
        scores = np.zeros(max(tot, 1), np.float64)
    nm = lib.orc_search(int(subdiv[0]), int(subdiv[1]), int(subdiv[2]), _p(feat), F, _p(exist_),
                        _p(axis_p), D, _p(fm), 0 if fm is None else fm.size, _p(axis_q), M, r,
                        int(ranges[0]), int(ranges[1]), int(ranges[2]), L.rank, int(thr), int(bool(rotate)),
                        int(bool(dbl)), _p(L.score), _p(L.x), _p(L.y), _p(L.z), _p(L.mode), _p(scores))
    if nm < 0:
        raise RuntimeError("orc_search failed %d" % nm)
    return L, nm, scores


def _mode_ranges(ranges, rotate):
    r1, r2, r3 = ranges
    R = {0: (r1, r2, r3), 1: (r1, r3, r2), 2: (r2, r1, r3), 3: (r2, r3, r1), 4: (r3, r1, r2), 5: (r3, r2, r1)}
    return [R[m] for m in mode_schedule(ranges, rotate)]


def mode_schedule(ranges, rotate=True):
    r1, r2, r3 = ranges
    if not rotate:
        return [0]
    if r1 == r2:
        return [0] if r2 == r3 else [0, 1, 4]
    if r2 == r3:
        return [0, 4, 5]
    if r1 == r3:
        return [0, 4, 2]
    return [0, 1, 2, 3, 4, 5]


def remove_overlap(L, ranges):
    load().orc_remove_overlap(L.M, L.rank, int(ranges[0]), int(ranges[1]), int(ranges[2]),
                              _p(L.score), _p(L.x), _p(L.y), _p(L.z), _p(L.mode))
    return L


def pca_read(path, ascii=False, max_dim=4096):
    buf = np.zeros(max_dim * max_dim, np.float32)
    var = np.zeros(max_dim, np.float32)
    mean = np.zeros(max_dim, np.float32)
    hm = C.c_int()
    dim = load().orc_pca_read(str(path).encode(), int(ascii), _p(buf), _p(var), _p(mean), C.byref(hm), max_dim)
    if dim < 0:
        raise RuntimeError("orc_pca_read failed %d" % dim)
    return buf[: dim * dim].reshape(dim, dim).T.copy(), var[:dim].copy(), (mean[:dim].copy() if hm.value else None)


def grid_inputs(words, div_b, leaf, min_b=(0, 0, 0)):
    """(grid dict, leaf_layout, cloud) for a packed colour/occupancy grid (uint32 words in
    z, y, x order, 0 = empty, else 1<<24 | rgb): the inputs getVoxelGrid would leave for a
    cloud with one point at the centre of every occupied cell, so centroid-derived and
    index-derived cells coincide (the grid-only entry points' definition)."""
    words = np.ascontiguousarray(words, np.uint32).reshape(-1)
    dx, dy, dz = (int(v) for v in div_b)
    assert words.size == dx * dy * dz
    occ = words != 0
    layout = np.full(words.size, -1, np.int32)
    idx = np.flatnonzero(occ)
    layout[idx] = np.arange(idx.size, dtype=np.int32)
    x, y, z = idx % dx, (idx // dx) % dy, idx // (dx * dy)
    lf = np.float64(np.float32(leaf))
    cloud = np.empty((idx.size, 4), np.float32)
    cloud[:, 0] = ((x + int(min_b[0]) + 0.5) * lf).astype(np.float32)
    cloud[:, 1] = ((y + int(min_b[1]) + 0.5) * lf).astype(np.float32)
    cloud[:, 2] = ((z + int(min_b[2]) + 0.5) * lf).astype(np.float32)
    cloud[:, 3] = (words[idx] & np.uint32(0xFFFFFF)).view(np.float32)
    g = OrcGrid()
    for a, (d, m) in enumerate(zip((dx, dy, dz), min_b)):
        g.div_b[a] = d
        g.min_b[a] = int(m)
        g.max_b[a] = int(m) + d - 1
    g.n_valid = idx.size
    g.n_occ = idx.size
    g.leaf = float(leaf)
    g.inv_leaf = float(np.float32(1) / np.float32(leaf))
    return g, layout, cloud
