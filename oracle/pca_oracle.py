"""CPU restatement of the reference's PCA training path (TEST INFRASTRUCTURE ONLY).

Only tests/ use this module: it is the checker of the GPU PCA training entry points
(csrc/pca.hip), never part of the product path.

Restates
  - pcl::rotateFeature90 (c3_hlac/src/c3_hlac.cpp:49-172): per mode, the 13 neighbour
    offset slots of every (centre colour i, neighbour colour j) block are permuted, and
    the slots whose offset the rotation reverses swap i and j;
  - the 24-rotation augmentation order of pca_models.cpp:109-171;
  - compressFeature (pca_models.cpp:48-63): float32 axis_t * f, whitened by sqrt(var);
  - PCA::addData (pca.cpp:48-69), PCA::solve (pca.cpp:73-105) with the eigensolve in
    float64 (Eigen's SelfAdjointEigenSolver<MatrixXf> is not available here) and
    sortVecAndVal's stable descending bubble sort (pca.cpp:244-271);
  - PCA::write (pca.cpp:190-240).
The eigen solve is therefore pinned only by this restatement (parity unpinned against
Eigen itself); the rotation maps are pinned by tests/golden/rotate90_map.json, which
oracle/gen_rotmap.py extracted mechanically from the reference source.
"""
import struct

import numpy as np

# input slot (first-order offsets 6..14, 60..63 of block (i, j)) -> (output slot,
# i/j swapped) per RotateMode, read off c3_hlac.cpp:77-160
_SLOTS = [6, 7, 8, 9, 10, 11, 12, 13, 14, 60, 61, 62, 63]
_MODES = {
    0: [(8, 0), (11, 0), (14, 0), (7, 0), (10, 0), (13, 0), (6, 0), (9, 0), (12, 0), (62, 0), (63, 1), (60, 1), (61, 0)],
    1: [(8, 0), (62, 0), (12, 1), (11, 0), (63, 1), (9, 1), (14, 0), (60, 1), (6, 1), (7, 0), (61, 0), (13, 1), (10, 0)],
    2: [(12, 0), (13, 0), (14, 0), (62, 1), (61, 1), (60, 1), (8, 1), (7, 1), (6, 1), (9, 0), (10, 0), (11, 0), (63, 0)],
    3: [(12, 0), (9, 0), (6, 0), (13, 0), (10, 0), (7, 0), (14, 0), (11, 0), (8, 0), (62, 1), (63, 0), (60, 0), (61, 1)],
}
R_MODE_1, R_MODE_2, R_MODE_3, R_MODE_4 = 0, 1, 2, 3


def _stride(slot):
    return 9 if slot < 60 else 4


def rotate_map_half(mode):
    """map[o] = input index of output o over one 495/486-dim half, indices 0..473."""
    m = np.arange(474)
    for (oslot, sw), islot in zip(_MODES[mode], _SLOTS):
        for i in range(6):
            for j in range(6):
                src = islot + i * _stride(islot) + j * 78
                a, b = (j, i) if sw else (i, j)
                m[oslot + a * _stride(oslot) + b * 78] = src
    return m


def rotate_map(dim, mode):
    """rotateFeature90 as a gather map over a whole vector (981 = 495 + 486 halves)."""
    if dim in (495, 486):
        m = np.arange(dim)
        m[:474] = rotate_map_half(mode)
        return m
    if dim == 981:
        return np.concatenate([rotate_map(495, mode), 495 + rotate_map(486, mode)])
    raise ValueError("rotateFeature90: improper dimension %d" % dim)


def rotate_feature90(v, mode):
    v = np.asarray(v)
    return v[..., rotate_map(v.shape[-1], mode)]


def rotations24(f):
    """The 24 vectors pca_models.cpp:109-171 adds for one feature f, in its order."""
    R = lambda v, m: rotate_feature90(v, m)
    out = [f]
    pre = f
    for _ in range(3):
        pre = R(pre, R_MODE_2)
        out.append(pre)
    pre2 = R(f, R_MODE_3)
    for _ in range(2):  # R3 f, then R3 R3 f (each followed by 3 x R2)
        out.append(pre2)
        pre = pre2
        for _ in range(3):
            pre = R(pre, R_MODE_2)
            out.append(pre)
        pre2 = R(pre2, R_MODE_3)
    out.append(pre2)  # R3^3 f
    pre = pre2
    for _ in range(3):
        pre = R(pre, R_MODE_2)
        out.append(pre)
    for m in (R_MODE_1, R_MODE_4):
        pre = R(f, m)
        out.append(pre)
        for _ in range(3):
            pre = R(pre, R_MODE_2)
            out.append(pre)
    assert len(out) == 24
    return out


def compress(f, axis, var, whitening=True):
    """compressFeature: axis F x D (the first D eigenvectors as columns), float32."""
    v = (axis.T.astype(np.float32) @ np.asarray(f, np.float32)).astype(np.float32)
    if whitening:
        v = (v / np.sqrt(np.asarray(var, np.float32))).astype(np.float32)
    return v


def train(rows, axis=None, var=None, rotate=False, mean_flg=False, reg=None, whitening=True, exact=False):
    """PCA of the vectors pca_models / pca_scene add: rows (n x F) -> each row (and its
    23 rotations if rotate) -> compress (if axis) -> addData.  float64 accumulation.
    exact: compress in float64 (the float32 compressFeature otherwise).
    Returns (axis dim x dim, columns = eigenvectors by descending variance, variance,
    mean or None, nsample, correlation before the eigensolve)."""
    rows = np.asarray(rows, np.float32)
    vecs = []
    for f in rows:
        vecs.extend(rotations24(f) if rotate else [f])
    X = np.asarray(vecs, np.float64)
    if axis is not None and exact:
        P = np.asarray(axis, np.float64)
        if whitening:
            P = P / np.sqrt(np.asarray(var, np.float32)).astype(np.float64)
        X = X @ P
    elif axis is not None:
        X = np.asarray([compress(g, axis, var, whitening) for g in X.astype(np.float32)], np.float64)
    n = X.shape[0]
    C = X.T @ X / n  # pca.cpp:80-88
    mean = None
    if mean_flg:
        mean = X.sum(0) / n
        C = C - np.outer(mean, mean)
    if reg is not None:
        C = C + float(np.float32(reg)) * np.eye(C.shape[0])  # regularization_nolm is a float
    w, V = np.linalg.eigh(C)
    order = sort_desc(w)
    return V[:, order], w[order], mean, n, C


def train_f32(rows, axis=None, var=None, rotate=False, mean_flg=False, reg=None, whitening=True):
    """The reference's own float32 numerics (pca.cpp:48-105), as pca_models / pca_scene run it:
    each vector (and its 23 rotations) compressed by compressFeature in float32, then
    PCA::addData one vector at a time -- `correlation(idx) += val * feature[j]` on the upper
    triangle of a float MatrixXf (product rounded to float, then added: no FMA in the x86-64
    build), `mean(i) += feature[i]` in float --, PCA::solve's `*= inv_nsample` (a double,
    the float result of float * double), the mirror, `mean *= inv_nsample`,
    `correlation -= mean * mean^T` (float), the float regularisation, and the eigensolve in
    float32 (Eigen's SelfAdjointEigenSolver<MatrixXf> is not available here: LAPACK ssyevd,
    also float32, stands in; both are backward-stable tridiagonal solvers, so only last-ulp
    eigenvector components and near-degenerate eigenvalues can differ).
    Returns as train(): (axis, variance, mean or None, nsample, correlation) in float32."""
    rows = np.asarray(rows, np.float32)
    vecs = []
    for f in rows:
        vecs.extend(rotations24(f) if rotate else [f])
    if axis is not None:
        vecs = [compress(g, axis, var, whitening) for g in vecs]
    X = np.asarray(vecs, np.float32)
    n, dim = X.shape
    C = np.zeros((dim, dim), np.float32)
    mean = np.zeros(dim, np.float32)
    iu = np.triu_indices(dim)
    for f in X:  # addData: sequential float accumulation, one vector at a time (the whole
        if mean_flg:  # square: f_j f_i == f_i f_j, so its upper triangle is addData's)
            mean += f
        C += np.outer(f, f)
    inv = 1.0 / float(n)  # solve: const double inv_nsample
    C[iu] = (C[iu].astype(np.float64) * inv).astype(np.float32)
    C = np.triu(C) + np.triu(C, 1).T
    if mean_flg:
        mean = (mean.astype(np.float64) * inv).astype(np.float32)
        C = (C - np.outer(mean, mean).astype(np.float32)).astype(np.float32)
    if reg is not None:
        C[np.diag_indices(dim)] += np.float32(reg)
    w, V = np.linalg.eigh(C)  # float32 in, float32 out
    order = sort_desc(w)
    return V[:, order], w[order], (mean if mean_flg else None), n, C


def sort_desc(vals):
    """sortVecAndVal's index order: bubble sort swapping only on strict '<' (stable)."""
    idx = list(range(len(vals)))
    for i in range(len(vals)):
        for j in range(1, len(vals) - i):
            if vals[idx[j - 1]] < vals[idx[j]]:
                idx[j - 1], idx[j] = idx[j], idx[j - 1]
    return np.asarray(idx)


def write_binary(axis, var, mean=None):
    """PCA::write(ascii=false) bytes: dim, axis(j, i) column by column, var, [mean]."""
    dim = len(var)
    out = struct.pack("<i", dim) + np.asarray(axis, np.float32).T.tobytes() + np.asarray(var, np.float32).tobytes()
    if mean is not None:
        out += np.asarray(mean, np.float32).tobytes()
    return out
