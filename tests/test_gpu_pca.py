"""GPU parity of the PCA training path (csrc/pca.hip) against the
restatement in oracle/pca_oracle.py.

- rotateFeature90 on device rows: bit-exact (a gather) for every mode and dimension.
- pca_scene.cpp shape: 981-dim rows, mean_flg false -> the correlation the solve
  decomposes within 1e-12 relative of the float64 oracle (the device sums are f64 from
  exact f32 x f32 products), eigenvalues within 1e-9 of the largest, eigenvectors of
  well-separated eigenvalues equal up to sign (|<u, v>| >= 1 - 1e-6).
- pca_models.cpp shape: rows compressed by a scene axis (D = 100, whitened) plus the 23
  rotations of each row -> the same checks against the oracle that rotates and compresses
  every vector explicitly; and against the float32 compressFeature order within 1e-4.
- mean_flg + regularisation, host vs device rows, batching, the error cases.
- write -> c3h_pca_read round trip of a trained subspace.
Eigenvector signs are arbitrary in the reference too (Eigen), hence "up to sign"."""
import numpy as np
import pytest

import c3hlac
import pca_oracle as pco

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(ctx):
    import torch
    return torch.device("cuda", 0)


def _rows(n, F, rank=12, seed=0):
    """non-negative feature-like rows with a decaying spectrum"""
    rng = np.random.default_rng(seed)
    Z = rng.random((n, rank)) * (0.6 ** np.arange(rank))
    B = rng.random((rank, F))
    X = Z @ B + 0.01 * rng.random((n, F))
    X[:, rng.random(F) < 0.05] = 0  # some bins never fire
    return X.astype(np.float32)


def _compare(pca, ref, what, k_vec=20):
    axis_r, var_r, mean_r, n_r, C_r = ref
    assert pca.nsample == n_r, what
    C = pca.correlation()
    scale = np.abs(C_r).max()
    assert np.abs(C - C_r).max() <= 1e-12 * scale, (what, np.abs(C - C_r).max() / scale)
    lam = np.asarray(var_r)
    np.testing.assert_allclose(pca.variance, lam.astype(np.float32), rtol=0, atol=1e-9 * lam[0] + 1e-30)
    d = len(lam)
    assert (np.diff(pca.variance) <= 0).all(), what  # sortVecAndVal: descending
    A = pca.axis.astype(np.float64)
    np.testing.assert_allclose(A.T @ A, np.eye(d), atol=1e-5)
    for i in range(min(k_vec, d)):
        gap = min(abs(lam[i] - lam[j]) for j in (i - 1, i + 1) if 0 <= j < d) / lam[0]
        if gap < 1e-5:
            continue
        dot = abs(float(A[:, i] @ axis_r[:, i]))
        assert dot >= 1 - 1e-6, (what, i, dot, gap)


@pytest.mark.parametrize("dim", [981, 495, 486])
def test_rotate_feature90_device(dev, dim):
    import torch
    x = _rows(37, dim, seed=dim)
    d_in = torch.from_numpy(x).to(dev)
    for mode in range(4):
        d_out = torch.empty_like(d_in)
        c3hlac.rotate_feature90(d_in, d_out, mode)
        torch.cuda.synchronize()
        assert np.array_equal(d_out.cpu().numpy(), pco.rotate_feature90(x, mode)), (dim, mode)


def test_pca_scene_shape(dev):
    import torch
    X = _rows(3000, 981, seed=1)
    pca = c3hlac.PCA(mean_flg=False)
    pca.add_data(torch.from_numpy(X[:1234]).to(dev))   # device rows
    pca.add_data(X[1234:])                              # host rows
    pca.solve()
    assert pca.axis.shape == (981, 981)
    _compare(pca, pco.train(X), "scene")
    pca.close()


def test_pca_models_shape_rotate24(dev):
    import torch
    scene = _rows(2000, 981, seed=2)
    sp = c3hlac.PCA(mean_flg=False)
    sp.add_data(scene)
    sp.solve()
    D = 100
    X = _rows(300, 981, rank=6, seed=3)
    mp = c3hlac.PCA(mean_flg=False)
    mp.set_compress(sp.axis, sp.variance, D)
    mp.add_data(torch.from_numpy(X).to(dev), rotate24=True)
    mp.solve()
    assert mp.axis.shape == (D, D) and mp.nsample == 24 * 300
    axis_d = sp.axis[:, :D]
    _compare(mp, pco.train(X, axis_d, sp.variance[:D], rotate=True, exact=True), "models exact")
    # the reference's float32 compressFeature order: same correlation within 1e-4
    ref32 = pco.train(X, axis_d, sp.variance[:D], rotate=True)
    C = mp.correlation()
    assert np.abs(C - ref32[4]).max() <= 1e-4 * np.abs(ref32[4]).max()
    sp.close()
    mp.close()


def test_pca_mean_regularisation_and_batches(dev):
    X = _rows(1500, 117, seed=4)
    pca = c3hlac.PCA(mean_flg=True)
    for a in range(0, 1500, 200):  # ragged batches
        pca.add_data(X[a:a + 200])
    pca.solve(True, 0.001)
    ref = pco.train(X, mean_flg=True, reg=0.001)
    _compare(pca, ref, "mean+reg")
    np.testing.assert_allclose(pca.getMean(), ref[2].astype(np.float32), rtol=1e-6)
    # solve again after more data: the accumulated sums are kept
    pca.add_data(X[:10])
    pca.solve()
    _compare(pca, pco.train(np.concatenate([X, X[:10]]), mean_flg=True), "resolve")
    pca.close()


def test_pca_errors(dev):
    pca = c3hlac.PCA(mean_flg=False)
    with pytest.raises(c3hlac._capi.C3HError, match="no data"):
        pca.solve()
    with pytest.raises(c3hlac._capi.C3HError, match="improper dimension"):
        pca.add_data(_rows(4, 117), rotate24=True)
    pca.add_data(_rows(4, 117))
    with pytest.raises(c3hlac._capi.C3HError, match="vector size differs"):
        pca.add_data(_rows(4, 118))
    with pytest.raises(c3hlac._capi.C3HError, match="data already added"):
        pca.set_compress(np.eye(117, dtype=np.float32), None, 10)
    pca.solve()
    with pytest.raises(c3hlac._capi.C3HError, match="no mean vector"):
        pca.getMean()
    pca.close()


def test_trained_subspace_round_trips_through_pca_read(dev, tmp_path):
    X = _rows(500, 137, seed=5)
    pca = c3hlac.PCA(mean_flg=True)
    pca.add_data(X)
    pca.solve()
    out = tmp_path / "pca_result"
    pca.write(out)
    a, v, m = c3hlac.pca_read(out)
    assert np.array_equal(a, pca.axis) and np.array_equal(v, pca.variance) and np.array_equal(m, pca.mean)
    pca.close()


@pytest.mark.parametrize("shape", ["scene", "models"])
def test_gpu_training_vs_reference_float32_order(dev, shape):
    """The GPU trains in f64 (exact products, f64 sums, dsyevd); the reference accumulates
    PCA::addData in a float MatrixXf and solves with a float SelfAdjointEigenSolver
    (pca.cpp:48-105).  Against pco.train_f32 -- that float32 order restated, compressFeature
    in float32, the eigensolve in float32 -- the stated tolerances: correlation within 1e-5
    of its largest entry, eigenvalues within 1e-5 of the largest, and the similarity scores
    |Q_r g| / |g| of held-out scenes through the first r = 5, 10, 20 axes (the SearchObj
    projection, search.cpp:915-968) within 1e-5 relative wherever the eigengap after axis r
    is at least 1e-4 of the largest eigenvalue.  Measured on the CPU restatements: 2e-6, 1e-6,
    3e-7 (the scene rows' noise eigenvalues are 6e-11 apart at r = 20: there neither float
    order determines the subspace, 7e-3)."""
    if shape == "scene":
        X = _rows(2000, 981, seed=11)
        pca = c3hlac.PCA(mean_flg=False)
        pca.add_data(X)
        pca.solve()
        ref = pco.train_f32(X)
        held = _rows(200, 981, seed=12).astype(np.float64)
    else:
        scene = _rows(2000, 981, seed=2)
        sp = c3hlac.PCA(mean_flg=False)
        sp.add_data(scene)
        sp.solve()
        D = 100
        X = _rows(300, 981, rank=6, seed=3)
        pca = c3hlac.PCA(mean_flg=False)
        pca.set_compress(sp.axis, sp.variance, D)
        pca.add_data(X, rotate24=True)
        pca.solve()
        ref = pco.train_f32(X, sp.axis[:, :D], sp.variance[:D], rotate=True)
        held = np.asarray([pco.compress(g, sp.axis[:, :D], sp.variance[:D]) for g in _rows(200, 981, rank=6, seed=9)],
                          np.float64)
        sp.close()
    axis32, lam32, _, n32, C32 = ref
    assert pca.nsample == n32
    C = pca.correlation()
    assert np.abs(C - C32).max() <= 1e-5 * np.abs(C32).max()
    k = 25
    assert (np.abs(pca.variance[:k].astype(np.float64) - lam32[:k]) <= 1e-5 * lam32[0]).all()
    checked = 0
    for r in (5, 10, 20):
        s_gpu = np.linalg.norm(held @ pca.axis[:, :r].astype(np.float64), axis=1) / np.linalg.norm(held, axis=1)
        s_ref = np.linalg.norm(held @ axis32[:, :r].astype(np.float64), axis=1) / np.linalg.norm(held, axis=1)
        gap = float(lam32[r - 1] - lam32[r]) / float(lam32[0])
        rel = float((np.abs(s_gpu - s_ref) / s_ref).max())
        print("%s r=%d eigengap %.1e score rel diff %.1e" % (shape, r, gap, rel))
        # a subspace whose last eigengap is below ~1e-4 of the largest eigenvalue is not
        # determined by the reference's own float32 arithmetic (perturbation ~ eps_f32 / gap):
        # the tolerance is stated for well-separated subspaces only
        if gap >= 1e-4:
            assert rel <= 1e-5, (shape, r, gap, rel)
            checked += 1
    assert checked >= 1
    pca.close()
