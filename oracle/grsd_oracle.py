"""CPU restatement of the GRSD / VOSCH feature path (TEST INFRASTRUCTURE ONLY).

Only tests/ use this module: it is the checker of the GPU normal / RSD / GRSD kernels
(csrc/rsd.hip), never part of the product path.

Restates, for pcl::PointXYZRGB clouds:
  - pcl::NormalEstimation with a radius search (grsd_colorCHLAC_tools.hpp:63-87,
    computeNormal; normals_radius_search = 0.02, grsd_colorCHLAC_tools.h:28): the PCL
    algorithm (third-party, PCL 1.x as shipped with ROS fuerte; not in /root/reference):
    covariance of the neighbours within the radius (the point itself included; fewer than
    3 -> NaN), the eigenvector of the smallest eigenvalue, flipped towards the viewpoint
    (0, 0, 0), curvature = lambda_min / trace.  float64 here.
  - pcl::RSDEstimation<..., PrincipalRadiiRSD> (grsd_colorCHLAC_tools.hpp:164-180): per
    downsampled point, the cloud points within max(rsd_radius_search, leaf/2*sqrt(3));
    PCL's computeRSD (nr_subdiv 5, plane_radius 0.2): angles between the normals of the
    nearest neighbour ("begin") and every other neighbour binned by their distance to it,
    min / max angle per bin, least-squares radii, x1.1 / x0.9, ordered.
  - get_type (grsd_colorCHLAC_tools.hpp:99-118) and extractGRSDSignature21 (:131-296):
    the 6 x 6 type transition counts over the 26 neighbour voxels of every occupied
    voxel (EMPTY for unoccupied), per subdivision, upper triangle i <= j, first 20 bins.
Ties in the neighbour order of a radius search (FLANN) are broken by point index here.
"""
import numpy as np

NOISE, PLANE, CYLINDER, SPHERE, EDGE, EMPTY = 0, 1, 2, 3, 4, 5


def _finite(p):
    return np.isfinite(p[:, :3]).all(1)


def normals(pts, radius, vp=(0.0, 0.0, 0.0)):
    """(n, 4) float32 x y z rgb -> (n, 4) float64 nx ny nz curvature (NaN where undefined)."""
    xyz = pts[:, :3].astype(np.float32)
    ok = _finite(pts)
    out = np.full((len(pts), 4), np.nan)
    idx_ok = np.flatnonzero(ok)
    P = xyz[idx_ok]
    r2 = np.float32(radius) * np.float32(radius)
    for a, i in enumerate(idx_ok):
        d = P - xyz[i]
        d2 = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
        nb = P[d2 < r2].astype(np.float64)
        if len(nb) < 3:
            continue
        m = nb.mean(0)
        C = (nb - m).T @ (nb - m) / len(nb)
        w, V = np.linalg.eigh(C)
        n = V[:, 0]
        if np.dot(np.asarray(vp, np.float64) - xyz[i].astype(np.float64), n) < 0:
            n = -n
        s = w.sum()
        out[i, :3] = n
        out[i, 3] = w[0] / s if s != 0 else 0.0
    return out


def compute_rsd(surface, nrm, centre, max_dist, nr_subdiv=5, plane_radius=0.2):
    """PCL computeRSD on the surface points within max_dist of centre -> (r_min, r_max)."""
    max_dist = float(np.float32(max_dist))  # the radius as the device holds it (float)
    xyz = surface[:, :3].astype(np.float32)
    ok = _finite(surface)
    d = xyz - centre.astype(np.float32)
    d2 = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
    cand = np.flatnonzero(ok & (d2 < np.float32(max_dist) * np.float32(max_dist)))
    if len(cand) < 2:
        return 0.0, 0.0
    order = cand[np.lexsort((cand, d2[cand]))]  # ascending distance, ties by index
    b = order[0]
    mn = [0.0] + [np.inf] * (nr_subdiv - 1)
    mx = [0.0] + [-np.inf] * (nr_subdiv - 1)
    nb = nrm[b, :3].astype(np.float32)
    for i in order[1:]:
        ni = nrm[i, :3].astype(np.float32)
        cosine = float(np.float32(np.float32(ni[0] * nb[0] + ni[1] * nb[1]) + ni[2] * nb[2]))
        cosine = min(max(cosine, -1.0), 1.0) if cosine == cosine else cosine
        angle = np.arccos(cosine) if cosine == cosine else np.nan
        if angle > np.pi / 2:
            angle = np.pi - angle
        dv = xyz[i] - xyz[b]
        dist = float(np.sqrt(np.float64(np.float32(np.float32(dv[0] * dv[0] + dv[1] * dv[1]) + dv[2] * dv[2]))))
        if dist > max_dist:
            continue
        bd = min(int(np.floor(nr_subdiv * dist / max_dist)), nr_subdiv - 1)
        if mn[bd] > angle:
            mn[bd] = angle
        if mx[bd] < angle:
            mx[bd] = angle
    aa = ad = xa = xd = 0.0
    for di in range(nr_subdiv):
        if mx[di] >= 0:
            f = (di + 0.5) * max_dist / nr_subdiv
            aa += mn[di] * mn[di]
            ad += mn[di] * f
            xa += mx[di] * mx[di]
            xd += mx[di] * f
    rmin = np.float32(plane_radius if aa == 0 else min(ad / aa, plane_radius))
    rmax = np.float32(plane_radius if xa == 0 else min(xd / xa, plane_radius))
    rmin = np.float32(np.float64(rmin) * 1.1)  # float *= double (C promotion)
    rmax = np.float32(np.float64(rmax) * 0.9)
    return (float(rmin), float(rmax)) if rmin < rmax else (float(rmax), float(rmin))


def get_type(rmin, rmax):
    if rmin > 0.100:
        return PLANE
    if rmax > 0.175:
        return CYLINDER
    if rmin < 0.015:
        return NOISE
    if rmax - rmin < 0.050:
        return SPHERE
    return EDGE


REL13 = [(i, j, -1) for i in (-1, 0, 1) for j in (-1, 0, 1)] + [(i, -1, 0) for i in (-1, 0, 1)] + [(-1, 0, 0)]
REL26 = REL13 + [(-a, -b, -c) for a, b, c in REL13]


def grsd(cloud_pts, nrm, g, layout, cent, leaf, subdiv=0, offset=(0, 0, 0), rsd_radius=0.01):
    """extractGRSDSignature21 on a voxelised cloud: g = oracle grid (div_b, min_b),
    layout = leaf layout (-1 empty), cent = downsampled centroids (n_occ, 4) in layout
    order.  Returns (features (hist_num, 20) raw counts, subdiv_b, radii (n_occ, 2), types)."""
    max_dist = max(rsd_radius, leaf / 2 * np.sqrt(3))
    radii = np.array([compute_rsd(cloud_pts, nrm, c[:3], max_dist) for c in cent])
    types = np.array([get_type(a, b) for a, b in radii], np.int32)
    div = np.array(g.div_b[:3])
    mnb = np.array(g.min_b[:3])
    if subdiv > 0:
        inv_s = np.float32(1.0 / subdiv)
        sb = [int(np.ceil(np.float32((div[a] - offset[a]) * inv_s))) for a in range(3)]
    else:
        sb = [1, 1, 1]
    H = sb[0] * sb[1] * sb[2]
    T = np.zeros((H, 6, 6), np.int64)
    inv = np.float32(1.0) / np.float32(leaf)
    for idx, c in enumerate(cent):
        if H == 1:
            h = 0
        else:
            t = [int(np.floor(np.float32(c[a]) / np.float32(leaf))) - mnb[a] - offset[a] for a in range(3)]
            if min(t) < 0:
                continue
            ijk = [int(np.floor(np.float32(t[a]) * inv_s)) for a in range(3)]
            if ijk[0] >= sb[0] or ijk[1] >= sb[1] or ijk[2] >= sb[2]:
                continue
            h = ijk[0] + sb[0] * (ijk[1] + sb[1] * ijk[2])
        base = [int(np.floor(np.float32(c[a]) * inv)) - mnb[a] for a in range(3)]
        for r in REL26:
            q = [base[a] + r[a] for a in range(3)]
            if min(q) < 0 or q[0] >= div[0] or q[1] >= div[1] or q[2] >= div[2]:
                nt = EMPTY
            else:
                li = layout[q[0] + div[0] * (q[1] + div[1] * q[2])]
                nt = EMPTY if li < 0 else types[li]
            T[h, types[idx], nt] += 1
    iu = [(i, j) for i in range(6) for j in range(i, 6)][:20]
    feat = np.array([[T[h, i, j] for i, j in iu] for h in range(H)], np.float64)
    return feat, sb, radii, types
