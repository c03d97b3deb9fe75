"""Independent numpy restatement of the C3-HLAC path (TEST INFRASTRUCTURE ONLY).

Second, independent restatement used to cross-check the C oracle and to generate the
committed golden fixtures.  It works on the dense grid (vectorised, exact integers)
and takes the bin layout straight from the tables extracted from the reference's
unrolled code (tests/golden/binmap_*.json, see oracle/gen_binmap.py) instead of the
closed form the C oracle and the HIP kernel use.
"""
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parents[1] / "tests" / "golden"
REL = [(-1, -1, -1), (-1, 0, -1), (-1, 1, -1), (0, -1, -1), (0, 0, -1), (0, 1, -1),
       (1, -1, -1), (1, 0, -1), (1, 1, -1), (-1, -1, 0), (0, -1, 0), (1, -1, 0), (-1, 0, 0)]
F32 = np.float32


def binmap(dim):
    return json.loads((GOLDEN / ("binmap_%d.json" % dim)).read_text())


def lut(color_mode=1):
    """setColor channel pairs: 0 C3 float sin/cos, 1 C3 double (default), 2 ColorCHLAC."""
    if color_mode == 2:  # ColorCHLAC{,_RI}Estimation::setColor (color_chlac.hpp:148-153)
        v = np.arange(256, dtype=np.int64)
        return np.stack([v, 255 - v], 1)
    an = F32(np.pi / 510)
    v = np.arange(256, dtype=np.float32) * an  # float multiply, as v * angle_norm
    if color_mode == 1:
        s = np.trunc(255 * np.sin(v.astype(np.float64))).astype(np.int64)
        c = np.trunc(255 * np.cos(v.astype(np.float64))).astype(np.int64)
    else:
        s = np.trunc(F32(255) * np.sin(v)).astype(np.int64)
        c = np.trunc(F32(255) * np.cos(v)).astype(np.int64)
    return np.stack([s, c], 1)


def voxelize(pts, leaf, z_limit=np.inf):
    """PCL VoxelGrid semantics -> (div_b, min_b, words[z,y,x] uint32, leaf_layout)."""
    pts = np.asarray(pts, np.float32)
    xyz = pts[:, :3]
    ok = np.isfinite(xyz).all(1) & (xyz[:, 2] < F32(z_limit))
    xyz = xyz[ok]
    rgb = pts[ok, 3].view(np.uint32)
    if xyz.shape[0] == 0:
        return (0, 0, 0), (0, 0, 0), np.zeros((0, 0, 0), np.uint32), np.zeros(0, np.int32)
    inv = F32(1) / F32(leaf)
    ijk_f = np.floor(xyz * inv)
    min_b = ijk_f.min(0).astype(np.int64)
    max_b = ijk_f.max(0).astype(np.int64)
    div = max_b - min_b + 1
    ijk = (ijk_f - min_b.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    nvox = int(np.prod(div))
    cnt = np.bincount(idx, minlength=nvox)
    chans = [(rgb >> 16) & 255, (rgb >> 8) & 255, rgb & 255]
    sums = [np.bincount(idx, weights=c.astype(np.float64), minlength=nvox) for c in chans]
    occ = cnt > 0
    words = np.zeros(nvox, np.uint32)
    # PCL 1.0 on Eigen 3.0: the channel sums times (1 / n) in float, truncated
    rn = F32(1) / cnt[occ].astype(np.float32)
    means = [np.trunc(s[occ].astype(np.float32) * rn).astype(np.uint32) for s in sums]
    words[occ] = (1 << 24) | (means[0] << 16) | (means[1] << 8) | means[2]
    layout = np.full(nvox, -1, np.int32)
    layout[occ] = np.arange(int(occ.sum()), dtype=np.int32)
    return tuple(int(d) for d in div), tuple(int(m) for m in min_b), words.reshape(div[2], div[1], div[0]), layout


def _shift(a, d):
    """out[z,y,x] = a[z+dz, y+dy, x+dx] with zero outside."""
    dx, dy, dz = d
    out = np.zeros_like(a)
    Z, Y, X = a.shape[-3:]
    def sl(n, o):
        return slice(max(0, -o), min(n, n - o)), slice(max(0, o), min(n, n + o))
    (zo, zi), (yo, yi), (xo, xi) = sl(Z, dz), sl(Y, dy), sl(X, dx)
    out[..., zo, yo, xo] = a[..., zi, yi, xi]
    return out


def subdivisions(div, subdiv, offset):
    """setVoxelFilter (c3_hlac.cpp:204-231) float arithmetic -> (sb, hist_num, ok)."""
    if subdiv == 0:
        return (0, 0, 0), 1, True
    if subdiv < 0 or any(div[a] <= offset[a] for a in range(3)):
        return (0, 0, 0), 0, False
    inv = F32(1.0 / subdiv)
    sb = tuple(int(np.ceil(F32(div[a] - offset[a]) * inv)) for a in range(3))
    return sb, sb[0] * sb[1] * sb[2], True


def c3hlac(words, variant, thr, subdiv=0, offset=(0, 0, 0), color_mode=1):
    """Exact-integer C3-HLAC on a dense packed grid words[z,y,x] -> (feat, exist, sb)."""
    Z, Y, X = words.shape
    div = (X, Y, Z)
    sb, hn, ok = subdivisions(div, subdiv, offset)
    if not ok or min(thr) < 0:
        return np.zeros((0, variant), np.float32), np.zeros(0, np.int32), sb
    occ = words != 0
    r = ((words >> 16) & 255).astype(np.int64)
    g = ((words >> 8) & 255).astype(np.int64)
    b = (words & 255).astype(np.int64)
    L = lut(color_mode)
    a = np.stack([L[r, 0], L[r, 1], L[g, 0], L[g, 1], L[b, 0], L[b, 1]]) * occ
    br, bg, bb = (r > thr[0]).astype(np.int64), (g > thr[1]).astype(np.int64), (b > thr[2]).astype(np.int64)
    be = np.stack([br, 1 - br, bg, 1 - bg, bb, 1 - bb]) * occ
    # centre -> subdivision index (float arithmetic of computeC3HLAC)
    if hn == 1:
        hidx = np.zeros((Z, Y, X), np.int64)
        center = occ
    else:
        zz, yy, xx = np.meshgrid(np.arange(Z), np.arange(Y), np.arange(X), indexing="ij")
        inv = F32(1.0 / subdiv)
        t = [xx - offset[0], yy - offset[1], zz - offset[2]]
        center = occ & (t[0] >= 0) & (t[1] >= 0) & (t[2] >= 0)
        s = [np.floor(np.maximum(ti, 0).astype(np.float32) * inv).astype(np.int64) for ti in t]
        hidx = s[0] + s[1] * sb[0] + s[2] * sb[0] * sb[1]
    hflat = hidx[center]
    acc = np.zeros((hn, 981), np.float64)

    def add(bin_, vals):
        acc[:, bin_] += np.bincount(hflat, weights=vals[center].astype(np.float64), minlength=hn)

    m981 = binmap(981)
    nb_a = [_shift(a, d) for d in REL]
    nb_b = [_shift(be, d) for d in REL]
    for c, b_ in m981["zero"]:
        add(b_, a[c])
    for c, n, b_ in m981["auto"]:
        add(b_, a[c] * a[n])
    for c, b_ in m981["bin_zero"]:
        add(b_, be[c])
    for c, n, b_ in m981["bin_pairs"]:
        add(b_, be[c] * be[n])
    for k, c, n, b_ in m981["first"]:
        add(b_, a[c] * nb_a[k][n])
    for k, c, n, b_ in m981["bin_first"]:
        add(b_, be[c] * nb_b[k][n])
    acc = acc.astype(np.int64)
    if variant == 981:
        feat = acc.astype(np.float32)
        norm = np.ones(981, np.float32)
        norm[:6] = F32(1 / 255.0)
        norm[6:495] = F32(1 / 65025.0)
    else:
        m117 = binmap(117)
        out = np.zeros((hn, 117), np.int64)
        for c, b_ in m117["zero"]:
            out[:, b_] = acc[:, c]
        auto981 = {(c, n): b_ for c, n, b_ in m981["auto"]}
        for c, n, b_ in m117["auto"]:
            out[:, b_] = acc[:, auto981[(c, n)]]
        for c, b_ in m117["bin_zero"]:
            out[:, b_] = acc[:, 495 + c]
        for i, (c, n, b_) in enumerate(m117["bin_pairs"]):
            src = [x[2] for x in m981["bin_pairs"] if x[0] == c and x[1] == n][0]
            out[:, b_] = acc[:, src]
        first981 = {(k, c, n): b_ for k, c, n, b_ in m981["first"]}
        bfirst981 = {(k, c, n): b_ for k, c, n, b_ in m981["bin_first"]}
        for _, c, n, b_ in m117["first"]:
            out[:, b_] = sum(acc[:, first981[(k, c, n)]] for k in range(13))
        for _, c, n, b_ in m117["bin_first"]:
            out[:, b_] = sum(acc[:, bfirst981[(k, c, n)]] for k in range(13))
        feat = out.astype(np.float32)
        norm = np.ones(117, np.float32)
        norm[:6] = F32(1 / 255.0)
        norm[6:42] = F32(1 / 845325.0)
        norm[42:63] = F32(1 / 65025.0)
        norm[69:105] = F32(1 / 13.0)
    feat = (feat * norm).astype(np.float32)
    f0 = acc[:, 0].astype(np.float32) * F32(1 / 255.0)
    f1 = acc[:, 1].astype(np.float32) * F32(1 / 255.0)
    ex = (((f0 + f1) * F32(2)).astype(np.float64) + 0.001).astype(np.int64).astype(np.int32)
    return feat, ex, sb


# ---------------------------------------------------------------- search (float64)
def _ranges(mode, r):
    r1, r2, r3 = r
    return {0: (r1, r2, r3), 1: (r1, r3, r2), 2: (r2, r1, r3), 3: (r2, r3, r1), 4: (r3, r1, r2), 5: (r3, r2, r1)}[mode]


def mode_schedule(r, rotate=True):
    r1, r2, r3 = r
    if not rotate:
        return [0]
    if r1 == r2:
        return [0] if r2 == r3 else [0, 1, 4]
    if r2 == r3:
        return [0, 4, 5]
    if r1 == r3:
        return [0, 4, 2]
    return [0, 1, 2, 3, 4, 5]


def box_sums(vol, xr, yr, zr):
    """vol[z,y,x,...] -> sums over [x,x+xr) x [y,y+yr) x [z,z+zr) for every valid origin."""
    Z, Y, X = vol.shape[:3]
    s = np.zeros((Z + 1, Y + 1, X + 1) + vol.shape[3:], vol.dtype)
    s[1:, 1:, 1:] = vol.cumsum(0).cumsum(1).cumsum(2)
    ze, ye, xe = Z - zr + 1, Y - yr + 1, X - xr + 1
    def S(z0, y0, x0):
        return s[z0:z0 + ze, y0:y0 + ye, x0:x0 + xe]
    return (S(zr, yr, xr) - S(0, yr, xr) - S(zr, 0, xr) - S(zr, yr, 0)
            + S(0, 0, xr) + S(0, yr, 0) + S(zr, 0, 0) - S(0, 0, 0))


def scores(sb, feat, exist, axis_p, axis_q, r, thr, rotate=True, fmax=None):
    """float64 per-position scores in the reference's (mode, z, y, x) order."""
    xn, yn, zn = sb
    if xn * yn * zn < 1 or xn * yn * zn != feat.shape[0]:
        return []  # setData returns early; the caller skips search()
    f = feat.astype(np.float64)
    if fmax is not None:
        fm = np.asarray(fmax, np.float32)
        f = feat.astype(np.float32).copy()
        L = min(len(fm), f.shape[1])
        for t in range(L):
            col = f[:, t]
            f[:, t] = np.where(fm[t] == 0, 0, np.where(col == fm[t], 1, col / fm[t]))
        f = f.astype(np.float64)
    G = f @ axis_p.astype(np.float64).T if axis_p is not None else f
    Gv = G.reshape(zn, yn, xn, -1)
    Ev = exist.astype(np.int64).reshape(zn, yn, xn)
    out = []
    for mode in mode_schedule(r, rotate):
        xr, yr, zr = _ranges(mode, r)
        if xn - xr + 1 <= 0 or yn - yr + 1 <= 0 or zn - zr + 1 <= 0:
            continue
        eb = box_sums(Ev, xr, yr, zr).reshape(-1)
        fb = box_sums(Gv, xr, yr, zr).reshape(eb.size, -1)
        ff = np.sqrt((fb * fb).sum(1))
        q = np.einsum("mrd,pd->mpr", axis_q.astype(np.float64), fb)
        sc = np.sqrt((q * q).sum(2)) / ff[None, :]
        sc[:, ~(eb > thr)] = -1.0
        out.append((mode, xn - xr + 1, yn - yr + 1, sc))
    return out


def replay(mode_scores, r, rank, lists=None):
    """Reference rank update (search.cpp:464-474, 327-356) over per-mode score arrays."""
    M = mode_scores[0][3].shape[0] if mode_scores else 1
    if lists is None:
        lists = [[[0.0, 0, 0, 0, 0] for _ in range(rank)] for _ in range(M)]
    for mode, xe, ye, sc in mode_scores:
        xr, yr, zr = _ranges(mode, r)
        for m in range(M):
            Lm = lists[m]
            # candidates at or below the current rank-th score can never enter (the
            # list only grows), so the scan can start from the strict-greater set
            for p in np.nonzero(sc[m] > Lm[rank - 1][0])[0]:
                dot = sc[m, p]
                x, y, z = int(p % xe), int((p // xe) % ye), int(p // (xe * ye))
                for i in range(rank):
                    if dot > Lm[i][0]:
                        num = 0
                        while num < rank - 1:
                            e = Lm[num]
                            oxr, oyr, ozr = _ranges(e[4], r)
                            v1 = e[1] - x
                            v1 = -v1 - oxr if v1 < 0 else v1 - xr
                            v2 = e[2] - y
                            v2 = -v2 - oyr if v2 < 0 else v2 - yr
                            v3 = e[3] - z
                            v3 = -v3 - ozr if v3 < 0 else v3 - zr
                            if v1 <= 0 and v2 <= 0 and v3 <= 0:
                                break
                            num += 1
                        for j in range(num - i):
                            Lm[num - j] = list(Lm[num - 1 - j])
                        if i <= num:
                            Lm[i] = [float(dot), x, y, z, mode]
                        break
    return lists


# ---------------------------------------------------------------- auto colour threshold
def color_histogram(words):
    """calc_scene_auto_threshold.cpp:92-108: per occupied voxel of the downsampled cloud
    (= the packed grid's non-empty words) one count in each channel's 256-bin histogram."""
    w = np.asarray(words, dtype=np.uint32).reshape(-1)
    w = w[w != 0]
    r, g, b = (w >> 16) & 255, (w >> 8) & 255, w & 255
    return np.stack([np.bincount(c.astype(np.int64), minlength=256) for c in (r, g, b)]).astype(np.int64)


def auto_threshold(hist):
    """calc_scene_auto_threshold.cpp:111-146, loop for loop (Python ints: exact where the
    tool's int sums are defined) -> (threshold[3], totalAve[3])."""
    hist = np.asarray(hist, dtype=np.int64)
    total = int(hist[0].sum())
    if total <= 0:
        raise ValueError("empty histogram (the tool divides by zero)")
    thr, ave = [], []
    for i in range(3):
        h = [int(v) for v in hist[i]]
        total_ave = 0.0
        for j in range(256):  # :113-118
            total_ave += j * h[j]
        total_ave *= 1 / float(total)
        each_ave, each_num = [0.0] * 256, [0] * 256  # :120-133
        each_num[0] = h[0]
        tmp = 0
        for j in range(1, 256):
            each_num[j] = each_num[j - 1] + h[j]
            tmp += j * h[j]
            each_ave[j] = 0.0 if each_num[j] == 0 else tmp / each_num[j]
        max_var, t = 0.0, 0  # :135-146
        for j in range(1, 256):
            if each_num[j] != 0:
                if each_num[j] == total:
                    break
                ave_sub = each_ave[j] - total_ave
                var = ave_sub * ave_sub * (each_num[j] / float(total - each_num[j]))
                if var > max_var:
                    max_var, t = var, j
        thr.append(t)
        ave.append(total_ave)
    return np.array(thr, np.int32), np.array(ave)
