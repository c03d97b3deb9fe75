"""MI355X-native colour-voxel C3-HLAC recognition (Python mirror of the C++ facade).

Names follow the reference's API (c3_hlac/include/c3_hlac/c3_hlac_tools.h,
color_voxel_recognition/include/color_voxel_recognition/search.h): every call goes
through the C-ABI of libc3hlac_mi355x.so (HIP kernels for gfx950); there is no CPU
fallback.  The C++ facade in host/ offers the same surface to C++ callers.
"""
import ctypes as C

import numpy as np

from . import _capi
from ._capi import DET_DTYPE, TIMER_NAMES, C3HError, check, i32x3, ptr  # noqa: F401

FRAME_INFO_DTYPE = np.dtype([("div_b", "<i4", 3), ("min_b", "<i4", 3), ("subdiv_b", "<i4", 3), ("status", "<i4"),
                             ("n_moved", "<i4"), ("n_valid", "<i8"), ("n_occ", "<i8")])
# c3h_frame_info as the C-ABI lays it out (with its padding word)
_FRAME_INFO_C = np.dtype([("div_b", "<i4", 3), ("min_b", "<i4", 3), ("subdiv_b", "<i4", 3), ("status", "<i4"),
                          ("n_moved", "<i4"), ("pad", "<i4"), ("n_valid", "<i8"), ("n_occ", "<i8")])
assert _FRAME_INFO_C.itemsize == C.sizeof(_capi.FrameInfo)


class PointFrames:
    """Point clouds validated for c3h_run_point_frames (Context.prepare_point_frames)."""

    def __init__(self, ptrs, ns, on_device, keep):
        self.ptrs, self.ns, self.on_device, self._keep = ptrs, ns, on_device, keep

    def __len__(self):
        return len(self.ns)


S_MODE = {"S_MODE_%d" % (i + 1): i for i in range(6)}
# setColor of the estimator (c3h_extract_params.color_mode, include/c3hlac_mi355x.h):
# C3HLAC with sin/cos in float or in double (the default), or ColorCHLAC's (v, 255 - v)
COLOR_C3_FLOAT, COLOR_C3_DOUBLE, COLOR_CHLAC = 0, 1, 2
DIM_C3HLAC_981_1_3_ALL = 981
DIM_C3HLAC_117_1_3_ALL = 117


class Context:
    """One device + one HIP stream (c3h_create)."""

    def __init__(self, device=0):
        self.lib = _capi.load()
        h = C.c_void_p()
        rc = self.lib.c3h_create(int(device), C.byref(h))
        if rc != 0:
            raise _capi.C3HError("c3h_create(%d) failed: %s" % (device, _capi.ERRORS.get(rc, rc)))
        self.h = h
        self.device = device
        self.info = None
        self.hist_num = 0
        self.subdiv = (0, 0, 0)
        self.variant = None
        self.M = 0
        self.rank = 1
        self.D = 0

    def close(self):
        if getattr(self, "h", None):
            self.lib.c3h_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc, what):
        return check(rc, self.h, what)

    def set_stream(self, stream_handle):
        """Bind the context to a HIP stream handle (torch.cuda.Stream.cuda_stream); None
        returns to the context's own non-blocking stream (NULL in the C-ABI).  Work queued
        on the previous stream is ordered before the new stream's.  The legacy default
        stream (integer handle 0) cannot be named through the C-ABI: run under a
        non-default torch stream instead, or synchronize() before torch reads results."""
        if stream_handle is None:
            self._chk(self.lib.c3h_set_stream(self.h, None), "set_stream")
            return
        if stream_handle == 0:
            raise ValueError("set_stream: handle 0 is the legacy default stream; use a torch.cuda.Stream() "
                             "or None for the context's own stream")
        self._chk(self.lib.c3h_set_stream(self.h, C.c_void_p(stream_handle)), "set_stream")

    def synchronize(self):
        self._chk(self.lib.c3h_synchronize(self.h), "synchronize")

    # --- voxel grid (getVoxelGrid + limitPoint) -------------------------------------
    def voxelize(self, xyzrgb, leaf, z_limit=float("inf")):
        """xyzrgb: (N,4) float32 host array or a device tensor (x,y,z, rgb bits)."""
        on_dev = not isinstance(xyzrgb, np.ndarray)
        if not on_dev:
            xyzrgb = np.ascontiguousarray(xyzrgb, dtype=np.float32)
            assert xyzrgb.ndim == 2 and xyzrgb.shape[1] == 4
        n = xyzrgb.shape[0]
        gi = _capi.GridInfo()
        self._chk(self.lib.c3h_voxelize(self.h, ptr(xyzrgb), n, int(on_dev), float(leaf),
                                        float(z_limit), C.byref(gi)), "voxelize")
        self.info = gi
        return gi

    def voxelize_pointcloud2(self, msg, leaf, z_limit=float("inf")):
        """sensor_msgs/PointCloud2 as a dict {height, width, point_step, row_step,
        is_bigendian, fields: {name: offset}, data: bytes / uint8 array / device tensor}."""
        f = msg["fields"]
        off = (C.c_int32 * 4)(f["x"], f["y"], f["z"], f.get("rgb", f.get("rgba", -1)))
        data = msg["data"]
        on_dev = hasattr(data, "data_ptr")
        if not on_dev:
            data = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data)
        gi = _capi.GridInfo()
        self._chk(self.lib.c3h_voxelize_pointcloud2(self.h, ptr(data), msg["height"], msg["width"], msg["point_step"],
                                                    msg["row_step"], off, int(bool(msg.get("is_bigendian", 0))),
                                                    int(on_dev), float(leaf), float(z_limit), C.byref(gi)),
                  "voxelize_pointcloud2")
        self.info = gi
        return gi

    def set_grid(self, words, div_b, min_b=(0, 0, 0), leaf=0.01):
        on_dev = not isinstance(words, np.ndarray)
        if not on_dev:
            words = np.ascontiguousarray(words, dtype=np.uint32)
        self._chk(self.lib.c3h_set_grid(self.h, ptr(words), i32x3(div_b), i32x3(min_b),
                                        float(leaf), int(on_dev)), "set_grid")
        gi = _capi.GridInfo()
        self._chk(self.lib.c3h_get_grid_info(self.h, C.byref(gi)), "get_grid_info")
        self.info = gi
        return gi

    def nvox(self):
        d = self.info.div_b
        return int(d[0]) * int(d[1]) * int(d[2])

    def grid(self):
        out = np.zeros(self.nvox(), np.uint32)
        if out.size:
            self._chk(self.lib.c3h_get_grid(self.h, ptr(out), 0), "get_grid")
        return out

    def leaf_layout(self):
        out = np.zeros(self.nvox(), np.int32)
        if out.size:
            self._chk(self.lib.c3h_get_leaf_layout(self.h, ptr(out), 0), "get_leaf_layout")
        return out

    def downsampled(self):
        out = np.zeros((max(int(self.info.n_occ), 0), 4), np.float32)
        if out.size:
            self._chk(self.lib.c3h_get_downsampled(self.h, ptr(out), 0), "get_downsampled")
        return out

    # --- C3-HLAC ----------------------------------------------------------------------
    def extract(self, variant, thr, subdiv=0, offset=(0, 0, 0), color_mode=COLOR_C3_DOUBLE):
        p = _capi.ExtractParams()
        p.variant = int(variant)
        p.thr = (C.c_int32 * 3)(*[int(t) for t in thr])
        p.subdiv = int(subdiv)
        p.offset = (C.c_int32 * 3)(*[int(o) for o in offset])
        p.color_mode = int(color_mode)
        sb = (C.c_int32 * 3)()
        hn = C.c_int64()
        self._chk(self.lib.c3h_extract(self.h, C.byref(p), sb, C.byref(hn)), "extract")
        self.hist_num = int(hn.value)
        self.subdiv = tuple(int(x) for x in sb)
        self.variant = int(variant)
        return self.subdiv, self.hist_num

    def features(self):
        out = np.zeros((self.hist_num, self.variant), np.float32)
        if out.size:
            self._chk(self.lib.c3h_get_features(self.h, ptr(out), 0), "get_features")
        return out

    def compute_normals(self, radius=0.02, viewpoint=(0.0, 0.0, 0.0)):
        vp = (C.c_float * 3)(*viewpoint)
        self._chk(self.lib.c3h_compute_normals(self.h, float(radius), vp), "compute_normals")

    def normals(self, n):
        out = np.zeros((n, 4), np.float32)
        self._chk(self.lib.c3h_get_normals(self.h, ptr(out), 0), "get_normals")
        return out

    @staticmethod
    def _grsd_params(subdiv, offset, rsd_radius, normalize):
        p = _capi.GrsdParams()
        p.subdiv = int(subdiv)
        p.offset = (C.c_int32 * 3)(*[int(o) for o in offset])
        p.rsd_radius = float(rsd_radius)
        p.normalize = int(bool(normalize))
        return p

    def extract_grsd(self, subdiv=0, offset=(0, 0, 0), rsd_radius=0.01, normalize=False):
        sb = (C.c_int32 * 3)()
        hn = C.c_int64()
        p = self._grsd_params(subdiv, offset, rsd_radius, normalize)
        self._chk(self.lib.c3h_extract_grsd(self.h, C.byref(p), sb, C.byref(hn)), "extract_grsd")
        self.hist_num, self.subdiv, self.variant = int(hn.value), tuple(int(x) for x in sb), 20
        return self.subdiv, self.hist_num

    def rsd(self):
        n = self._chk(self.lib.c3h_get_rsd(self.h, None, None, 0), "get_rsd")
        radii = np.zeros((n, 2), np.float32)
        types = np.zeros(n, np.int32)
        self._chk(self.lib.c3h_get_rsd(self.h, ptr(radii), ptr(types), 0), "get_rsd")
        return radii, types

    def extract_vosch(self, thr, subdiv=0, offset=(0, 0, 0), rsd_radius=0.01, normalize=False, color_mode=COLOR_C3_DOUBLE):
        sb = (C.c_int32 * 3)()
        hn = C.c_int64()
        p = self._grsd_params(subdiv, offset, rsd_radius, normalize)
        t = (C.c_int32 * 3)(*[int(x) for x in thr])
        self._chk(self.lib.c3h_extract_vosch(self.h, C.byref(p), t, int(color_mode), sb, C.byref(hn)),
                  "extract_vosch")
        self.hist_num, self.subdiv, self.variant = int(hn.value), tuple(int(x) for x in sb), 137
        return self.subdiv, self.hist_num

    def set_score_engine(self, engine):
        """c3h_set_score_engine: 0 automatic, 1 VALU, 2 matrix cores (single-frame search)."""
        self._chk(self.lib.c3h_set_score_engine(self.h, int(engine)), "set_score_engine")

    def set_search_precision(self, fp16):
        """c3h_set_search_precision: fp16 matrix-core compress for large grids."""
        self._chk(self.lib.c3h_set_search_precision(self.h, int(bool(fp16))), "set_search_precision")

    def set_features(self, feat, subdiv, exist=None, rule=0):
        """SearchObj::setData with caller-computed features (c3h_set_features): feat
        (hist_num, dim) numpy or torch device tensor, exist None -> derived by rule
        (0 setC3HLAC, 1 setVOSCH / setConVOSCH, 2 setGRSD)."""
        on_dev = hasattr(feat, "data_ptr")
        if not on_dev:
            feat = np.ascontiguousarray(feat, np.float32)
            if exist is not None:
                exist = np.ascontiguousarray(exist, np.int32)
        sb = (C.c_int32 * 3)(*[int(v) for v in subdiv])
        self._chk(self.lib.c3h_set_features(self.h, ptr(feat), sb, int(feat.shape[1]), ptr(exist), int(rule),
                                            int(on_dev)), "set_features")
        self.hist_num = int(feat.shape[0])
        self.subdiv = tuple(int(v) for v in subdiv)
        self.variant = int(feat.shape[1])

    def exist(self):
        out = np.zeros(self.hist_num, np.int32)
        if out.size:
            self._chk(self.lib.c3h_get_exist(self.h, ptr(out), 0), "get_exist")
        return out

    def color_histogram(self, hist=None):
        """Per-channel 256-bin histograms (3, 256) int64 of the current grid's occupied voxel
        colours (calc_scene_auto_threshold.cpp:92-108); adds into `hist` when given."""
        out = np.zeros((3, 256), np.int64) if hist is None else hist
        assert out.dtype == np.int64 and out.shape == (3, 256) and out.flags.c_contiguous
        self._chk(self.lib.c3h_color_histogram(self.h, ptr(out), 0 if hist is None else 1), "color_histogram")
        return out

    # --- search -----------------------------------------------------------------------
    def search_setup(self, axis_p, var, axis_q, feature_max=None):
        """axis_p: (D,F) or None; var: (D,) or None (whitening); axis_q: (M,r,D)."""
        axis_q = np.ascontiguousarray(axis_q, dtype=np.float32)
        M, r, D = axis_q.shape
        if axis_p is not None:
            axis_p = np.ascontiguousarray(axis_p, dtype=np.float32)
            assert axis_p.shape[0] == D
            F = axis_p.shape[1]
        else:
            F = D
        if var is not None:
            var = np.ascontiguousarray(var, dtype=np.float32)
        fm = None if feature_max is None else np.ascontiguousarray(feature_max, dtype=np.float32)
        self._chk(self.lib.c3h_search_setup(self.h, ptr(axis_p), ptr(var), D, F, ptr(axis_q), M, r,
                                            ptr(fm), 0 if fm is None else fm.size), "search_setup")
        self.M, self.D = M, D

    def set_rank(self, rank):
        self._chk(self.lib.c3h_set_rank(self.h, int(rank)), "set_rank")
        self.rank = int(rank)

    def clean_max(self):
        self._chk(self.lib.c3h_clean_max(self.h), "clean_max")

    def search(self, ranges, exist_threshold, rotate=True, remove_overlap=False):
        out = np.zeros(max(self.M, 1) * self.rank, DET_DTYPE)
        nm = self._chk(self.lib.c3h_search(self.h, i32x3(ranges), int(exist_threshold), int(bool(rotate)),
                                           int(bool(remove_overlap)), ptr(out)), "search")
        return out.reshape(max(self.M, 1), self.rank), nm

    def search_async(self, ranges, exist_threshold, rotate=True, d_out=None):
        return self._chk(self.lib.c3h_search_async(self.h, i32x3(ranges), int(exist_threshold),
                                                   int(bool(rotate)), ptr(d_out)), "search_async")

    def run_frames(self, grid_ptrs, div_b, min_b, leaf, variant, thr, subdiv, ranges, exist_threshold,
                   rotate=True, d_out=None, offset=(0, 0, 0), color_mode=COLOR_C3_DOUBLE, stream=False):
        """c3h_run_frames (stream=True: c3h_stream_frames, the pipeline stays filled;
        call stream_flush() before reading the last batches): grid_ptrs = uint64 numpy
        array of device pointers."""
        gp = np.ascontiguousarray(grid_ptrs, dtype=np.uint64)
        fn = self.lib.c3h_stream_frames if stream else self.lib.c3h_run_frames
        p = _capi.ExtractParams()
        p.variant = int(variant)
        p.thr = (C.c_int32 * 3)(*[int(t) for t in thr])
        p.subdiv = int(subdiv)
        p.offset = (C.c_int32 * 3)(*[int(o) for o in offset])
        p.color_mode = int(color_mode)
        nm = self._chk(fn(self.h, ptr(gp), gp.size, i32x3(div_b), i32x3(min_b), float(leaf),
                          C.byref(p), i32x3(ranges), int(exist_threshold),
                          int(bool(rotate)), ptr(d_out)), "run_frames")
        if not stream:  # the context holds the last frame's grid, features and search
            self._refresh()
        return nm

    def prepare_point_frames(self, frames):
        """Validates a list of point clouds for run_point_frames once: all numpy (n, 4) host
        arrays (pinned or not) or all contiguous (n, 4) float32 torch tensors on this
        context's device.  Returns a PointFrames (the pointer and count arrays the C-ABI
        takes, and references keeping the clouds alive) that run_point_frames accepts in
        place of the list: a caller pushing the same frames repeatedly -- the bench -- pays
        the per-frame Python checks (~3 us per frame) once, as a C++ caller holding its
        pointer array would."""
        on_dev = hasattr(frames[0], "data_ptr") if len(frames) else False
        keep = []
        ptrs = np.zeros(len(frames), np.uint64)
        ns = np.zeros(len(frames), np.int64)
        for i, fr in enumerate(frames):
            if on_dev:
                import torch
                if fr.dtype != torch.float32 or fr.ndim != 2 or fr.shape[1] != 4 or not fr.is_contiguous():
                    raise ValueError("run_point_frames: frame %d must be a contiguous (n, 4) float32 tensor" % i)
                if fr.device.type != "cuda" or (fr.device.index or 0) != self.device:
                    raise ValueError("run_point_frames: frame %d is on %s, the context on cuda:%d"
                                     % (i, fr.device, self.device))
                keep.append(fr)
                ptrs[i] = fr.data_ptr()
            else:
                fr = np.ascontiguousarray(fr, dtype=np.float32)
                if fr.ndim != 2 or fr.shape[1] != 4:
                    raise ValueError("run_point_frames: frame %d must be (n, 4)" % i)
                keep.append(fr)
                ptrs[i] = fr.ctypes.data
            ns[i] = fr.shape[0]
        return PointFrames(ptrs, ns, on_dev, keep)

    def run_point_frames(self, frames, leaf, canvas, variant, thr, subdiv, ranges, exist_threshold, rotate=True,
                         d_out=None, z_limit=float("inf"), offset=(0, 0, 0), color_mode=COLOR_C3_DOUBLE):
        """c3h_run_point_frames: frames = list of (n, 4) float32 point clouds, all numpy host
        arrays (pinned or not) or all torch device tensors, or a PointFrames from
        prepare_point_frames; d_out = device pointer (int) or tensor of len(frames) * M * rank
        records.  Returns (modes, info) with info a numpy structured array (div_b, min_b,
        subdiv_b, status, n_valid, n_occ) per frame."""
        if not isinstance(frames, PointFrames):
            frames = self.prepare_point_frames(frames)
        ptrs, ns, on_dev = frames.ptrs, frames.ns, frames.on_device
        if d_out is not None and hasattr(d_out, "data_ptr"):
            need = len(frames) * max(self.M, 1) * self.rank * DET_DTYPE.itemsize
            have = d_out.numel() * d_out.element_size()
            if have < need or not d_out.is_contiguous() or d_out.device.type != "cuda" or \
                    (d_out.device.index or 0) != self.device:
                raise ValueError("run_point_frames: d_out must be a contiguous tensor of >= %d bytes on cuda:%d"
                                 % (need, self.device))
        p = _capi.ExtractParams()
        p.variant = int(variant)
        p.thr = (C.c_int32 * 3)(*[int(t) for t in thr])
        p.subdiv = int(subdiv)
        p.offset = (C.c_int32 * 3)(*[int(o) for o in offset])
        p.color_mode = int(color_mode)
        info = (_capi.FrameInfo * max(len(frames), 1))()
        nm = self._chk(self.lib.c3h_run_point_frames(self.h, ptr(ptrs), ptr(ns), len(frames), int(on_dev),
                                                     float(leaf), float(z_limit), i32x3(canvas), C.byref(p),
                                                     i32x3(ranges), int(exist_threshold), int(bool(rotate)),
                                                     ptr(d_out), info), "run_point_frames")
        raw = np.frombuffer(info, _FRAME_INFO_C, count=len(frames))
        out = np.zeros(len(frames), FRAME_INFO_DTYPE)
        for f in FRAME_INFO_DTYPE.names:
            out[f] = raw[f]
        return nm, out

    def _refresh(self):
        """Re-read the grid / feature state the library holds (after run_frames)."""
        gi = _capi.GridInfo()
        if self.lib.c3h_get_grid_info(self.h, C.byref(gi)) == 0:
            self.info = gi
        sb = (C.c_int32 * 3)()
        hn = C.c_int64()
        dim = C.c_int32()
        self._chk(self.lib.c3h_get_feature_info(self.h, sb, C.byref(hn), C.byref(dim)), "get_feature_info")
        self.subdiv = tuple(int(x) for x in sb)
        self.hist_num = int(hn.value)
        self.variant = int(dim.value) or self.variant

    def stream_flush(self):
        """c3h_stream_flush: the remaining ticks of an open frame stream (no host sync)."""
        self._chk(self.lib.c3h_stream_flush(self.h), "stream_flush")

    def set_lanes(self, n):
        """Frames in flight in run_frames (child contexts on their own streams)."""
        self._chk(self.lib.c3h_set_lanes(self.h, int(n)), "set_lanes")

    def set_batch(self, n):
        """Frames per pipeline batch / launch in run_frames (1..64)."""
        self._chk(self.lib.c3h_set_batch(self.h, int(n)), "set_batch")

    @staticmethod
    def point_batch(n_frames):
        """Batch size for a c3h_run_point_frames call of n_frames 1M-point frames (round 6,
        measured on MI355X at 128^3, C3-HLAC-981: profiles/r6/shard/): 32 frames per batch
        from 256 frames up (512 frames: 117k frames/s against 109k at 64), 64 below, where a
        call has few batches and each tick's fill and drain cost more than the finer
        overlap of smaller batches gains (64 frames: 85-89k at 64, 80-83k at 32)."""
        return 32 if n_frames >= 256 else 64

    def set_pipeline(self, on):
        """run_frames scheduling: True = pipelined tick launches, False = lanes."""
        self._chk(self.lib.c3h_set_pipeline(self.h, int(bool(on))), "set_pipeline")

    def compressed(self):
        out = np.zeros((self.hist_num, self.D), np.float32)
        self._chk(self.lib.c3h_get_compressed(self.h, ptr(out), 0), "get_compressed")
        return out

    def scores(self):
        n = C.c_int64()
        self._chk(self.lib.c3h_get_scores(self.h, None, C.byref(n), 0), "get_scores")
        out = np.zeros(n.value, np.float64)
        if out.size:
            self._chk(self.lib.c3h_get_scores(self.h, ptr(out), C.byref(n), 0), "get_scores")
        return out

    # --- timing -----------------------------------------------------------------------
    def timing(self, enable=True):
        """True/False: all slots / off; an int: C3H_TIMING_* mask (e.g. timing_mask("c3hlac"))."""
        v = int(enable) if not isinstance(enable, bool) else int(enable)
        self._chk(self.lib.c3h_timing(self.h, v), "timing")

    def kernel_times(self, reset=True):
        ms = np.zeros(_capi.NTIMERS, np.float32)
        cnt = np.zeros(_capi.NTIMERS, np.int32)
        self._chk(self.lib.c3h_kernel_times(self.h, ptr(ms), ptr(cnt), int(bool(reset))), "kernel_times")
        return {n: (float(ms[i]), int(cnt[i])) for i, n in enumerate(TIMER_NAMES)}


def auto_threshold(hist):
    """calc_scene_auto_threshold.cpp:111-146 on (3, 256) histograms -> (thr (3,), total_ave (3,))."""
    h = np.ascontiguousarray(hist, dtype=np.int64)
    thr = np.zeros(3, np.int32)
    ave = np.zeros(3, np.float64)
    check(_capi.load().c3h_auto_threshold(ptr(h), ptr(thr), ptr(ave)), None, "auto_threshold")
    return thr, ave


def read_pcd(path):
    """c3h_pcd_read_xyzrgb -> (n, 4) float32 x, y, z, rgb-bits (the c3h_voxelize input)."""
    lib = _capi.load()
    n = C.c_int64(0)
    check(lib.c3h_pcd_read_xyzrgb(str(path).encode(), None, C.byref(n)), None, "pcd_read")
    out = np.zeros((n.value, 4), np.float32)
    if n.value:
        check(lib.c3h_pcd_read_xyzrgb(str(path).encode(), ptr(out), C.byref(n)), None, "pcd_read")
    return out


def read_feature(path):
    """readFeature (c3_hlac_tools.hpp:46-71) -> (rows, dim) float32."""
    lib = _capi.load()
    rows, dim = C.c_int64(0), C.c_int32(0)
    check(lib.c3h_feature_pcd_read(str(path).encode(), None, C.byref(rows), C.byref(dim)), None, "feature_read")
    out = np.zeros((rows.value, dim.value), np.float32)
    if out.size:
        check(lib.c3h_feature_pcd_read(str(path).encode(), ptr(out), C.byref(rows), C.byref(dim)), None,
              "feature_read")
    return out


def write_feature(path, feat, remove_zero=True, fields=None):
    """writeFeature (c3_hlac_tools.hpp:83-113)."""
    f = np.ascontiguousarray(feat, dtype=np.float32)
    if f.ndim == 1:
        f = f[None, :]
    check(_capi.load().c3h_feature_pcd_write(str(path).encode(), ptr(f), f.shape[0], f.shape[1],
                                             int(bool(remove_zero)), None if fields is None else fields.encode()),
          None, "feature_write")


def replay_scores(scores, subdiv_b, ranges, lists, rotate=True, floors=False):
    """c3h_replay_scores: searchPart's rank update over score arrays in c3h_get_scores'
    layout (host function); lists: (M, rank) DET_DTYPE, continued from their state.
    floors=True (c3h_replay_scores_floor): returns (lists, row floors), the floors per
    searched mode as M x ze x ye doubles, concatenated in the scores' mode order."""
    lists = np.ascontiguousarray(lists, dtype=DET_DTYPE)
    M, rank = lists.shape
    sc = np.ascontiguousarray(scores, dtype=np.float64)
    lib = _capi.load()
    if not floors:
        check(lib.c3h_replay_scores(M, rank, i32x3(ranges), int(bool(rotate)), i32x3(subdiv_b), ptr(sc),
                                    ptr(lists)), None, "replay_scores")
        return lists
    from .dist import mode_schedule, mode_ranges
    n = 0
    for md in mode_schedule(ranges, rotate):
        xr, yr, zr = mode_ranges(md, ranges)
        xe, ye, ze = subdiv_b[0] - xr + 1, subdiv_b[1] - yr + 1, subdiv_b[2] - zr + 1
        if xe > 0 and ye > 0 and ze > 0:
            n += M * ze * ye
    fl = np.zeros(max(n, 1), np.float64)
    check(lib.c3h_replay_scores_floor(M, rank, i32x3(ranges), int(bool(rotate)), i32x3(subdiv_b), ptr(sc),
                                      ptr(lists), ptr(fl)), None, "replay_scores_floor")
    return lists, fl[:n]


def remove_overlap(lists, ranges):
    """SearchObjMulti::removeOverlap on (M, rank) DET_DTYPE lists (host function)."""
    lists = np.ascontiguousarray(lists, dtype=DET_DTYPE)
    M, rank = lists.shape
    check(_capi.load().c3h_remove_overlap(M, rank, i32x3(ranges), ptr(lists)), None, "remove_overlap")
    return lists


def pca_read(path, ascii=False, max_dim=4096):
    """PCA::read -> (axis (dim,dim) with axis[:, i] = eigenvector i, variance, mean or None)."""
    buf = np.zeros(max_dim * max_dim, np.float32)
    var = np.zeros(max_dim, np.float32)
    mean = np.zeros(max_dim, np.float32)
    hm = C.c_int32()
    dim = check(_capi.load().c3h_pca_read(str(path).encode(), int(bool(ascii)), ptr(buf), ptr(var),
                                          ptr(mean), C.byref(hm), max_dim), None, "pca_read")
    axis = buf[: dim * dim].reshape(dim, dim).T.copy()  # column i = eigenvector i
    return axis, var[:dim].copy(), (mean[:dim].copy() if hm.value else None)


def timing_mask(*slots):
    """C3H_TIMING_* mask for the named slots (TIMER_NAMES)."""
    return sum(2 << TIMER_NAMES.index(n) for n in slots)


def read_axis(axis, variance, dim, dim_model, multiple_similarity=True):
    """SearchObj::readAxis transform (search.cpp:153-165): (dim_model, dim) float32."""
    q = np.ascontiguousarray(axis[:, :dim_model].T, dtype=np.float32)
    if multiple_similarity:
        for i in range(1, dim_model):
            q[i, :dim] = (q[i, :dim].astype(np.float64) * np.sqrt(np.float64(variance[i]))
                          / np.sqrt(np.float64(variance[0]))).astype(np.float32)
    return q


def box_size(size_m, region_size):
    """Sliding-box size in subdivisions (detect_object.cpp:254-266)."""
    t = np.float32(size_m) / np.float32(region_size)
    s = int(t)
    if (t - s) >= 0.5 or s == 0:
        s += 1
    return s


R_MODE_1, R_MODE_2, R_MODE_3, R_MODE_4 = 0, 1, 2, 3


def rotate_map(dim, mode):
    """pcl::rotateFeature90 (c3_hlac.cpp:49-172) as a gather map: out[o] = in[map[o]]."""
    out = np.zeros(dim, np.int32)
    check(_capi.load().c3h_rotate_map(dim, mode, ptr(out)), None, "rotate_map")
    return out


def rotate_feature90(d_in, d_out, mode, stream=None):
    """pcl::rotateFeature90 on device rows: d_in / d_out torch float32 tensors (n, dim)."""
    n, dim = d_in.shape
    assert d_out.shape == d_in.shape and d_in.is_contiguous() and d_out.is_contiguous()
    s = None if stream is None else C.c_void_p(stream)
    check(_capi.load().c3h_rotate_feature90(ptr(d_in), ptr(d_out), n, dim, dim, mode, s), None,
          "rotate_feature90")


def pca_write(path, axis, var, mean=None, ascii=False):
    """PCA::write (pca.cpp:190-240); axis (dim, dim) with axis[:, i] = eigenvector i."""
    dim = len(var)
    a = np.ascontiguousarray(np.asarray(axis, np.float32).T)  # eigenvector i contiguous
    v = np.ascontiguousarray(var, np.float32)
    m = None if mean is None else np.ascontiguousarray(mean, np.float32)
    check(_capi.load().c3h_pca_write(str(path).encode(), int(bool(ascii)), dim, ptr(a), ptr(v), ptr(m)), None,
          "pca_write")


class PCA:
    """class PCA (color_voxel_recognition/include/color_voxel_recognition/pca.h:45-81) with
    the correlation accumulated on the GPU (csrc/pca.hip).

    add_data takes a batch of rows (numpy host array or torch device tensor) instead of
    one std::vector per call; set_compress + rotate24 give pca_models.cpp's augmented,
    compressed training in one pass (see c3h_pca_add_data)."""

    def __init__(self, mean_flg=True, device=0):
        self.lib = _capi.load()
        h = C.c_void_p()
        check(self.lib.c3h_pca_create(device, int(bool(mean_flg)), C.byref(h)), None, "pca_create")
        self.h = h
        self.mean_flg = bool(mean_flg)

    def close(self):
        if getattr(self, "h", None):
            self.lib.c3h_pca_destroy(self.h)
            self.h = None

    __del__ = close

    def _check(self, rc, what):
        if rc < 0:
            m = self.lib.c3h_pca_last_error(self.h)
            raise _capi.C3HError("%s failed: %s %s" % (what, _capi.ERRORS.get(rc, rc), m.decode() if m else ""))
        return rc

    def set_compress(self, axis, var, dim):
        """compressFeature's projection: the first dim columns of axis (F, F'), whitened by var."""
        F = axis.shape[0]
        a = np.ascontiguousarray(np.asarray(axis, np.float32)[:, :dim].T)  # column d contiguous
        v = None if var is None else np.ascontiguousarray(np.asarray(var, np.float32)[:dim])
        self._check(self.lib.c3h_pca_set_compress(self.h, ptr(a), ptr(v), F, dim), "pca_set_compress")

    def add_data(self, rows, rotate24=False):
        on_dev = hasattr(rows, "data_ptr")
        if not on_dev:
            rows = np.ascontiguousarray(rows, np.float32)
            if rows.ndim == 1:
                rows = rows[None, :]
        else:
            assert rows.is_contiguous()
        n, F = rows.shape
        self._check(self.lib.c3h_pca_add_data(self.h, ptr(rows), n, F, F, int(bool(rotate24)), int(on_dev)),
                    "pca_add_data")

    addData = add_data

    def solve(self, regularization_flg=False, regularization_nolm=0.0001):
        self._check(self.lib.c3h_pca_solve(self.h, int(bool(regularization_flg)), regularization_nolm), "pca_solve")
        d = self._check(self.lib.c3h_pca_get(self.h, None, None, None, None, 0), "pca_get")
        a = np.zeros((d, d), np.float32)
        v = np.zeros(d, np.float32)
        m = np.zeros(d, np.float32) if self.mean_flg else None
        n = C.c_int64()
        self._check(self.lib.c3h_pca_get(self.h, ptr(a), ptr(v), ptr(m), C.byref(n), 0), "pca_get")
        self.axis, self.variance, self.mean, self.nsample = a.T.copy(), v, m, n.value
        return self

    def correlation(self):
        d = self.axis.shape[0]
        out = np.zeros((d, d), np.float64)
        self._check(self.lib.c3h_pca_get_correlation(self.h, ptr(out)), "pca_get_correlation")
        return out

    def getAxis(self):
        return self.axis

    def getVariance(self):
        return self.variance

    def getMean(self):
        if not self.mean_flg:
            raise _capi.C3HError("getMean: There is no mean vector (mean_flg=false).")
        return self.mean

    def write(self, path, ascii=False):
        pca_write(path, self.axis, self.variance, self.mean if self.mean_flg else None, ascii)
