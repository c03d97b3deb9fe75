"""ctypes binding of libc3hlac_mi355x.so (include/c3hlac_mi355x.h).

The HIP library is the only implementation: importing this module fails loudly when
the shared object is missing (no CPU fallback exists in the product path).
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parents[1]          # mapping-private_amd/
LIB_DIR = PKG_ROOT / "lib"
LIB_PATH = LIB_DIR / "libc3hlac_mi355x.so"
HEADER = PKG_ROOT.parent / "include" / "c3hlac_mi355x.h"

C3H_OK = 0
ERRORS = {
    -1: "C3H_ERR_ARG", -2: "C3H_ERR_HIP", -3: "C3H_ERR_STATE", -4: "C3H_ERR_NOMEM",
    -5: "C3H_ERR_RANGE", -6: "C3H_ERR_NOTFOUND", -7: "C3H_ERR_FORMAT",
}
NTIMERS = 6
TIMER_NAMES = ("voxelize", "c3hlac", "compress", "score", "replay", "pipeline")


class GridInfo(C.Structure):
    _fields_ = [("div_b", C.c_int32 * 3), ("min_b", C.c_int32 * 3), ("max_b", C.c_int32 * 3),
                ("n_valid", C.c_int64), ("n_occ", C.c_int64), ("leaf", C.c_float),
                ("inv_leaf", C.c_float)]


class ExtractParams(C.Structure):
    _fields_ = [("variant", C.c_int32), ("thr", C.c_int32 * 3), ("subdiv", C.c_int32),
                ("offset", C.c_int32 * 3), ("color_mode", C.c_int32)]


class GrsdParams(C.Structure):
    _fields_ = [("subdiv", C.c_int32), ("offset", C.c_int32 * 3), ("rsd_radius", C.c_float),
                ("normalize", C.c_int32)]


class Det(C.Structure):
    _fields_ = [("score", C.c_double), ("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32),
                ("mode", C.c_int32)]


class FrameInfo(C.Structure):
    _fields_ = [("div_b", C.c_int32 * 3), ("min_b", C.c_int32 * 3), ("subdiv_b", C.c_int32 * 3),
                ("status", C.c_int32), ("n_moved", C.c_int32), ("pad", C.c_int32), ("n_valid", C.c_int64),
                ("n_occ", C.c_int64)]


DET_DTYPE = np.dtype([("score", "<f8"), ("x", "<i4"), ("y", "<i4"), ("z", "<i4"), ("mode", "<i4")])
assert DET_DTYPE.itemsize == C.sizeof(Det)

_P = C.c_void_p
_SIGS = {
    "c3h_version": (C.c_int, []),
    "c3h_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "c3h_destroy": (None, [_P]),
    "c3h_set_stream": (C.c_int, [_P, _P]),
    "c3h_synchronize": (C.c_int, [_P]),
    "c3h_last_error": (C.c_char_p, [_P]),
    "c3h_build_info": (C.c_char_p, []),
    "c3h_voxelize": (C.c_int, [_P, _P, C.c_int64, C.c_int, C.c_float, C.c_float, C.POINTER(GridInfo)]),
    "c3h_voxelize_pointcloud2": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.POINTER(C.c_int32), C.c_int32, C.c_int, C.c_float, C.c_float,
                                            C.POINTER(GridInfo)]),
    "c3h_pointcloud2_to_xyzrgb": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                             C.POINTER(C.c_int32), C.c_int32, _P, _P]),
    "c3h_get_leaf_layout": (C.c_int, [_P, _P, C.c_int]),
    "c3h_get_downsampled": (C.c_int, [_P, _P, C.c_int]),
    "c3h_get_grid": (C.c_int, [_P, _P, C.c_int]),
    "c3h_set_grid": (C.c_int, [_P, _P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_float, C.c_int]),
    "c3h_get_grid_info": (C.c_int, [_P, C.POINTER(GridInfo)]),
    "c3h_grid_device_ptr": (C.c_int, [_P, C.POINTER(_P)]),
    "c3h_color_histogram": (C.c_int, [_P, _P, C.c_int32]),
    "c3h_auto_threshold": (C.c_int, [_P, _P, _P]),
    "c3h_pcd_read_xyzrgb": (C.c_int, [C.c_char_p, _P, C.POINTER(C.c_int64)]),
    "c3h_feature_pcd_read": (C.c_int, [C.c_char_p, _P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "c3h_feature_pcd_write": (C.c_int, [C.c_char_p, _P, C.c_int64, C.c_int32, C.c_int32, C.c_char_p]),
    "c3h_extract": (C.c_int, [_P, C.POINTER(ExtractParams), C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "c3h_get_feature_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "c3h_get_features": (C.c_int, [_P, _P, C.c_int]),
    "c3h_get_exist": (C.c_int, [_P, _P, C.c_int]),
    "c3h_search_setup": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int32, _P, C.c_int32, C.c_int32, _P, C.c_int32]),
    "c3h_set_rank": (C.c_int, [_P, C.c_int32]),
    "c3h_clean_max": (C.c_int, [_P]),
    "c3h_search": (C.c_int, [_P, C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_int32, _P]),
    "c3h_search_async": (C.c_int, [_P, C.POINTER(C.c_int32), C.c_int32, C.c_int32, _P]),
    "c3h_run_frames": (C.c_int, [_P, _P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_float,
                                 C.POINTER(ExtractParams), C.POINTER(C.c_int32), C.c_int32, C.c_int32, _P]),
    "c3h_stream_frames": (C.c_int, [_P, _P, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_float,
                                    C.POINTER(ExtractParams), C.POINTER(C.c_int32), C.c_int32, C.c_int32, _P]),
    "c3h_stream_flush": (C.c_int, [_P]),
    "c3h_run_point_frames": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int, C.c_float, C.c_float, C.POINTER(C.c_int32),
                                       C.POINTER(ExtractParams), C.POINTER(C.c_int32), C.c_int32, C.c_int32, _P,
                                       _P]),
    "c3h_set_lanes": (C.c_int, [_P, C.c_int32]),
    "c3h_set_batch": (C.c_int, [_P, C.c_int32]),
    "c3h_set_pipeline": (C.c_int, [_P, C.c_int32]),
    "c3h_get_compressed": (C.c_int, [_P, _P, C.c_int]),
    "c3h_get_scores": (C.c_int, [_P, _P, C.POINTER(C.c_int64), C.c_int]),
    "c3h_remove_overlap": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_int32), _P]),
    "c3h_replay_scores": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_int32),
                                    _P, _P]),
    "c3h_replay_scores_floor": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                          C.POINTER(C.c_int32), _P, _P, _P]),
    "c3h_pca_read": (C.c_int, [C.c_char_p, C.c_int32, _P, _P, _P, C.POINTER(C.c_int32), C.c_int32]),
    "c3h_allgather_detections": (C.c_int, [_P, _P, _P, C.c_int64, _P]),
    "c3h_compute_normals": (C.c_int, [_P, C.c_float, _P]),
    "c3h_get_normals": (C.c_int, [_P, _P, C.c_int]),
    "c3h_extract_grsd": (C.c_int, [_P, C.POINTER(GrsdParams), C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "c3h_get_rsd": (C.c_int, [_P, _P, _P, C.c_int]),
    "c3h_extract_vosch": (C.c_int, [_P, C.POINTER(GrsdParams), C.POINTER(C.c_int32), C.c_int32,
                                    C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "c3h_set_search_precision": (C.c_int, [_P, C.c_int32]),
    "c3h_set_score_engine": (C.c_int, [_P, C.c_int32]),
    "c3h_set_features": (C.c_int, [_P, _P, C.POINTER(C.c_int32), C.c_int32, _P, C.c_int32, C.c_int]),
    "c3h_pca_write": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, _P, _P, _P]),
    "c3h_pca_create": (C.c_int, [C.c_int, C.c_int32, C.POINTER(_P)]),
    "c3h_pca_destroy": (None, [_P]),
    "c3h_pca_last_error": (C.c_char_p, [_P]),
    "c3h_pca_set_stream": (C.c_int, [_P, _P]),
    "c3h_pca_set_compress": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int32]),
    "c3h_pca_add_data": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int]),
    "c3h_pca_solve": (C.c_int, [_P, C.c_int32, C.c_float]),
    "c3h_pca_get": (C.c_int, [_P, _P, _P, _P, C.POINTER(C.c_int64), C.c_int]),
    "c3h_pca_get_correlation": (C.c_int, [_P, _P]),
    "c3h_rotate_feature90": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P]),
    "c3h_rotate_map": (C.c_int, [C.c_int32, C.c_int32, _P]),
    "c3h_timing": (C.c_int, [_P, C.c_int32]),
    "c3h_kernel_times": (C.c_int, [_P, _P, _P, C.c_int32]),
}

_lib = None


def load(path=None):
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("C3HLAC_LIB", LIB_PATH))
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same SONAME as
    # /opt/rocm's).  Loading torch first makes this library bind to that already-loaded
    # runtime; loading it first would leave torch to start a second runtime, which
    # cannot open the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise RuntimeError(
            "libc3hlac_mi355x.so not found at %s: build it with `make -C mapping-private_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback" % p)
    lib = C.CDLL(str(p))
    # a diagnostics override (C3HLAC_LIB: an older build in an A/B) may lack newer entry
    # points; the product library must export every one
    lenient = path is None and "C3HLAC_LIB" in os.environ
    for name, (res, args) in _SIGS.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def exported_symbols():
    return sorted(_SIGS)


class C3HError(RuntimeError):
    pass


def check(rc, ctx=None, what=""):
    if rc < 0:
        msg = ""
        if ctx is not None:
            m = load().c3h_last_error(ctx)
            msg = m.decode() if m else ""
        raise C3HError("%s failed: %s %s" % (what, ERRORS.get(rc, rc), msg))
    return rc


def ptr(a):
    """Host numpy array -> void*, torch tensor -> device pointer."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
        return a.ctypes.data_as(C.c_void_p)
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return C.c_void_p(a)
    raise TypeError(type(a))


def i32x3(v):
    return (C.c_int32 * 3)(*[int(x) for x in v])


def build_provenance():
    """Which build the process loaded: the library's c3h_build_info() (sha256 of the sources
    it was compiled from, build host and time) beside the same hash of the sources in this
    tree (the Makefile's HASHSRC: csrc/*.hip, csrc/*.h, ../include/c3hlac_mi355x.h, sorted
    by path string, contents concatenated)."""
    import hashlib
    lib = load()
    try:
        info = dict(kv.split("=", 1) for kv in lib.c3h_build_info().decode().split())
    except AttributeError:  # a diagnostics build (C3HLAC_LIB) without the provenance record
        info = {}
    pkg = Path(__file__).resolve().parents[1]
    names = sorted(["csrc/" + p.name for p in (pkg / "csrc").glob("*.hip")]
                   + ["csrc/" + p.name for p in (pkg / "csrc").glob("*.h")]
                   + ["../include/c3hlac_mi355x.h"])
    h = hashlib.sha256()
    for n in names:
        h.update((pkg / n).read_bytes())
    tree = h.hexdigest()
    return {"lib": os.path.relpath(os.path.realpath(lib._name), pkg.parent), "lib_src_sha256": info.get("src"),
            "tree_src_sha256": tree, "lib_matches_tree": info.get("src") == tree,
            "built_on": info.get("host"), "built_at": info.get("built"), "arch": info.get("arch")}
