"""ctypes front-end of oracle/libgeom_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. It is the checker for the HIP preprocessing kernels, never the
product. The C restatement it loads is documented in oracle/geom_oracle.c.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, 'libgeom_oracle.so')
_lib = None

INDEX, DIST = 0, 1


def build():
    subprocess.check_call(['make', '-s', '-C', HERE, 'all'])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, f32 = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_float
        L.oracle_grid_count.restype = i64
        L.oracle_grid_count.argtypes = [vp, vp, ctypes.c_int, f32, vp]
        L.oracle_grid_fill.restype = None
        L.oracle_grid_fill.argtypes = [vp, vp, ctypes.c_int, f32, vp, vp]
        L.oracle_radius_count.restype = i64
        L.oracle_radius_count.argtypes = [vp, vp, vp, vp, ctypes.c_int, f32, vp]
        L.oracle_radius_fill.restype = None
        L.oracle_radius_fill.argtypes = [vp, vp, vp, vp, ctypes.c_int, f32, ctypes.c_int,
                                         ctypes.c_int, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def grid_subsample(points, lengths, dl, return_keys=False):
    """(N,3) f32 packed clouds + (C,) lengths -> (M,3) f32 barycentres, (C,) int64 lengths.

    Voxels come out in ascending voxel-key order within each cloud.
    """
    pts = np.ascontiguousarray(points, dtype=np.float32)
    lens = np.ascontiguousarray(lengths, dtype=np.int64)
    out_lens = np.zeros_like(lens)
    L = lib()
    m = L.oracle_grid_count(_p(pts), _p(lens), len(lens), float(dl), _p(out_lens))
    out = np.zeros((m, 3), np.float32)
    keys = np.zeros((m,), np.int64)
    L.oracle_grid_fill(_p(pts), _p(lens), len(lens), float(dl), _p(out), _p(keys))
    return (out, out_lens, keys) if return_keys else (out, out_lens)


def radius_counts(queries, q_lengths, supports, s_lengths, radius):
    q = np.ascontiguousarray(queries, dtype=np.float32)
    s = np.ascontiguousarray(supports, dtype=np.float32)
    ql = np.ascontiguousarray(q_lengths, dtype=np.int64)
    sl = np.ascontiguousarray(s_lengths, dtype=np.int64)
    counts = np.zeros((len(q),), np.int64)
    mx = lib().oracle_radius_count(_p(q), _p(ql), _p(s), _p(sl), len(ql), float(radius),
                                   _p(counts))
    return counts, int(mx)


def radius_search(queries, q_lengths, supports, s_lengths, radius, limit, mode=INDEX):
    """Neighbour table (Nq, width) int64, shadow index = total supports.

    mode INDEX: ball_query semantics, width = limit.
    mode DIST:  nanoflann semantics, width = min(max_count, limit) (limit <= 0: uncapped).
    """
    q = np.ascontiguousarray(queries, dtype=np.float32)
    s = np.ascontiguousarray(supports, dtype=np.float32)
    ql = np.ascontiguousarray(q_lengths, dtype=np.int64)
    sl = np.ascontiguousarray(s_lengths, dtype=np.int64)
    if mode == INDEX:
        width = int(limit)
    else:
        _, mx = radius_counts(q, ql, s, sl, radius)
        width = mx if limit <= 0 else min(mx, int(limit))
    out = np.zeros((len(q), width), np.int64)
    lib().oracle_radius_fill(_p(q), _p(ql), _p(s), _p(sl), len(ql), float(radius), int(mode),
                             width, _p(out))
    return out
