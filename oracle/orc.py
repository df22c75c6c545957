"""orc -- ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product.  See oracle.h for what is
restated and the parity status ("parity unpinned").
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

SWS_ACCURATE_RND, SWS_BITEXACT = 0x40000, 0x80000
PARAM_DEFAULT = 123456.0
_lib = None


class OrcQStat(ctypes.Structure):
    _fields_ = [("sse", ctypes.c_uint64 * 3), ("mse", ctypes.c_double * 3), ("mse_avg", ctypes.c_double),
                ("psnr", ctypes.c_double * 3), ("psnr_avg", ctypes.c_double), ("ssim", ctypes.c_double * 3),
                ("ssim_all", ctypes.c_double), ("ssim_db", ctypes.c_double)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built at {LIB_PATH}; run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.orc_init_filter.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32,
                                      ctypes.POINTER(ctypes.c_double), i32, i32]
        L.orc_get_local_pos.argtypes = [i32, i32]
        L.orc_scale_frame.argtypes = [i32, i32, i32, ctypes.POINTER(vp), ctypes.POINTER(i64), i32, i32, i32,
                                      ctypes.POINTER(vp), ctypes.POINTER(i64), i32, ctypes.POINTER(ctypes.c_double)]
        L.orc_scale_frame_range.argtypes = [i32, i32, i32, ctypes.POINTER(vp), ctypes.POINTER(i64), i32, i32, i32,
                                            ctypes.POINTER(vp), ctypes.POINTER(i64), i32,
                                            ctypes.POINTER(ctypes.c_double), i32, i32]
        L.orc_plane_sse8.argtypes = [vp, i64, vp, i64, i32, i32]
        L.orc_plane_sse8.restype = ctypes.c_uint64
        L.orc_plane_ssim8.argtypes = [vp, i64, vp, i64, i32, i32]
        L.orc_plane_ssim8.restype = ctypes.c_double
        L.orc_quality_frame420.argtypes = [i32, i32, ctypes.POINTER(vp), ctypes.POINTER(i64),
                                           ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.POINTER(OrcQStat)]
        L.orc_fps_map.argtypes = [i64, i32, i32, i32, i32, vp, i32]
        d = ctypes.c_double
        L.orc_hdr_to_sdr_frame.argtypes = [i32, i32, ctypes.POINTER(vp), ctypes.POINTER(i64), i32,
                                           ctypes.POINTER(vp), ctypes.POINTER(i64), i32, d, d, d, d, i32]
        L.orc_tonemap_param.argtypes = [i32, d]
        L.orc_tonemap_param.restype = d
        L.orc_bt2020_to_bt709.argtypes = [ctypes.POINTER(d * 3)]
        L.orc_yadif_frame.argtypes = [i32, i32, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                      ctypes.POINTER(i64), ctypes.POINTER(vp), ctypes.POINTER(i64), i32, i32, i32]
        _lib = L
    return _lib


def init_filter(src_n, dst_n, flags, one=1 << 14, align=4, pos=128, param=(PARAM_DEFAULT, PARAM_DEFAULT), cap=256):
    """libswscale initFilter restated: returns (coeff[dst_n, size], filterPos[dst_n])."""
    inc = ((src_n << 16) + (dst_n >> 1)) // dst_n
    c = np.zeros(dst_n * cap, np.int16)
    p = np.zeros(dst_n, np.int32)
    par = (ctypes.c_double * 2)(*param)
    n = lib().orc_init_filter(c.ctypes.data, p.ctypes.data, cap, inc, src_n, dst_n, align, one,
                              flags | SWS_ACCURATE_RND | SWS_BITEXACT, par, pos, pos)
    if n <= 0:
        raise RuntimeError(f"orc_init_filter failed ({n})")
    return c[:dst_n * n].reshape(dst_n, n), p


def _ptrs(planes):
    data = (ctypes.c_void_p * 3)()
    pitch = (ctypes.c_int64 * 3)()
    for i, p in enumerate(planes):
        if p is not None:
            data[i] = p.ctypes.data
            pitch[i] = p.strides[0]
    return data, pitch


def _alloc(w, h, fmt):
    cw, ch = (w + 1) // 2, (h + 1) // 2
    if fmt == 0:
        return [np.zeros((h, w), np.uint8), np.zeros((ch, cw), np.uint8), np.zeros((ch, cw), np.uint8)]
    if fmt == 2:
        return [np.zeros((h, 2 * w), np.uint8), np.zeros((ch, 4 * cw), np.uint8), None]
    return [np.zeros((h, w), np.uint8), np.zeros((ch, 2 * cw), np.uint8), None]


def scale_frame(src_planes, src_w, src_h, src_fmt, dst_w, dst_h, dst_fmt, method,
                param=(PARAM_DEFAULT, PARAM_DEFAULT), src_range=0, dst_range=0):
    """sws_scale of one frame through the restated C path; returns dst planes.
    src_range / dst_range: 0 MPEG (limited), 1 JPEG (full) (libswscale range conversion)."""
    dst = _alloc(dst_w, dst_h, dst_fmt)
    sd, sp = _ptrs(src_planes)
    dd, dp = _ptrs(dst)
    par = (ctypes.c_double * 2)(*param)
    r = lib().orc_scale_frame_range(src_w, src_h, src_fmt, sd, sp, dst_w, dst_h, dst_fmt, dd, dp,
                                    method | SWS_ACCURATE_RND | SWS_BITEXACT, par, src_range, dst_range)
    if r != 0:
        raise RuntimeError(f"orc_scale_frame failed ({r})")
    return dst


def nv12_to_planar(planes):
    uv = planes[1]
    return [planes[0], np.ascontiguousarray(uv[:, 0::2]), np.ascontiguousarray(uv[:, 1::2])]


def quality_frame(w, h, a_planes, b_planes):
    """vf_psnr + vf_ssim frame record for two yuv420p frames."""
    ad, ap = _ptrs(a_planes)
    bd, bp = _ptrs(b_planes)
    q = OrcQStat()
    lib().orc_quality_frame420(w, h, ad, ap, bd, bp, ctypes.byref(q))
    return {"sse": list(q.sse), "mse": list(q.mse), "mse_avg": q.mse_avg, "psnr": list(q.psnr),
            "psnr_avg": q.psnr_avg, "ssim": list(q.ssim), "ssim_all": q.ssim_all, "ssim_db": q.ssim_db}


def plane_ssim(a, b):
    return lib().orc_plane_ssim8(a.ctypes.data, a.strides[0], b.ctypes.data, b.strides[0], a.shape[1], a.shape[0])


def plane_sse(a, b):
    return lib().orc_plane_sse8(a.ctypes.data, a.strides[0], b.ctypes.data, b.strides[0], a.shape[1], a.shape[0])


def fps_map(nb_in, in_rate, out_rate, cap=1 << 20):
    out = np.zeros(cap, np.int64)
    n = lib().orc_fps_map(nb_in, in_rate[0], in_rate[1], out_rate[0], out_rate[1], out.ctypes.data, cap)
    return out[:n]


TM_MODES = {"none": 0, "linear": 1, "gamma": 2, "clip": 3, "reinhard": 4, "hable": 5, "mobius": 6}


def hdr_to_sdr(src_planes, w, h, dst_fmt, mode=5, param=float("nan"), desat=2.0, peak=0.0, npl=0.0, full=False):
    """HDR10 p010 -> SDR bt709 8-bit (zscale + vf_tonemap restated, double precision);
    full: the last zscale's r=pc (else r=tv)."""
    dst = _alloc(w, h, dst_fmt)
    sd, sp = _ptrs(src_planes)
    dd, dp = _ptrs(dst)
    r = lib().orc_hdr_to_sdr_frame(w, h, sd, sp, dst_fmt, dd, dp, mode, param, desat, peak, npl, 1 if full else 0)
    if r != 0:
        raise RuntimeError(f"orc_hdr_to_sdr_frame failed ({r})")
    return dst


def bt2020_to_bt709():
    m = ((ctypes.c_double * 3) * 3)()
    lib().orc_bt2020_to_bt709(m)
    return np.array([[m[i][j] for j in range(3)] for i in range(3)])


def yadif_frame(prev, cur, nxt, w, h, mode=0, tff=1, is_second=0):
    """vf_yadif on one yuv420p frame (planes of prev/cur/next must share pitches)."""
    pd, pp = _ptrs(prev)
    cd, cp = _ptrs(cur)
    nd, np_ = _ptrs(nxt)
    assert list(pp) == list(cp) == list(np_), "prev/cur/next must share plane pitches"
    dst = _alloc(w, h, 0)
    dd, dp = _ptrs(dst)
    r = lib().orc_yadif_frame(w, h, pd, cd, nd, cp, dd, dp, mode, tff, is_second)
    if r != 0:
        raise RuntimeError(f"orc_yadif_frame failed ({r})")
    return dst
