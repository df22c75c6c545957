"""dtsffi -- ctypes binding of libdts (include/dts.h) for tests and bench.py.

Plumbing only: the product is libdts.so (HIP kernels + C-ABI) and the Node
worker above it (../lib, ../addon).  This module loads the in-tree
``lib/libdts.so`` and fails loudly when it is missing -- there is no CPU
fallback anywhere in the product path.

Frames are lists of 2-D numpy uint8 planes: yuv420p -> [Y, U, V];
nv12 / p010le -> [Y, UV, None] (p010 planes hold raw little-endian bytes).
"""
import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.environ.get("DTS_LIB") or os.path.join(PKG, "lib", "libdts.so")

FMT_YUV420P, FMT_NV12, FMT_P010LE = 0, 1, 2
FMT_NAMES = {"yuv420p": FMT_YUV420P, "nv12": FMT_NV12, "p010le": FMT_P010LE, "p010": FMT_P010LE}
SCALE_BILINEAR, SCALE_BICUBIC, SCALE_X, SCALE_POINT = 0x2, 0x4, 0x8, 0x10
SCALE_AREA, SCALE_GAUSS, SCALE_SINC, SCALE_LANCZOS = 0x20, 0x80, 0x100, 0x200
METHODS = {"bilinear": SCALE_BILINEAR, "bicubic": SCALE_BICUBIC, "x": SCALE_X, "point": SCALE_POINT,
           "neighbor": SCALE_POINT, "area": SCALE_AREA, "gauss": SCALE_GAUSS, "sinc": SCALE_SINC,
           "lanczos": SCALE_LANCZOS}
PARAM_DEFAULT = 123456.0
Q_NONE, Q_PSNR, Q_SSIM, Q_BOTH = 0, 1, 2, 3
QREF_EXTERNAL = -1           # dts_output_spec.qref_method: references passed with every run (dts.h)
# vf_tonemap.c enum TonemapAlgorithm
TM_NONE, TM_LINEAR, TM_GAMMA, TM_CLIP, TM_REINHARD, TM_HABLE, TM_MOBIUS = range(7)
TM_MODES = {"none": TM_NONE, "linear": TM_LINEAR, "gamma": TM_GAMMA, "clip": TM_CLIP, "reinhard": TM_REINHARD,
            "hable": TM_HABLE, "mobius": TM_MOBIUS}
MAX_OUTPUTS = 4
ABI_VERSION = 7              # include/dts.h DTS_ABI_VERSION this binding lays its structs out for

E_INVAL, E_NOMEM, E_RANGE, E_UNSUPPORTED, E_BUSY, E_NODEV, E_HIP = -22, -12, -34, -95, -16, -19, -1000


class OutputSpec(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int32), ("h", ctypes.c_int32), ("fmt", ctypes.c_int32),
                ("method", ctypes.c_int32), ("param", ctypes.c_double * 2),
                ("quality", ctypes.c_int32), ("qref_method", ctypes.c_int32)]


class TonemapSpec(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("pad_", ctypes.c_int32), ("param", ctypes.c_double),
                ("desat", ctypes.c_double), ("peak", ctypes.c_double), ("npl", ctypes.c_double)]


class GraphSpec(ctypes.Structure):
    _fields_ = [("src_w", ctypes.c_int32), ("src_h", ctypes.c_int32), ("src_fmt", ctypes.c_int32),
                ("nout", ctypes.c_int32), ("out", OutputSpec * MAX_OUTPUTS),
                ("quality", ctypes.c_int32), ("quality_out", ctypes.c_int32), ("max_batch", ctypes.c_int32),
                ("hdr_to_sdr", ctypes.c_int32), ("tonemap", TonemapSpec),
                ("deint", ctypes.c_int32), ("deint_mode", ctypes.c_int32), ("deint_tff", ctypes.c_int32),
                ("range", ctypes.c_int32)]


class Frame(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * 3), ("pitch", ctypes.c_int64 * 3)]


class DevFrames(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * 3), ("pitch", ctypes.c_int64 * 3), ("frame_stride", ctypes.c_int64)]


class QRaw(ctypes.Structure):
    _fields_ = [("sse", ctypes.c_uint64 * 3), ("ssim_sum", ctypes.c_double * 3)]


class QStat(ctypes.Structure):
    _fields_ = [("sse", ctypes.c_uint64 * 3), ("mse", ctypes.c_double * 3), ("mse_avg", ctypes.c_double),
                ("psnr", ctypes.c_double * 3), ("psnr_avg", ctypes.c_double),
                ("ssim", ctypes.c_double * 3), ("ssim_all", ctypes.c_double), ("ssim_db", ctypes.c_double)]

    def as_dict(self):
        return {"sse": list(self.sse), "mse": list(self.mse), "mse_avg": self.mse_avg,
                "psnr": list(self.psnr), "psnr_avg": self.psnr_avg, "ssim": list(self.ssim),
                "ssim_all": self.ssim_all, "ssim_db": self.ssim_db}


class GraphInfo(ctypes.Structure):
    _fields_ = [("src_frame_bytes", ctypes.c_int64), ("out_frame_bytes", ctypes.c_int64 * MAX_OUTPUTS),
                ("algo_bytes_per_frame", ctypes.c_int64), ("njobs", ctypes.c_int32),
                ("lds_bytes", ctypes.c_int32), ("h_taps", (ctypes.c_int32 * 2) * MAX_OUTPUTS),
                ("v_taps", (ctypes.c_int32 * 2) * MAX_OUTPUTS),
                ("sws_h_size", (ctypes.c_int32 * 2) * MAX_OUTPUTS),
                ("sws_v_size", (ctypes.c_int32 * 2) * MAX_OUTPUTS), ("ladder_v4_mask", ctypes.c_int32),
                ("h_pairs4", (ctypes.c_int32 * 2) * MAX_OUTPUTS), ("ladder_v5", ctypes.c_int32),
                ("v5_strip_width", ctypes.c_int32 * 2), ("v5_strips", ctypes.c_int32 * 2)]


# Every symbol include/dts.h declares (checked by tests/test_abi.py).
EXPORTS = ["dts_version", "dts_strerror", "dts_device_count", "dts_ctx_create", "dts_ctx_destroy",
           "dts_ctx_last_hip_error", "dts_graph_create", "dts_graph_destroy", "dts_graph_info_get",
           "dts_graph_submit", "dts_graph_wait", "dts_graph_run_device", "dts_quality_run_device",
           "dts_qstat_finalize", "dts_synth_host", "dts_synth_device", "dts_frame_layout",
           "dts_sws_filter", "dts_fps_map", "dts_graph_plan", "dts_yadif_run_device", "dts_quality_run_host",
           "dts_qraw_sum_device", "dts_qstat_stream", "dts_abi_version", "dts_abi_struct_size",
           "dts_host_alloc", "dts_host_free", "dts_host_register", "dts_host_unregister"]

# DTS_STRUCT_* ids of dts_abi_struct_size and the ctypes layout of each (filled below)
STRUCT_IDS = {}

_lib = None


def lib():
    """Load libdts.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libdts.so not built at {LIB_PATH}; run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
    L.dts_version.restype = ctypes.c_char_p
    L.dts_strerror.restype = ctypes.c_char_p
    L.dts_strerror.argtypes = [i32]
    L.dts_device_count.argtypes = [ctypes.POINTER(i32)]
    L.dts_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.dts_ctx_destroy.argtypes = [vp]
    L.dts_ctx_destroy.restype = None
    L.dts_ctx_last_hip_error.argtypes = [vp]
    L.dts_graph_create.argtypes = [vp, ctypes.POINTER(GraphSpec), ctypes.POINTER(vp)]
    L.dts_graph_destroy.argtypes = [vp]
    L.dts_graph_destroy.restype = None
    L.dts_graph_info_get.argtypes = [vp, ctypes.POINTER(GraphInfo)]
    L.dts_graph_plan.argtypes = [ctypes.POINTER(GraphSpec), ctypes.POINTER(GraphInfo)]
    L.dts_graph_submit.argtypes = [vp, ctypes.POINTER(Frame), i32, ctypes.POINTER(Frame),
                                   ctypes.POINTER(Frame), ctypes.POINTER(QStat)]
    L.dts_graph_wait.argtypes = [vp]
    L.dts_graph_run_device.argtypes = [vp, ctypes.POINTER(DevFrames), i32, ctypes.POINTER(DevFrames),
                                       ctypes.POINTER(DevFrames), vp, vp]
    L.dts_quality_run_device.argtypes = [vp, i32, i32, i32, ctypes.POINTER(DevFrames),
                                         ctypes.POINTER(DevFrames), i32, vp, vp]
    L.dts_qstat_finalize.argtypes = [i32, i32, ctypes.POINTER(QRaw), i32, ctypes.POINTER(QStat)]
    L.dts_qraw_sum_device.argtypes = [vp, vp, i32, vp, vp]
    L.dts_qstat_stream.argtypes = [i32, i32, ctypes.POINTER(QRaw), i64, ctypes.POINTER(QStat)]
    L.dts_quality_run_host.argtypes = [vp, i32, i32, i32, ctypes.POINTER(Frame), ctypes.POINTER(Frame), i32,
                                       ctypes.POINTER(QStat)]
    L.dts_synth_host.argtypes = [i32, i32, i32, i32, u32, i64, ctypes.POINTER(Frame)]
    L.dts_synth_device.argtypes = [vp, i32, i32, i32, i32, u32, i64, ctypes.POINTER(DevFrames), i32, vp]
    L.dts_frame_layout.argtypes = [i32, i32, i32, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.dts_sws_filter.argtypes = [i32, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_double), i32, vp, vp, i32]
    L.dts_fps_map.argtypes = [i64, i32, i32, i32, i32, vp, i64]
    L.dts_fps_map.restype = i64
    L.dts_yadif_run_device.argtypes = [vp, i32, i32, i32, i32, ctypes.POINTER(DevFrames), i32, i32, i32,
                                       ctypes.POINTER(DevFrames), vp]
    L.dts_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
    L.dts_host_free.argtypes = [vp]
    L.dts_host_free.restype = None
    L.dts_host_register.argtypes = [vp, ctypes.c_size_t]
    L.dts_host_unregister.argtypes = [vp]
    L.dts_abi_version.argtypes = []
    L.dts_abi_struct_size.argtypes = [i32]
    L.dts_abi_struct_size.restype = i64
    abi_check(L)
    _lib = L
    return L


def abi_check(L):
    """Refuse a library whose ABI or struct layouts differ from this binding's (a binding
    built against another dts.h would pass misaligned specs without an error)."""
    v = L.dts_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"libdts ABI {v}, dtsffi expects {ABI_VERSION} ({LIB_PATH})")
    for which, cls in STRUCT_IDS.items():
        n = L.dts_abi_struct_size(which)
        if n != ctypes.sizeof(cls):
            raise RuntimeError(f"libdts sizeof({cls.__name__}) = {n}, dtsffi lays out {ctypes.sizeof(cls)}")


STRUCT_IDS.update({0: TonemapSpec, 1: OutputSpec, 2: GraphSpec, 3: Frame, 4: DevFrames, 5: QRaw, 6: QStat,
                   7: GraphInfo})


class DtsError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {lib().dts_strerror(code).decode()} ({code})")


def check(code, what=""):
    if code < 0:
        raise DtsError(code, what)
    return code


# ---------------------------------------------------------------------------
# host frames (numpy)
# ---------------------------------------------------------------------------
def plane_shapes(w, h, fmt):
    """(rows, row_bytes) per plane; None for the unused third plane."""
    cw, ch = (w + 1) // 2, (h + 1) // 2
    if fmt == FMT_YUV420P:
        return [(h, w), (ch, cw), (ch, cw)]
    if fmt == FMT_NV12:
        return [(h, w), (ch, 2 * cw), None]
    return [(h, 2 * w), (ch, 4 * cw), None]


def alloc_frame(w, h, fmt, pad=0):
    """Planes with an optional row padding (pitch > row bytes)."""
    planes = []
    for s in plane_shapes(w, h, fmt):
        if s is None:
            planes.append(None)
        else:
            buf = np.zeros((s[0], s[1] + pad), np.uint8)
            planes.append(buf[:, :s[1]])
    return planes


class PinnedBuffer:
    """dts_host_alloc memory as a uint8 numpy array (`.array`); freed with dts_host_free when
    the object goes away.  Frames carved from it take the host path's direct DMA (ABI 7)."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        check(lib().dts_host_alloc(nbytes, ctypes.byref(p)), "host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self._arr = None

    @property
    def array(self):
        """The buffer as a uint8 array.  Every view of it keeps this object (and so the pinned
        memory) alive: the ctypes array under the numpy base holds a reference to it, so
        dropping the PinnedBuffer while frames carved from it live frees nothing."""
        a = self._arr() if self._arr is not None else None
        if a is None:
            carr = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
            carr._owner = self
            a = np.ctypeslib.as_array(carr)
            self._arr = weakref.ref(a)
        return a

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().dts_host_free(self.ptr)
            self.ptr = None


def alloc_frames_pinned(w, h, fmt, n, pitch_align=16):
    """n frames of (w, h, fmt) in one pinned buffer: ([planes per frame], the PinnedBuffer,
    which must outlive the frames).  Row pitches are rounded up to pitch_align bytes and planes
    to 256: with 16 this is the host path's device batch layout (api.cpp DevLayout, tight), so
    every plane crosses PCIe by DMA and consecutive frames of the buffer as one DMA (ABI 7)."""
    shapes = plane_shapes(w, h, fmt)
    pitches = [None if s is None else (s[1] + pitch_align - 1) // pitch_align * pitch_align for s in shapes]
    sizes = [0 if s is None else (s[0] * p + 255) // 256 * 256 for s, p in zip(shapes, pitches)]
    fb = sum(sizes)
    buf = PinnedBuffer(max(1, fb * n))
    arr = buf.array
    frames = []
    for i in range(n):
        off, planes = i * fb, []
        for s, p, z in zip(shapes, pitches, sizes):
            if s is None:
                planes.append(None)
                continue
            planes.append(arr[off:off + s[0] * p].reshape(s[0], p)[:, :s[1]])
            off += z
        frames.append(planes)
    return frames, buf


def frame_struct(planes):
    f = Frame()
    for i, p in enumerate(planes):
        if p is None:
            f.data[i] = None
            f.pitch[i] = 0
        else:
            assert p.dtype == np.uint8 and p.strides[1] == 1
            f.data[i] = p.ctypes.data
            f.pitch[i] = p.strides[0]
    return f


def synth_host(w, h, fmt, pattern=0, seed=0x5EED, frame=0):
    planes = alloc_frame(w, h, fmt)
    check(lib().dts_synth_host(w, h, fmt, pattern, seed, frame, ctypes.byref(frame_struct(planes))), "synth_host")
    return planes


def sws_filter(src_n, dst_n, one, align, method, pos=128, param=(PARAM_DEFAULT, PARAM_DEFAULT), cap=256):
    coeff = np.zeros(dst_n * cap, np.int16)
    fpos = np.zeros(dst_n, np.int32)
    par = (ctypes.c_double * 2)(*param)
    n = check(lib().dts_sws_filter(src_n, dst_n, one, align, method, par, pos, coeff.ctypes.data,
                                   fpos.ctypes.data, cap), "sws_filter")
    return coeff[:dst_n * n].reshape(dst_n, n), fpos


def fps_map(nb_in, in_rate, out_rate):
    in_num, in_den = in_rate
    out_num, out_den = out_rate
    n = check(lib().dts_fps_map(nb_in, in_num, in_den, out_num, out_den, None, 0), "fps_map")
    out = np.zeros(max(n, 1), np.int64)
    lib().dts_fps_map(nb_in, in_num, in_den, out_num, out_den, out.ctypes.data, n)
    return out[:n]


def qstat_finalize(w, h, raws):
    n = len(raws)
    arr = (QRaw * n)(*raws)
    out = (QStat * n)()
    check(lib().dts_qstat_finalize(w, h, arr, n, out), "qstat_finalize")
    return [out[i].as_dict() for i in range(n)]


def qstat_stream(w, h, raw_sum, nframes):
    """dts_qstat_stream: vf_psnr / vf_ssim end-of-stream averages of nframes frames
    from their summed record (a QRaw)."""
    out = QStat()
    check(lib().dts_qstat_stream(w, h, ctypes.byref(raw_sum), nframes, ctypes.byref(out)), "qstat_stream")
    return out.as_dict()


def qraw_sum_host(raws):
    """The sum of QRaw records (u64 SSE, f64 SSIM sums) on the host, in list order."""
    s = QRaw()
    for r in raws:
        for c in range(3):
            s.sse[c] += r.sse[c]
            s.ssim_sum[c] += r.ssim_sum[c]
    return s


def graph_plan(spec):
    """dts_graph_plan: the graph's info (filter sizes, kernel choice) without a device."""
    info = GraphInfo()
    check(lib().dts_graph_plan(ctypes.byref(spec), ctypes.byref(info)), "graph_plan")
    return info


def make_spec(src_w, src_h, src_fmt, outputs, quality=Q_NONE, quality_out=0, max_batch=0, tonemap=None,
              deint=None, src_range=0, dst_range=0):
    """outputs: list of (w, h, fmt, method[, (p0, p1)[, (quality, qref_method)]]): the last
    turns on rendition quality (dts_output_spec.quality / qref_method).  tonemap: None, or a dict
    {mode, param, desat, peak, npl} turning on HDR10 -> SDR (dts_tonemap_spec).
    deint: None, or (mode, tff) for yadif ahead of the ladder (sources then carry one
    context frame on each side: dts_graph_spec.deint)."""
    s = GraphSpec()
    s.src_w, s.src_h, s.src_fmt = src_w, src_h, src_fmt
    s.nout = len(outputs)
    for i, o in enumerate(outputs):
        s.out[i].w, s.out[i].h, s.out[i].fmt, s.out[i].method = o[0], o[1], o[2], o[3]
        par = o[4] if len(o) > 4 and o[4] is not None else (PARAM_DEFAULT, PARAM_DEFAULT)
        s.out[i].param[0], s.out[i].param[1] = par
        if len(o) > 5 and o[5] is not None:
            s.out[i].quality, s.out[i].qref_method = o[5]
    s.quality, s.quality_out, s.max_batch = quality, quality_out, max_batch
    if tonemap is not None:
        s.hdr_to_sdr = 1
        s.tonemap.mode = tonemap.get("mode", TM_HABLE)
        s.tonemap.param = tonemap.get("param", float("nan"))
        s.tonemap.desat = tonemap.get("desat", 2.0)          # vf_tonemap's default (FFmpeg 4.4)
        s.tonemap.peak = tonemap.get("peak", 0.0)
        s.tonemap.npl = tonemap.get("npl", 100.0)
    if deint is not None:
        s.deint, s.deint_mode, s.deint_tff = 1, deint[0], deint[1]
    s.range = (src_range & 1) | ((dst_range & 1) << 4)   # DTS_RANGE_*: 0 MPEG (limited), 1 JPEG (full)
    return s


# ---------------------------------------------------------------------------
# device objects
# ---------------------------------------------------------------------------
def device_count():
    n = ctypes.c_int(0)
    lib().dts_device_count(ctypes.byref(n))
    return n.value


class Context:
    def __init__(self, device=0):
        self.h = ctypes.c_void_p()
        check(lib().dts_ctx_create(device, ctypes.byref(self.h)), "ctx_create")
        self.device = device

    def close(self):
        if self.h:
            lib().dts_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def quality_device(self, w, h, fmt, a, b, nframes, qraw_ptr, stream=None):
        check(lib().dts_quality_run_device(self.h, w, h, fmt, ctypes.byref(a), ctypes.byref(b), nframes,
                                           ctypes.c_void_p(qraw_ptr), ctypes.c_void_p(stream or 0)),
              "quality_run_device")

    def qraw_sum_device(self, raw_ptr, n, sum_ptr, stream=None):
        check(lib().dts_qraw_sum_device(self.h, ctypes.c_void_p(raw_ptr), n, ctypes.c_void_p(sum_ptr),
                                        ctypes.c_void_p(stream or 0)), "qraw_sum_device")

    def quality_host(self, w, h, fmt, a_frames, b_frames):
        """vf_psnr + vf_ssim of host frames a[i] vs b[i] (plane lists) -> [qstat dict]."""
        n = len(a_frames)
        a = (Frame * n)(*[frame_struct(f) for f in a_frames])
        b = (Frame * n)(*[frame_struct(f) for f in b_frames])
        q = (QStat * n)()
        check(lib().dts_quality_run_host(self.h, w, h, fmt, a, b, n, q), "quality_run_host")
        return [q[i].as_dict() for i in range(n)]

    def yadif_device(self, w, h, mode, tff, seq, nseq, first, count, dst, stream=None):
        check(lib().dts_yadif_run_device(self.h, w, h, mode, tff, ctypes.byref(seq), nseq, first, count,
                                         ctypes.byref(dst), ctypes.c_void_p(stream or 0)), "yadif_run_device")

    def synth_device(self, w, h, fmt, pattern, seed, first, dst, nframes, stream=None):
        check(lib().dts_synth_device(self.h, w, h, fmt, pattern, seed, first, ctypes.byref(dst), nframes,
                                     ctypes.c_void_p(stream or 0)), "synth_device")


class Graph:
    def __init__(self, ctx, spec):
        self.ctx = ctx
        self.spec = spec
        self.h = ctypes.c_void_p()
        check(lib().dts_graph_create(ctx.h, ctypes.byref(spec), ctypes.byref(self.h)), "graph_create")
        self.info = GraphInfo()
        check(lib().dts_graph_info_get(self.h, ctypes.byref(self.info)), "graph_info")

    def close(self):
        if self.h:
            lib().dts_graph_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run_host(self, frames, qref=None, pinned_out=False):
        """frames: list of source frames (plane lists; with deint, n + 2 of them: one
        context frame each side).  Returns (outputs, qstats): outputs[f][k] is output
        k of frame f as a plane list.  pinned_out: the outputs are allocated with
        dts_host_alloc (the library DMAs straight into them; ABI 7); an int is the outputs'
        row-pitch alignment (16, the default for True: every plane direct)."""
        s = self.spec
        ns = len(frames)
        n = ns - 2 if s.deint else ns
        src = (Frame * ns)(*[frame_struct(f) for f in frames])
        if pinned_out:
            pa = 16 if pinned_out is True else int(pinned_out)
            # (each output plane is a view that keeps its PinnedBuffer alive)
            per = [alloc_frames_pinned(s.out[k].w, s.out[k].h, s.out[k].fmt, n, pa) for k in range(s.nout)]
            outs = [[per[k][0][f] for k in range(s.nout)] for f in range(n)]
        else:
            outs = [[alloc_frame(s.out[k].w, s.out[k].h, s.out[k].fmt) for k in range(s.nout)] for _ in range(n)]
        dst = (Frame * (n * s.nout))(*[frame_struct(outs[f][k]) for f in range(n) for k in range(s.nout)])
        rq = any(s.out[k].quality for k in range(s.nout))
        if rq:                      # rendition quality: q[f * nout + k]
            qs = (QStat * (n * s.nout))()
            check(lib().dts_graph_submit(self.h, src, n, dst, None, qs), "graph_submit")
            check(lib().dts_graph_wait(self.h), "graph_wait")
            return outs, [[qs[f * s.nout + k].as_dict() if s.out[k].quality else None for k in range(s.nout)]
                          for f in range(n)]
        qr = (Frame * n)(*[frame_struct(q) for q in qref]) if qref is not None else None
        qs = (QStat * n)() if qref is not None else None
        check(lib().dts_graph_submit(self.h, src, n, dst, qr, qs), "graph_submit")
        check(lib().dts_graph_wait(self.h), "graph_wait")
        return outs, ([qs[i].as_dict() for i in range(n)] if qs is not None else None)

    def run_device(self, src, nframes, dsts, qref=None, qraw_ptr=0, stream=None):
        """qref: the quality_out reference batch (DevFrames), or with rendition quality against
        external references (qref_method QREF_EXTERNAL) a list of one DevFrames per output"""
        k = len(dsts)
        arr = (DevFrames * k)(*dsts)
        if isinstance(qref, (list, tuple)):
            qarg = (DevFrames * len(qref))(*[q if q is not None else DevFrames() for q in qref])
        else:
            qarg = ctypes.byref(qref) if qref is not None else None
        check(lib().dts_graph_run_device(self.h, ctypes.byref(src), nframes, arr, qarg,
                                         ctypes.c_void_p(qraw_ptr), ctypes.c_void_p(stream or 0)),
              "graph_run_device")
