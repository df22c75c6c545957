/*
 * dts_napi.c -- thin N-API binding of include/dts.h for the Node.js worker.
 *
 * The reference server is Node.js (index.js); its worker would spawn the
 * ffmpeg-static binary (index.js:9).  This addon is the in-process
 * replacement: the worker builds a graph from the job row
 * (database.js:73-79) and runs segment frames through libdts.so.  Frame
 * processing runs in napi_async_work on the libuv pool so the event loop never
 * blocks; results resolve a Promise.  Written for Node 12 / N-API 8 (plain C,
 * no node-addon-api), built by gcc against /usr/include/node.
 */
#include <pthread.h>
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include "dts.h"

#define NAPI_OK(env, call)                                                    \
    do {                                                                      \
        if ((call) != napi_ok) {                                              \
            napi_throw_error((env), NULL, "N-API call failed: " #call);       \
            return NULL;                                                      \
        }                                                                     \
    } while (0)

static napi_value throw_dts(napi_env env, int code, const char *what)
{
    char msg[256];
    snprintf(msg, sizeof msg, "%s: %s (%d)", what, dts_strerror(code), code);
    char codebuf[32];
    snprintf(codebuf, sizeof codebuf, "%d", code);
    napi_throw_error(env, codebuf, msg);
    return NULL;
}

static int get_i32(napi_env env, napi_value obj, const char *key, int32_t dflt, int32_t *out)
{
    bool has = false;
    napi_value v;
    *out = dflt;
    if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return 0;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return -1;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_undefined || t == napi_null) return 0;
    return napi_get_value_int32(env, v, out) == napi_ok ? 0 : -1;
}

static int get_f64(napi_env env, napi_value obj, const char *key, double dflt, double *out)
{
    bool has = false;
    napi_value v;
    *out = dflt;
    if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return 0;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return -1;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_undefined || t == napi_null) return 0;
    return napi_get_value_double(env, v, out) == napi_ok ? 0 : -1;
}

static void finalize_ctx(napi_env env, void *data, void *hint)
{
    (void)env;
    (void)hint;
    dts_ctx_destroy((dts_ctx *)data);
}

/* A graph external: the libdts graph plus the spec it was made from (run()
 * validates every caller frame against it).  libdts reference-counts the
 * context, so the graph stays valid whichever finalizer runs first. */
typedef struct {
    dts_graph *g;
    dts_graph_spec spec;
} graph_box;

static void finalize_graph(napi_env env, void *data, void *hint)
{
    (void)env;
    (void)hint;
    graph_box *b = (graph_box *)data;
    dts_graph_destroy(b->g);
    free(b);
}

static graph_box *get_graph(napi_env env, napi_value v)
{
    graph_box *b = NULL;
    if (napi_get_value_external(env, v, (void **)&b) != napi_ok || !b || !b->g) return NULL;
    return b;
}

/* ---- version(), deviceCount() ------------------------------------------ */
static napi_value js_version(napi_env env, napi_callback_info info)
{
    (void)info;
    napi_value s;
    NAPI_OK(env, napi_create_string_utf8(env, dts_version(), NAPI_AUTO_LENGTH, &s));
    return s;
}

static napi_value js_device_count(napi_env env, napi_callback_info info)
{
    (void)info;
    int n = 0;
    dts_device_count(&n);
    napi_value v;
    NAPI_OK(env, napi_create_int32(env, n, &v));
    return v;
}

/* ---- createContext(device) -> external ---------------------------------- */
static napi_value js_create_context(napi_env env, napi_callback_info info)
{
    size_t argc = 1;
    napi_value argv[1];
    int32_t dev = 0;
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc >= 1) napi_get_value_int32(env, argv[0], &dev);
    dts_ctx *ctx = NULL;
    int e = dts_ctx_create(dev, &ctx);
    if (e) return throw_dts(env, e, "dts_ctx_create");
    napi_value ext;
    NAPI_OK(env, napi_create_external(env, ctx, finalize_ctx, NULL, &ext));
    return ext;
}

/* ---- createGraph(ctx, spec) -> external --------------------------------- */
static int parse_spec(napi_env env, napi_value o, dts_graph_spec *s)
{
    memset(s, 0, sizeof *s);
    napi_value src, outs;
    if (napi_get_named_property(env, o, "src", &src) != napi_ok) return -1;
    if (get_i32(env, src, "w", 0, &s->src_w) || get_i32(env, src, "h", 0, &s->src_h) ||
        get_i32(env, src, "fmt", 0, &s->src_fmt))
        return -1;
    if (napi_get_named_property(env, o, "outputs", &outs) != napi_ok) return -1;
    uint32_t n = 0;
    if (napi_get_array_length(env, outs, &n) != napi_ok || n < 1 || n > DTS_MAX_OUTPUTS) return -1;
    s->nout = (int32_t)n;
    for (uint32_t i = 0; i < n; ++i) {
        napi_value oi, par;
        bool has = false;
        napi_get_element(env, outs, i, &oi);
        dts_output_spec *os = &s->out[i];
        if (get_i32(env, oi, "w", 0, &os->w) || get_i32(env, oi, "h", 0, &os->h) ||
            get_i32(env, oi, "fmt", DTS_FMT_NV12, &os->fmt) || get_i32(env, oi, "method", DTS_SCALE_BICUBIC, &os->method))
            return -1;
        /* rendition quality: {quality: DTS_Q_*, qrefMethod: DTS_SCALE_*} (dts_output_spec, ABI 6) */
        if (get_i32(env, oi, "quality", 0, &os->quality) ||
            get_i32(env, oi, "qrefMethod", DTS_SCALE_LANCZOS, &os->qref_method))
            return -1;
        os->param[0] = os->param[1] = DTS_PARAM_DEFAULT;
        napi_has_named_property(env, oi, "param", &has);
        if (has) {
            napi_get_named_property(env, oi, "param", &par);
            uint32_t pn = 0;
            if (napi_get_array_length(env, par, &pn) == napi_ok)
                for (uint32_t k = 0; k < pn && k < 2; ++k) {
                    napi_value pv;
                    napi_get_element(env, par, k, &pv);
                    napi_valuetype t;
                    napi_typeof(env, pv, &t);
                    if (t == napi_number) napi_get_value_double(env, pv, &os->param[k]);
                }
        }
    }
    if (get_i32(env, o, "quality", 0, &s->quality) || get_i32(env, o, "qualityOut", 0, &s->quality_out) ||
        get_i32(env, o, "maxBatch", 0, &s->max_batch))
        return -1;
    /* srcRange / dstRange: 0 = tv (limited), 1 = pc (full) -> dts_graph_spec.range */
    {
        int32_t sr = 0, dr = 0;
        if (get_i32(env, o, "srcRange", 0, &sr) || get_i32(env, o, "dstRange", 0, &dr)) return -1;
        s->range = (sr & 1) | ((dr & 1) << 4);
    }
    /* deint: {mode, tff} -> yadif ahead of the ladder (sources carry a context frame each side) */
    bool has_di = false;
    napi_has_named_property(env, o, "deint", &has_di);
    if (has_di) {
        napi_value di;
        napi_valuetype t;
        if (napi_get_named_property(env, o, "deint", &di) != napi_ok) return -1;
        napi_typeof(env, di, &t);
        if (t == napi_object) {
            s->deint = 1;
            if (get_i32(env, di, "mode", 0, &s->deint_mode) || get_i32(env, di, "tff", 1, &s->deint_tff)) return -1;
        }
    }
    /* tonemap: {mode, param, desat, peak, npl} -> HDR10 -> SDR (vf_tonemap / zscale) */
    bool has_tm = false;
    napi_has_named_property(env, o, "tonemap", &has_tm);
    if (has_tm) {
        napi_value tm;
        napi_valuetype t;
        if (napi_get_named_property(env, o, "tonemap", &tm) != napi_ok) return -1;
        napi_typeof(env, tm, &t);
        if (t == napi_object) {
            s->hdr_to_sdr = 1;
            if (get_i32(env, tm, "mode", DTS_TM_HABLE, &s->tonemap.mode) ||
                get_f64(env, tm, "param", NAN, &s->tonemap.param) ||
                get_f64(env, tm, "desat", 2.0, &s->tonemap.desat) /* vf_tonemap default */ ||
                get_f64(env, tm, "peak", 0.0, &s->tonemap.peak) || get_f64(env, tm, "npl", 100.0, &s->tonemap.npl))
                return -1;
        }
    }
    return 0;
}

static napi_value js_create_graph(napi_env env, napi_callback_info info)
{
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 2) return throw_dts(env, DTS_E_INVAL, "createGraph(ctx, spec)");
    dts_ctx *ctx = NULL;
    if (napi_get_value_external(env, argv[0], (void **)&ctx) != napi_ok || !ctx)
        return throw_dts(env, DTS_E_INVAL, "createGraph: ctx");
    dts_graph_spec s;
    if (parse_spec(env, argv[1], &s)) return throw_dts(env, DTS_E_INVAL, "createGraph: spec");
    graph_box *b = (graph_box *)calloc(1, sizeof(graph_box));
    if (!b) return throw_dts(env, DTS_E_NOMEM, "createGraph");
    int e = dts_graph_create(ctx, &s, &b->g);
    if (e) {
        free(b);
        return throw_dts(env, e, "dts_graph_create");
    }
    b->spec = s;
    napi_value ext;
    if (napi_create_external(env, b, finalize_graph, NULL, &ext) != napi_ok) {
        dts_graph_destroy(b->g);
        free(b);
        return throw_dts(env, DTS_E_NOMEM, "createGraph: external");
    }
    return ext;
}

static napi_value set_num(napi_env env, napi_value obj, const char *k, double v)
{
    napi_value n;
    napi_create_double(env, v, &n);
    napi_set_named_property(env, obj, k, n);
    return obj;
}

static napi_value js_graph_info(napi_env env, napi_callback_info info)
{
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    graph_box *b = argc >= 1 ? get_graph(env, argv[0]) : NULL;
    if (!b) return throw_dts(env, DTS_E_INVAL, "graphInfo(graph)");
    dts_graph_info gi;
    int e = dts_graph_info_get(b->g, &gi);
    if (e) return throw_dts(env, e, "dts_graph_info_get");
    napi_value o;
    NAPI_OK(env, napi_create_object(env, &o));
    set_num(env, o, "srcFrameBytes", (double)gi.src_frame_bytes);
    set_num(env, o, "algoBytesPerFrame", (double)gi.algo_bytes_per_frame);
    set_num(env, o, "jobs", gi.njobs);
    set_num(env, o, "ldsBytes", gi.lds_bytes);
    napi_value arr;
    napi_create_array(env, &arr);
    for (int k = 0; k < DTS_MAX_OUTPUTS; ++k) {
        napi_value n;
        napi_create_double(env, (double)gi.out_frame_bytes[k], &n);
        napi_set_element(env, arr, (uint32_t)k, n);
    }
    napi_set_named_property(env, o, "outFrameBytes", arr);
    return o;
}

/* ---- frames ------------------------------------------------------------- */
/* {data: [Buffer, Buffer, Buffer|null], pitch: [n, n, n]}; len[p] = byte
 * length of plane p's Buffer (0 when it is not a Buffer) */
static int parse_frame(napi_env env, napi_value o, dts_frame *f, size_t len[3])
{
    napi_value data, pitch;
    memset(f, 0, sizeof *f);
    len[0] = len[1] = len[2] = 0;
    if (napi_get_named_property(env, o, "data", &data) != napi_ok ||
        napi_get_named_property(env, o, "pitch", &pitch) != napi_ok)
        return -1;
    for (uint32_t p = 0; p < 3; ++p) {
        napi_value b, pv;
        bool isbuf = false;
        if (napi_get_element(env, data, p, &b) != napi_ok) return -1;
        napi_is_buffer(env, b, &isbuf);
        if (isbuf) {
            if (napi_get_buffer_info(env, b, &f->data[p], &len[p]) != napi_ok) return -1;
        } else {
            f->data[p] = NULL;
        }
        if (napi_get_element(env, pitch, p, &pv) != napi_ok) return -1;
        int64_t pi = 0;
        napi_valuetype t;
        napi_typeof(env, pv, &t);
        if (t == napi_number) napi_get_value_int64(env, pv, &pi);
        f->pitch[p] = pi;
    }
    return 0;
}

/* Every plane the format declares is a Buffer whose pitch covers a row and
 * whose length covers pitch * (rows - 1) + row bytes (libdts reads and
 * writes exactly that much through the caller's pointers). */
static int frame_fits(const dts_frame *f, const size_t len[3], int w, int h, int fmt)
{
    int64_t rowb[3], rows[3];
    if (dts_frame_layout(w, h, fmt, rowb, rows, NULL)) return 0;
    for (int p = 0; p < 3; ++p) {
        if (!rowb[p]) continue;
        if (!f->data[p] || f->pitch[p] < rowb[p]) return 0;
        if ((uint64_t)len[p] < (uint64_t)(f->pitch[p] * (rows[p] - 1) + rowb[p])) return 0;
    }
    return 1;
}

/* frames i of arr must each fit geometry (w[i % nw], h[i % nw], fmt[i % nw]) */
static int parse_frames(napi_env env, napi_value arr, dts_frame **out, uint32_t *n, const int32_t *w,
                        const int32_t *h, const int32_t *fmt, int nw)
{
    *out = NULL;
    if (napi_get_array_length(env, arr, n) != napi_ok) return -1;
    *out = (dts_frame *)calloc(*n ? *n : 1, sizeof(dts_frame));
    if (!*out) return -1;
    for (uint32_t i = 0; i < *n; ++i) {
        napi_value fo;
        size_t len[3];
        if (napi_get_element(env, arr, i, &fo) != napi_ok) return -1;
        if (parse_frame(env, fo, &(*out)[i], len)) return -1;
        const int k = (int)(i % (uint32_t)nw);
        if (!frame_fits(&(*out)[i], len, w[k], h[k], fmt[k])) return -1;
    }
    return 0;
}

/* ---- run(graph, src[], dst[], qref[]|null) -> Promise<qstat[]|null> ---- */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref keep[4];            /* graph, src, dst, qref arrays kept alive */
    dts_graph *g;
    dts_frame *src, *dst, *qref;
    dts_qstat *q;
    int n, nq, status;           /* nq: statistics per frame (rendition quality: nout) */
    int rq[DTS_MAX_OUTPUTS];     /* output k carries rendition quality */
    int nout;
} run_job;

static void free_job(run_job *j)
{
    free(j->src);
    free(j->dst);
    free(j->qref);
    free(j->q);
    free(j);
}

static void run_execute(napi_env env, void *data)
{
    (void)env;
    run_job *j = (run_job *)data;
    j->status = dts_graph_submit(j->g, j->src, j->n, j->dst, j->qref, j->q);
    int w = dts_graph_wait(j->g);
    if (!j->status) j->status = w;
}

static napi_value qstat_obj(napi_env env, const dts_qstat *q)
{
    napi_value o, a;
    napi_create_object(env, &o);
    const char *comp[3] = {"y", "u", "v"};
    napi_create_object(env, &a);
    for (int c = 0; c < 3; ++c) set_num(env, a, comp[c], (double)q->sse[c]);
    napi_set_named_property(env, o, "sse", a);
    napi_create_object(env, &a);
    for (int c = 0; c < 3; ++c) set_num(env, a, comp[c], q->psnr[c]);
    napi_set_named_property(env, o, "psnr", a);
    napi_create_object(env, &a);
    for (int c = 0; c < 3; ++c) set_num(env, a, comp[c], q->ssim[c]);
    napi_set_named_property(env, o, "ssim", a);
    set_num(env, o, "mseAvg", q->mse_avg);
    set_num(env, o, "psnrAvg", q->psnr_avg);
    set_num(env, o, "ssimAll", q->ssim_all);
    set_num(env, o, "ssimDb", q->ssim_db);
    return o;
}

static void run_complete(napi_env env, napi_status st, void *data)
{
    run_job *j = (run_job *)data;
    if (st != napi_ok || j->status) {
        napi_value err, msg, code;
        char buf[160], cb[32];
        int e = j->status ? j->status : DTS_E_INVAL;
        snprintf(buf, sizeof buf, "dts run: %s (%d)", dts_strerror(e), e);
        snprintf(cb, sizeof cb, "%d", e);
        napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &msg);
        napi_create_string_utf8(env, cb, NAPI_AUTO_LENGTH, &code);
        napi_create_error(env, code, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    } else {
        napi_value res;
        if (j->q && j->nq > 1) {        /* rendition quality: res[f][k] (null for outputs without it) */
            napi_create_array_with_length(env, (size_t)j->n, &res);
            for (int i = 0; i < j->n; ++i) {
                napi_value row;
                napi_create_array_with_length(env, (size_t)j->nout, &row);
                for (int k = 0; k < j->nout; ++k) {
                    napi_value v;
                    if (j->rq[k])
                        v = qstat_obj(env, &j->q[(size_t)i * j->nout + k]);
                    else
                        napi_get_null(env, &v);
                    napi_set_element(env, row, (uint32_t)k, v);
                }
                napi_set_element(env, res, (uint32_t)i, row);
            }
        } else if (j->q) {
            napi_create_array_with_length(env, (size_t)j->n, &res);
            for (int i = 0; i < j->n; ++i) napi_set_element(env, res, (uint32_t)i, qstat_obj(env, &j->q[i]));
        } else {
            napi_get_null(env, &res);
        }
        napi_resolve_deferred(env, j->deferred, res);
    }
    for (int k = 0; k < 4; ++k)
        if (j->keep[k]) napi_delete_reference(env, j->keep[k]);
    napi_delete_async_work(env, j->work);
    free_job(j);
}

static napi_value js_run(napi_env env, napi_callback_info info)
{
    size_t argc = 4;
    napi_value argv[4];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 3) return throw_dts(env, DTS_E_INVAL, "run(graph, src, dst[, qref])");
    graph_box *b = get_graph(env, argv[0]);
    if (!b) return throw_dts(env, DTS_E_INVAL, "run: graph");
    const dts_graph_spec *s = &b->spec;
    run_job *j = (run_job *)calloc(1, sizeof(run_job));
    if (!j) return throw_dts(env, DTS_E_NOMEM, "run");
    j->g = b->g;
    int32_t ow[DTS_MAX_OUTPUTS], oh[DTS_MAX_OUTPUTS], of[DTS_MAX_OUTPUTS];
    for (int k = 0; k < s->nout; ++k) {
        ow[k] = s->out[k].w;
        oh[k] = s->out[k].h;
        of[k] = s->out[k].fmt;
    }
    uint32_t ns = 0, nd = 0, nq = 0;
    if (parse_frames(env, argv[1], &j->src, &ns, &s->src_w, &s->src_h, &s->src_fmt, 1) ||
        parse_frames(env, argv[2], &j->dst, &nd, ow, oh, of, s->nout)) {
        free_job(j);
        return throw_dts(env, DTS_E_INVAL, "run: frames (a plane is missing, or its Buffer / pitch is too small)");
    }
    const uint32_t cf = s->deint ? 2u : 0u;       /* deint: one context frame each side of the segment */
    if (ns < cf || (uint64_t)nd != (uint64_t)(ns - cf) * (uint64_t)s->nout) {
        free_job(j);
        return throw_dts(env, DTS_E_INVAL, "run: dst must hold (src.length - context) * outputs frames (frame-major)");
    }
    j->n = (int)(ns - cf);
    j->nout = s->nout;
    int any_rq = 0;
    for (int k = 0; k < s->nout; ++k) any_rq |= j->rq[k] = s->out[k].quality != 0;
    if (any_rq) {                                 /* rendition quality: nout statistics per frame */
        j->nq = s->nout;
        j->q = (dts_qstat *)calloc(j->n ? (size_t)j->n * s->nout : 1, sizeof(dts_qstat));
        if (!j->q) {
            free_job(j);
            return throw_dts(env, DTS_E_NOMEM, "run");
        }
    }
    napi_valuetype qt = napi_undefined;
    if (argc >= 4) napi_typeof(env, argv[3], &qt);
    if (qt == napi_object && !any_rq) {
        const int qo = s->quality_out;
        if (!s->quality || parse_frames(env, argv[3], &j->qref, &nq, &ow[qo], &oh[qo], &of[qo], 1) ||
            nq != (uint32_t)j->n) {
            free_job(j);
            return throw_dts(env, DTS_E_INVAL, "run: qref frames");
        }
        j->q = (dts_qstat *)calloc(j->n ? (size_t)j->n : 1, sizeof(dts_qstat));
        if (!j->q) {
            free_job(j);
            return throw_dts(env, DTS_E_NOMEM, "run");
        }
    } else if (s->quality) {
        free_job(j);
        return throw_dts(env, DTS_E_INVAL, "run: the graph has quality on and needs qref frames");
    }
    for (int k = 0; k < 4 && (size_t)k < argc; ++k) {
        napi_valuetype t;
        napi_typeof(env, argv[k], &t);
        if (t == napi_object || t == napi_external) napi_create_reference(env, argv[k], 1, &j->keep[k]);
    }
    napi_value promise, name;
    NAPI_OK(env, napi_create_promise(env, &j->deferred, &promise));
    napi_create_string_utf8(env, "dts_run", NAPI_AUTO_LENGTH, &name);
    NAPI_OK(env, napi_create_async_work(env, NULL, name, run_execute, run_complete, j, &j->work));
    NAPI_OK(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* ---- quality(ctx, w, h, fmt, a[], b[]) -> Promise<qstat[]> --------------- */
/* vf_psnr + vf_ssim of a[i] against b[i] (8-bit yuv420p / nv12 frames of one size)
 * on the ctx's GPU, off the event loop (dts_quality_run_host). */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref keep[3];            /* ctx, a, b kept alive */
    dts_ctx *ctx;
    dts_frame *a, *b;
    dts_qstat *q;
    int w, h, fmt, n, status;
} quality_job;

static void free_qjob(quality_job *j)
{
    free(j->a);
    free(j->b);
    free(j->q);
    free(j);
}

static void quality_execute(napi_env env, void *data)
{
    (void)env;
    quality_job *j = (quality_job *)data;
    j->status = dts_quality_run_host(j->ctx, j->w, j->h, j->fmt, j->a, j->b, j->n, j->q);
}

static void quality_complete(napi_env env, napi_status st, void *data)
{
    quality_job *j = (quality_job *)data;
    if (st != napi_ok || j->status) {
        napi_value err, msg, code;
        char buf[160], cb[32];
        int e = j->status ? j->status : DTS_E_INVAL;
        snprintf(buf, sizeof buf, "dts quality: %s (%d)", dts_strerror(e), e);
        snprintf(cb, sizeof cb, "%d", e);
        napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &msg);
        napi_create_string_utf8(env, cb, NAPI_AUTO_LENGTH, &code);
        napi_create_error(env, code, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    } else {
        napi_value res;
        napi_create_array_with_length(env, (size_t)j->n, &res);
        for (int i = 0; i < j->n; ++i) napi_set_element(env, res, (uint32_t)i, qstat_obj(env, &j->q[i]));
        napi_resolve_deferred(env, j->deferred, res);
    }
    for (int k = 0; k < 3; ++k)
        if (j->keep[k]) napi_delete_reference(env, j->keep[k]);
    napi_delete_async_work(env, j->work);
    free_qjob(j);
}

static napi_value js_quality(napi_env env, napi_callback_info info)
{
    size_t argc = 6;
    napi_value argv[6];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 6) return throw_dts(env, DTS_E_INVAL, "quality(ctx, w, h, fmt, a, b)");
    quality_job *j = (quality_job *)calloc(1, sizeof(quality_job));
    if (!j) return throw_dts(env, DTS_E_NOMEM, "quality");
    if (napi_get_value_external(env, argv[0], (void **)&j->ctx) != napi_ok || !j->ctx) {
        free_qjob(j);
        return throw_dts(env, DTS_E_INVAL, "quality: ctx");
    }
    napi_get_value_int32(env, argv[1], &j->w);
    napi_get_value_int32(env, argv[2], &j->h);
    napi_get_value_int32(env, argv[3], &j->fmt);
    uint32_t na = 0, nb = 0;
    if (j->w < 1 || j->h < 1 || (j->fmt != DTS_FMT_YUV420P && j->fmt != DTS_FMT_NV12) ||
        parse_frames(env, argv[4], &j->a, &na, &j->w, &j->h, &j->fmt, 1) ||
        parse_frames(env, argv[5], &j->b, &nb, &j->w, &j->h, &j->fmt, 1) || na != nb) {
        free_qjob(j);
        return throw_dts(env, DTS_E_INVAL, "quality: frames (8-bit 4:2:0, equal counts, planes that fit)");
    }
    j->n = (int)na;
    j->q = (dts_qstat *)calloc(na ? na : 1, sizeof(dts_qstat));
    if (!j->q) {
        free_qjob(j);
        return throw_dts(env, DTS_E_NOMEM, "quality");
    }
    napi_create_reference(env, argv[0], 1, &j->keep[0]);
    napi_create_reference(env, argv[4], 1, &j->keep[1]);
    napi_create_reference(env, argv[5], 1, &j->keep[2]);
    napi_value promise, name;
    NAPI_OK(env, napi_create_promise(env, &j->deferred, &promise));
    napi_create_string_utf8(env, "dts_quality", NAPI_AUTO_LENGTH, &name);
    NAPI_OK(env, napi_create_async_work(env, NULL, name, quality_execute, quality_complete, j, &j->work));
    NAPI_OK(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* ---- synthFrame(w, h, fmt, pattern, seed, index, frame) ---------------- */
/* ---- qstatStream(w, h, sse[3], ssimSum[3], frames) -> qstat ---------------- */
/* vf_psnr / vf_ssim end-of-stream averages from a summed record (dts_qstat_stream) */
static napi_value js_qstat_stream(napi_env env, napi_callback_info info)
{
    size_t argc = 5;
    napi_value argv[5];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 5) return throw_dts(env, DTS_E_INVAL, "qstatStream(w, h, sse, ssimSum, frames)");
    int32_t w = 0, h = 0;
    int64_t n = 0;
    napi_get_value_int32(env, argv[0], &w);
    napi_get_value_int32(env, argv[1], &h);
    napi_get_value_int64(env, argv[4], &n);
    dts_qraw r;
    memset(&r, 0, sizeof r);
    for (uint32_t c = 0; c < 3; ++c) {
        napi_value v;
        double d = 0;
        if (napi_get_element(env, argv[2], c, &v) != napi_ok || napi_get_value_double(env, v, &d) != napi_ok)
            return throw_dts(env, DTS_E_INVAL, "qstatStream: sse");
        r.sse[c] = (uint64_t)d;
        if (napi_get_element(env, argv[3], c, &v) != napi_ok || napi_get_value_double(env, v, &r.ssim_sum[c]) != napi_ok)
            return throw_dts(env, DTS_E_INVAL, "qstatStream: ssimSum");
    }
    dts_qstat q;
    const int e = dts_qstat_stream(w, h, &r, n, &q);
    if (e) return throw_dts(env, e, "dts_qstat_stream");
    return qstat_obj(env, &q);
}

static napi_value js_synth_frame(napi_env env, napi_callback_info info)
{
    size_t argc = 7;
    napi_value argv[7];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 7) return throw_dts(env, DTS_E_INVAL, "synthFrame(w, h, fmt, pattern, seed, index, frame)");
    int32_t w, h, fmt, pat;
    uint32_t seed;
    int64_t idx;
    napi_get_value_int32(env, argv[0], &w);
    napi_get_value_int32(env, argv[1], &h);
    napi_get_value_int32(env, argv[2], &fmt);
    napi_get_value_int32(env, argv[3], &pat);
    napi_get_value_uint32(env, argv[4], &seed);
    napi_get_value_int64(env, argv[5], &idx);
    dts_frame f;
    size_t len[3];
    if (parse_frame(env, argv[6], &f, len) || !frame_fits(&f, len, w, h, fmt))
        return throw_dts(env, DTS_E_INVAL, "synthFrame: frame");
    int e = dts_synth_host(w, h, fmt, pat, seed, idx, &f);
    if (e) return throw_dts(env, e, "dts_synth_host");
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

/* ---- hostAlloc(bytes) -> Buffer in pinned memory (dts_host_alloc, ABI 7) ----------
 * Frames whose planes are views of such a Buffer (pitches = the device layout's, i.e.
 * row bytes rounded up to 16) cross PCIe by one DMA per plane in run(), without the
 * library's ring copies.  The memory is released (dts_host_free) after the Buffer is
 * garbage collected; keep it alive until run() settles.  The release runs on a detached
 * thread of its own, never in the finalizer on the event loop: hipHostFree synchronises
 * the device, which would block the loop until every slot's in-flight work had drained
 * (ADVICE r05). */
static void *host_free_thread(void *p)
{
    dts_host_free(p);
    return NULL;
}

static void host_free_cb(napi_env env, void *data, void *hint)
{
    (void)env;
    (void)hint;
    pthread_t t;
    pthread_attr_t a;
    if (pthread_attr_init(&a) == 0) {
        pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
        const int ok = pthread_create(&t, &a, host_free_thread, data) == 0;
        pthread_attr_destroy(&a);
        if (ok) return;
    }
    dts_host_free(data);                /* (no thread: free here rather than leak) */
}

static napi_value js_host_alloc(napi_env env, napi_callback_info info)
{
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    double nb = 0;
    if (argc < 1 || napi_get_value_double(env, argv[0], &nb) != napi_ok || !(nb >= 1) || nb > 1e12)
        return throw_dts(env, DTS_E_INVAL, "hostAlloc(bytes)");
    void *p = NULL;
    const int e = dts_host_alloc((size_t)nb, &p);
    if (e) return throw_dts(env, e, "dts_host_alloc");
    napi_value buf;
    if (napi_create_external_buffer(env, (size_t)nb, p, host_free_cb, NULL, &buf) != napi_ok) {
        dts_host_free(p);
        return throw_dts(env, DTS_E_NOMEM, "hostAlloc: external buffer");
    }
    return buf;
}

/* ---- frameLayout(w, h, fmt) -> {pitch, rows, bytes} --------------------- */
static napi_value js_frame_layout(napi_env env, napi_callback_info info)
{
    size_t argc = 3;
    napi_value argv[3];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t w = 0, h = 0, fmt = 0;
    if (argc < 3) return throw_dts(env, DTS_E_INVAL, "frameLayout(w, h, fmt)");
    napi_get_value_int32(env, argv[0], &w);
    napi_get_value_int32(env, argv[1], &h);
    napi_get_value_int32(env, argv[2], &fmt);
    int64_t pitch[3], rows[3], bytes = 0;
    int e = dts_frame_layout(w, h, fmt, pitch, rows, &bytes);
    if (e) return throw_dts(env, e, "dts_frame_layout");
    napi_value o, pa, ra;
    napi_create_object(env, &o);
    napi_create_array(env, &pa);
    napi_create_array(env, &ra);
    for (uint32_t p = 0; p < 3; ++p) {
        napi_value a, b;
        napi_create_double(env, (double)pitch[p], &a);
        napi_create_double(env, (double)rows[p], &b);
        napi_set_element(env, pa, p, a);
        napi_set_element(env, ra, p, b);
    }
    napi_set_named_property(env, o, "pitch", pa);
    napi_set_named_property(env, o, "rows", ra);
    set_num(env, o, "bytes", (double)bytes);
    return o;
}

/* ---- fpsMap(nbIn, inNum, inDen, outNum, outDen) -> number[] ------------- */
static napi_value js_fps_map(napi_env env, napi_callback_info info)
{
    size_t argc = 5;
    napi_value argv[5];
    NAPI_OK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 5) return throw_dts(env, DTS_E_INVAL, "fpsMap(nbIn, inNum, inDen, outNum, outDen)");
    int64_t nb;
    int32_t a, b, c, d;
    napi_get_value_int64(env, argv[0], &nb);
    napi_get_value_int32(env, argv[1], &a);
    napi_get_value_int32(env, argv[2], &b);
    napi_get_value_int32(env, argv[3], &c);
    napi_get_value_int32(env, argv[4], &d);
    int64_t n = dts_fps_map(nb, a, b, c, d, NULL, 0);
    if (n < 0) return throw_dts(env, (int)n, "dts_fps_map");
    int64_t *idx = (int64_t *)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    if (!idx) return throw_dts(env, DTS_E_NOMEM, "fpsMap");
    dts_fps_map(nb, a, b, c, d, idx, n);
    napi_value arr;
    napi_create_array_with_length(env, (size_t)n, &arr);
    for (int64_t i = 0; i < n; ++i) {
        napi_value v;
        napi_create_double(env, (double)idx[i], &v);
        napi_set_element(env, arr, (uint32_t)i, v);
    }
    free(idx);
    return arr;
}

/* The library this addon loads must have the ABI and struct layouts of the header it was
 * compiled against (dts.h DTS_ABI_VERSION); a mismatch would pass misaligned specs. */
static int abi_mismatch(char *msg, size_t cap)
{
    static const struct { int id; int64_t size; const char *name; } st[] = {
        {DTS_STRUCT_TONEMAP_SPEC, (int64_t)sizeof(dts_tonemap_spec), "dts_tonemap_spec"},
        {DTS_STRUCT_OUTPUT_SPEC, (int64_t)sizeof(dts_output_spec), "dts_output_spec"},
        {DTS_STRUCT_GRAPH_SPEC, (int64_t)sizeof(dts_graph_spec), "dts_graph_spec"},
        {DTS_STRUCT_FRAME, (int64_t)sizeof(dts_frame), "dts_frame"},
        {DTS_STRUCT_DEV_FRAMES, (int64_t)sizeof(dts_dev_frames), "dts_dev_frames"},
        {DTS_STRUCT_QRAW, (int64_t)sizeof(dts_qraw), "dts_qraw"},
        {DTS_STRUCT_QSTAT, (int64_t)sizeof(dts_qstat), "dts_qstat"},
        {DTS_STRUCT_GRAPH_INFO, (int64_t)sizeof(dts_graph_info), "dts_graph_info"},
    };
    const int v = dts_abi_version();
    if (v != DTS_ABI_VERSION) {
        snprintf(msg, cap, "libdts ABI %d, the addon was built for ABI %d", v, DTS_ABI_VERSION);
        return 1;
    }
    for (size_t i = 0; i < sizeof st / sizeof st[0]; ++i) {
        const int64_t n = dts_abi_struct_size(st[i].id);
        if (n != st[i].size) {
            snprintf(msg, cap, "libdts sizeof(%s) = %lld, the addon's %lld", st[i].name, (long long)n,
                     (long long)st[i].size);
            return 1;
        }
    }
    return 0;
}

static napi_value init(napi_env env, napi_value exports)
{
    char msg[160];
    if (abi_mismatch(msg, sizeof msg)) {
        napi_throw_error(env, "DTS_ABI", msg);
        return NULL;
    }
    napi_property_descriptor props[] = {
        {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
        {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_default, NULL},
        {"createContext", NULL, js_create_context, NULL, NULL, NULL, napi_default, NULL},
        {"createGraph", NULL, js_create_graph, NULL, NULL, NULL, napi_default, NULL},
        {"graphInfo", NULL, js_graph_info, NULL, NULL, NULL, napi_default, NULL},
        {"run", NULL, js_run, NULL, NULL, NULL, napi_default, NULL},
        {"synthFrame", NULL, js_synth_frame, NULL, NULL, NULL, napi_default, NULL},
        {"frameLayout", NULL, js_frame_layout, NULL, NULL, NULL, napi_default, NULL},
        {"fpsMap", NULL, js_fps_map, NULL, NULL, NULL, napi_default, NULL},
        {"hostAlloc", NULL, js_host_alloc, NULL, NULL, NULL, napi_default, NULL},
        {"quality", NULL, js_quality, NULL, NULL, NULL, napi_default, NULL},
        {"qstatStream", NULL, js_qstat_stream, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

NAPI_MODULE(dts_napi, init)
