"use strict";
// filtergraph.js -- the ffmpeg `-vf` filtergraph a CPU worker would spawn with (SURVEY.md §8b:
// spawn(ffmpeg-static, [..., "-vf", "scale=1920:1080:flags=bicubic+accurate_rnd+bitexact,format=nv12",
// ...]), index.js:9) read into the settings object ladder.js takes from Jobs.codecSettings
// (database.js:78), so a job row written for an ffmpeg worker runs on the GPU worker unchanged.
//
// One linear chain of the FFmpeg 4.4 filters on the path, with their option syntax (positional
// values in the filter's option order, or key=value, ':'-separated; filters ','-separated):
//   scale     w:h:flags:...  (vf_scale.c: w / width, h / height, flags, in_range, out_range,
//                             param0, param1; sizes -1 / -2 / expressions keep the Jobs row's)
//   format    pix_fmts       (the first of '|'-separated formats the GPU path writes: yuv420p,
//                             nv12, p010le; gbrpf32le / gbrp inside the HDR chain)
//   yadif     mode:parity:deint (vf_yadif.c; the frame-rate modes 0 / 2 -- one output per frame)
//   zscale    t / transfer, npl, p / primaries, m / matrix, r / range (vf_zscale.c: the HDR10 ->
//                             SDR chain's linearise and bt709 steps; npl, and r of a zscale after
//                             the tonemap -- the SDR output's range, tv or pc -- are the ones that
//                             matter)
// In an HDR graph the GPU scales the p010 source before the tone map (dts.h hdr_to_sdr), so a
// scale must come ahead of the zscale / tonemap chain and carry no range conversion.
//   tonemap   tonemap:param:desat:peak (vf_tonemap.c)
//   fps       fps            (vf_fps.c: checked against the Jobs row's framerate)
// Anything else is an error: the worker refuses a graph it would not run exactly.
//
// Node 12 (this image): no `??` / `?.`.

const SCALE_FLAGS = { bilinear: "bilinear", bicubic: "bicubic", neighbor: "neighbor", point: "point",
                      area: "area", gauss: "gauss", sinc: "sinc", lanczos: "lanczos", x: "x", experimental: "x" };
// flags that select libswscale's exact C paths or do not change the arithmetic of the ones above
const SCALE_MODIFIERS = { accurate_rnd: 1, bitexact: 1, full_chroma_int: 0, full_chroma_inp: 0, print_info: 1 };
const OUT_FORMATS = { yuv420p: "yuv420p", nv12: "nv12", p010le: "p010le", p010: "p010le" };
const HDR_INTERMEDIATE = { gbrpf32le: 1, gbrpf32: 1, gbrp: 1, gbrp16le: 1 };
const RANGES = { tv: "tv", mpeg: "tv", limited: "tv", pc: "pc", jpeg: "pc", full: "pc" };
const YADIF_MODES = { send_frame: 0, send_field: 1, send_frame_nospatial: 2, send_field_nospatial: 3 };
const YADIF_PARITY = { tff: "tff", bff: "bff", auto: "tff" };   // auto: the frames carry no field order here
const TONEMAPS = { none: 1, linear: 1, gamma: 1, clip: 1, reinhard: 1, hable: 1, mobius: 1 };

// option order of each filter's positional values (FFmpeg 4.4 AVOption tables)
const ORDER = {
    scale: ["w", "h", "flags"],
    format: ["pix_fmts"],
    yadif: ["mode", "parity", "deint"],
    zscale: ["w", "h"],
    tonemap: ["tonemap", "param", "desat", "peak"],
    fps: ["fps"],
};
const ALIAS = {
    scale: { width: "w", height: "h" },
    zscale: { transfer: "t", primaries: "p", matrix: "m", range: "r", t: "t", p: "p", m: "m", r: "r" },
};

function fail(msg) {
    throw new Error("filtergraph: " + msg);
}

// "name=a:b:k=v" -> {name, opts: {key: value}} with positional values named by ORDER
function parseFilter(text) {
    const eq = text.indexOf("=");
    const name = (eq < 0 ? text : text.slice(0, eq)).trim();
    if (!ORDER[name]) fail("unsupported filter '" + name + "' (the GPU path runs scale, format, yadif, zscale, tonemap, fps)");
    const opts = {};
    if (eq >= 0) {
        const parts = text.slice(eq + 1).split(":");
        let pos = 0;
        parts.forEach(function (p) {
            if (p === "") return;
            const k = p.indexOf("=");
            let key, val;
            if (k < 0) {
                if (pos >= ORDER[name].length) fail(name + ": too many values in '" + text + "'");
                key = ORDER[name][pos++];
                val = p;
            } else {
                key = p.slice(0, k).trim();
                val = p.slice(k + 1);
            }
            const al = ALIAS[name];
            if (al && al[key]) key = al[key];
            opts[key] = val.trim();
        });
    }
    return { name: name, opts: opts };
}

function num(v, what) {
    const m = /^(-?\d+(?:\.\d+)?)(?:\/(\d+(?:\.\d+)?))?$/.exec(String(v));
    if (!m) fail(what + ": not a number: " + v);
    return m[2] ? Number(m[1]) / Number(m[2]) : Number(m[1]);
}

function checkKeys(f, allowed) {
    Object.keys(f.opts).forEach(function (k) {
        if (allowed.indexOf(k) < 0) fail(f.name + ": unsupported option '" + k + "'");
    });
}

// The filtergraph -> the settings object of ladder.js (scale, param, format, inRange, outRange,
// deinterlace, tonemap) plus {size: [w, h] | null, fps: number | null} for the caller to check
// against the Jobs row.
function parseFiltergraph(graph) {
    const s = {};
    let size = null, fps = null, linear = false, npl = null, scaleRange = false, tmOutRange = null;
    const filters = String(graph).split(",").map(function (t) { return t.trim(); }).filter(function (t) { return t; });
    if (!filters.length) fail("empty graph");
    filters.forEach(function (text) {
        const f = parseFilter(text);
        const o = f.opts;
        switch (f.name) {
        case "scale": {
            checkKeys(f, ["w", "h", "flags", "in_range", "out_range", "param0", "param1"]);
            if (s.scale) fail("one scale per graph");
            if (linear || s.tonemap) fail("scale after zscale / tonemap (the GPU graph scales the p010 source first)");
            scaleRange = o.in_range !== undefined || o.out_range !== undefined;
            let method = null;
            String(o.flags || "bicubic").split("+").forEach(function (t) {
                t = t.trim();
                if (!t) return;
                if (SCALE_FLAGS[t]) {
                    if (method) fail("scale: two scale methods in flags=" + o.flags);
                    method = SCALE_FLAGS[t];
                } else if (SCALE_MODIFIERS[t] === undefined) {
                    fail("scale: unsupported flag '" + t + "'");
                } else if (SCALE_MODIFIERS[t] === 0) {
                    fail("scale: flag '" + t + "' changes the chroma path (not on the GPU path)");
                }
            });
            s.scale = method || "bicubic";
            const wh = [o.w, o.h].map(function (v) { return /^\d+$/.test(String(v)) ? Number(v) : null; });
            if (wh[0] !== null && wh[1] !== null) size = wh;
            if (o.param0 !== undefined || o.param1 !== undefined) {
                const dflt = 123456;                         // SWS_PARAM_DEFAULT
                s.param = [o.param0 !== undefined ? num(o.param0, "param0") : dflt,
                           o.param1 !== undefined ? num(o.param1, "param1") : dflt];
            }
            if (o.in_range !== undefined) {
                if (!RANGES[o.in_range]) fail("scale: in_range=" + o.in_range);
                s.inRange = RANGES[o.in_range];
            }
            if (o.out_range !== undefined) {
                if (!RANGES[o.out_range]) fail("scale: out_range=" + o.out_range);
                s.outRange = RANGES[o.out_range];
            }
            break;
        }
        case "format": {
            checkKeys(f, ["pix_fmts"]);
            const fmts = String(o.pix_fmts || "").split("|").map(function (t) { return t.trim(); });
            const out = fmts.filter(function (t) { return OUT_FORMATS[t]; });
            if (out.length) s.format = OUT_FORMATS[out[0]];
            else if (!fmts.every(function (t) { return HDR_INTERMEDIATE[t]; })) fail("format: unsupported " + o.pix_fmts);
            break;
        }
        case "yadif": {
            checkKeys(f, ["mode", "parity", "deint"]);
            let mode = o.mode === undefined ? 0 : (YADIF_MODES[o.mode] !== undefined ? YADIF_MODES[o.mode] : num(o.mode, "yadif mode"));
            const par = o.parity === undefined ? "auto" : String(o.parity);
            const parity = { "-1": "tff", "0": "tff", "1": "bff" }[par] || YADIF_PARITY[par];
            if (!parity) fail("yadif: parity=" + par);
            const deint = o.deint === undefined ? "0" : String(o.deint);
            if (deint !== "0" && deint !== "all") fail("yadif: deint=" + deint + " (every frame is deinterlaced: 0 / all)");
            s.deinterlace = { mode: mode, parity: parity };
            break;
        }
        case "zscale": {
            checkKeys(f, ["t", "npl", "p", "m", "r", "w", "h"]);
            if (o.t === "linear") linear = true;
            if (o.npl !== undefined) npl = num(o.npl, "zscale npl");
            if (o.r !== undefined && s.tonemap) {        // the SDR output's quantisation
                if (!RANGES[o.r]) fail("zscale: r=" + o.r);
                tmOutRange = RANGES[o.r];
            }
            break;
        }
        case "tonemap": {
            checkKeys(f, ["tonemap", "param", "desat", "peak"]);
            const mode = String(o.tonemap || "none");
            if (!TONEMAPS[mode]) fail("tonemap: unsupported curve " + mode);
            const t = { mode: mode };
            ["param", "desat", "peak"].forEach(function (k) { if (o[k] !== undefined) t[k] = num(o[k], "tonemap " + k); });
            s.tonemap = t;
            break;
        }
        case "fps": {
            checkKeys(f, ["fps"]);
            fps = num(o.fps, "fps");
            break;
        }
        }
    });
    if (s.tonemap) {
        if (!linear) fail("tonemap needs the linear light of zscale=t=linear ahead of it");
        if (npl !== null) s.tonemap.npl = npl;
        if (scaleRange) fail("scale: in_range / out_range on the HDR source (the output range is zscale's r=)");
        if (tmOutRange === "pc") s.outRange = "pc";
    }
    return { settings: s, size: size, fps: fps };
}

// Jobs.codecSettings text that is not JSON: an ffmpeg argument string.  The graph of its
// -vf / -filter:v / -filter:V option (or the whole text when it is a bare graph) -> the
// settings object; null when the text carries no filtergraph (plain encoder options).
function graphOfArgs(text) {
    const t = String(text || "").trim();
    if (!t) return null;
    const m = /(?:^|\s)-(?:vf|filter:v|filter:V)\s+("([^"]*)"|'([^']*)'|(\S+))/.exec(t);
    if (m) return m[2] !== undefined ? m[2] : (m[3] !== undefined ? m[3] : m[4]);
    if (!/\s/.test(t) && /^(scale|format|yadif|zscale|tonemap|fps)\b/.test(t)) return t;
    return null;
}

module.exports = { parseFiltergraph: parseFiltergraph, graphOfArgs: graphOfArgs };
