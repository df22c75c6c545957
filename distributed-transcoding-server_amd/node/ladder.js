"use strict";
// ladder.js -- Jobs rows -> one libdts graph spec per source (SURVEY.md §8b/§8f).
//
// In the reference a rendition is one `job_list` row (database.js:61-94:
// width, height, framerate, bitrate, codec, codecSettings, chunks) that points
// at its source (`sourceID`, database.js:66-72).  A CPU worker would run one
// ffmpeg per row and segment; the GPU worker groups the rows that share a
// source into ONE graph with an output per row -- the `split=N` ladder -- so
// the source segment is read from HBM once for all renditions.
//
// Node 12 (this image): no `??` / `?.`.

const filtergraph = require("./filtergraph");

const FMT = { yuv420p: 0, nv12: 1, p010le: 2, p010: 2 };
// libswscale SWS_* flag values (swscale.h), as include/dts.h DTS_SCALE_*
const METHOD = { bilinear: 0x2, bicubic: 0x4, x: 0x8, point: 0x10, neighbor: 0x10, area: 0x20, gauss: 0x80,
                 sinc: 0x100, lanczos: 0x200 };
// vf_tonemap.c enum TonemapAlgorithm (include/dts.h DTS_TM_*)
const TONEMAP = { none: 0, linear: 1, gamma: 2, clip: 3, reinhard: 4, hable: 5, mobius: 6 };
const MAX_OUTPUTS = 4;

// Jobs.codecSettings is free text in the reference (database.js:78).  The GPU
// worker reads an optional JSON object from it with the filtergraph knobs a CPU
// worker would put on its ffmpeg command line:
//   {"scale": "bicubic", "format": "nv12", "param": [b, c], "tonemap": {"mode": "hable", ...},
//    "quality": "psnr" | "ssim" | "both", "qualityRef": "lanczos",
//    "deinterlace": "yadif" | {"mode": 0 | 2, "parity": "tff" | "bff"},
//    "inRange": "tv" | "pc", "outRange": "tv" | "pc"}
// inRange / outRange: `scale=in_range=R:out_range=R` (libswscale range conversion on
// the horizontally scaled lines; dts_graph_spec.range).
// deinterlace: `yadif=MODE:PARITY` ahead of the scale (frame-rate modes; vf_yadif.c),
// run on the GPU in the same graph (dts_graph_spec.deint).
// quality: `[rendition][reference]psnr` / `ssim` per segment against a reference
// rendition of the same size -- the source scaled with `qualityRef` (default
// lanczos) -- reported in JobChunks.result.quality.
// Or (round 6) the ffmpeg arguments / filtergraph a CPU worker would run with -- e.g.
//   -vf scale=1920:1080:flags=bicubic+accurate_rnd+bitexact,format=nv12 -preset fast
// -- read by filtergraph.js into the same object (its scale size and fps, when given, must agree
// with the row's width / height / framerate).
function parseSettings(text) {
    if (!text) return {};
    let o = null;
    try {
        o = JSON.parse(text);
    } catch (e) {
        const g = filtergraph.graphOfArgs(text);
        if (g === null) return {};        // plain encoder options: nothing for the filtergraph
        const r = filtergraph.parseFiltergraph(g);
        const st = r.settings;
        if (r.size) st._size = r.size;
        if (r.fps) st._fps = r.fps;
        return st;
    }
    return o && typeof o === "object" ? o : {};
}

function outputOf(job) {
    const s = parseSettings(job.codecSettings);
    const method = METHOD[String(s.scale || "bicubic").toLowerCase()];
    if (method === undefined) throw new Error("job " + job.id + ": unknown scale method " + s.scale);
    const fmt = FMT[String(s.format || "nv12").toLowerCase()];
    if (fmt === undefined) throw new Error("job " + job.id + ": unknown output format " + s.format);
    const o = { w: job.width | 0, h: job.height | 0, fmt: fmt, method: method };
    if (s._size && (s._size[0] !== o.w || s._size[1] !== o.h))
        throw new Error("job " + job.id + ": the graph scales to " + s._size.join("x") + ", the row asks " + o.w + "x" + o.h);
    if (s._fps && job.framerate && Math.abs(s._fps - job.framerate) > 1e-3 * job.framerate)
        throw new Error("job " + job.id + ": the graph's fps=" + s._fps + " is not the row's framerate " + job.framerate);
    if (Array.isArray(s.param)) o.param = s.param.slice(0, 2);
    return o;
}

const QUALITY = { psnr: 1, ssim: 2, both: 3, true: 3 };
const RANGE = { tv: 0, mpeg: 0, limited: 0, pc: 1, jpeg: 1, full: 1 };

// {src, dst}: DTS_RANGE_* of the source and of the renditions
function rangeOf(job) {
    const s = parseSettings(job.codecSettings);
    const r = function (v, what) {
        if (v === undefined) return 0;
        const x = RANGE[String(v).toLowerCase()];
        if (x === undefined) throw new Error("job " + job.id + ": unknown " + what + " " + v);
        return x;
    };
    return { src: r(s.inRange, "inRange"), dst: r(s.outRange, "outRange") };
}

// {mode, tff} or null
function deintOf(job) {
    const s = parseSettings(job.codecSettings);
    if (!s.deinterlace) return null;
    const d = typeof s.deinterlace === "object" ? s.deinterlace : {};
    if (typeof s.deinterlace === "string" && s.deinterlace.toLowerCase() !== "yadif")
        throw new Error("job " + job.id + ": unknown deinterlacer " + s.deinterlace);
    const mode = d.mode === undefined ? 0 : d.mode | 0;
    if (mode !== 0 && mode !== 2) throw new Error("job " + job.id + ": yadif mode " + mode + " (frame-rate modes 0 / 2 only)");
    const parity = String(d.parity || "tff").toLowerCase();
    if (parity !== "tff" && parity !== "bff") throw new Error("job " + job.id + ": yadif parity " + d.parity);
    return { mode: mode, tff: parity === "tff" ? 1 : 0 };
}

// {mode: DTS_Q_*, ref: DTS_SCALE_*} or null
function qualityOf(job) {
    const s = parseSettings(job.codecSettings);
    if (!s.quality) return null;
    const mode = QUALITY[String(s.quality).toLowerCase()];
    if (mode === undefined) throw new Error("job " + job.id + ": unknown quality " + s.quality);
    const ref = METHOD[String(s.qualityRef || "lanczos").toLowerCase()];
    if (ref === undefined) throw new Error("job " + job.id + ": unknown qualityRef " + s.qualityRef);
    return { mode: mode, ref: ref };
}

function tonemapOf(job) {
    const s = parseSettings(job.codecSettings);
    if (!s.tonemap) return null;
    const t = typeof s.tonemap === "string" ? { mode: s.tonemap } : s.tonemap;
    const mode = TONEMAP[String(t.mode || "hable").toLowerCase()];
    if (mode === undefined) throw new Error("job " + job.id + ": unknown tonemap " + t.mode);
    const r = { mode: mode };
    ["param", "desat", "peak", "npl"].forEach(function (k) { if (typeof t[k] === "number") r[k] = t[k]; });
    return r;
}

// Group rendition rows by source.  src: {w, h, fmt, fps: [num, den]} per sourceID.
// Returns [{sourceID, jobs: [row...], spec}] with at most MAX_OUTPUTS rows per graph
// (a larger ladder is split into several graphs over the same source).
function planLadders(jobs, sources) {
    const bySrc = new Map();                   // one ladder per (source, output frame rate)
    jobs.forEach(function (j) {
        const key = j.sourceID + "@" + (j.framerate || 0);
        if (!bySrc.has(key)) bySrc.set(key, []);
        bySrc.get(key).push(j);
    });
    const plans = [];
    bySrc.forEach(function (rows) {
        const sid = rows[0].sourceID;
        const src = sources[sid];
        if (!src) throw new Error("source " + sid + " has no stream info");
        rows.sort(function (a, b) { return b.width * b.height - a.width * a.height || a.id - b.id; });
        for (let i = 0; i < rows.length; i += MAX_OUTPUTS) {
            const part = rows.slice(i, i + MAX_OUTPUTS);
            const tm = tonemapOf(part[0]);
            part.forEach(function (r) {
                if (JSON.stringify(tonemapOf(r)) !== JSON.stringify(tm))
                    throw new Error("jobs " + part[0].id + "/" + r.id + ": one graph needs one tonemap setting");
            });
            const spec = { src: { w: src.w, h: src.h, fmt: src.fmt }, outputs: part.map(outputOf), quality: 0,
                           maxBatch: 32 };
            if (tm) spec.tonemap = tm;
            const di = deintOf(part[0]);
            part.forEach(function (r) {
                if (JSON.stringify(deintOf(r)) !== JSON.stringify(di))
                    throw new Error("jobs " + part[0].id + "/" + r.id + ": one graph needs one deinterlace setting");
            });
            if (di) spec.deint = di;
            const rg = rangeOf(part[0]);
            part.forEach(function (r) {
                if (JSON.stringify(rangeOf(r)) !== JSON.stringify(rg))
                    throw new Error("jobs " + part[0].id + "/" + r.id + ": one graph needs one range setting");
            });
            if (rg.src || rg.dst) { spec.srcRange = rg.src; spec.dstRange = rg.dst; }
            // per-rendition quality (codecSettings.quality): each requesting row against its
            // reference rendition, made and scored inside the same graph on the GPU
            // (dts_output_spec.quality / qref_method): no rendition crosses PCIe twice
            const q = part.map(qualityOf);
            const quality = q.some(function (x) { return x; }) ? { rows: q.map(function (x) { return x ? x.mode : 0; }) } : null;
            if (quality) spec.outputs.forEach(function (o, k) {
                if (q[k]) {
                    o.quality = q[k].mode;
                    o.qrefMethod = q[k].ref;
                }
            });
            if (quality && tm) throw new Error("job " + part[0].id + ": quality with tonemap is not supported");
            plans.push({ sourceID: sid, framerate: part[0].framerate || 0, jobs: part, spec: spec, quality: quality });
        }
    });
    return plans;
}

// Jobs.framerate (database.js:75) vs the source rate: the vf_fps (round=near)
// input frame of every output frame of a segment of `n` source frames.
function rateOf(fps) {
    return Number.isInteger(fps) ? [fps, 1] : [Math.round(fps * 1001), 1001];      // 29.97 -> 30000/1001
}

function fpsFrames(addon, n, srcFps, outFps) {
    if (!outFps || !srcFps) return null;
    const r = rateOf(outFps);
    if (r[0] * srcFps[1] === srcFps[0] * r[1]) return null;                       // same rate: identity
    return addon.fpsMap(n, srcFps[0], srcFps[1], r[0], r[1]);
}

// A segment's summed quality record from per-frame statistics (the addon's qstat
// objects): {frames, sse: [y, u, v], ssimSum: [y, u, v]} -- the running sums vf_psnr /
// vf_ssim keep (SSE exact; SSIM as the per-plane window sums), which add across segments.
// The per-plane window sums come back as ssim x windows (exact to the f64 rounding of the
// library's one division); a plane smaller than 8x8 has no SSIM window (vf_ssim scores none)
// and adds 0 (ADVICE r03: its NaN / negative count poisoned the job's sums).
function ssimWindows(pw, ph) {
    return Math.max(0, (pw >> 2) - 1) * Math.max(0, (ph >> 2) - 1);
}

function rawQuality(stats, w, h) {
    const pw = [w, (w + 1) >> 1, (w + 1) >> 1], ph = [h, (h + 1) >> 1, (h + 1) >> 1];
    const nw = [0, 1, 2].map(function (c) { return ssimWindows(pw[c], ph[c]); });
    const comp = ["y", "u", "v"], raw = { frames: stats.length, sse: [0, 0, 0], ssimSum: [0, 0, 0] };
    stats.forEach(function (q) {
        comp.forEach(function (c, i) {
            raw.sse[i] += q.sse[c];
            if (nw[i] > 0) raw.ssimSum[i] += q.ssim[c] * nw[i];
        });
    });
    return raw;
}

function addRaw(list) {
    const r = { frames: 0, sse: [0, 0, 0], ssimSum: [0, 0, 0] };
    list.forEach(function (x) {
        r.frames += x.frames;
        for (let i = 0; i < 3; ++i) {
            r.sse[i] += x.sse[i];
            r.ssimSum[i] += x.ssimSum[i];
        }
    });
    return r;
}

// vf_psnr / vf_ssim end-of-stream averages of a summed record: PSNR from the mean MSE
// (per plane and area-weighted overall), mean SSIM (as dts_qstat_stream)
function summarizeRaw(raw, w, h) {
    const pw = [w, (w + 1) >> 1, (w + 1) >> 1], ph = [h, (h + 1) >> 1, (h + 1) >> 1];
    const area = pw[0] * ph[0] + pw[1] * ph[1] + pw[2] * ph[2], n = raw.frames;
    const psnr = function (m) { return m === 0 ? "inf" : 10 * Math.log10(255 * 255 / m); };   // JSON has no Infinity
    const comp = ["y", "u", "v"], r = { frames: n, psnr: {}, ssim: {} };
    let mseAvg = 0, ssimAll = 0;
    let noWindows = false;
    comp.forEach(function (c, i) {
        const mse = raw.sse[i] / (n * pw[i] * ph[i]);
        const nw = ssimWindows(pw[i], ph[i]);
        r.psnr[c] = psnr(mse);
        r.ssim[c] = nw > 0 ? raw.ssimSum[i] / (n * nw) : null;      // no 8x8 window: no SSIM (not NaN)
        noWindows = noWindows || nw <= 0;
        mseAvg += mse * pw[i] * ph[i] / area;
        if (nw > 0) ssimAll += r.ssim[c] * pw[i] * ph[i] / area;
    });
    r.psnr.avg = psnr(mseAvg);
    r.ssim.all = noWindows ? null : ssimAll;
    return r;
}

// the same from the addon's qstatStream() object
function summaryOfStat(q, raw) {
    const f = function (x) { return x === Infinity ? "inf" : x; };
    const g = function (x) { return typeof x === "number" && isFinite(x) ? x : null; };   // 0/0 windows -> null
    return { frames: raw.frames, psnr: { y: f(q.psnr.y), u: f(q.psnr.u), v: f(q.psnr.v), avg: f(q.psnrAvg) },
             ssim: { y: g(q.ssim.y), u: g(q.ssim.u), v: g(q.ssim.v), all: g(q.ssimAll) } };
}

// Segment summary of per-frame statistics, as vf_psnr / vf_ssim print at the end of
// a stream: PSNR from the mean MSE (per plane and area-weighted overall), mean SSIM.
function summarizeQuality(stats, w, h) {
    const pw = [w, (w + 1) >> 1, (w + 1) >> 1], ph = [h, (h + 1) >> 1, (h + 1) >> 1];
    const area = pw[0] * ph[0] + pw[1] * ph[1] + pw[2] * ph[2];
    const comp = ["y", "u", "v"], n = stats.length;
    const mse = [0, 0, 0], ssim = [0, 0, 0];
    let ssimAll = 0;
    stats.forEach(function (q) {
        comp.forEach(function (c, i) {
            mse[i] += q.sse[c] / (pw[i] * ph[i]) / n;
            ssim[i] += q.ssim[c] / n;
        });
        ssimAll += q.ssimAll / n;
    });
    const psnr = function (m) { return m === 0 ? Infinity : 10 * Math.log10(255 * 255 / m); };
    const mseAvg = mse.reduce(function (a, m, i) { return a + m * pw[i] * ph[i] / area; }, 0);
    const r = { frames: n, psnr: {}, ssim: {} };
    comp.forEach(function (c, i) {
        r.psnr[c] = psnr(mse[i]);
        r.ssim[c] = ssim[i];
    });
    r.psnr.avg = psnr(mseAvg);
    r.ssim.all = ssimAll;
    return r;
}

module.exports = { FMT: FMT, METHOD: METHOD, TONEMAP: TONEMAP, MAX_OUTPUTS: MAX_OUTPUTS, parseSettings: parseSettings,
                   outputOf: outputOf, tonemapOf: tonemapOf, qualityOf: qualityOf, deintOf: deintOf, rangeOf: rangeOf,
                   planLadders: planLadders,
                   rateOf: rateOf, fpsFrames: fpsFrames, summarizeQuality: summarizeQuality, rawQuality: rawQuality,
                   addRaw: addRaw, summarizeRaw: summarizeRaw, summaryOfStat: summaryOfStat };
