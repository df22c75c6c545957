"use strict";
// CPU test of the Node GPU worker's scheduler and JobChunks state machine
// against a stand-in addon (same interface as dts_napi.node, no device).
// Run by tests/test_node.py; exits non-zero on the first failed check.
const assert = require("assert");
const path = require("path");
const NODE = path.join(__dirname, "..", "..", "distributed-transcoding-server_amd", "node");
const fs = require("fs");
const os = require("os");
const { GpuSegmentScheduler } = require(path.join(NODE, "scheduler"));
const ladder = require(path.join(NODE, "ladder"));
const y4m = require(path.join(NODE, "y4m"));
const assemble = require(path.join(NODE, "assemble"));

function fakeAddon(opts) {
    opts = opts || {};
    const stats = { graphs: 0, runs: 0, byDev: {} };
    return {
        stats: stats,
        deviceCount: function () { return opts.devices === undefined ? 4 : opts.devices; },
        createContext: function (dev) { return { dev: dev }; },
        createGraph: function (ctx, spec) { stats.graphs++; return { ctx: ctx, spec: spec }; },
        synthFrame: function (w, h, fmt, pat, seed, idx, f) { f.data[0][0] = idx & 255; },
        // vf_fps round=near for a constant-rate input (oracle/swscale_ref.c orc_fps_map)
        fpsMap: function (n, a, b, c, d) {
            const B = b * c, C = a * d, near = function (x) { return Math.floor((x * B + Math.floor(C / 2)) / C); };
            const nout = near(n), out = [];
            let i = 0;
            for (let k = 0; k < nout; k++) { while (i + 1 < n && near(i + 1) <= k) i++; out.push(i); }
            return out;
        },
        // stand-in vf_psnr: identical frames -> sse 0, otherwise 1 per byte of the first plane differing
        quality: function (ctx, w, h, fmt, a, b) {
            stats.quality = (stats.quality || 0) + 1;
            return Promise.resolve(a.map(function (fa, i) {
                const d = fa.data[0][0] === b[i].data[0][0] ? 0 : 1;
                return { sse: { y: d, u: 0, v: 0 }, psnr: {}, ssim: { y: 1 - d / 2, u: 1, v: 1 }, ssimAll: 1 - d / 4 };
            }));
        },
        run: function (g, src, dst, q) {
            stats.runs++;
            stats.byDev[g.ctx.dev] = (stats.byDev[g.ctx.dev] || 0) + 1;
            const cf = g.spec.deint ? 1 : 0;             // deint: one context frame each side
            stats.srcFirst = src.map(function (f) { return f.data[0][0]; });
            assert.strictEqual(dst.length, (src.length - 2 * cf) * g.spec.outputs.length);
            return new Promise(function (resolve, reject) {
                setTimeout(function () {
                    if (opts.fail && opts.fail(g.ctx.dev, stats.runs)) return reject(new Error("dts run: HIP error (-1000)"));
                    dst.forEach(function (f, i) { f.data[0][0] = src[cf + Math.floor(i / g.spec.outputs.length)].data[0][0]; });
                    // rendition quality: stats[f][k] (stand-in vf_psnr: odd frames differ by one luma level)
                    const rq = g.spec.outputs.some(function (o) { return o.quality; });
                    if (!rq) return resolve(null);
                    stats.quality = (stats.quality || 0) + 1;
                    resolve(Array.from({ length: src.length - 2 * cf }, function (_, fi) {
                        return g.spec.outputs.map(function (o) {
                            if (!o.quality) return null;
                            const d = src[cf + fi].data[0][0] & 1;
                            return { sse: { y: d, u: 0, v: 0 }, psnr: {}, ssim: { y: 1 - d / 2, u: 1, v: 1 }, ssimAll: 1 - d / 4 };
                        });
                    }));
                }, opts.delay === undefined ? 2 : opts.delay);
            });
        },
    };
}

function jobSet(nseg, fps) {
    const jobs = [
        { id: 11, sourceID: 7, width: 192, height: 108, framerate: fps || 60, codecSettings: null },
        { id: 12, sourceID: 7, width: 128, height: 72, framerate: fps || 60, codecSettings: '{"scale": "lanczos"}' },
        { id: 13, sourceID: 7, width: 86, height: 48, framerate: fps || 60, codecSettings: "-preset slow" },
    ];
    const chunks = [];
    let id = 1;
    jobs.forEach(function (j) {
        for (let o = 0; o < nseg; o++) chunks.push({ id: id++, mainJob: j.id, chunkOffset: o, assignedTo: null, status: null, result: null });
    });
    return { jobs: jobs, chunks: chunks, sources: { 7: { w: 384, h: 216, fmt: 0, fps: [60, 1] } } };
}

async function testAllDoneAndBalanced() {
    const addon = fakeAddon({ devices: 4 });
    const js = jobSet(16);
    const seen = {};
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 42, segmentFrames: 6,
        onUpdate: function (row, f) { (seen[row.id] = seen[row.id] || []).push(f.status); } });
    const sum = await s.runJobs(js.jobs, js.chunks, js.sources);
    assert.strictEqual(sum.segments, 16);
    js.chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done");
        assert.strictEqual(c.assignedTo, 42);
        const r = JSON.parse(c.result);
        assert.strictEqual(r.frames, 6);
        assert.ok(r.gpu >= 0 && r.gpu < 4);
        assert.strictEqual(r.sha1.length, 40);
        assert.deepStrictEqual(seen[c.id], ["assigned", "processing", "done"]);
    });
    // one graph per (ladder, GPU): the 3 renditions share one launch per segment
    assert.ok(addon.stats.graphs <= 4, "graphs " + addon.stats.graphs);
    assert.strictEqual(addon.stats.runs, 16);
    sum.gpus.forEach(function (g) { assert.ok(g.segments >= 2, "GPU " + g.device + " got " + g.segments); });
    const r12 = JSON.parse(js.chunks.find(function (c) { return c.mainJob === 12; }).result);
    assert.strictEqual(r12.width, 128);
    assert.strictEqual(r12.bytes, 6 * (128 * 72 * 3 / 2));
}

async function testRetryOnAnotherGpu() {
    const addon = fakeAddon({ devices: 3, fail: function (dev) { return dev === 1; } });
    const js = jobSet(9);
    let retries = 0;
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 1, segmentFrames: 2 });
    s.on("retry", function () { retries++; });
    const sum = await s.runJobs(js.jobs, js.chunks, js.sources);
    js.chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done");
        assert.notStrictEqual(JSON.parse(c.result).gpu, 1);
    });
    assert.ok(retries > 0);
    assert.ok(sum.gpus[1].failures > 0 && sum.gpus[1].segments === 0);
}

async function testGiveUpAfterRetries() {
    const addon = fakeAddon({ devices: 2, fail: function () { return true; } });
    const js = jobSet(3);
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 1, segmentFrames: 2, maxRetries: 2 });
    await s.runJobs(js.jobs, js.chunks, js.sources);
    js.chunks.forEach(function (c) {
        assert.strictEqual(c.status, "failed");
        const r = JSON.parse(c.result);
        assert.strictEqual(r.tries, 3);
        assert.ok(/HIP/.test(r.error));
    });
    assert.strictEqual(addon.stats.runs, 9);
}

async function testFpsMapAndResume() {
    const addon = fakeAddon({ devices: 2 });
    const js = jobSet(4, 30);                      // 60 fps source -> 30 fps renditions
    js.chunks[0].status = "done";                  // already finished: not re-run
    js.chunks[0].result = "{}";
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 1, segmentFrames: 10 });
    await s.runJobs(js.jobs, js.chunks, js.sources);
    js.chunks.forEach(function (c, i) {
        assert.strictEqual(c.status, "done");
        if (i > 0) assert.strictEqual(JSON.parse(c.result).frames, 5);
    });
    assert.strictEqual(js.chunks[0].result, "{}");
    assert.deepStrictEqual(ladder.fpsFrames(addon, 10, [60, 1], 30), [0, 2, 4, 6, 8]);
    assert.strictEqual(ladder.fpsFrames(addon, 10, [60, 1], 60), null);
}

function testLadderPlanning() {
    const js = jobSet(1);
    const plans = ladder.planLadders(js.jobs, js.sources);
    assert.strictEqual(plans.length, 1);
    assert.deepStrictEqual(plans[0].spec.outputs.map(function (o) { return o.method; }), [0x4, 0x200, 0x4]);
    const many = [];
    for (let i = 0; i < 6; i++) many.push({ id: i, sourceID: 7, width: 64 + 2 * i, height: 36, framerate: 60 });
    assert.strictEqual(ladder.planLadders(many, js.sources).length, 2);      // > 4 renditions: two graphs
    const hdr = [{ id: 1, sourceID: 8, width: 1920, height: 1080, codecSettings: '{"tonemap": {"mode": "hable", "desat": 0}, "format": "yuv420p"}' }];
    const p = ladder.planLadders(hdr, { 8: { w: 3840, h: 2160, fmt: 2 } });
    assert.deepStrictEqual(p[0].spec.tonemap, { mode: 5, desat: 0 });
    assert.strictEqual(p[0].spec.outputs[0].fmt, 0);
    assert.throws(function () { ladder.planLadders([{ id: 1, sourceID: 9, width: 2, height: 2 }], {}); });
    assert.throws(function () { ladder.outputOf({ id: 1, width: 2, height: 2, codecSettings: '{"scale": "nope"}' }); });
    assert.deepStrictEqual(ladder.rateOf(29.97), [30000, 1001]);
}

async function testThrowingUpdateDoesNotHang() {
    // a failing JobChunks.update (onUpdate throws) must not leave a slot busy or hang runJobs
    const addon = fakeAddon({ devices: 2 });
    const js = jobSet(5);
    let errors = 0;
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 1, segmentFrames: 2,
        onUpdate: function (row, f) { if (f.status === "done" && row.id % 2) throw new Error("db down"); } });
    s.on("updateError", function () { errors++; });
    const sum = await s.runJobs(js.jobs, js.chunks, js.sources);
    assert.strictEqual(sum.segments, 5);
    assert.strictEqual(addon.stats.runs, 5);
    assert.ok(errors > 0);
    js.chunks.forEach(function (c) { assert.strictEqual(c.status, "done"); });
}

function tmpdir() {
    return fs.mkdtempSync(path.join(os.tmpdir(), "dts-node-"));
}

function testY4MRoundTrip() {
    const d = tmpdir(), p = path.join(d, "a.y4m");
    const w = 37, h = 23, cw = 19, ch = 12;
    y4m.writeFile(p, w, h, [30000, 1001], 5, function (i) {
        const f = { data: [Buffer.alloc(w * h, i), Buffer.alloc(cw * ch, 100 + i), Buffer.alloc(cw * ch, 200 + i)],
                    pitch: [w, cw, cw] };
        f.data[0][3] = 7;
        return f;
    });
    const r = new y4m.Y4MReader(p);
    assert.deepStrictEqual([r.hdr.w, r.hdr.h, r.frames], [w, h, 5]);
    assert.deepStrictEqual(r.hdr.fps, [30000, 1001]);
    const f3 = r.read(3);
    assert.strictEqual(f3.data[0][0], 3);
    assert.strictEqual(f3.data[0][3], 7);
    assert.strictEqual(f3.data[1][cw * ch - 1], 103);
    assert.strictEqual(f3.data[2][0], 203);
    assert.strictEqual(r.read(5), null);                                  // past the end
    r.close();
    // nv12 rendition -> planar Y4M record (de-interleaved chroma)
    const nv = { data: [Buffer.alloc(w * h, 1), Buffer.alloc(ch * 2 * cw), null], pitch: [w, 2 * cw, 0] };
    for (let i = 0; i < cw * ch; ++i) { nv.data[1][2 * i] = 10; nv.data[1][2 * i + 1] = 20; }
    const rec = y4m.frameRecord(nv, w, h, 1);
    assert.strictEqual(rec.length, 6 + y4m.frameBytes(w, h));
    assert.strictEqual(rec[6 + w * h], 10);
    assert.strictEqual(rec[6 + w * h + cw * ch], 20);
    assert.throws(function () { y4m.parseHeader(Buffer.from("YUV4MPEG2 W4 H4 C444\n")); }, /4:2:0/);
}

function testAssembleBlocks() {
    const d = tmpdir();
    const sizes = [700000, 1048576, 5, 1500000];
    const files = sizes.map(function (n, i) {
        const p = path.join(d, "s" + i);
        const b = Buffer.alloc(n);
        for (let k = 0; k < n; ++k) b[k] = (k * 7 + i) & 255;
        fs.writeFileSync(p, b);
        return p;
    });
    const a = assemble.assembleFiles(files, path.join(d, "blocks"));
    const total = sizes.reduce(function (x, y) { return x + y; }, 0);
    assert.strictEqual(a.size, total);
    assert.strictEqual(a.chunk.length, Math.ceil(total / 1048576));
    const whole = Buffer.concat(files.map(function (f) { return fs.readFileSync(f); }));
    // index.js block arithmetic: any byte range reads back from the blocks
    [[0, 10], [1048570, 1048600], [total - 3, total + 100], [700000, 1748576]].forEach(function (rg) {
        const got = assemble.readRange(a, path.join(d, "blocks"), rg[0], rg[1]);
        assert.ok(got.equals(whole.slice(rg[0], Math.min(rg[1], total - 1) + 1)), "range " + rg);
    });
}

function testQualitySummary() {
    // two frames, luma MSE 1 and 3 -> mean 2; chroma exact -> inf; area-weighted average
    const w = 4, h = 4;
    const st = [1, 3].map(function (m) {
        return { sse: { y: m * 16, u: 0, v: 0 }, ssim: { y: 0.5, u: 1, v: 1 }, ssimAll: 0.75 };
    });
    const r = ladder.summarizeQuality(st, w, h);
    assert.ok(Math.abs(r.psnr.y - 10 * Math.log10(255 * 255 / 2)) < 1e-9);
    assert.strictEqual(r.psnr.u, Infinity);
    assert.ok(Math.abs(r.psnr.avg - 10 * Math.log10(255 * 255 / (2 * 16 / 24))) < 1e-9);
    assert.strictEqual(r.ssim.all, 0.75);
    assert.deepStrictEqual(ladder.qualityOf({ id: 1, codecSettings: '{"quality": "ssim"}' }), { mode: 2, ref: 0x200 });
    assert.strictEqual(ladder.qualityOf({ id: 1, codecSettings: "-crf 20" }), null);
}

async function testY4MJobAssembled() {
    // a Y4M source, renditions written per segment, quality on one row, every job assembled
    const d = tmpdir(), src = path.join(d, "src.y4m");
    const W = 64, H = 36;
    y4m.writeFile(src, W, H, [60, 1], 14, function (i) {
        return { data: [Buffer.alloc(W * H, i), Buffer.alloc(32 * 18, 128), Buffer.alloc(32 * 18, 128)], pitch: [W, 32, 32] };
    });
    const addon = fakeAddon({ devices: 2 });
    const jobs = [{ id: 21, sourceID: 3, width: 32, height: 18, framerate: 60, chunks: 3, codecSettings: '{"quality": "both"}' },
                  { id: 22, sourceID: 3, width: 16, height: 10, framerate: 60, chunks: 3, codecSettings: null }];
    const chunks = [];
    let id = 1;
    jobs.forEach(function (j) { for (let o = 0; o < 3; o++) chunks.push({ id: id++, mainJob: j.id, chunkOffset: o, status: null }); });
    const updates = [];
    const s = new GpuSegmentScheduler({ addon: addon, segmentFrames: 6, outDir: d,
                                        onJobUpdate: function (j, f) { updates.push([j.id, f.finished]); } });
    await s.runJobs(jobs, chunks, { 3: { path: src } });
    chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done");
        const r = JSON.parse(c.result);
        assert.strictEqual(r.frames, c.chunkOffset < 2 ? 6 : 2);             // 14 frames: 6 + 6 + 2
        assert.ok(r.readMs >= 0 && r.gpuMs >= 0 && r.writeMs >= 0);
        assert.strictEqual(fs.statSync(r.file).size, r.fileBytes);
        if (c.mainJob === 21) assert.ok(r.quality && r.quality.psnr && r.quality.ssim);
        else assert.strictEqual(r.quality, undefined);
        // the rendition file reads back: first luma byte = the source frame index (stand-in ladder)
        const rd = new y4m.Y4MReader(r.file);
        assert.strictEqual(rd.frames, r.frames);
        assert.strictEqual(rd.read(0).data[0][0], 6 * c.chunkOffset);
        rd.close();
    });
    jobs.forEach(function (j) {
        assert.strictEqual(j.finished, true);
        const a = JSON.parse(j.assembledData);
        const files = chunks.filter(function (c) { return c.mainJob === j.id; })
            .sort(function (x, y) { return x.chunkOffset - y.chunkOffset; })
            .map(function (c) { return JSON.parse(c.result).file; });
        // one YUV4MPEG2 stream: the first segment's header, every segment's FRAME records
        const hb = y4m.headerBytes(files[0]);
        const total = files.reduce(function (x, f) { return x + fs.statSync(f).size; }, 0) - (files.length - 1) * hb;
        assert.strictEqual(a.size, total);
        assert.strictEqual(a.chunk.length, Math.ceil(total / 1048576));
        const whole = path.join(d, "whole" + j.id + ".y4m");
        fs.writeFileSync(whole, assemble.readRange(a, path.join(d, "blocks"), 0, a.size - 1));
        const rd = new y4m.Y4MReader(whole);
        assert.strictEqual(rd.frames, 14);
        for (let i = 0; i < 14; ++i) assert.strictEqual(rd.read(i).data[0][0], i);
        rd.close();
    });
    assert.deepStrictEqual(updates.sort(), [[21, true], [22, true]]);
    // job-level quality on the row that asked for it: the summed segment records
    const q21 = JSON.parse(jobs[0].quality);
    assert.strictEqual(q21.frames, 14);
    assert.strictEqual(q21.segments, 3);
    // stand-in: odd source frames (7 of 14) carry luma SSE 1 over 32x18 -> mean MSE 0.5 / 576
    assert.ok(Math.abs(q21.psnr.y - 10 * Math.log10(255 * 255 / (0.5 / 576))) < 1e-9, JSON.stringify(q21));
    assert.ok(q21.ssim.y < 1 && q21.ssim.u === 1, JSON.stringify(q21));
    assert.strictEqual(jobs[1].quality, undefined);
    assert.ok(addon.stats.quality >= 3);
    assert.strictEqual(addon.stats.graphs, 2);          // one graph per GPU: the references are inside it
}

async function testDeinterlaceWithRateChange() {
    // yadif + 60 -> 30 fps over a 14-frame Y4M source in segments of 6: the graph sees the
    // contiguous segment plus a context frame each side (clamped at the ends), and the
    // vf_fps pick (every other frame) is applied to its outputs
    const d = tmpdir(), src = path.join(d, "src.y4m");
    y4m.writeFile(src, 32, 18, [60, 1], 14, function (i) {
        return { data: [Buffer.alloc(32 * 18, i), Buffer.alloc(16 * 9, 128), Buffer.alloc(16 * 9, 128)], pitch: [32, 16, 16] };
    });
    const addon = fakeAddon({ devices: 1 });
    const jobs = [{ id: 41, sourceID: 9, width: 16, height: 10, framerate: 30,
                    codecSettings: '{"deinterlace": {"mode": 2, "parity": "bff"}}' }];
    const chunks = [0, 1, 2].map(function (o) { return { id: 50 + o, mainJob: 41, chunkOffset: o, status: null }; });
    const firsts = [];
    addon.run = (function (run) {
        return function (g, s, dst, q) {
            assert.deepStrictEqual(g.spec.deint, { mode: 2, tff: 0 });
            firsts.push(s.map(function (f) { return f.data[0][0]; }));
            return run(g, s, dst, q);
        };
    })(addon.run);
    const s = new GpuSegmentScheduler({ addon: addon, segmentFrames: 6, outDir: d });
    await s.runJobs(jobs, chunks, { 9: { path: src } });
    firsts.sort(function (a, b) { return a[1] - b[1]; });
    assert.deepStrictEqual(firsts, [[0, 0, 1, 2, 3, 4, 5, 6], [5, 6, 7, 8, 9, 10, 11, 12], [11, 12, 13, 13]]);
    chunks.forEach(function (c) {
        const r = JSON.parse(c.result);
        const rd = new y4m.Y4MReader(r.file);
        const got = Array.from({ length: rd.frames }, function (_, i) { return rd.read(i).data[0][0]; });
        assert.strictEqual(jobs[0].finished, undefined);            // Jobs.chunks unknown: not assembled
        rd.close();
        const want = { 0: [0, 2, 4], 1: [6, 8, 10], 2: [12] }[c.chunkOffset];
        assert.deepStrictEqual(got, want, "chunk " + c.chunkOffset);
    });
    assert.throws(function () {
        ladder.planLadders([{ id: 1, sourceID: 1, width: 8, height: 8, codecSettings: '{"deinterlace": {"mode": 1}}' }],
                           { 1: { w: 16, h: 16, fmt: 0 } });
    }, /frame-rate modes/);
}

async function testY4M10BitAndHeaders() {
    // C420p10 <-> p010 host frames; a long header line; FRAME parameters on a stream
    const d = tmpdir(), p = path.join(d, "p10.y4m");
    const w = 6, h = 4, cw = 3, ch = 2;
    const f = { data: [Buffer.alloc(2 * w * h), Buffer.alloc(4 * cw * ch), null], pitch: [2 * w, 4 * cw, 0] };
    for (let i = 0; i < w * h; ++i) f.data[0].writeUInt16LE(((i * 37) & 1023) << 6, 2 * i);
    for (let i = 0; i < cw * ch; ++i) {
        f.data[1].writeUInt16LE(((i * 91 + 5) & 1023) << 6, 4 * i);
        f.data[1].writeUInt16LE(((i * 13 + 700) & 1023) << 6, 4 * i + 2);
    }
    const wr = new y4m.Y4MWriter(p, w, h, [24, 1], y4m.FMT_P010LE);
    wr.write(f);
    wr.write(f);
    assert.strictEqual(wr.close(), fs.statSync(p).size);
    const r = new y4m.Y4MReader(p);
    assert.deepStrictEqual([r.hdr.bits, r.hdr.fmt, r.frames], [10, y4m.FMT_P010LE, 2]);
    const g = r.read(1);
    assert.ok(g.data[0].equals(f.data[0]) && g.data[1].equals(f.data[1]));
    r.close();
    // record layout: planar 10-bit little-endian samples
    const raw = fs.readFileSync(p);
    const o = y4m.headerBytes(p) + 6;
    assert.strictEqual(raw.readUInt16LE(o + 2), 37);
    assert.strictEqual(raw.readUInt16LE(o + 2 * w * h + 2), 96);                  // U[1]
    assert.strictEqual(raw.readUInt16LE(o + 2 * (w * h + cw * ch)), 700);         // V[0]
    // a header with many tags (> 512 bytes) and FRAME parameters, read as a stream
    const q = path.join(d, "long.y4m");
    const tags = Array.from({ length: 80 }, function (_, i) { return "XTAG" + i + "=abcdef"; }).join(" ");
    const rec = Buffer.alloc(w * h + 2 * cw * ch, 9);
    fs.writeFileSync(q, Buffer.concat([Buffer.from("YUV4MPEG2 W6 H4 F30:1 C420jpeg " + tags + "\n"),
                                       Buffer.from("FRAME Ixyz\n"), rec, Buffer.from("FRAME\n"), rec]));
    assert.ok(y4m.headerBytes(q) > 512);
    // the same file through a FIFO (a real stream: buffered in-order reads, FRAME parameters)
    const fifo = path.join(d, "long.fifo");
    require("child_process").execFileSync("mkfifo", [fifo]);
    const feeder = require("child_process").spawn("sh", ["-c", "cat \"$0\" > \"$1\"", q, fifo]);
    const st = await y4m.open(fifo);
    assert.strictEqual(st.seekable, false);
    assert.strictEqual(st.hdr.headerBytes, y4m.headerBytes(q));
    assert.strictEqual((await st.read(1)).data[0][0], 9);
    assert.strictEqual((await st.read(0)).data[2][0], 9);         // kept until released
    st.release(2);
    await assert.rejects(st.read(0), /released/);
    assert.strictEqual(await st.read(2), null);
    assert.strictEqual(st.frames, 2);
    st.close();
    assert.throws(function () { new y4m.Y4MReader(fifo); }, /not a regular file/);
    return new Promise(function (res) { feeder.on("exit", res); if (feeder.exitCode !== null) res(); });
}

async function testPipeSourceAndPartialJob() {
    // a FIFO source (read in order, never seeked) through the scheduler; a job whose
    // Jobs.chunks exceeds the rows this worker got is left unassembled (ADVICE r02)
    const d = tmpdir(), src = path.join(d, "src.y4m"), fifo = path.join(d, "src.fifo");
    y4m.writeFile(src, 32, 18, [60, 1], 10, function (i) {
        return { data: [Buffer.alloc(32 * 18, i), Buffer.alloc(16 * 9, 128), Buffer.alloc(16 * 9, 128)], pitch: [32, 16, 16] };
    });
    require("child_process").execFileSync("mkfifo", [fifo]);
    const feeder = require("child_process").spawn("sh", ["-c", "cat \"$0\" > \"$1\"", src, fifo]);
    const addon = fakeAddon({ devices: 2 });
    const jobs = [{ id: 51, sourceID: 4, width: 16, height: 10, framerate: 30, chunks: 3, codecSettings: null },
                  { id: 52, sourceID: 4, width: 8, height: 6, framerate: 60, chunks: 4, codecSettings: null }];
    const chunks = [];
    [0, 1, 2].forEach(function (o) { chunks.push({ id: 60 + o, mainJob: 51, chunkOffset: o, status: null }); });
    [0, 1, 2].forEach(function (o) { chunks.push({ id: 70 + o, mainJob: 52, chunkOffset: o, status: null }); });
    const s = new GpuSegmentScheduler({ addon: addon, segmentFrames: 4, outDir: d });
    await s.runJobs(jobs, chunks, { 4: { path: fifo } });
    await new Promise(function (res) { feeder.on("exit", res); if (feeder.exitCode !== null) res(); });
    chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done", c.result);
        const r = JSON.parse(c.result);
        const rd = new y4m.Y4MReader(r.file);
        const got = Array.from({ length: rd.frames }, function (_, i) { return rd.read(i).data[0][0]; });
        rd.close();
        const base = 4 * c.chunkOffset;
        const want = (c.mainJob === 51 ? [0, 2] : [0, 1, 2, 3]).map(function (i) { return base + i; })
            .filter(function (i) { return i < 10; });
        assert.deepStrictEqual(got, want, "job " + c.mainJob + " chunk " + c.chunkOffset);
    });
    assert.strictEqual(jobs[0].finished, true);
    assert.strictEqual(jobs[1].finished, undefined);             // 3 of 4 chunks here: not this worker's to assemble
    assert.deepStrictEqual(Object.keys(s.readers), []);          // readers closed
}

async function testFfmpegBoundary() {
    // decode and encode through ffmpeg children (tests/node/ffmpeg_stub.js as the binary):
    // frames bigger than a pipe's buffer, several segments (the decoder's pipe read across
    // awaits), every rendition segment encoded with its row's codec, the job concatenated
    const d = tmpdir(), src = path.join(d, "src.mkv"), W = 320, H = 180, N = 7;
    y4m.writeFile(src, W, H, [60, 1], N, function (i) {
        return { data: [Buffer.alloc(W * H, i), Buffer.alloc(W * H / 4, 90), Buffer.alloc(W * H / 4, 160)],
                 pitch: [W, W / 2, W / 2] };
    });
    const jobs = [{ id: 41, sourceID: 8, width: 320, height: 180, framerate: 60, chunks: 3, codec: "h264", bitrate: 1500000 },
                  { id: 42, sourceID: 8, width: 96, height: 54, framerate: 60, chunks: 3, codec: "vp9" }];
    const chunks = [];
    jobs.forEach(function (j, k) { [0, 1, 2].forEach(function (o) { chunks.push({ id: 300 + 3 * k + o, mainJob: j.id, chunkOffset: o, status: null }); }); });
    const s = new GpuSegmentScheduler({ addon: fakeAddon({ devices: 1 }), segmentFrames: 3, outDir: path.join(d, "out"),
                                        encode: true, ffmpeg: path.join(__dirname, "ffmpeg_stub.js") });
    await s.runJobs(jobs, chunks, { 8: { path: src, decode: "ffmpeg" } });
    chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done", c.result);
        const r = JSON.parse(c.result);
        assert.ok(r.encodeMs >= 0 && r.file.endsWith(c.mainJob === 41 ? ".mp4" : ".webm"));
        const body = fs.readFileSync(r.file), nl = body.indexOf(0x0a);
        const seg = path.join(d, "seg.y4m");
        fs.writeFileSync(seg, body.slice(nl + 1));
        const rd = new y4m.Y4MReader(seg);
        const got = Array.from({ length: rd.frames }, function (_, i) { return rd.read(i).data[0][0]; });
        rd.close();
        const base = 3 * c.chunkOffset;
        assert.deepStrictEqual(got, [base, base + 1, base + 2].filter(function (i) { return i < N; }), "chunk " + c.chunkOffset);
    });
    jobs.forEach(function (j) { assert.strictEqual(j.finished, true); });
}

async function testSlowEncodersKeepTheLoopFree() {
    // SURVEY §8b "Threading": one Node process drives every GPU slot, so a slow encoder must
    // not stall the event loop.  Two slots, three renditions per segment, a stub encoder that
    // takes 40 ms per frame: each segment's three encoders consume in overlapping windows, the
    // other slot's GPU runs start while an encode is in progress, an event-loop lag probe
    // stays under 50 ms, and the whole run takes <= 0.6x the encoders' summed time.
    const d = tmpdir(), times = path.join(d, "times.jsonl");
    process.env.STUB_ENC_MS_PER_FRAME = "40";
    process.env.STUB_TIMES = times;
    // GPU 1's runs take longer, so the two slots' segments drift apart
    const addon = fakeAddon({ devices: 2, delay: 5 });
    const runs = [];
    addon.run = (function (run) {
        return function (g, src, dst, q) {
            runs.push({ t: Date.now(), dev: g.ctx.dev });
            const p = run(g, src, dst, q);
            return g.ctx.dev ? p.then(function (r) {
                return new Promise(function (res) { setTimeout(function () { res(r); }, 60); });
            }) : p;
        };
    })(addon.run);
    const js = jobSet(6);
    js.jobs.forEach(function (j) { j.codec = "h264"; });
    let last = Date.now(), lag = 0;
    const lags = [];
    const probe = setInterval(function () {
        const now = Date.now();
        lag = Math.max(lag, now - last - 5);
        if (now - last - 5 > 20) lags.push([now - t0, now - last - 5]);
        last = now;
    }, 5);
    const t0 = Date.now();
    const s = new GpuSegmentScheduler({ addon: addon, workerId: 1, segmentFrames: 6, outDir: d, encode: true,
                                        ffmpeg: path.join(__dirname, "ffmpeg_stub.js") });
    await s.runJobs(js.jobs, js.chunks, js.sources);
    const wall = Date.now() - t0;
    clearInterval(probe);
    delete process.env.STUB_ENC_MS_PER_FRAME;
    delete process.env.STUB_TIMES;
    const win = fs.readFileSync(times, "utf8").trim().split("\n").map(JSON.parse);
    assert.strictEqual(win.length, 18);
    const slotOf = {};
    js.chunks.forEach(function (c) {
        assert.strictEqual(c.status, "done", c.result);
        const r = JSON.parse(c.result);
        slotOf[r.file] = r.gpu;
    });
    for (let off = 0; off < 6; ++off) {                  // the renditions of a segment encode together
        const w = win.filter(function (x) { return path.basename(x.out).split(".")[0] === String(off); });
        assert.strictEqual(w.length, 3);
        const start = Math.max.apply(null, w.map(function (x) { return x.t0; }));
        const end = Math.min.apply(null, w.map(function (x) { return x.t1; }));
        assert.ok(start < end, "segment " + off + " encoders ran one after another: " + JSON.stringify(w));
    }
    // the other slot starts a GPU run while an encode is in progress
    const during = win.some(function (x) {
        return runs.some(function (r) { return r.dev !== slotOf[x.out] && r.t > x.t0 && r.t < x.t1; });
    });
    assert.ok(during, "no GPU run started during any encode");
    assert.ok(lag < 50, "event loop lag " + lag + " ms " + JSON.stringify(lags) + " wall " + wall);
    const seq = win.reduce(function (a, x) { return a + (x.t1 - x.t0); }, 0);
    assert.ok(wall <= 0.6 * seq, "wall " + wall + " ms vs sequential " + seq + " ms");
}

function testNoDevicesIsLoud() {
    assert.throws(function () { new GpuSegmentScheduler({ addon: fakeAddon({ devices: 0 }) }); }, /no CPU fallback/);
}

(async function () {
    const tests = [testLadderPlanning, testNoDevicesIsLoud, testAllDoneAndBalanced, testRetryOnAnotherGpu,
                   testGiveUpAfterRetries, testFpsMapAndResume, testThrowingUpdateDoesNotHang, testY4MRoundTrip,
                   testAssembleBlocks, testQualitySummary, testY4MJobAssembled, testDeinterlaceWithRateChange,
                   testY4M10BitAndHeaders, testPipeSourceAndPartialJob, testFfmpegBoundary,
                   testSlowEncodersKeepTheLoopFree];
    for (let i = 0; i < tests.length; ++i) {
        if (process.env.TEST_VERBOSE) process.stderr.write(tests[i].name + "\n");
        await tests[i]();
    }
    process.stdout.write("node scheduler tests ok\n");
})().catch(function (e) { process.stderr.write((e && e.stack || e) + "\n"); process.exit(1); });
