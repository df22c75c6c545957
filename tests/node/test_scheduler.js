"use strict";
// CPU test of the Node GPU worker's scheduler and JobChunks state machine
// against a stand-in addon (same interface as dts_napi.node, no device).
// Run by tests/test_node.py; exits non-zero on the first failed check.
const assert = require("assert");
const path = require("path");
const NODE = path.join(__dirname, "..", "..", "distributed-transcoding-server_amd", "node");
const { GpuSegmentScheduler } = require(path.join(NODE, "scheduler"));
const ladder = require(path.join(NODE, "ladder"));

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
        run: function (g, src, dst, q) {
            stats.runs++;
            stats.byDev[g.ctx.dev] = (stats.byDev[g.ctx.dev] || 0) + 1;
            assert.strictEqual(dst.length, src.length * g.spec.outputs.length);
            return new Promise(function (resolve, reject) {
                setTimeout(function () {
                    if (opts.fail && opts.fail(g.ctx.dev, stats.runs)) return reject(new Error("dts run: HIP error (-1000)"));
                    dst.forEach(function (f, i) { f.data[0][0] = src[Math.floor(i / g.spec.outputs.length)].data[0][0]; });
                    resolve(null);
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

function testNoDevicesIsLoud() {
    assert.throws(function () { new GpuSegmentScheduler({ addon: fakeAddon({ devices: 0 }) }); }, /no CPU fallback/);
}

(async function () {
    testLadderPlanning();
    testNoDevicesIsLoud();
    await testAllDoneAndBalanced();
    await testRetryOnAnotherGpu();
    await testGiveUpAfterRetries();
    await testFpsMapAndResume();
    await testThrowingUpdateDoesNotHang();
    process.stdout.write("node scheduler tests ok\n");
})().catch(function (e) { process.stderr.write((e && e.stack || e) + "\n"); process.exit(1); });
