"use strict";
// GPU test (run by tests/test_node.py, -m gpu): the scheduler with the real addon on
// gpus [0, 0] -- two libdts contexts on one device, driven from two libuv threads --
// with one segment's source failing once.  Prints the chunk rows and the summary as
// JSON; the Python side checks every written frame against the oracle.
const path = require("path");
const fs = require("fs");
process.env.UV_THREADPOOL_SIZE = "4";
const NODE = path.join(__dirname, "..", "..", "distributed-transcoding-server_amd", "node");
const addon = require(path.join(__dirname, "..", "..", "distributed-transcoding-server_amd", "addon", "dts_napi.node"));
const { GpuSegmentScheduler, synthSource } = require(path.join(NODE, "scheduler"));

(async function () {
    const out = process.argv[2];
    const synth = synthSource(addon, 0x5EED);
    let failed = 0;
    const threads = new Set();
    const source = function (plan, idx) {
        if (idx[0] === 4 * 3 && !failed) {                 // chunk 3's first attempt: a decoder error
            failed++;
            throw new Error("injected source failure");
        }
        return synth(plan, idx);
    };
    const jobs = [{ id: 81, sourceID: 1, width: 192, height: 108, framerate: 60, chunks: 6,
                    codecSettings: JSON.stringify({ quality: "both" }) },
                  { id: 82, sourceID: 1, width: 128, height: 72, framerate: 60, chunks: 6,
                    codecSettings: JSON.stringify({ scale: "lanczos", format: "yuv420p" }) }];
    const chunks = [];
    jobs.forEach(function (j) { for (let o = 0; o < 6; o++) chunks.push({ id: chunks.length + 1, mainJob: j.id, chunkOffset: o, status: null }); });
    const sink = function (plan, rows, per) {
        per.forEach(function (frames, k) {
            frames.forEach(function (f, i) {
                fs.writeFileSync(path.join(out, plan.jobs[k].id + "_" + rows[k].chunkOffset + "_" + i + ".raw"),
                                 Buffer.concat(f.data.filter(function (b) { return b; })));
            });
        });
    };
    const s = new GpuSegmentScheduler({ addon: addon, gpus: [0, 0], workerId: 9, segmentFrames: 4, source: source, sink: sink });
    let retries = 0;
    s.on("retry", function () { retries++; });
    const sum = await s.runJobs(jobs, chunks, { 1: { w: 384, h: 216, fmt: 0, fps: [60, 1] } });
    process.stdout.write(JSON.stringify({ chunks: chunks, jobs: jobs, summary: sum, retries: retries, failed: failed }) + "\n");
})().catch(function (e) { process.stderr.write((e && e.stack || e) + "\n"); process.exit(1); });
