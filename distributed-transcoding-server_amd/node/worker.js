"use strict";
// worker.js -- the GPU transcoding worker entry: Jobs/JobChunks rows in,
// renditions + updated JobChunks rows out (the drop-in for a CPU worker that
// spawns ffmpeg-static per segment, index.js:9).
//
//   node worker.js <job.json> [--out DIR [--encode] | --dump DIR]
//
// job.json: {"workerId": 1, "segmentFrames": 600, "gpus": [0, ...] (optional),
//            "sources": {"<sourceID>": {"path": "src.y4m"} or {"w": 3840, "h": 2160, "fmt": 0,
//                                                             "fps": [60, 1]}},
//            "jobs": [Jobs rows], "chunks": [JobChunks rows]}
// Prints one JSON object: {"chunks": [updated rows], "jobs": [rows], "summary": {...}}.
// --out DIR: sources with a `path` are read from their Y4M file, every rendition
// segment is written as DIR/job<id>/<chunkOffset>.y4m and finished jobs get
// Jobs.assembledData (1 MiB blocks in DIR/blocks) and finished = true.
// --dump DIR writes every output frame as DIR/<jobId>_<chunkOffset>_<frame>.raw
// (packed planes) for offline checks.  Without a path the source is libdts's
// synthetic one.  Decode / encode stay in ffmpeg child processes (ffpipe.js): a source
// path that is not .y4m is decoded by one, and --encode (or "encode": true) hands each
// rendition segment to one with the Jobs row's codec and bitrate; the binary is
// cfg.ffmpeg, $DTS_FFMPEG, ffmpeg-static or `ffmpeg` on PATH.
const path = require("path");
const fs = require("fs");

function threadPool(n) {
    // before any async work starts: one libuv worker per GPU slot (+ 2 spare)
    if (!process.env.UV_THREADPOOL_SIZE) process.env.UV_THREADPOOL_SIZE = String(Math.max(4, n + 2));
}

function loadAddon() {
    const p = process.env.DTS_ADDON || path.join(__dirname, "..", "addon", "dts_napi.node");
    return require(p);
}

async function main(argv) {
    const cfg = JSON.parse(fs.readFileSync(argv[0], "utf8"));
    const di = argv.indexOf("--dump");
    const dump = di >= 0 ? argv[di + 1] : null;
    const oi = argv.indexOf("--out");
    const outDir = oi >= 0 ? argv[oi + 1] : cfg.outDir || null;
    threadPool(cfg.gpus ? cfg.gpus.length : 8);
    const addon = loadAddon();
    const { GpuSegmentScheduler } = require("./scheduler");
    const sink = dump ? function (plan, rows, per) {
        per.forEach(function (frames, k) {
            frames.forEach(function (f, i) {
                const off = rows[k] ? rows[k].chunkOffset : "x";
                const name = path.join(dump, plan.jobs[k].id + "_" + off + "_" + i + ".raw");
                fs.writeFileSync(name, Buffer.concat(f.data.filter(function (b) { return b; })));
            });
        });
    } : null;
    const sched = new GpuSegmentScheduler({ addon: addon, gpus: cfg.gpus, workerId: cfg.workerId,
                                            segmentFrames: cfg.segmentFrames, sink: sink, outDir: outDir,
                                            encode: argv.indexOf("--encode") >= 0 || !!cfg.encode, ffmpeg: cfg.ffmpeg });
    const summary = await sched.runJobs(cfg.jobs, cfg.chunks, cfg.sources);
    process.stdout.write(JSON.stringify({ chunks: cfg.chunks, jobs: cfg.jobs, summary: summary }) + "\n");
}

if (require.main === module) {
    main(process.argv.slice(2)).catch(function (e) {
        process.stderr.write("worker: " + (e && e.stack || e) + "\n");
        process.exitCode = 1;
    });
}

module.exports = { main: main };
