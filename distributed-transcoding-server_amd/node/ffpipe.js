"use strict";
// ffpipe.js -- the ffmpeg process boundary of the GPU worker (SURVEY.md §8f rank 2, rows
// a14 / f2).  The reference resolves a static ffmpeg binary (index.js:9,
// `require("ffmpeg-static")`) and would spawn it per segment with the job's codec
// settings (Jobs.codec / bitrate / codecSettings, database.js:76-78; containers by codec as
// index.js:108-118 getContentType).  The GPU worker keeps ffmpeg for what stays on the
// host -- entropy decode and encode -- and takes the pixel filtergraph itself, so the
// child processes talk rawvideo to it over pipes (`-f yuv4mpegpipe`):
//
//   decode:  ffmpeg -i SOURCE -f yuv4mpegpipe -pix_fmt yuv420p|yuv420p10le -   -> Y4MStream
//   encode:  Y4MSink -> ffmpeg -f yuv4mpegpipe -i - -c:v CODEC -b:v BITRATE ... SEGMENT
//   concat:  ffmpeg -f concat -safe 0 -i LIST -c copy OUTPUT  (a job's encoded segments)
//
// Both pipes are the children's stdio as Node streams, polled by libuv on the event loop:
// the decoder's stdout is read in paused mode (y4m.Y4MStream pulls only the frames the
// segments ask for, so the child waits on a full pipe), the encoders' stdin is written
// with 'drain' backpressure (y4m.Y4MSink), and stderr is always drained (an ffmpeg that
// logs a lot never blocks on it).  No call here blocks the event loop: one Node process
// drives every GPU slot of the node (SURVEY.md §8b "Threading"), and an encode waiting on a
// slow libx264 must not hold back the other slots.  Every rendition of a segment gets its
// own encoder child, all started before the first frame is written and fed concurrently
// (encodeRenditions).  Decode time lands in JobChunks.result.readMs and encode time in
// writeMs / encodeMs, apart from gpuMs.  The binary: opts.ffmpeg, $DTS_FFMPEG,
// ffmpeg-static if installed, else `ffmpeg` on PATH; none -> null (the worker then reads and
// writes Y4M files only).  libavcodec is not in this image: tests run a stub executable that
// speaks yuv4mpegpipe.
//
// Node 12: no `??` / `?.`.

const cp = require("child_process");
const fs = require("fs");
const path = require("path");
const y4m = require("./y4m");

// Jobs.codec -> ffmpeg encoder and container extension (index.js:108-118: h264 / h265 in mp4,
// vp9 in webm); an unknown codec is passed to -c:v as it is, in Matroska
const CODECS = { h264: ["libx264", "mp4"], h265: ["libx265", "mp4"], hevc: ["libx265", "mp4"], vp9: ["libvpx-vp9", "webm"] };

function onPath(name) {
    const dirs = String(process.env.PATH || "").split(path.delimiter);
    for (let i = 0; i < dirs.length; ++i) {
        const p = path.join(dirs[i], name);
        try {
            fs.accessSync(p, fs.constants.X_OK);
            if (fs.statSync(p).isFile()) return p;
        } catch (e) { /* next */ }
    }
    return null;
}

// the ffmpeg binary to spawn, or null
function ffmpegBinary(opts) {
    if (opts && opts.ffmpeg) return opts.ffmpeg;
    if (process.env.DTS_FFMPEG) return process.env.DTS_FFMPEG;
    try {
        const p = require("ffmpeg-static");               // the reference's dependency (index.js:9)
        if (p && fs.existsSync(p)) return p;
    } catch (e) { /* not installed */ }
    return onPath("ffmpeg");
}

function codecOf(job) {
    const c = CODECS[String(job.codec || "").toLowerCase()];
    return c ? { encoder: c[0], ext: c[1] } : { encoder: String(job.codec || "rawvideo"), ext: "mkv" };
}

// the encoder options a CPU worker would put on its command line: -b:v from Jobs.bitrate,
// then codecSettings.encoderArgs (an array of ffmpeg arguments), if any
function encodeArgs(job, settings) {
    const a = ["-c:v", codecOf(job).encoder];
    if (job.bitrate) a.push("-b:v", String(job.bitrate));
    if (settings && Array.isArray(settings.encoderArgs)) settings.encoderArgs.forEach(function (x) { a.push(String(x)); });
    return a;
}

function collect(child) {
    const err = [];
    let kept = 0;
    // drained whatever the child writes (a full stderr pipe would block it); the first 64 KB kept
    if (child.stderr) child.stderr.on("data", function (d) { if (kept < 65536) { err.push(d); kept += d.length; } });
    return function () { return Buffer.concat(err).toString("utf8").trim(); };
}

function exitOf(child) {
    return new Promise(function (resolve) {
        child.on("exit", function (code, sig) { resolve({ code: code, signal: sig }); });
        child.on("error", function (e) { resolve({ code: -1, error: e }); });
    });
}

// A decoder child: its stdout is a Y4M stream read in order (y4m.Y4MStream: frames kept
// until released).  fmt: the libdts source format wanted (8-bit -> yuv420p, p010 ->
// yuv420p10le, which y4m.js turns into p010 host frames).  FfmpegDecoder.open resolves once
// the stream's header has arrived.
class FfmpegDecoder {
    static async open(bin, input, opts) {
        const d = new FfmpegDecoder(bin, input, opts);
        try {
            d.reader = await y4m.Y4MStream.open(d.child.stdout);
        } catch (e) {
            d.kill();
            const st = await d.exited;
            throw new Error("ffmpeg decode of " + input + ": " + e.message + " (" + (st.error || st.signal || st.code) + ") " +
                            d.stderr());
        }
        d.hdr = d.reader.hdr;
        return d;
    }
    constructor(bin, input, opts) {
        opts = opts || {};
        const pf = opts.fmt === y4m.FMT_P010LE ? "yuv420p10le" : "yuv420p";
        this.args = ["-v", "error", "-nostdin", "-i", input, "-f", "yuv4mpegpipe", "-pix_fmt", pf, "-strict", "-1", "-"];
        this.t0 = Date.now();
        this.child = cp.spawn(bin, this.args, { stdio: ["ignore", "pipe", "pipe"] });
        this.stderr = collect(this.child);
        this.exited = exitOf(this.child);
        this.reader = null;
    }
    get frames() { return this.reader.frames; }
    read(i) { return this.reader.read(i); }
    release(below) { this.reader.release(below); }
    kill() {
        try { this.child.kill("SIGKILL"); } catch (e) { /* gone */ }
    }
    close() {
        if (this.reader) this.reader.close();
        if (this.child.exitCode === null) this.kill();
    }
}

// An encoder child: Y4M records written to its stdin become SEGMENT (codec, bitrate and
// options of the Jobs row).  write(frame) resolves when the child's pipe takes more;
// close() ends the stream and resolves once the child exits, with the encode time and the
// file size.
class FfmpegEncoder {
    constructor(bin, out, w, h, fps, fmt, job, settings) {
        this.out = out;
        this.args = ["-v", "error", "-nostdin", "-f", "yuv4mpegpipe", "-i", "-"].concat(encodeArgs(job || {}, settings),
                                                                                       ["-y", out]);
        this.t0 = Date.now();
        this.child = cp.spawn(bin, this.args, { stdio: ["pipe", "ignore", "pipe"] });
        this.stderr = collect(this.child);
        this.exited = exitOf(this.child);
        this.sink = new y4m.Y4MSink(this.child.stdin, w, h, fps, fmt);
    }
    write(frame) { return this.sink.write(frame); }
    kill() {
        try { this.child.kill("SIGKILL"); } catch (e) { /* gone */ }
    }
    async close() {
        let werr = null;
        try {
            await this.sink.end();                        // EOF: the encoder flushes and exits
        } catch (e) {
            werr = e;                                     // EPIPE: the exit status says why
        }
        const st = await this.exited;
        if (st.code !== 0 || werr)
            throw new Error("ffmpeg encode of " + this.out + " failed (" + (st.error || st.signal || st.code) + ")" +
                            (werr ? " " + werr.message : "") + ": " + this.stderr());
        return { file: this.out, bytes: fs.statSync(this.out).size, encodeMs: Date.now() - this.t0 };
    }
}

// one rendition segment through an encoder child; resolves to {file, bytes, encodeMs}
async function encodeSegment(bin, out, frames, w, h, fmt, fps, job, settings) {
    return (await encodeRenditions(bin, [{ out: out, frames: frames, w: w, h: h, fmt: fmt, fps: fps, job: job,
                                           settings: settings }]))[0];
}

// Every rendition segment of a launch through its own encoder child: all children are started
// first, then each is fed by its own loop (the loops interleave on the event loop, each
// paced by its child's pipe).  items: [{out, frames, w, h, fmt, fps, job, settings}];
// resolves to [{file, bytes, encodeMs}] in item order, or rejects with the first failure
// once every child has ended (the others are killed).
async function encodeRenditions(bin, items) {
    const encs = [];
    try {
        // one spawn per turn of the event loop: a spawn forks this process (~10 ms each), and
        // a burst of them would hold the loop -- and every other GPU slot -- for all of them
        for (let k = 0; k < items.length; ++k) {
            const it = items[k];
            if (k) await new Promise(setImmediate);
            encs.push(new FfmpegEncoder(bin, it.out, it.w, it.h, it.fps, it.fmt, it.job, it.settings));
        }
    } catch (e) {
        encs.forEach(function (en) { en.kill(); });
        throw new Error("ffmpeg encode: " + e.message);
    }
    const runs = encs.map(async function (en, k) {
        try {
            const fr = items[k].frames;
            for (let i = 0; i < fr.length; ++i) await en.write(fr[i]);
        } catch (e) { /* a dead child: close() reports it with its exit status */ }
        return en.close();
    });
    const res = await Promise.all(runs.map(function (p) {
        return p.then(function (r) { return { ok: r }; }, function (e) { return { err: e }; });
    }));
    const bad = res.find(function (r) { return r.err; });
    if (bad) {
        encs.forEach(function (en) { en.kill(); });
        throw bad.err;
    }
    return res.map(function (r) { return r.ok; });
}

// a job's encoded segments (chunkOffset order) -> one file, stream-copied by ffmpeg's
// concat demuxer (the container is rewritten; the bitstreams are not re-encoded); resolves
// to the output path
async function concatSegments(bin, files, out) {
    const list = out + ".txt";
    fs.writeFileSync(list, files.map(function (f) { return "file '" + path.resolve(f).replace(/'/g, "'\\''") + "'\n"; }).join(""));
    const child = cp.spawn(bin, ["-v", "error", "-nostdin", "-f", "concat", "-safe", "0", "-i", list, "-c", "copy", "-y", out],
                           { stdio: ["ignore", "ignore", "pipe"] });
    const err = collect(child);
    const st = await exitOf(child);
    fs.unlinkSync(list);
    if (st.code !== 0) throw new Error("ffmpeg concat of " + out + " failed (" + (st.error || st.signal || st.code) + "): " + err());
    return out;
}

module.exports = { CODECS: CODECS, ffmpegBinary: ffmpegBinary, codecOf: codecOf, encodeArgs: encodeArgs,
                   FfmpegDecoder: FfmpegDecoder, FfmpegEncoder: FfmpegEncoder, encodeSegment: encodeSegment,
                   encodeRenditions: encodeRenditions, concatSegments: concatSegments };
