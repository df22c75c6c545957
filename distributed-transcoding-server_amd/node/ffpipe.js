"use strict";
// ffpipe.js -- the ffmpeg process boundary of the GPU worker (SURVEY.md §8f rank 2, rows
// a14 / f2).  The reference resolves a static ffmpeg binary (index.js:9,
// `require("ffmpeg-static")`) and would spawn it per segment with the job's codec
// settings (Jobs.codec / bitrate / codecSettings, database.js:76-78; containers by codec as
// index.js:108-118 getContentType).  The GPU worker keeps ffmpeg for what stays on the
// host -- entropy decode and encode -- and takes the pixel filtergraph itself, so the
// child processes talk rawvideo to it over pipes (`-f yuv4mpegpipe`):
//
//   decode:  ffmpeg -i SOURCE -f yuv4mpegpipe -pix_fmt yuv420p|yuv420p10le -   -> Y4MReader
//   encode:  Y4MWriter -> ffmpeg -f yuv4mpegpipe -i - -c:v CODEC -b:v BITRATE ... SEGMENT
//   concat:  ffmpeg -f concat -safe 0 -i LIST -c copy OUTPUT  (a job's encoded segments)
//
// Both pipes are the children's stdio, made from a FIFO whose two ends are opened here (a
// Node stream on a child's stdio would read ahead into its own buffer whenever the event loop
// runs and take bytes from under the synchronous reader): the child's end in blocking mode,
// the worker's end non-blocking, read / written synchronously (y4m.js retries EAGAIN; a
// dead encoder is EPIPE, a finished decoder EOF).  Decode time lands in
// JobChunks.result.readMs and encode time in writeMs / encodeMs, apart from gpuMs.  The binary: opts.ffmpeg, $DTS_FFMPEG,
// ffmpeg-static if installed, else `ffmpeg` on PATH; none -> null (the worker then reads and
// writes Y4M files only).  libavcodec is not in this image: tests run a stub executable that
// speaks yuv4mpegpipe.
//
// Node 12: no `??` / `?.`.

const cp = require("child_process");
const fs = require("fs");
const os = require("os");
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

// A pipe as {mine, theirs}: `theirs` (blocking) for the child's stdin (toChild) or stdout,
// `mine` (non-blocking) for this process.  Made from a FIFO opened from both sides, then
// unlinked; the child's end is closed here once the child has it.
let fifoSeq = 0;
function pipePair(toChild) {
    const p = path.join(os.tmpdir(), "dts-ff-" + process.pid + "-" + (fifoSeq++) + ".fifo");
    cp.execFileSync("mkfifo", ["-m", "600", p]);
    const C = fs.constants;
    try {
        if (toChild) {                         // we write, the child reads
            const tmp = fs.openSync(p, C.O_RDONLY | C.O_NONBLOCK);      // a reader, so the next open does not block
            const mine = fs.openSync(p, C.O_WRONLY | C.O_NONBLOCK);
            const theirs = fs.openSync(p, C.O_RDONLY);                  // a writer exists: no block
            fs.closeSync(tmp);
            return { mine: mine, theirs: theirs };
        }
        const mine = fs.openSync(p, C.O_RDONLY | C.O_NONBLOCK);         // we read, the child writes
        const theirs = fs.openSync(p, C.O_WRONLY);                      // a reader exists: no block
        return { mine: mine, theirs: theirs };
    } finally {
        fs.unlinkSync(p);
    }
}

function collect(child) {
    const err = [];
    if (child.stderr) child.stderr.on("data", function (d) { if (err.length < 64) err.push(d); });
    return function () { return Buffer.concat(err).toString("utf8").trim(); };
}

// A decoder child: its stdout is a Y4M stream read by a Y4MReader (stream mode: frames in
// order, kept until released).  fmt: the libdts source format wanted (8-bit -> yuv420p,
// p010 -> yuv420p10le, which y4m.js turns into p010 host frames).
class FfmpegDecoder {
    constructor(bin, input, opts) {
        opts = opts || {};
        const pf = opts.fmt === y4m.FMT_P010LE ? "yuv420p10le" : "yuv420p";
        this.args = ["-v", "error", "-nostdin", "-i", input, "-f", "yuv4mpegpipe", "-pix_fmt", pf, "-strict", "-1", "-"];
        this.t0 = Date.now();
        const pp = pipePair(false);
        try {
            this.child = cp.spawn(bin, this.args, { stdio: ["ignore", pp.theirs, "pipe"] });
        } finally {
            fs.closeSync(pp.theirs);
        }
        this.fd = pp.mine;
        this.stderr = collect(this.child);
        const self = this;
        this.exited = new Promise(function (resolve) {
            self.child.on("exit", function (code, sig) { resolve({ code: code, signal: sig }); });
            self.child.on("error", function (e) { resolve({ code: -1, error: e }); });
        });
        try {
            this.reader = new y4m.Y4MReader(this.fd);
        } catch (e) {
            this.kill();
            fs.closeSync(this.fd);
            throw new Error("ffmpeg decode of " + input + ": " + e.message);
        }
        this.hdr = this.reader.hdr;
    }
    get frames() { return this.reader.frames; }
    read(i) { return this.reader.read(i); }
    release(below) { this.reader.release(below); }
    kill() {
        try { this.child.kill("SIGKILL"); } catch (e) { /* gone */ }
    }
    close() {
        this.reader.close();
        if (this.fd !== null) fs.closeSync(this.fd);
        this.fd = null;
        if (this.child.exitCode === null) this.kill();
    }
}

// An encoder child: Y4M records written to its stdin become SEGMENT (codec, bitrate and
// options of the Jobs row).  close() ends the stream and resolves once the child exits, with
// the encode time and the file size.
class FfmpegEncoder {
    constructor(bin, out, w, h, fps, fmt, job, settings) {
        this.out = out;
        this.args = ["-v", "error", "-nostdin", "-f", "yuv4mpegpipe", "-i", "-"].concat(encodeArgs(job || {}, settings),
                                                                                       ["-y", out]);
        this.t0 = Date.now();
        const pp = pipePair(true);
        try {
            this.child = cp.spawn(bin, this.args, { stdio: [pp.theirs, "ignore", "pipe"] });
        } finally {
            fs.closeSync(pp.theirs);
        }
        this.fd = pp.mine;
        this.stderr = collect(this.child);
        const self = this;
        this.exited = new Promise(function (resolve) {
            self.child.on("exit", function (code, sig) { resolve({ code: code, signal: sig }); });
            self.child.on("error", function (e) { resolve({ code: -1, error: e }); });
        });
        try {
            this.writer = new y4m.Y4MWriter(this.fd, w, h, fps, fmt);
        } catch (e) {
            e.encoder = this;
            throw e;
        }
    }
    write(frame) { this.writer.write(frame); }
    _closeFd() {
        if (this.fd !== null) fs.closeSync(this.fd);
        this.fd = null;
    }
    close() {
        const self = this;
        this.writer.close();
        this._closeFd();                                  // EOF: the encoder flushes and exits
        return this.exited.then(function (st) {
            if (st.code !== 0)
                throw new Error("ffmpeg encode of " + self.out + " failed (" + (st.error || st.signal || st.code) + "): " +
                                self.stderr());
            return { file: self.out, bytes: fs.statSync(self.out).size, encodeMs: Date.now() - self.t0 };
        });
    }
}

// a rendition segment through an encoder child; resolves to {file, bytes, encodeMs}
function encodeSegment(bin, out, frames, w, h, fmt, fps, job, settings) {
    let enc = null;
    try {
        enc = new FfmpegEncoder(bin, out, w, h, fps, fmt, job, settings);
        frames.forEach(function (f) { enc.write(f); });
    } catch (e) {                              // e.g. EPIPE: the child is gone
        enc = enc || e.encoder || null;
        if (!enc) return Promise.reject(new Error("ffmpeg encode of " + out + ": " + e.message));
        enc.child.kill("SIGKILL");
        enc._closeFd();
        return enc.exited.then(function () {
            throw new Error("ffmpeg encode of " + out + ": " + e.message + " " + enc.stderr());
        });
    }
    return enc.close();
}

// a job's encoded segments (chunkOffset order) -> one file, stream-copied by ffmpeg's
// concat demuxer (the container is rewritten; the bitstreams are not re-encoded)
function concatSegments(bin, files, out) {
    const list = out + ".txt";
    fs.writeFileSync(list, files.map(function (f) { return "file '" + path.resolve(f).replace(/'/g, "'\\''") + "'\n"; }).join(""));
    const r = cp.spawnSync(bin, ["-v", "error", "-nostdin", "-f", "concat", "-safe", "0", "-i", list, "-c", "copy", "-y", out],
                           { stdio: ["ignore", "ignore", "pipe"] });
    fs.unlinkSync(list);
    if (r.status !== 0) throw new Error("ffmpeg concat of " + out + " failed: " + String(r.stderr || r.error || r.status));
    return out;
}

module.exports = { CODECS: CODECS, ffmpegBinary: ffmpegBinary, codecOf: codecOf, encodeArgs: encodeArgs,
                   FfmpegDecoder: FfmpegDecoder, FfmpegEncoder: FfmpegEncoder, encodeSegment: encodeSegment,
                   concatSegments: concatSegments };
