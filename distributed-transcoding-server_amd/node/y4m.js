"use strict";
// y4m.js -- YUV4MPEG2 (rawvideo) source and sink of the GPU worker (SURVEY.md §8f
// rows f2 / a14).  The reference's worker would hand ffmpeg-static a segment of the
// job's source and collect the encoded renditions (index.js:9; Jobs.codec /
// codecSettings, database.js:76-78).  libavcodec is not part of this build, so the
// worker's file interface is the uncompressed one ffmpeg itself reads and writes
// (`-f yuv4mpegpipe`): 4:2:0 in 8 bits (C420jpeg / C420mpeg2 / C420paldv / C420) or
// 10 bits (C420p10, little-endian 16-bit samples: yuv420p10le), one "FRAME" record per
// picture.  Decode / encode slot in before / after this module (segment frames in,
// rendition frames out) without changing the scheduler: `ffmpeg -i in.mkv -f
// yuv4mpegpipe -` into a pipe is a source, `... | ffmpeg -f yuv4mpegpipe -i - -c:v
// libx264 out.mp4` a sink.
//
// Sources are read either at random (a regular file: frame i at a fixed offset) or in
// order (a pipe / FIFO / stdin: frames are read forward as segments ask for them and
// kept until the scheduler releases them).  10-bit sources become p010 host frames (the layout libdts
// takes: value << 6 in 16-bit words, U / V interleaved); p010 renditions are written
// back as C420p10.
//
// Node 12: no `??` / `?.`.

const fs = require("fs");

const FMT_YUV420P = 0, FMT_NV12 = 1, FMT_P010LE = 2;
const MAX_HEADER = 65536;           // a header line longer than this is not a Y4M stream

// bytes of one planar 4:2:0 picture with `bps` bytes per sample
function frameBytes(w, h, bps) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    return (w * h + 2 * cw * ch) * (bps || 1);
}

// "YUV4MPEG2 W3840 H2160 F60:1 Ip A1:1 C420mpeg2" -> {w, h, fps: [n, d], chroma, bits, fmt}
function parseHeader(line) {
    if (Buffer.isBuffer(line)) {
        const nl = line.indexOf(0x0a);
        if (nl < 0) throw new Error("y4m: no header line");
        line = line.toString("latin1", 0, nl);
    }
    const tok = line.split(" ");
    if (tok[0] !== "YUV4MPEG2") throw new Error("y4m: not a YUV4MPEG2 stream");
    const h = { w: 0, h: 0, fps: [25, 1], chroma: "420jpeg", interlace: "p" };
    tok.slice(1).forEach(function (t) {
        const v = t.slice(1);
        switch (t[0]) {
        case "W": h.w = parseInt(v, 10); break;
        case "H": h.h = parseInt(v, 10); break;
        case "F": h.fps = v.split(":").map(function (x) { return parseInt(x, 10); }); break;
        case "C": h.chroma = v; break;
        case "I": h.interlace = v; break;
        default: break;
        }
    });
    if (!(h.w > 0 && h.h > 0)) throw new Error("y4m: bad size " + line);
    if (/^420(jpeg|mpeg2|paldv)?$/.test(h.chroma)) {
        h.bits = 8;
        h.fmt = FMT_YUV420P;
    } else if (h.chroma === "420p10") {
        h.bits = 10;
        h.fmt = FMT_P010LE;
    } else {
        throw new Error("y4m: only 4:2:0 in 8 or 10 bits is supported (C" + h.chroma + ")");
    }
    return h;
}

// A non-blocking descriptor (a child process's pipe, stdin after the parent set
// O_NONBLOCK) answers EAGAIN while the producer has nothing yet: wait a millisecond and try
// again (ADVICE r03), up to `EAGAIN_MS` in all, then fail clearly.
const EAGAIN_MS = 600000;
const SLEEP = new Int32Array(new SharedArrayBuffer(4));
function retryAgain(fn) {
    for (let waited = 0;; ++waited) {
        try {
            return fn();
        } catch (e) {
            if (e.code !== "EAGAIN" || waited >= EAGAIN_MS) throw e;
            Atomics.wait(SLEEP, 0, 0, 1);
        }
    }
}

function readSync(fd, buf, off, len, pos) {
    return retryAgain(function () { return fs.readSync(fd, buf, off, len, pos); });
}

// Buffered in-order reads of a stream (pipe / FIFO / stdin): header and FRAME lines are
// parsed from 1 MiB reads instead of one read per byte (ADVICE r03); frame payloads copy
// what is buffered and read the rest straight into the record.
class StreamIn {
    constructor(fd) {
        this.fd = fd;
        this.buf = Buffer.alloc(1 << 20);
        this.start = 0;
        this.end = 0;
        this.eof = false;
    }
    _fill() {
        if (this.eof) return 0;
        if (this.start === this.end) {
            this.start = this.end = 0;
        } else if (this.end === this.buf.length) {
            this.buf.copy(this.buf, 0, this.start, this.end);
            this.end -= this.start;
            this.start = 0;
        }
        const n = readSync(this.fd, this.buf, this.end, this.buf.length - this.end, null);
        if (n <= 0) this.eof = true;
        else this.end += n;
        return Math.max(n, 0);
    }
    // {line, bytes} up to and without "\n", or null at the end of the stream
    line(limit) {
        for (;;) {
            const nl = this.buf.indexOf(0x0a, this.start);
            if (nl >= 0 && nl < this.end) {
                const r = { line: this.buf.toString("latin1", this.start, nl), bytes: nl + 1 - this.start };
                this.start = nl + 1;
                return r;
            }
            if (this.end - this.start > limit) throw new Error("y4m: header line longer than " + limit + " bytes");
            if (!this._fill()) {
                if (this.start === this.end) return null;
                throw new Error("y4m: stream ends inside a header line");
            }
        }
    }
    // fill dst; returns the bytes read (short at the end of the stream)
    read(dst) {
        const have = Math.min(this.end - this.start, dst.length);
        this.buf.copy(dst, 0, this.start, this.start + have);
        this.start += have;
        let off = have;
        while (off < dst.length && !this.eof) {
            const n = readSync(this.fd, dst, off, dst.length - off, null);
            if (n <= 0) this.eof = true;
            else off += n;
        }
        return off;
    }
}

// one line (up to and without "\n") of a regular file at `pos`; returns {line, bytes} or
// null at the end of the file
function readLine(fd, pos, limit) {
    const one = Buffer.alloc(1), out = [];
    let n = 0;
    for (;;) {
        const got = readSync(fd, one, 0, 1, pos + n);
        if (got <= 0) {
            if (n === 0) return null;
            throw new Error("y4m: stream ends inside a header line");
        }
        ++n;
        if (one[0] === 0x0a) break;
        if (n > limit) throw new Error("y4m: header line longer than " + limit + " bytes");
        out.push(one[0]);
    }
    return { line: Buffer.from(out).toString("latin1"), bytes: n };
}

// fill buf from fd (a stream may return short reads); returns the bytes read
function readFull(fd, buf, pos) {
    let off = 0;
    while (off < buf.length) {
        const n = readSync(fd, buf, off, buf.length - off, pos === null ? null : pos + off);
        if (n <= 0) break;
        off += n;
    }
    return off;
}

// a planar record's bytes -> a host frame for the addon ({data, pitch}):
// 8 bit: yuv420p planes (views of the record); 10 bit: p010 (Y << 6, U / V interleaved << 6)
function recordToFrame(rec, w, h, bits) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    if (bits === 8)
        return { data: [rec.slice(0, w * h), rec.slice(w * h, w * h + cw * ch), rec.slice(w * h + cw * ch)],
                 pitch: [w, cw, cw] };
    const s = new Uint16Array(rec.buffer, rec.byteOffset, rec.length >> 1);
    const y = Buffer.alloc(2 * w * h), uv = Buffer.alloc(4 * cw * ch);
    const yv = new Uint16Array(y.buffer, y.byteOffset, w * h), uvv = new Uint16Array(uv.buffer, uv.byteOffset, 2 * cw * ch);
    for (let i = 0; i < w * h; ++i) yv[i] = s[i] << 6;
    const u0 = w * h, v0 = u0 + cw * ch;
    for (let i = 0; i < cw * ch; ++i) {
        uvv[2 * i] = s[u0 + i] << 6;
        uvv[2 * i + 1] = s[v0 + i] << 6;
    }
    return { data: [y, uv, null], pitch: [2 * w, 4 * cw, 0] };
}

class Y4MReader {
    // src: a path ("-" = stdin) or an open file descriptor
    constructor(src) {
        this.path = typeof src === "string" ? src : null;
        this.fd = typeof src === "number" ? src : (src === "-" ? 0 : fs.openSync(src, "r"));
        this.ownFd = typeof src === "string" && src !== "-";
        const st = fs.fstatSync(this.fd);
        this.seekable = st.isFile();
        if (!this.seekable) this.sin = new StreamIn(this.fd);
        const hl = this.seekable ? readLine(this.fd, 0, MAX_HEADER) : this.sin.line(MAX_HEADER);
        if (!hl) throw new Error("y4m: empty stream");
        this.hdr = parseHeader(hl.line);
        this.hdr.headerBytes = hl.bytes;
        this.bps = this.hdr.bits > 8 ? 2 : 1;
        this.frameBytes = frameBytes(this.hdr.w, this.hdr.h, this.bps);
        if (this.seekable) {
            this.stride = 6 + this.frameBytes;             // "FRAME\n" + planes (no frame parameters)
            this.frames = Math.floor((st.size - hl.bytes) / this.stride);
        } else {
            this.frames = Infinity;                        // known at the end of the stream
            this.next = 0;                                 // index of the next record in the stream
            this.kept = new Map();                         // frames read, not yet released
        }
    }

    // frame i as a host frame for the addon, or null past the end of the stream.  A
    // stream keeps every frame it has read until release() drops it (segments are
    // requested roughly in order, so at most a few segments are held; a frame may be
    // asked for twice: vf_fps repeats, yadif context frames, two ladders of one source).
    read(i) {
        if (i < 0) throw new Error("y4m: frame " + i);
        if (this.seekable) {
            if (i >= this.frames) return null;
            const off = this.hdr.headerBytes + i * this.stride;
            const tag = Buffer.alloc(6);
            readFull(this.fd, tag, off);
            if (tag.toString("latin1") !== "FRAME\n")
                throw new Error("y4m: frame " + i + ": FRAME parameters need a stream (pipe) reader");
            const rec = Buffer.alloc(this.frameBytes);
            if (readFull(this.fd, rec, off + 6) !== rec.length) throw new Error("y4m: frame " + i + " is truncated");
            return recordToFrame(rec, this.hdr.w, this.hdr.h, this.hdr.bits);
        }
        if (this.kept.has(i)) return this.kept.get(i);
        if (i < this.next) throw new Error("y4m: frame " + i + " of a stream was already released");
        while (this.next <= i) {
            const tl = this.sin.line(MAX_HEADER);
            if (!tl) {
                this.frames = this.next;
                return null;
            }
            if (tl.line.slice(0, 5) !== "FRAME") throw new Error("y4m: record " + this.next + " is not a FRAME");
            const rec = Buffer.alloc(this.frameBytes);
            if (this.sin.read(rec) !== rec.length) throw new Error("y4m: frame " + this.next + " is truncated");
            this.kept.set(this.next++, recordToFrame(rec, this.hdr.w, this.hdr.h, this.hdr.bits));
        }
        return this.kept.get(i);
    }

    // a stream forgets the frames below `below` (no pending segment asks for them again)
    release(below) {
        if (!this.kept) return;
        const self = this;
        Array.from(this.kept.keys()).forEach(function (k) { if (k < below) self.kept.delete(k); });
    }

    close() {
        if (this.fd !== null && this.ownFd) fs.closeSync(this.fd);
        this.fd = null;
        if (this.kept) this.kept.clear();
    }
}

function header(w, h, fps, fmt) {
    const f = fps || [25, 1];
    const c = fmt === FMT_P010LE ? "C420p10 XYSCSS=420P10" : "C420mpeg2";
    return Buffer.from("YUV4MPEG2 W" + w + " H" + h + " F" + f[0] + ":" + f[1] + " Ip A1:1 " + c + "\n", "latin1");
}

// One host frame (yuv420p planes, nv12 Y + interleaved UV, or p010 Y + interleaved UV)
// as a Y4M FRAME record (planar 4:2:0, as ffmpeg's yuv4mpegpipe muxer writes it:
// interleaved chroma de-interleaved, p010 as 10-bit samples >> 6 in 16-bit words)
function frameRecord(f, w, h, fmt) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    if (fmt === FMT_P010LE) {
        const out = Buffer.alloc(6 + frameBytes(w, h, 2));
        out.write("FRAME\n", 0, "latin1");
        const y = f.data[0], uv = f.data[1];
        let o = 6;
        for (let r = 0; r < h; ++r)
            for (let x = 0; x < w; ++x, o += 2) out.writeUInt16LE(y.readUInt16LE(r * f.pitch[0] + 2 * x) >> 6, o);
        const u0 = o, v0 = o + 2 * cw * ch;
        for (let r = 0; r < ch; ++r)
            for (let x = 0; x < cw; ++x) {
                const p = r * f.pitch[1] + 4 * x, d = 2 * (r * cw + x);
                out.writeUInt16LE(uv.readUInt16LE(p) >> 6, u0 + d);
                out.writeUInt16LE(uv.readUInt16LE(p + 2) >> 6, v0 + d);
            }
        return out;
    }
    const out = Buffer.alloc(6 + frameBytes(w, h, 1));
    out.write("FRAME\n", 0, "latin1");
    let o = 6;
    for (let y = 0; y < h; ++y, o += w) f.data[0].copy(out, o, y * f.pitch[0], y * f.pitch[0] + w);
    if (fmt === FMT_NV12) {
        const uv = f.data[1], p = f.pitch[1], u0 = o, v0 = o + cw * ch;
        for (let y = 0; y < ch; ++y)
            for (let x = 0; x < cw; ++x) {
                out[u0 + y * cw + x] = uv[y * p + 2 * x];
                out[v0 + y * cw + x] = uv[y * p + 2 * x + 1];
            }
    } else if (fmt === FMT_YUV420P) {
        for (let pl = 1; pl < 3; ++pl)
            for (let y = 0; y < ch; ++y, o += cw) f.data[pl].copy(out, o, y * f.pitch[pl], y * f.pitch[pl] + cw);
    } else {
        throw new Error("y4m: unknown rendition format " + fmt);
    }
    return out;
}

// A streaming sink: the header, then one record per frame written as it comes (a
// segment of any size never sits in memory as one Buffer; ADVICE r02)
class Y4MWriter {
    // dst: a path or an open file descriptor (e.g. a pipe into an encoder)
    constructor(dst, w, h, fps, fmt) {
        this.fd = typeof dst === "number" ? dst : fs.openSync(dst, "w");
        this.ownFd = typeof dst !== "number";
        this.w = w;
        this.h = h;
        this.fmt = fmt;
        this.bytes = 0;
        this.frames = 0;
        this._put(header(w, h, fps, fmt));
    }

    _put(buf) {
        let off = 0;
        const fd = this.fd;
        while (off < buf.length) {
            const o = off;
            off += retryAgain(function () { return fs.writeSync(fd, buf, o, buf.length - o); });
        }
        this.bytes += buf.length;
    }

    write(frame) {
        this._put(frameRecord(frame, this.w, this.h, this.fmt));
        ++this.frames;
    }

    close() {
        if (this.fd !== null && this.ownFd) fs.closeSync(this.fd);
        this.fd = null;
        return this.bytes;
    }
}

// write a whole rendition segment, frame by frame; returns the bytes written
function writeSegment(path, frames, w, h, fmt, fps) {
    const wr = new Y4MWriter(path, w, h, fps, fmt);
    try {
        frames.forEach(function (f) { wr.write(f); });
    } finally {
        wr.close();
    }
    return wr.bytes;
}

// a complete 8-bit Y4M file from frames made by gen(i) (tests, fixtures)
function writeFile(path, w, h, fps, n, gen) {
    const wr = new Y4MWriter(path, w, h, fps, FMT_YUV420P);
    for (let i = 0; i < n; ++i) wr.write(gen(i));
    wr.close();
}

// bytes of the header line of a Y4M file (assembly keeps the first segment's only)
function headerBytes(path) {
    const fd = fs.openSync(path, "r");
    try {
        const hl = readLine(fd, 0, MAX_HEADER);
        if (!hl) throw new Error("y4m: empty file " + path);
        parseHeader(hl.line);
        return hl.bytes;
    } finally {
        fs.closeSync(fd);
    }
}

module.exports = { Y4MReader: Y4MReader, Y4MWriter: Y4MWriter, parseHeader: parseHeader, frameBytes: frameBytes,
                   header: header, frameRecord: frameRecord, writeSegment: writeSegment, writeFile: writeFile,
                   headerBytes: headerBytes, recordToFrame: recordToFrame,
                   FMT_YUV420P: FMT_YUV420P, FMT_NV12: FMT_NV12, FMT_P010LE: FMT_P010LE };
