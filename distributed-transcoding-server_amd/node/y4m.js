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
// Sources are read either at random (a regular file: frame i at a fixed offset; Y4MReader)
// or in order (a pipe / FIFO / stdin / a decoder child's stdout: Y4MStream, frames read
// forward as segments ask for them and kept until the scheduler releases them).  10-bit
// sources become p010 host frames (the layout libdts takes: value << 6 in 16-bit words,
// U / V interleaved); p010 renditions are written back as C420p10.
//
// Nothing here blocks the event loop on a pipe: a stream is read through a paused Node
// Readable (libuv polls the descriptor; the reader pulls only as many bytes as the frames
// asked for, so the producer is held back by the pipe itself), and sinks (Y4MSink: an
// encoder child's stdin, a segment file) are Writables awaited on 'drain'.  One Node
// process drives every GPU slot of a node (SURVEY.md §8b "Threading"), so a decode or an
// encode must never stall the other slots.  Y4MReader / Y4MWriter keep synchronous calls
// for regular files only (fixtures, tests, random access).
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

const readP = require("util").promisify(fs.read);

// Bytes of a Readable in paused mode: chunks are pulled with read() only when the parser
// needs more, and a pull with nothing buffered waits for 'readable' / 'end' / 'error' --
// a Promise, never a loop on the event loop's thread.
class ByteQueue {
    constructor(rs) {
        this.rs = rs;
        this.bufs = [];
        this.have = 0;
        this.ended = false;
        this.err = null;
        this.wake = null;
        const self = this;
        rs.on("readable", function () { self._wake(); });
        rs.on("end", function () { self.ended = true; self._wake(); });
        rs.on("close", function () { self.ended = true; self._wake(); });
        rs.on("error", function (e) { self.err = self.err || e; self._wake(); });
    }
    _wake() {
        const w = this.wake;
        this.wake = null;
        if (w) w();
    }
    // one more chunk into the queue; false at the end of the stream
    async _more() {
        for (;;) {
            if (this.err) throw this.err;
            const c = this.rs.read();
            if (c !== null) {
                this.bufs.push(c);
                this.have += c.length;
                return true;
            }
            if (this.ended) return false;
            const self = this;
            await new Promise(function (res) { self.wake = res; });
        }
    }
    _consume(n) {
        this.have -= n;
        while (n > 0) {
            const b = this.bufs[0];
            if (b.length <= n) {
                this.bufs.shift();
                n -= b.length;
            } else {
                this.bufs[0] = b.subarray(n);
                n = 0;
            }
        }
    }
    // {line, bytes} up to and without "\n", or null at the end of the stream
    async line(limit) {
        let scanned = 0;
        for (;;) {
            if (this.bufs.length > 1) this.bufs = [Buffer.concat(this.bufs, this.have)];
            const b = this.bufs[0];
            const nl = b ? b.indexOf(0x0a, scanned) : -1;
            if (nl >= 0) {
                const r = { line: b.toString("latin1", 0, nl), bytes: nl + 1 };
                this._consume(nl + 1);
                return r;
            }
            scanned = this.have;
            if (this.have > limit) throw new Error("y4m: header line longer than " + limit + " bytes");
            if (!(await this._more())) {
                if (!this.have) return null;
                throw new Error("y4m: stream ends inside a header line");
            }
        }
    }
    // fill dst; resolves to the bytes read (short at the end of the stream)
    async read(dst) {
        let off = 0;
        while (off < dst.length) {
            if (!this.have && !(await this._more())) break;
            const b = this.bufs[0], n = Math.min(b.length, dst.length - off);
            b.copy(dst, off, 0, n);
            this._consume(n);
            off += n;
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
        const got = fs.readSync(fd, one, 0, 1, pos + n);
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

// fill buf from a regular file at pos; returns the bytes read
function readFull(fd, buf, pos) {
    let off = 0;
    while (off < buf.length) {
        const n = fs.readSync(fd, buf, off, buf.length - off, pos + off);
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

// Random access to a Y4M regular file: frame i at a fixed offset.  read(i) is synchronous
// (fixtures, tests); readAsync(i) is what the worker uses (the reads run on the libuv pool).
class Y4MReader {
    // src: the path of a regular file (pipes, FIFOs and stdin: y4m.open -> Y4MStream)
    constructor(src) {
        this.path = src;
        if (!fs.statSync(src).isFile())             // (opening a FIFO would wait for its writer)
            throw new Error("y4m: " + src + " is not a regular file (read pipes through y4m.open)");
        this.fd = fs.openSync(src, "r");
        const st = fs.fstatSync(this.fd);
        this.seekable = true;
        const hl = readLine(this.fd, 0, MAX_HEADER);
        if (!hl) throw new Error("y4m: empty stream");
        this.hdr = parseHeader(hl.line);
        this.hdr.headerBytes = hl.bytes;
        this.bps = this.hdr.bits > 8 ? 2 : 1;
        this.frameBytes = frameBytes(this.hdr.w, this.hdr.h, this.bps);
        this.stride = 6 + this.frameBytes;                 // "FRAME\n" + planes (no frame parameters)
        this.frames = Math.floor((st.size - hl.bytes) / this.stride);
    }

    // frame i as a host frame for the addon, or null past the end of the file
    read(i) {
        if (i < 0) throw new Error("y4m: frame " + i);
        if (i >= this.frames) return null;
        const off = this.hdr.headerBytes + i * this.stride;
        const rec = Buffer.alloc(this.stride);
        if (readFull(this.fd, rec, off) !== rec.length) throw new Error("y4m: frame " + i + " is truncated");
        return this._frame(i, rec);
    }

    async readAsync(i) {
        if (i < 0) throw new Error("y4m: frame " + i);
        if (i >= this.frames) return null;
        const off = this.hdr.headerBytes + i * this.stride;
        const rec = Buffer.alloc(this.stride);
        let got = 0;
        while (got < rec.length) {
            const r = await readP(this.fd, rec, got, rec.length - got, off + got);
            if (r.bytesRead <= 0) break;
            got += r.bytesRead;
        }
        if (got !== rec.length) throw new Error("y4m: frame " + i + " is truncated");
        return this._frame(i, rec);
    }

    _frame(i, rec) {
        if (rec.toString("latin1", 0, 6) !== "FRAME\n")
            throw new Error("y4m: frame " + i + ": FRAME parameters need a stream (pipe) reader");
        return recordToFrame(rec.subarray(6), this.hdr.w, this.hdr.h, this.hdr.bits);
    }

    release() {}

    close() {
        if (this.fd !== null) fs.closeSync(this.fd);
        this.fd = null;
    }
}

// In-order reads of a Y4M byte stream (a Readable: a decoder child's stdout, a FIFO, stdin).
// open() resolves once the header is parsed; read(i) resolves to frame i (or null past the
// end).  Calls are served one after another in call order (two GPU slots may ask at once);
// every frame read is kept until release() drops it (segments are requested roughly in
// order, so at most a few segments are held; a frame may be asked for twice: vf_fps
// repeats, yadif context frames, two ladders of one source).
class Y4MStream {
    static async open(rs) {
        const q = new ByteQueue(rs);
        const hl = await q.line(MAX_HEADER);
        if (!hl) throw new Error("y4m: empty stream");
        return new Y4MStream(rs, q, hl);
    }
    constructor(rs, q, hl) {
        this.rs = rs;
        this.q = q;
        this.seekable = false;
        this.hdr = parseHeader(hl.line);
        this.hdr.headerBytes = hl.bytes;
        this.bps = this.hdr.bits > 8 ? 2 : 1;
        this.frameBytes = frameBytes(this.hdr.w, this.hdr.h, this.bps);
        this.frames = Infinity;                            // known at the end of the stream
        this.next = 0;                                     // index of the next record in the stream
        this.kept = new Map();                             // frames read, not yet released
        this.chain = Promise.resolve();
    }

    read(i) {
        const self = this;
        const p = this.chain.then(function () { return self._read(i); });
        this.chain = p.catch(function () {});
        return p;
    }

    async _read(i) {
        if (i < 0) throw new Error("y4m: frame " + i);
        if (this.kept.has(i)) return this.kept.get(i);
        if (i < this.next) throw new Error("y4m: frame " + i + " of a stream was already released");
        while (this.next <= i) {
            if (this.next >= this.frames) return null;
            const tl = await this.q.line(MAX_HEADER);
            if (!tl) {
                this.frames = this.next;
                return null;
            }
            if (tl.line.slice(0, 5) !== "FRAME") throw new Error("y4m: record " + this.next + " is not a FRAME");
            const rec = Buffer.alloc(this.frameBytes);
            if ((await this.q.read(rec)) !== rec.length) throw new Error("y4m: frame " + this.next + " is truncated");
            this.kept.set(this.next++, recordToFrame(rec, this.hdr.w, this.hdr.h, this.hdr.bits));
        }
        return this.kept.get(i);
    }

    // forget the frames below `below` (no pending segment asks for them again)
    release(below) {
        const self = this;
        Array.from(this.kept.keys()).forEach(function (k) { if (k < below) self.kept.delete(k); });
    }

    close() {
        this.kept.clear();
        if (this.rs && this.rs !== process.stdin) this.rs.destroy();
        this.rs = null;
    }
}

// A source by path: a regular file -> Y4MReader (random access); "-" -> stdin, any other
// path (a FIFO, a device) -> opened on the libuv pool (a FIFO's open waits for its writer
// there, not on the event loop) and polled as a pipe -> Y4MStream.
async function open(src) {
    if (src === "-") return Y4MStream.open(process.stdin);
    if (fs.statSync(src).isFile()) return new Y4MReader(src);
    const fd = await require("util").promisify(fs.open)(src, "r");
    const sock = new (require("net").Socket)({ fd: fd, readable: true, writable: false });
    try {
        return await Y4MStream.open(sock);
    } catch (e) {
        sock.destroy();
        throw e;
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

// A synchronous writer of a regular file (fixtures, tests): the header, then one record
// per frame as it comes (a segment of any size never sits in memory as one Buffer)
class Y4MWriter {
    constructor(path, w, h, fps, fmt) {
        this.fd = fs.openSync(path, "w");
        this.w = w;
        this.h = h;
        this.fmt = fmt;
        this.bytes = 0;
        this.frames = 0;
        this._put(header(w, h, fps, fmt));
    }

    _put(buf) {
        let off = 0;
        while (off < buf.length) off += fs.writeSync(this.fd, buf, off, buf.length - off);
        this.bytes += buf.length;
    }

    write(frame) {
        this._put(frameRecord(frame, this.w, this.h, this.fmt));
        ++this.frames;
    }

    close() {
        if (this.fd !== null) fs.closeSync(this.fd);
        this.fd = null;
        return this.bytes;
    }
}

// The worker's sink: Y4M records into a Writable (an encoder child's stdin, a file stream).
// write(frame) resolves once the Writable takes more (its 'drain'), so at most one record
// per sink waits in memory and a slow consumer holds back only its own writer; a failed
// Writable (EPIPE: the encoder died) rejects the pending and every later write.
class Y4MSink {
    constructor(ws, w, h, fps, fmt) {
        this.ws = ws;
        this.w = w;
        this.h = h;
        this.fmt = fmt;
        this.bytes = 0;
        this.frames = 0;
        this.err = null;
        this.waiters = [];
        const self = this;
        ws.on("error", function (e) {
            self.err = self.err || e;
            self._wake();
        });
        ws.on("drain", function () { self._wake(); });
        this.pending = this._put(header(w, h, fps, fmt));
    }
    _wake() {
        const ws = this.waiters;
        this.waiters = [];
        ws.forEach(function (f) { f(); });
    }
    async _put(buf) {
        if (this.err) throw this.err;
        this.bytes += buf.length;
        if (this.ws.write(buf)) return;
        const self = this;
        await new Promise(function (res) { self.waiters.push(res); });
        if (this.err) throw this.err;
    }
    async write(frame) {
        await this.pending;
        this.pending = this._put(frameRecord(frame, this.w, this.h, this.fmt));
        ++this.frames;
        return this.pending;
    }
    // resolves with the bytes written once the Writable has flushed them ('finish')
    async end() {
        await this.pending;
        if (this.err) throw this.err;
        const self = this;
        await new Promise(function (res, rej) {
            if (self.err) return rej(self.err);
            self.waiters.push(function () { if (self.err) rej(self.err); });
            self.ws.end(function () { res(); });
        });
        return this.bytes;
    }
}

// a rendition segment as a Y4M file, written through a file stream (the libuv pool); resolves
// to the bytes written
async function writeSegment(path, frames, w, h, fmt, fps) {
    const ws = fs.createWriteStream(path);
    const sink = new Y4MSink(ws, w, h, fps, fmt);
    try {
        for (let i = 0; i < frames.length; ++i) await sink.write(frames[i]);
        const n = await sink.end();
        await new Promise(function (res) { if (ws.closed || ws.destroyed) res(); else ws.once("close", res); });
        return n;
    } catch (e) {
        ws.destroy();
        throw e;
    }
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

module.exports = { Y4MReader: Y4MReader, Y4MStream: Y4MStream, Y4MWriter: Y4MWriter, Y4MSink: Y4MSink, open: open,
                   parseHeader: parseHeader, frameBytes: frameBytes,
                   header: header, frameRecord: frameRecord, writeSegment: writeSegment, writeFile: writeFile,
                   headerBytes: headerBytes, recordToFrame: recordToFrame,
                   FMT_YUV420P: FMT_YUV420P, FMT_NV12: FMT_NV12, FMT_P010LE: FMT_P010LE };
