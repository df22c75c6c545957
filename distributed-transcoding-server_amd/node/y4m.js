"use strict";
// y4m.js -- YUV4MPEG2 (rawvideo) source and sink of the GPU worker (SURVEY.md §8f
// rows f2 / a14).  The reference's worker would hand ffmpeg-static a segment of the
// job's source and collect the encoded renditions (index.js:9; Jobs.codec /
// codecSettings, database.js:76-78).  libavcodec is not part of this build, so the
// worker's file interface is the uncompressed one ffmpeg itself reads and writes
// (`-f yuv4mpegpipe`): 8-bit 4:2:0, one "FRAME" record per picture.  Decode /
// encode slot in before / after this module (segment frames in, rendition frames
// out) without changing the scheduler.
//
// Node 12: no `??` / `?.`.

const fs = require("fs");

const FMT_YUV420P = 0, FMT_NV12 = 1;

function frameBytes(w, h) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    return w * h + 2 * cw * ch;
}

// "YUV4MPEG2 W3840 H2160 F60:1 Ip A1:1 C420mpeg2\n" -> {w, h, fps: [n, d], chroma, headerBytes}
function parseHeader(buf) {
    const nl = buf.indexOf(0x0a);
    if (nl < 0) throw new Error("y4m: no header line");
    const line = buf.toString("latin1", 0, nl);
    const tok = line.split(" ");
    if (tok[0] !== "YUV4MPEG2") throw new Error("y4m: not a YUV4MPEG2 stream");
    const h = { w: 0, h: 0, fps: [25, 1], chroma: "420jpeg", interlace: "p", headerBytes: nl + 1 };
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
    if (!/^420(jpeg|mpeg2|paldv)?$/.test(h.chroma)) throw new Error("y4m: only 8-bit 4:2:0 is supported (C" + h.chroma + ")");
    return h;
}

class Y4MReader {
    constructor(path) {
        this.path = path;
        this.fd = fs.openSync(path, "r");
        const head = Buffer.alloc(512);
        const n = fs.readSync(this.fd, head, 0, head.length, 0);
        this.hdr = parseHeader(head.slice(0, n));
        this.frameBytes = frameBytes(this.hdr.w, this.hdr.h);
        this.stride = 6 + this.frameBytes;                 // "FRAME\n" + planes (no frame parameters)
        const size = fs.fstatSync(this.fd).size;
        this.frames = Math.floor((size - this.hdr.headerBytes) / this.stride);
    }

    // frame i as a yuv420p host frame for the addon ({data: [Y, U, V], pitch})
    read(i) {
        if (i < 0 || i >= this.frames) throw new Error("y4m: frame " + i + " out of range (" + this.frames + ")");
        const off = this.hdr.headerBytes + i * this.stride;
        const tag = Buffer.alloc(6);
        fs.readSync(this.fd, tag, 0, 6, off);
        if (tag.toString("latin1") !== "FRAME\n") throw new Error("y4m: frame " + i + ": FRAME parameters are not supported");
        const w = this.hdr.w, h = this.hdr.h, cw = (w + 1) >> 1, ch = (h + 1) >> 1;
        const all = Buffer.alloc(this.frameBytes);
        fs.readSync(this.fd, all, 0, this.frameBytes, off + 6);
        return { data: [all.slice(0, w * h), all.slice(w * h, w * h + cw * ch), all.slice(w * h + cw * ch)],
                 pitch: [w, cw, cw] };
    }

    close() {
        if (this.fd !== null) fs.closeSync(this.fd);
        this.fd = null;
    }
}

function header(w, h, fps) {
    const f = fps || [25, 1];
    return Buffer.from("YUV4MPEG2 W" + w + " H" + h + " F" + f[0] + ":" + f[1] + " Ip A1:1 C420mpeg2\n", "latin1");
}

// One host frame (yuv420p planes, or nv12 Y + interleaved UV) as a Y4M FRAME record
// (planar 4:2:0: nv12 chroma is de-interleaved, as ffmpeg's yuv4mpegpipe muxer needs)
function frameRecord(f, w, h, fmt) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    const out = Buffer.alloc(6 + frameBytes(w, h));
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
        throw new Error("y4m: 8-bit 4:2:0 renditions only (fmt " + fmt + ")");
    }
    return out;
}

// write a whole rendition segment; returns the bytes written
function writeSegment(path, frames, w, h, fmt, fps) {
    const parts = [header(w, h, fps)];
    frames.forEach(function (f) { parts.push(frameRecord(f, w, h, fmt)); });
    const buf = Buffer.concat(parts);
    fs.writeFileSync(path, buf);
    return buf.length;
}

// a complete Y4M file from frames made by gen(i) (tests, fixtures)
function writeFile(path, w, h, fps, n, gen) {
    const fd = fs.openSync(path, "w");
    fs.writeSync(fd, header(w, h, fps));
    for (let i = 0; i < n; ++i) fs.writeSync(fd, frameRecord(gen(i), w, h, FMT_YUV420P));
    fs.closeSync(fd);
}

module.exports = { Y4MReader: Y4MReader, parseHeader: parseHeader, frameBytes: frameBytes, header: header,
                   frameRecord: frameRecord, writeSegment: writeSegment, writeFile: writeFile };
