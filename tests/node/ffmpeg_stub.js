#!/usr/bin/env node
"use strict";
// A stand-in for the ffmpeg binary (the image has none; tests only).  It speaks the three
// command lines node/ffpipe.js builds and logs each argv as a JSON line to $STUB_LOG:
//   ... -i SOURCE -f yuv4mpegpipe -pix_fmt PF ... -      decode: SOURCE is a Y4M file under any
//                                                           name, copied to stdout
//   ... -f yuv4mpegpipe -i - -c:v ENC [-b:v B] ... -y OUT  encode: "STUBENC <json argv>\n" and the
//                                                           Y4M stream from stdin into OUT
//   ... -f concat -safe 0 -i LIST -c copy -y OUT           concat: the listed files into OUT
const fs = require("fs");
const argv = process.argv.slice(2);
if (process.env.STUB_LOG) fs.appendFileSync(process.env.STUB_LOG, JSON.stringify(argv) + "\n");
const at = function (flag) { const i = argv.indexOf(flag); return i >= 0 ? argv[i + 1] : null; };
const out = argv[argv.length - 1];
if (at("-f") === "concat") {
    const files = fs.readFileSync(at("-i"), "utf8").split("\n").filter(function (l) { return l; })
        .map(function (l) { return l.replace(/^file '/, "").replace(/'$/, ""); });
    fs.writeFileSync(out, Buffer.concat(files.map(function (f) { return fs.readFileSync(f); })));
} else if (at("-i") === "-") {
    // $STUB_ENC_MS_PER_FRAME: consume at most one Y4M frame record per that many ms (a slow
    // encoder: the pipe fills and the writer has to wait); $STUB_TIMES: append
    // {out, t0, t1} (first input byte, end of the "encode", ms since the epoch)
    const msPer = Number(process.env.STUB_ENC_MS_PER_FRAME || 0);
    const chunks = [];
    let total = 0, rec = 0, t0 = 0;
    process.stdin.on("data", function (d) {
        if (!t0) t0 = Date.now();
        chunks.push(d);
        total += d.length;
        if (!msPer) return;
        if (!rec) {
            const hdr = Buffer.concat(chunks).toString("latin1");
            const nl = hdr.indexOf("\n");
            if (nl < 0) return;
            const tok = hdr.slice(0, nl).split(" ");
            const w = parseInt(tok.find(function (t) { return t[0] === "W"; }).slice(1), 10);
            const h = parseInt(tok.find(function (t) { return t[0] === "H"; }).slice(1), 10);
            const bps = /C420p10/.test(hdr.slice(0, nl)) ? 2 : 1;
            rec = 6 + (w * h + 2 * ((w + 1) >> 1) * ((h + 1) >> 1)) * bps;
        }
        const due = t0 + Math.floor(total / rec) * msPer - Date.now();
        if (due > 0) {
            process.stdin.pause();
            setTimeout(function () { process.stdin.resume(); }, due);
        }
    });
    process.stdin.on("end", function () {
        // the last frames still "encode" after EOF (a pipe holds several small records)
        const due = rec ? t0 + Math.floor(total / rec) * msPer - Date.now() : 0;
        setTimeout(function () {
            fs.writeFileSync(out, Buffer.concat([Buffer.from("STUBENC " + JSON.stringify(argv) + "\n"), Buffer.concat(chunks)]));
            if (process.env.STUB_TIMES)
                fs.appendFileSync(process.env.STUB_TIMES, JSON.stringify({ out: out, t0: t0, t1: Date.now() }) + "\n");
        }, Math.max(0, due));
    });
} else {
    const data = fs.readFileSync(at("-i"));
    let off = 0;
    (function pump() {                        // in pieces, so the reader sees a live pipe
        while (off < data.length) {
            const n = Math.min(65536, data.length - off);
            const ok = process.stdout.write(data.slice(off, off + n));
            off += n;
            if (!ok) return process.stdout.once("drain", pump);
        }
    })();
}
