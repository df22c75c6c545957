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
    const chunks = [];
    process.stdin.on("data", function (d) { chunks.push(d); });
    process.stdin.on("end", function () {
        fs.writeFileSync(out, Buffer.concat([Buffer.from("STUBENC " + JSON.stringify(argv) + "\n"), Buffer.concat(chunks)]));
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
