"use strict";
// CPU test of node/ffpipe.js (the ffmpeg process boundary) with tests/node/ffmpeg_stub.js as
// the binary: a decoder child's yuv4mpegpipe read in order, an encoder child fed the same
// frames with the Jobs row's codec / bitrate / encoderArgs, and the concat of two segments.
const assert = require("assert");
const fs = require("fs");
const os = require("os");
const path = require("path");
const NODE = path.join(__dirname, "..", "..", "distributed-transcoding-server_amd", "node");
const ffpipe = require(path.join(NODE, "ffpipe"));
const y4m = require(path.join(NODE, "y4m"));

const dir = fs.mkdtempSync(path.join(os.tmpdir(), "ffpipe-"));
const stub = path.join(__dirname, "ffmpeg_stub.js");
process.env.STUB_LOG = path.join(dir, "argv.log");
const w = 48, h = 20, n = 5;
function gen(i) {
    const cw = w >> 1, ch = h >> 1;
    const f = { data: [Buffer.alloc(w * h, i), Buffer.alloc(cw * ch, 100 + i), Buffer.alloc(cw * ch, 200 - i)],
                pitch: [w, cw, cw] };
    f.data[0][3] = 7 * i;
    return f;
}
const src = path.join(dir, "in.mkv");                    // a Y4M file under a container's name
y4m.writeFile(src, w, h, [30, 1], n, gen);

(async function () {
    assert.strictEqual(ffpipe.ffmpegBinary({ ffmpeg: stub }), stub);
    assert.deepStrictEqual(ffpipe.codecOf({ codec: "vp9" }), { encoder: "libvpx-vp9", ext: "webm" });
    assert.deepStrictEqual(ffpipe.encodeArgs({ codec: "h264", bitrate: 3000000 }, { encoderArgs: ["-preset", "fast"] }),
                           ["-c:v", "libx264", "-b:v", "3000000", "-preset", "fast"]);
    // decode: frames in order from the child's pipe
    const dec = await ffpipe.FfmpegDecoder.open(stub, src, { fmt: 0 });
    assert.strictEqual(dec.hdr.w, w);
    const frames = [];
    for (let i = 0; ; ++i) {
        const f = await dec.read(i);
        if (!f) break;
        assert.strictEqual(f.data[0][0], i);
        assert.strictEqual(f.data[0][3], 7 * i);
        frames.push(f);
        dec.release(i);
    }
    assert.strictEqual(frames.length, n);
    assert.strictEqual(dec.frames, n);
    dec.close();
    // encode: two segments, then their concat
    const segs = [];
    for (let s = 0; s < 2; ++s) {
        const out = path.join(dir, s + ".mp4");
        const r = await ffpipe.encodeSegment(stub, out, frames.slice(s * 3, s * 3 + 3), w, h, 0, [30, 1],
                                             { codec: "h264", bitrate: 2500000 }, { encoderArgs: ["-crf", "20"] });
        assert.strictEqual(r.file, out);
        assert.strictEqual(r.bytes, fs.statSync(out).size);
        assert.ok(r.encodeMs >= 0);
        const body = fs.readFileSync(out);
        const nl = body.indexOf(0x0a);
        const args = JSON.parse(body.toString("utf8", 8, nl));
        assert.deepStrictEqual(args.slice(args.indexOf("-c:v"), args.indexOf("-c:v") + 6),
                               ["-c:v", "libx264", "-b:v", "2500000", "-crf", "20"]);
        const expect = Buffer.concat([y4m.header(w, h, [30, 1], 0)].concat(frames.slice(s * 3, s * 3 + 3).map(function (f) {
            return y4m.frameRecord(f, w, h, 0);
        })));
        assert.ok(body.slice(nl + 1).equals(expect), "segment " + s + " carries the Y4M records");
        segs.push(out);
    }
    const all = await ffpipe.concatSegments(stub, segs, path.join(dir, "output.mp4"));
    assert.ok(fs.readFileSync(all).equals(Buffer.concat(segs.map(function (f) { return fs.readFileSync(f); }))));
    // a failing encoder is an error, not a hang
    await ffpipe.encodeSegment("/bin/false", path.join(dir, "x.mp4"), frames.slice(0, 1), w, h, 0, [30, 1],
                               { codec: "h264" }, {}).then(function () { assert.fail("no error"); }, function (e) {
        assert.ok(/ffmpeg encode/.test(e.message), e.message);
    });
    const log = fs.readFileSync(process.env.STUB_LOG, "utf8").trim().split("\n").map(JSON.parse);
    assert.ok(log.some(function (a) { return a.indexOf("yuv4mpegpipe") >= 0 && a.indexOf(src) >= 0; }));
    assert.ok(log.some(function (a) { return a.indexOf("concat") >= 0; }));
    console.log("ok");
})().catch(function (e) {
    console.error(e && e.stack || e);
    process.exit(1);
});
