"use strict";
// scheduler.js -- GPU-slot-aware segment scheduler and the JobChunks state
// machine of the GPU worker (SURVEY.md §8e / §8f rank 1).
//
// The reference keeps segments as `job_chunks` rows (database.js:97-129:
// mainJob, chunkOffset, assignedTo, status, result) and reads them back per job
// (index.js:178-209), but its dispatch is empty (index.js:13: socket.io with no
// handlers).  This module is that dispatch for one GPU node:
//
//   * segments are independent (no data exchange): every (ladder, chunkOffset)
//     pair is one task, pulled by whichever GPU slot is free first (a shared
//     work queue = least-loaded assignment, no static i mod G split);
//   * one libdts context per GPU, one graph per (ladder, GPU), created lazily
//     and reused for every segment of the ladder;
//   * a chunk row goes null -> "assigned" -> "processing" -> "done", or back to
//     the queue on failure (another GPU first) until maxRetries, then "failed";
//     `assignedTo` is the worker account id, `result` a JSON record (frames,
//     output bytes, sha1 of each rendition, GPU, ms, quality);
//   * every status change is reported through `onUpdate(row, fields)`, which is
//     where a maintainer calls JobChunks.update(...) (database.js:97-129);
//   * with `outDir`, the source comes from the Y4M file named by the source row
//     (`sources[id].path`) and every rendition segment is written as
//     outDir/job<id>/<chunkOffset>.y4m; once all of a job's chunks are done the
//     segments are assembled into Jobs.assembledData = {size, chunk: [1 MiB block
//     ids]} (assemble.js) and reported through `onJobUpdate(job, fields)`;
//   * with an ffmpeg binary (opts.ffmpeg, $DTS_FFMPEG, ffmpeg-static or PATH; ffpipe.js), a
//     source row may name a compressed file (`decode: "ffmpeg"`, or any path that is not
//     .y4m): an ffmpeg child decodes it into a yuv4mpegpipe the worker reads in order; and
//     with `encode` each rendition segment goes to an ffmpeg child encoding it with the Jobs
//     row's codec / bitrate / codecSettings.encoderArgs (outDir/job<id>/<off>.mp4|webm|mkv),
//     a finished job's segments stream-copied into one file before its blocks are cut;
//   * `result` carries per-phase timings (readMs, gpuMs, qualityMs, writeMs; encodeMs) and,
//     for rows whose codecSettings ask for it, the segment's PSNR / SSIM against
//     the reference rendition (ladder.js qualityOf) with its summed record (`raw`);
//     a job whose chunks are all done gets the whole stream's averages (Jobs row
//     field `quality`, from the summed records: vf_psnr / vf_ssim end of stream).
//
// The addon's run() executes on the libuv thread pool: set UV_THREADPOOL_SIZE
// >= the GPU count before the first async call (worker.js does).  Source reads, encoder
// feeds and segment writes are asynchronous too (y4m.js / ffpipe.js): while one slot's
// segment is decoding or encoding, the event loop completes and starts the other slots'.
// Node 12: no `??` / `?.`.

const crypto = require("crypto");
const EventEmitter = require("events");
const fs = require("fs");
const path = require("path");
const ladder = require("./ladder");
const y4m = require("./y4m");
const assemble = require("./assemble");
const ffpipe = require("./ffpipe");

function planeShapes(w, h, fmt) {
    const cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    if (fmt === 0) return [[h, w], [ch, cw], [ch, cw]];
    if (fmt === 1) return [[h, w], [ch, 2 * cw], null];
    return [[h, 2 * w], [ch, 4 * cw], null];
}

// a tightly packed host frame for the addon: {data: [Buffer...], pitch: [...]}
function allocFrame(w, h, fmt) {
    const data = [], pitch = [];
    planeShapes(w, h, fmt).forEach(function (s) {
        data.push(s ? Buffer.alloc(s[0] * s[1]) : null);
        pitch.push(s ? s[1] : 0);
    });
    return { data: data, pitch: pitch };
}

// A source maps (plan, frame indices) to host frames, each carrying its source index
// (`frame.index`); indices past the end of the stream are dropped (the last segment of
// a job is usually short).
// default source: the deterministic testsrc2-like generator of libdts (the
// segment's frames are its global frame indices); a real deployment passes a
// decoder here (host libavcodec, out of the GPU path)
function synthSource(addon, seed) {
    return function (plan, frameIdx) {
        const s = plan.spec.src;
        return frameIdx.map(function (i) {
            const f = allocFrame(s.w, s.h, s.fmt);
            addon.synthFrame(s.w, s.h, s.fmt, 0, seed >>> 0, i, f);
            f.index = i;
            return f;
        });
    };
}

// Y4M source (a file read at random: y4m.Y4MReader.readAsync, or a pipe read in order:
// y4m.Y4MStream / an ffmpeg decoder child).  Each index is read once per request (vf_fps may
// repeat a frame); a stream reader keeps the frames it has read until the scheduler
// releases them (release(sourceID, below)).  Reads resolve asynchronously: the event loop
// keeps serving the other GPU slots while a segment's frames arrive.
function y4mSource(readers) {
    const src = async function (plan, frameIdx) {
        const r = readers[plan.sourceID];
        if (!r) throw new Error("source " + plan.sourceID + " has no Y4M path");
        const got = new Map();
        for (let k = 0; k < frameIdx.length; ++k) {
            const i = frameIdx[k];
            if (got.has(i) || i >= r.frames) continue;
            const f = r.readAsync ? await r.readAsync(i) : await r.read(i);
            if (f) {
                f.index = i;
                got.set(i, f);
            }
        }
        return frameIdx.filter(function (i) { return got.has(i); }).map(function (i) { return got.get(i); });
    };
    src.release = function (sourceID, below) {
        const r = readers[sourceID];
        if (r && r.release) r.release(below);
    };
    return src;
}

// a regular file that starts with the YUV4MPEG2 signature, or anything that is not a regular
// file (a pipe, a FIFO, "-": read as Y4M, never sniffed)
function isY4MFile(p) {
    if (p === "-") return true;
    try {
        if (!fs.statSync(p).isFile()) return true;
        const fd = fs.openSync(p, "r"), b = Buffer.alloc(9);
        try {
            return fs.readSync(fd, b, 0, 9, 0) === 9 && b.toString("latin1") === "YUV4MPEG2";
        } finally {
            fs.closeSync(fd);
        }
    } catch (e) {
        return true;                          // let the Y4M reader report it
    }
}

class GpuSegmentScheduler extends EventEmitter {
    // opts: addon (dts_napi.node or a stand-in), gpus ([device...], default all),
    // workerId (WorkerAccounts id written to assignedTo), maxRetries (2),
    // segmentFrames (source frames per chunk), source (plan, frameIdx) -> frames,
    // sink (plan, chunkRows, outputs[k][f]) -> Promise|void, onUpdate(row, fields)
    constructor(opts) {
        super();
        this.addon = opts.addon;
        const n = opts.gpus ? opts.gpus.length : this.addon.deviceCount();
        if (!n) throw new Error("no GPU slots (deviceCount() == 0): the GPU worker has no CPU fallback");
        this.gpus = opts.gpus ? opts.gpus.slice() : Array.from({ length: n }, function (_, i) { return i; });
        this.workerId = opts.workerId === undefined ? null : opts.workerId;
        this.maxRetries = opts.maxRetries === undefined ? 2 : opts.maxRetries;
        this.segmentFrames = opts.segmentFrames || 600;
        this.source = opts.source || synthSource(this.addon, 0x5EED);
        this._userSource = !!opts.source;
        this.sink = opts.sink || null;
        this.outDir = opts.outDir || null;
        this.ffmpeg = ffpipe.ffmpegBinary(opts);              // null: Y4M files only
        this.encode = !!opts.encode;
        if (this.encode && !this.ffmpeg) throw new Error("encode needs an ffmpeg binary (DTS_FFMPEG / ffmpeg-static / PATH)");
        this.onUpdate = opts.onUpdate || function () {};
        this.onJobUpdate = opts.onJobUpdate || function () {};
        this.readers = {};
        // a slot = one libdts context on one device; several slots may share a device
        // (gpus: [0, 0] drives GPU 0 from two libuv threads)
        this.slots = this.gpus.map(function (dev, i) {
            return { id: i, dev: dev, ctx: null, graphs: new Map(), busy: false, done: 0, failed: 0, ms: 0 };
        });
    }

    _ctx(slot) {
        if (!slot.ctx) slot.ctx = this.addon.createContext(slot.dev);
        return slot.ctx;
    }

    _graph(slot, plan) {
        if (!slot.graphs.has(plan.key)) slot.graphs.set(plan.key, this.addon.createGraph(this._ctx(slot), plan.spec));
        return slot.graphs.get(plan.key);
    }

    _segmentPath(jobId, off, ext) {
        return path.join(this.outDir, "job" + jobId, off + "." + (ext || "y4m"));
    }

    _update(row, fields) {
        Object.keys(fields).forEach(function (k) { row[k] = fields[k]; });
        this.onUpdate(row, fields);
        this.emit("update", row, fields);
    }

    // frames of segment `off` in source-frame indices, after the vf_fps map
    _frames(plan, off, srcFps) {
        const n = this.segmentFrames, base = off * n;
        const map = ladder.fpsFrames(this.addon, n, srcFps, plan.framerate);
        const local = map ? Array.from(map) : Array.from({ length: n }, function (_, i) { return i; });
        return local.map(function (i) { return base + i; });
    }

    _allocOutputs(outs, n) {
        const dst = [], per = outs.map(function () { return []; });
        for (let i = 0; i < n; ++i)
            outs.forEach(function (o, k) {
                const f = allocFrame(o.w, o.h, o.fmt);
                dst.push(f);
                per[k].push(f);
            });
        return { dst: dst, per: per };
    }

    async _runSegment(slot, task) {
        const self = this;
        const plan = task.plan;
        const t0 = Date.now();
        const g = this._graph(slot, plan);
        const idx = this._frames(plan, task.chunkOffset, plan.srcFps);
        let sel = null, src;
        if (plan.spec.deint) {
            // yadif needs each frame's neighbours in the source stream: the graph runs on the
            // segment's contiguous frames plus one context frame each side (yadif's clone of
            // the first / last frame at the stream ends); the vf_fps selection is applied to
            // its outputs.  The stream's length need not be known up front (a pipe).
            const segN = this.segmentFrames, base = task.chunkOffset * segN;
            const want = (base > 0 ? [base - 1] : []).concat(Array.from({ length: segN + 1 }, function (_, i) { return base + i; }));
            const got = await this.source(plan, want);
            const real = got.filter(function (f) { return f.index >= base && f.index < base + segN; });
            const n = real.length;
            sel = idx.map(function (i) { return i - base; }).filter(function (i) { return i < n; });
            src = [];
            if (n) {
                const prev = got.find(function (f) { return f.index === base - 1; }) || real[0];
                const next = got.find(function (f) { return f.index === base + n; }) || real[n - 1];
                src = [prev].concat(real, [next]);
            }
        } else {
            src = await this.source(plan, idx);
        }
        const t1 = Date.now();
        const outs = plan.spec.outputs;
        const nout = plan.spec.deint ? Math.max(0, src.length - 2) : src.length;
        const o = this._allocOutputs(outs, nout);
        // with rendition quality the graph also returns, per frame, each rendition's vf_psnr /
        // vf_ssim against its reference rendition (made and scored on the GPU: qs[f][k])
        let qs = nout ? await this.addon.run(g, src, o.dst, null) : null;
        if (sel) {
            o.per = o.per.map(function (fr) { return sel.map(function (j) { return fr[j]; }); });
            if (qs) qs = sel.map(function (j) { return qs[j]; });
        }
        const t2 = Date.now();
        const quality = outs.map(function () { return null; });
        if (plan.quality && qs && qs.length) {
            for (let k = 0; k < outs.length; ++k) {
                if (!plan.quality.rows[k]) continue;
                const st = qs.map(function (fq) { return fq[k]; });
                const sum = this._qsummary(ladder.rawQuality(st, outs[k].w, outs[k].h), outs[k].w, outs[k].h);
                if (!(plan.quality.rows[k] & 1)) delete sum.psnr;
                if (!(plan.quality.rows[k] & 2)) delete sum.ssim;
                quality[k] = sum;
            }
        }
        const t3 = Date.now();
        const files = outs.map(function () { return null; }), written = outs.map(function () { return 0; });
        const encMs = outs.map(function () { return null; });
        if (this.sink) {
            await this.sink(plan, task.rows, o.per);
        } else if (this.outDir) {
            const fps = plan.framerate ? ladder.rateOf(plan.framerate) : (plan.srcFps || [25, 1]);
            const ks = [], items = [];
            task.rows.forEach(function (row, k) {
                if (!row) return;
                const job = plan.jobs[k];
                const p = self._segmentPath(row.mainJob, row.chunkOffset, self.encode ? ffpipe.codecOf(job).ext : "y4m");
                fs.mkdirSync(path.dirname(p), { recursive: true });
                ks.push(k);
                items.push({ out: p, frames: o.per[k], w: outs[k].w, h: outs[k].h, fmt: outs[k].fmt, fps: fps, job: job,
                             settings: ladder.parseSettings(job.codecSettings) });
            });
            if (this.encode) {
                // an ffmpeg child per rendition segment, all started before the first frame and
                // fed concurrently (ffpipe.encodeRenditions); the event loop stays free meanwhile
                const rs = await ffpipe.encodeRenditions(this.ffmpeg, items);
                rs.forEach(function (r, i) {
                    files[ks[i]] = r.file;
                    written[ks[i]] = r.bytes;
                    encMs[ks[i]] = r.encodeMs;
                });
            } else {
                const ns = await Promise.all(items.map(function (it) {
                    return y4m.writeSegment(it.out, it.frames, it.w, it.h, it.fmt, it.fps);
                }));
                ns.forEach(function (n, i) {
                    files[ks[i]] = items[i].out;
                    written[ks[i]] = n;
                });
            }
        }
        const t4 = Date.now();
        return task.rows.map(function (row, k) {
            const h = crypto.createHash("sha1");
            let bytes = 0;
            o.per[k].forEach(function (f) {
                f.data.forEach(function (b) { if (b) { h.update(b); bytes += b.length; } });
            });
            const r = { frames: o.per[k].length, bytes: bytes, sha1: h.digest("hex"), gpu: slot.dev, slot: slot.id, ms: t4 - t0,
                        readMs: t1 - t0, gpuMs: t2 - t1, qualityMs: t3 - t2, writeMs: t4 - t3,
                        width: outs[k].w, height: outs[k].h, fmt: outs[k].fmt };
            if (quality[k]) r.quality = quality[k];
            if (encMs[k] !== null) {
                r.encodeMs = encMs[k];
                r.codec = plan.jobs[k].codec;
            }
            if (files[k]) {
                r.file = files[k];
                r.fileBytes = written[k];
            }
            return r;
        });
    }

    // vf_psnr / vf_ssim end-of-stream averages of a summed record (the addon's
    // dts_qstat_stream when it has it, else the same formulas in ladder.js)
    _qsummary(raw, w, h) {
        const r = this.addon.qstatStream ? ladder.summaryOfStat(this.addon.qstatStream(w, h, raw.sse, raw.ssimSum, raw.frames), raw)
                                         : ladder.summarizeRaw(raw, w, h);
        r.raw = raw;
        return r;
    }

    // A job whose chunks are all here and done: chunkOffsets exactly 0 .. Jobs.chunks - 1
    // (database.js:79).  A worker that was given only some of a job's chunks -- the usual
    // case in a pool -- leaves the job alone (ADVICE r02: it used to publish a truncated
    // output as finished); the worker the job names in Jobs.assemble gets every row.
    _completeJob(job, chunks) {
        const mine = chunks.filter(function (c) { return c.mainJob === job.id; });
        if (!mine.length || mine.some(function (c) { return c.status !== "done"; })) return null;
        mine.sort(function (a, b) { return a.chunkOffset - b.chunkOffset; });
        const n = typeof job.chunks === "number" ? job.chunks : NaN;
        if (mine.length !== n || mine.some(function (c, i) { return c.chunkOffset !== i; })) return null;
        return mine;
    }

    // every chunk of a job done -> the job's quality (every segment's summed record,
    // combined as vf_psnr / vf_ssim average a whole stream) and, with outDir, its
    // segments assembled into 1 MiB blocks of one Y4M stream
    async _assembleJobs(jobs, chunks) {
        const self = this;
        for (let ji = 0; ji < jobs.length; ++ji) {
            const job = jobs[ji];
            const mine = self._completeJob(job, chunks);
            if (!mine) continue;
            try {
                const fields = {};
                const recs = mine.map(function (c) {
                    try {
                        return JSON.parse(c.result || "{}");
                    } catch (e) {
                        return {};
                    }
                });
                if (recs.every(function (r) { return r.quality && r.quality.raw; })) {
                    const raw = ladder.addRaw(recs.map(function (r) { return r.quality.raw; }));
                    const q = self._qsummary(raw, recs[0].width, recs[0].height);
                    delete q.raw;
                    q.segments = mine.length;
                    fields.quality = JSON.stringify(q);
                }
                if (self.outDir && !self.sink) {
                    const ext = self.encode ? ffpipe.codecOf(job).ext : "y4m";
                    const files = mine.map(function (c, i) { return recs[i].file || self._segmentPath(job.id, c.chunkOffset, ext); });
                    const a = self.encode
                        ? assemble.assembleFiles([await ffpipe.concatSegments(self.ffmpeg, files,
                                                                              path.join(self.outDir, "job" + job.id, "output." + ext))],
                                                 path.join(self.outDir, "blocks"))
                        : assemble.assembleY4M(files, path.join(self.outDir, "blocks"));
                    fields.assembledData = JSON.stringify(a);
                    fields.finished = true;
                }
                if (!Object.keys(fields).length) continue;
                Object.keys(fields).forEach(function (k) { job[k] = fields[k]; });
                self.onJobUpdate(job, fields);
                self.emit("jobUpdate", job, fields);
            } catch (e) {
                self.emit("updateError", e, job, null);
            }
        }
    }

    // a stream source keeps frames until no pending segment can ask for them again
    _releaseFrames(queue, inflight) {
        if (!this.source.release) return;
        const self = this, low = new Map();
        queue.concat(inflight).forEach(function (t) {
            const sid = String(t.plan.sourceID), b = t.chunkOffset * self.segmentFrames - 1;
            low.set(sid, low.has(sid) ? Math.min(low.get(sid), b) : b);
        });
        Object.keys(this.readers).forEach(function (sid) {
            self.source.release(sid, low.has(sid) ? low.get(sid) : Infinity);
        });
    }

    _closeReaders() {
        const self = this;
        Object.keys(this.readers).forEach(function (sid) { self.readers[sid].close(); });
        this.readers = {};
    }

    // jobs: Jobs rows of one or more ladders; chunks: their JobChunks rows;
    // sources: {sourceID: {w, h, fmt, fps: [num, den]}}.  Resolves to a summary
    // once every chunk is "done" or "failed".
    async runJobs(jobs, chunks, sources) {
        if (this.outDir && !this.sink) await this._openSources(sources);
        return this._schedule(jobs, chunks, sources);
    }

    // Y4M / compressed sources: stream geometry and rate from the stream header.  A compressed
    // source (decode: "ffmpeg", or a regular file that is not YUV4MPEG2) is decoded by an ffmpeg
    // child into a pipe; pipes / FIFOs / stdin are read as Y4M streams, regular Y4M files at
    // random.  Opening waits for the header without blocking the event loop.
    async _openSources(sources) {
        const sids = Object.keys(sources);
        for (let i = 0; i < sids.length; ++i) {
            const sid = sids[i], s = sources[sid];
            if (!s.path || this.readers[sid]) continue;
            const viaFfmpeg = s.decode === "ffmpeg" || (s.decode === undefined && !isY4MFile(s.path));
            if (viaFfmpeg && !this.ffmpeg) throw new Error("source " + sid + ": " + s.path + " needs an ffmpeg binary to decode");
            const r = viaFfmpeg ? await ffpipe.FfmpegDecoder.open(this.ffmpeg, s.path, { fmt: s.fmt }) : await y4m.open(s.path);
            this.readers[sid] = r;
            s.w = s.w || r.hdr.w;
            s.h = s.h || r.hdr.h;
            s.fmt = s.fmt === undefined ? r.hdr.fmt : s.fmt;
            s.fps = s.fps || r.hdr.fps;
        }
        if (Object.keys(this.readers).length && !this._userSource) this.source = y4mSource(this.readers);
    }

    _schedule(jobs, chunks, sources) {
        const self = this;
        const plans = ladder.planLadders(jobs, sources);
        const queue = [];
        plans.forEach(function (plan, pi) {
            plan.key = "p" + pi + ":" + JSON.stringify(plan.spec);
            plan.srcFps = sources[plan.sourceID].fps || null;
            const byOff = new Map();
            chunks.forEach(function (c) {
                const k = plan.jobs.findIndex(function (j) { return j.id === c.mainJob; });
                if (k < 0 || c.status === "done") return;
                if (!byOff.has(c.chunkOffset)) byOff.set(c.chunkOffset, new Array(plan.jobs.length).fill(null));
                byOff.get(c.chunkOffset)[k] = c;
            });
            Array.from(byOff.keys()).sort(function (a, b) { return a - b; }).forEach(function (off) {
                const rows = byOff.get(off);
                // a rendition without a row at this offset still runs (it shares the launch); only
                // rows that exist are updated
                queue.push({ plan: plan, chunkOffset: off, rows: rows, tries: 0, lastGpu: -1, lastSlot: -1 });
            });
        });
        // segments in stream order across ladders (a pipe source is read once, front to back)
        queue.sort(function (a, b) { return a.chunkOffset - b.chunkOffset; });
        const total = queue.length;
        let finished = 0;
        function safeUpdate(r, fields) {
            try {
                self._update(r, fields);
            } catch (e) {
                self.emit("updateError", e, r, fields);
            }
        }
        const inflight = [];
        return new Promise(function (resolve) {
            function finish() {
                self._assembleJobs(jobs, chunks).catch(function (e) {
                    self.emit("updateError", e, null, null);
                }).then(function () {
                    self._closeReaders();
                    resolve(self._summary(total));
                });
            }
            if (!total) return finish();
            function pull(slot) {
                if (slot.busy) return;
                // prefer a task that did not just fail on this GPU, then one that did not fail
                // on this slot; a task that failed here waits for another slot unless this is
                // the only one
                let i = queue.findIndex(function (t) { return t.lastGpu !== slot.dev; });
                if (i < 0) i = queue.findIndex(function (t) { return t.lastSlot !== slot.id; });
                if (i < 0 && queue.length && self.slots.length === 1) i = 0;
                if (i < 0) return;
                const task = queue.splice(i, 1)[0];
                inflight.push(task);
                slot.busy = true;
                task.rows.forEach(function (r) {
                    if (r) safeUpdate(r, { assignedTo: self.workerId, status: "assigned" });
                });
                task.rows.forEach(function (r) { if (r) safeUpdate(r, { status: "processing" }); });
                // a throw from onUpdate / an 'update' listener must neither leave the slot busy
                // nor lose the task from the count (ADVICE r01): every handler is guarded, and
                // the release runs whatever happened before it
                let counted = false;
                self._runSegment(slot, task).then(function (res) {
                    counted = true;
                    finished++;
                    slot.done++;
                    slot.ms += res.length ? res[0].ms : 0;
                    task.rows.forEach(function (r, k) {
                        if (r) safeUpdate(r, { status: "done", result: JSON.stringify(res[k]) });
                    });
                }, function (err) {
                    task.tries++;
                    task.lastGpu = slot.dev;
                    task.lastSlot = slot.id;
                    slot.failed++;
                    if (task.tries > self.maxRetries) {
                        counted = true;
                        finished++;
                        task.rows.forEach(function (r) {
                            if (r) safeUpdate(r, { status: "failed", result: JSON.stringify({ error: String(err && err.message || err), gpu: slot.dev, tries: task.tries }) });
                        });
                    } else {
                        task.rows.forEach(function (r) { if (r) safeUpdate(r, { status: null, assignedTo: null }); });
                        queue.push(task);
                        try {
                            self.emit("retry", task, err);
                        } catch (e) {
                            self.emit("updateError", e, null, null);
                        }
                    }
                }).catch(function (e) {
                    // a bug in the handlers above: count the task as failed rather than hang
                    if (!counted && queue.indexOf(task) < 0) finished++;
                    self.emit("updateError", e, null, null);
                }).then(function () {
                    slot.busy = false;
                    inflight.splice(inflight.indexOf(task), 1);
                    try {
                        self._releaseFrames(queue, inflight);
                    } catch (e) {
                        self.emit("updateError", e, null, null);
                    }
                    if (finished === total) return finish();
                    self.slots.forEach(pull);
                });
            }
            self.slots.forEach(pull);
        });
    }

    _summary(total) {
        return { segments: total, gpus: this.slots.map(function (s) {
            return { device: s.dev, slot: s.id, segments: s.done, failures: s.failed, ms: s.ms };
        }) };
    }
}

module.exports = { GpuSegmentScheduler: GpuSegmentScheduler, allocFrame: allocFrame, planeShapes: planeShapes,
                   synthSource: synthSource, y4mSource: y4mSource };
