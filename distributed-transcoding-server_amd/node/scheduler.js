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
//   * `result` carries per-phase timings (readMs, gpuMs, qualityMs, writeMs) and,
//     for rows whose codecSettings ask for it, the segment's PSNR / SSIM against
//     the reference rendition (ladder.js qualityOf).
//
// The addon's run() executes on the libuv thread pool: set UV_THREADPOOL_SIZE
// >= the GPU count before the first async call (worker.js does).
// Node 12: no `??` / `?.`.

const crypto = require("crypto");
const EventEmitter = require("events");
const fs = require("fs");
const path = require("path");
const ladder = require("./ladder");
const y4m = require("./y4m");
const assemble = require("./assemble");

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

// default source: the deterministic testsrc2-like generator of libdts (the
// segment's frames are its global frame indices); a real deployment passes a
// decoder here (host libavcodec, out of the GPU path)
function synthSource(addon, seed) {
    return function (plan, frameIdx) {
        const s = plan.spec.src;
        return frameIdx.map(function (i) {
            const f = allocFrame(s.w, s.h, s.fmt);
            addon.synthFrame(s.w, s.h, s.fmt, 0, seed >>> 0, i, f);
            return f;
        });
    };
}

// Y4M source: frame indices past the end of the file are dropped (the last segment
// of a job is usually short)
function y4mSource(readers) {
    return function (plan, frameIdx) {
        const r = readers[plan.sourceID];
        if (!r) throw new Error("source " + plan.sourceID + " has no Y4M path");
        return frameIdx.filter(function (i) { return i < r.frames; }).map(function (i) { return r.read(i); });
    };
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
        this.onUpdate = opts.onUpdate || function () {};
        this.onJobUpdate = opts.onJobUpdate || function () {};
        this.readers = {};
        this.slots = this.gpus.map(function (dev) {
            return { dev: dev, ctx: null, graphs: new Map(), busy: false, done: 0, failed: 0, ms: 0 };
        });
    }

    _ctx(slot) {
        if (!slot.ctx) slot.ctx = this.addon.createContext(slot.dev);
        return slot.ctx;
    }

    _graph(slot, plan, ref) {
        const key = ref ? plan.key + ":ref" : plan.key;
        if (!slot.graphs.has(key))
            slot.graphs.set(key, this.addon.createGraph(this._ctx(slot), ref ? plan.quality.refSpec : plan.spec));
        return slot.graphs.get(key);
    }

    _segmentPath(jobId, off) {
        return path.join(this.outDir, "job" + jobId, off + ".y4m");
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

    // source frames a stream holds (Y4M file), Infinity for the synthetic source
    _sourceFrames(plan) {
        const r = this.readers[plan.sourceID];
        return r ? r.frames : Infinity;
    }

    async _runSegment(slot, task) {
        const self = this;
        const plan = task.plan;
        const t0 = Date.now();
        const g = this._graph(slot, plan);
        let idx = this._frames(plan, task.chunkOffset, plan.srcFps);
        let sel = null;
        if (plan.spec.deint) {
            // yadif needs each frame's neighbours in the source stream: the graph runs on the
            // segment's contiguous frames plus one context frame each side (clamped: yadif's
            // clone at the stream ends); the vf_fps selection is applied to its outputs
            const base = task.chunkOffset * this.segmentFrames, total = this._sourceFrames(plan);
            const n = Math.max(0, Math.min(this.segmentFrames, total - base));
            sel = idx.filter(function (i) { return i < base + n; }).map(function (i) { return i - base; });
            idx = n ? [Math.max(base - 1, 0)].concat(Array.from({ length: n }, function (_, i) { return base + i; }),
                                                      [Math.min(base + n, total - 1)]) : [];
        }
        const src = await this.source(plan, idx);
        const t1 = Date.now();
        const outs = plan.spec.outputs;
        const nout = plan.spec.deint ? Math.max(0, src.length - 2) : src.length;
        const o = this._allocOutputs(outs, nout);
        if (nout) await this.addon.run(g, src, o.dst, null);
        if (sel) o.per = o.per.map(function (fr) { return sel.map(function (j) { return fr[j]; }); });
        const t2 = Date.now();
        // per-rendition PSNR / SSIM against the reference rendition of the same source frames
        const quality = outs.map(function () { return null; });
        if (plan.quality && nout) {
            const ref = this._allocOutputs(plan.quality.refSpec.outputs, nout);
            await this.addon.run(this._graph(slot, plan, true), src, ref.dst, null);
            if (sel) ref.per = ref.per.map(function (fr) { return sel.map(function (j) { return fr[j]; }); });
            for (let k = 0; k < outs.length; ++k) {
                if (!plan.quality.rows[k]) continue;
                const st = await this.addon.quality(this._ctx(slot), outs[k].w, outs[k].h, outs[k].fmt, o.per[k],
                                                    ref.per[k]);
                const sum = ladder.summarizeQuality(st, outs[k].w, outs[k].h);
                if (!(plan.quality.rows[k] & 1)) delete sum.psnr;
                if (!(plan.quality.rows[k] & 2)) delete sum.ssim;
                quality[k] = sum;
            }
        }
        const t3 = Date.now();
        const files = outs.map(function () { return null; }), written = outs.map(function () { return 0; });
        if (this.sink) {
            await this.sink(plan, task.rows, o.per);
        } else if (this.outDir) {
            task.rows.forEach(function (row, k) {
                if (!row) return;
                const p = self._segmentPath(row.mainJob, row.chunkOffset);
                fs.mkdirSync(path.dirname(p), { recursive: true });
                const fps = plan.framerate ? ladder.rateOf(plan.framerate) : (plan.srcFps || [25, 1]);
                written[k] = y4m.writeSegment(p, o.per[k], outs[k].w, outs[k].h, outs[k].fmt, fps);
                files[k] = p;
            });
        }
        const t4 = Date.now();
        return task.rows.map(function (row, k) {
            const h = crypto.createHash("sha1");
            let bytes = 0;
            o.per[k].forEach(function (f) {
                f.data.forEach(function (b) { if (b) { h.update(b); bytes += b.length; } });
            });
            const r = { frames: o.per[k].length, bytes: bytes, sha1: h.digest("hex"), gpu: slot.dev, ms: t4 - t0,
                        readMs: t1 - t0, gpuMs: t2 - t1, qualityMs: t3 - t2, writeMs: t4 - t3,
                        width: outs[k].w, height: outs[k].h, fmt: outs[k].fmt };
            if (quality[k]) r.quality = quality[k];
            if (files[k]) {
                r.file = files[k];
                r.fileBytes = written[k];
            }
            return r;
        });
    }

    // every chunk of a job done -> its segments assembled into 1 MiB blocks
    _assembleJobs(jobs, chunks) {
        const self = this;
        if (!this.outDir || this.sink) return;
        jobs.forEach(function (job) {
            const mine = chunks.filter(function (c) { return c.mainJob === job.id; });
            if (!mine.length || mine.some(function (c) { return c.status !== "done"; })) return;
            mine.sort(function (a, b) { return a.chunkOffset - b.chunkOffset; });
            const files = mine.map(function (c) { return self._segmentPath(job.id, c.chunkOffset); });
            try {
                const a = assemble.assembleFiles(files, path.join(self.outDir, "blocks"));
                const fields = { assembledData: JSON.stringify(a), finished: true };
                Object.keys(fields).forEach(function (k) { job[k] = fields[k]; });
                self.onJobUpdate(job, fields);
                self.emit("jobUpdate", job, fields);
            } catch (e) {
                self.emit("updateError", e, job, null);
            }
        });
    }

    // jobs: Jobs rows of one or more ladders; chunks: their JobChunks rows;
    // sources: {sourceID: {w, h, fmt, fps: [num, den]}}.  Resolves to a summary
    // once every chunk is "done" or "failed".
    runJobs(jobs, chunks, sources) {
        const self = this;
        if (this.outDir && !this.sink) {          // Y4M sources: stream geometry / rate from the file header
            const self = this;
            Object.keys(sources).forEach(function (sid) {
                const s = sources[sid];
                if (!s.path || self.readers[sid]) return;
                const r = new y4m.Y4MReader(s.path);
                self.readers[sid] = r;
                s.w = s.w || r.hdr.w;
                s.h = s.h || r.hdr.h;
                s.fmt = s.fmt || 0;
                s.fps = s.fps || r.hdr.fps;
            });
            if (Object.keys(this.readers).length && !this._userSource) this.source = y4mSource(this.readers);
        }
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
                queue.push({ plan: plan, chunkOffset: off, rows: rows, tries: 0, lastGpu: -1 });
            });
        });
        const total = queue.length;
        let finished = 0;
        function safeUpdate(r, fields) {
            try {
                self._update(r, fields);
            } catch (e) {
                self.emit("updateError", e, r, fields);
            }
        }
        return new Promise(function (resolve) {
            if (!total) {
                self._assembleJobs(jobs, chunks);
                return resolve(self._summary(0));
            }
            function pull(slot) {
                if (slot.busy) return;
                // prefer a task that did not just fail on this GPU
                let i = queue.findIndex(function (t) { return t.lastGpu !== slot.dev; });
                if (i < 0 && queue.length && self.slots.length === 1) i = 0;
                if (i < 0) return;
                const task = queue.splice(i, 1)[0];
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
                    if (finished === total) {
                        self._assembleJobs(jobs, chunks);
                        return resolve(self._summary(total));
                    }
                    self.slots.forEach(pull);
                });
            }
            self.slots.forEach(pull);
        });
    }

    _summary(total) {
        return { segments: total, gpus: this.slots.map(function (s) {
            return { device: s.dev, segments: s.done, failures: s.failed, ms: s.ms };
        }) };
    }
}

module.exports = { GpuSegmentScheduler: GpuSegmentScheduler, allocFrame: allocFrame, planeShapes: planeShapes,
                   synthSource: synthSource, y4mSource: y4mSource };
