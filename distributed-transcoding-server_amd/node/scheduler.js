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
//     where a maintainer calls JobChunks.update(...) (database.js:97-129).
//
// The addon's run() executes on the libuv thread pool: set UV_THREADPOOL_SIZE
// >= the GPU count before the first async call (worker.js does).
// Node 12: no `??` / `?.`.

const crypto = require("crypto");
const EventEmitter = require("events");
const ladder = require("./ladder");

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
        this.sink = opts.sink || null;
        this.onUpdate = opts.onUpdate || function () {};
        this.slots = this.gpus.map(function (dev) {
            return { dev: dev, ctx: null, graphs: new Map(), busy: false, done: 0, failed: 0, ms: 0 };
        });
    }

    _ctx(slot) {
        if (!slot.ctx) slot.ctx = this.addon.createContext(slot.dev);
        return slot.ctx;
    }

    _graph(slot, plan) {
        const key = plan.key;
        if (!slot.graphs.has(key)) slot.graphs.set(key, this.addon.createGraph(this._ctx(slot), plan.spec));
        return slot.graphs.get(key);
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

    async _runSegment(slot, task) {
        const plan = task.plan;
        const t0 = Date.now();
        const g = this._graph(slot, plan);
        const idx = this._frames(plan, task.chunkOffset, plan.srcFps);
        const src = await this.source(plan, idx);
        const outs = plan.spec.outputs;
        const dst = [], per = outs.map(function () { return []; });
        src.forEach(function () {
            outs.forEach(function (o, k) {
                const f = allocFrame(o.w, o.h, o.fmt);
                dst.push(f);
                per[k].push(f);
            });
        });
        const quality = await this.addon.run(g, src, dst, null);
        if (this.sink) await this.sink(plan, task.rows, per);
        const ms = Date.now() - t0;
        return task.rows.map(function (row, k) {
            const h = crypto.createHash("sha1");
            let bytes = 0;
            per[k].forEach(function (f) {
                f.data.forEach(function (b) { if (b) { h.update(b); bytes += b.length; } });
            });
            return { frames: per[k].length, bytes: bytes, sha1: h.digest("hex"), gpu: slot.dev, ms: ms,
                     width: outs[k].w, height: outs[k].h, fmt: outs[k].fmt, quality: quality };
        });
    }

    // jobs: Jobs rows of one or more ladders; chunks: their JobChunks rows;
    // sources: {sourceID: {w, h, fmt, fps: [num, den]}}.  Resolves to a summary
    // once every chunk is "done" or "failed".
    runJobs(jobs, chunks, sources) {
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
            if (!total) return resolve(self._summary(0));
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
                    if (finished === total) return resolve(self._summary(total));
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
                   synthSource: synthSource };
