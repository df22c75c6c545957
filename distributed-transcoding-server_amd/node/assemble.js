"use strict";
// assemble.js -- a finished job's segments -> Jobs.assembledData (SURVEY.md §8f row f3).
//
// The reference serves a finished job from `Jobs.assembledData` = JSON
// {size, chunk: [id...]} (database.js:89-93): the job's output file cut into
// 1 MiB blocks, chunk[i] the content id of block i (index.js:57-66 maps a byte
// range to blocks of 1048576 and fetches chunk[i] from IPFS by CID).  This is the
// producer side: the rendition segment files, in chunkOffset order, are
// concatenated into one stream, cut into 1 MiB blocks, and each block is stored
// content-addressed as blockDir/<sha256 hex> (the id that goes into `chunk`).
// Files are streamed block by block, so segment size is not limited by memory.
//
// Node 12: no `??` / `?.`.

const crypto = require("crypto");
const fs = require("fs");
const path = require("path");

const BLOCK = 1048576;

function storeBlock(blockDir, buf) {
    const id = crypto.createHash("sha256").update(buf).digest("hex");
    const p = path.join(blockDir, id);
    if (!fs.existsSync(p)) fs.writeFileSync(p, buf);
    return id;
}

// files: segment paths in playback order -> {size, chunk: [block ids]}.
// skip(i): bytes at the start of file i that are not part of the stream (Y4M segments:
// every segment file carries its own header line, the assembled stream one -- the
// first segment's; ADVICE r02: concatenated headers made an invalid Y4M stream).
function assembleFiles(files, blockDir, skip) {
    fs.mkdirSync(blockDir, { recursive: true });
    const block = Buffer.alloc(BLOCK);
    let fill = 0, size = 0;
    const chunk = [];
    files.forEach(function (f, fi) {
        const fd = fs.openSync(f, "r");
        let pos = skip ? skip(fi, f) : 0;
        try {
            for (;;) {
                const n = fs.readSync(fd, block, fill, BLOCK - fill, pos);
                pos += Math.max(n, 0);
                if (n <= 0) break;
                fill += n;
                size += n;
                if (fill === BLOCK) {
                    chunk.push(storeBlock(blockDir, block));
                    fill = 0;
                }
            }
        } finally {
            fs.closeSync(fd);
        }
    });
    if (fill > 0) chunk.push(storeBlock(blockDir, block.slice(0, fill)));
    return { size: size, chunk: chunk };
}

// the byte range [first, last] of an assembled job, read back from its blocks
// (index.js downloadChunkData's block arithmetic, for tests and local serving)
function readRange(assembled, blockDir, first, last) {
    const out = [];
    const end = Math.min(last, assembled.size - 1);
    for (let b = Math.floor(first / BLOCK); b * BLOCK <= end && b < assembled.chunk.length; ++b) {
        const data = fs.readFileSync(path.join(blockDir, assembled.chunk[b]));
        const s = Math.max(first - b * BLOCK, 0), e = Math.min(end - b * BLOCK + 1, data.length);
        out.push(data.slice(s, e));
    }
    return Buffer.concat(out);
}

// Y4M rendition segments -> one YUV4MPEG2 stream: the first file whole, the header
// line of every later one dropped (all segments of a rendition share it)
function assembleY4M(files, blockDir) {
    const y4m = require("./y4m");
    return assembleFiles(files, blockDir, function (i, f) { return i ? y4m.headerBytes(f) : 0; });
}

module.exports = { BLOCK: BLOCK, assembleFiles: assembleFiles, assembleY4M: assembleY4M, readRange: readRange };
