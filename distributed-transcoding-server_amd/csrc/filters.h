// filters.h -- host-side polyphase table construction for the GPU ladder.
//
// Builds libswscale-identical integer filters (FFmpeg 4.4 utils.c
// initFilter semantics under SWS_BITEXACT|SWS_ACCURATE_RND on x86-64) and
// repacks them into the layouts the HIP kernels consume:
//   H u8   : per output column a 4-aligned source window of nd dwords; each
//            int16 tap c split into c = 256*hi + lo (hi, lo signed i8) so a
//            v_dot4_i32_i8 pair over (src ^ 0x80) computes sum(src*c) exactly
//            with the constant 128*sum(c) folded into the accumulator.
//   H p010 : 2-aligned window of nd int16x2 tap pairs (v_dot2_i32_i16).
//   V      : even-aligned window of nv int16x2 row pairs per output row.
#pragma once

#include <stdint.h>
#include <vector>

#include "dts_internal.h"

namespace dts {

struct SwsFilter {
    int size = 0;                    // taps per output (libswscale filterSize)
    std::vector<int16_t> coeff;      // [n * size]
    std::vector<int32_t> pos;        // [n]
};

// utils.c get_local_pos(): 0..256 siting of sample 0 in 1/256 units.
int sws_local_pos(int chr_subsample, int pos);

// initFilter(); returns 0 or a DTS_E_* code.  one = 1<<14 (H) or 1<<12 (V),
// align = x86 filterAlign (H 4, V 2).
int sws_build_filter(int srcN, int dstN, int one, int align, int flags,
                     const double param[2], int srcPos, int dstPos, SwsFilter &out);

struct HTable {                      // H pass tables for one plane kind
    int nd = 0;                      // dwords per output
    int span = 0;                    // max window taps actually used
    std::vector<int32_t> pos, bias;
    std::vector<uint32_t> hi, lo;    // [nd][n]
};

struct VTable {
    int nv = 0;                      // row pairs per output row
    int span = 0;
    std::vector<int32_t> pos;        // even
    std::vector<uint32_t> coef;      // [n][nv]
};

int pack_h_u8(const SwsFilter &f, int dstN, HTable &out);
int pack_h_p010(const SwsFilter &f, int dstN, HTable &out);
int pack_v(const SwsFilter &f, int dstN, VTable &out);

// Output rows whose V window is complete once `rows_done` source rows are
// available, for each pipeline step of kBlkRows rows.  Also checks the ring
// capacity (pairs); returns false if the ring is too small.
bool plan_vlimits(const VTable &v, int srcH, int dstH, int ring_pairs, std::vector<int32_t> &vlim);

// v4 ladder plan of one (rendition, plane kind) (ladder4.hip): strips of C
// output columns, each split into four wave groups.
struct Plan4 {
    int N = 0;                       // H tap pairs per output (kernel bucket)
    int NV = 0;                      // V row pairs per output row
    int C = 0, nstrips = 0, nsteps = 0;
    std::vector<HGroup4> groups;     // [nstrips][4]
    std::vector<uint32_t> hcoef;     // int16x2 tap pairs, group after group
    std::vector<int32_t> vslot, vlim;
    std::vector<uint32_t> vcoef;     // [dstH][NV]
};

// fh: the libswscale H filter; v: the packed V table; bps: bytes per sample
// in the source row (1 u8, 2 nv12 chroma / p010 luma, 4 p010 chroma); nlmax:
// 16-B loads per row the kernel holds; cap: sample pairs its H code
// addresses; row_bytes: source row bytes; ring: ring slots.  Returns false
// when the geometry does not fit k_ladder4 (upscaling, > 16 tap pairs ...):
// that (rendition, kind) then runs on the v3 kernel.
bool plan4_kind(const SwsFilter &fh, const VTable &v, int srcH, int dstW, int dstH, int bps, int nlmax, int cap,
                int maxcols, int64_t row_bytes, int ring, Plan4 &out);

// v5 ladder plan of one plane kind (plan5.cpp, ladder5.hip).
struct Plan5Rung {
    const SwsFilter *fh;             // the libswscale H filter
    const VTable *v;                 // the packed V table
    int dstW, dstH, fmt;             // plane size and the rendition's output format
};

struct Plan5In {
    bool chroma = false;             // U + V planes (else luma)
    bool nv12_chroma = false;        // chroma staged from an interleaved nv12 plane
    bool p10 = false;                // 16-bit (p010) source samples (k_ladder7 only)
    int srcW = 0, srcH = 0;          // plane size
    int lds_cap = 160 * 1024;        // bytes per workgroup (one per CU)
    int range_conv = 0;              // 0 none, 1 *RangeToJpeg, 2 *RangeFromJpeg (k_ladder7 only)
    std::vector<Plan5Rung> rungs;
};

struct Plan5Kind {
    int nplanes = 1, nsteps = 0, nlp = 1, stage = 0, SB = 0, FA = 0, FB = 0, nrings = 0, lds_bytes = 0, strip_width = 0;
    Ring5 ring[kL5MaxRings]{};
    Out5 out[DTS_MAX_OUTPUTS]{};
    std::vector<Strip5> strips;
    std::vector<Ent5> ents;
    std::vector<uint32_t> bfrag;     // H then V fragment pairs
    std::vector<VEnt5> vsched;
    std::vector<int32_t> vstep;      // [nsteps + 1][4]
};

// false: the geometry / format does not fit k_ladder5 (the kind then runs on v4 / v3)
bool plan5_kind(const Plan5In &in, Plan5Kind &out);

// ladder work-unit plan (plan6.cpp): the work units of one frame (both plane kinds,
// every rendition), their B fragments and the V fire tables; plan7_graph groups them.
struct Plan6 {
    std::vector<Unit6> units;
    std::vector<uint32_t> frag;      // fragment pairs, 512 dwords each
    std::vector<int32_t> fire;
};

// kinds[0] luma, kinds[1] chroma (Plan5In: same inputs as v5).  false: the graph
// does not fit the walks (planes narrower than 64 or 128 columns, windows wider
// than two K blocks ...): it then runs on k_ladder5.
// align: the H K windows start on multiples of align source columns (16 for k_ladder7,
// whose A operands are 16-B LDS reads; 0: 8 or 16); sort: heaviest units first.
// narrow (k_ladder7): the one-K-block walks get 2 tiles per plane (luma) / 1 (chroma), not 4 / 2
// fs_window: granules whose firing row blocks share the V fragment slots
// hsplit: the H taps as hsplit * hi + lo (256: lo a signed byte; 128: lo in
// [0, 127], k_ladder7's one-shift epilogue; false if a tap does not split)
bool plan6_graph(const Plan5In kinds[2], Plan6 &out, int align = 4, bool sort = true, bool narrow = false,
                 int fs_window = kL6Stages, int hsplit = 256);

// v7 ladder plan: the work units (align 16) in groups of at most wmax waves over one
// source strip (Group7, Unit7).  false: the graph does not fit k_ladder7 (plane widths
// not multiples of 16, strips wider than the plane ...): k_ladder5 / k_ladder4 run it.
struct Plan7 {
    std::vector<Group7> groups;
    std::vector<Unit7> units;
    std::vector<uint32_t> frag;
    std::vector<int32_t> fire;
    int lds_bytes = 0, waves = 0;    // per workgroup: LDS, waves (max over groups)
    int hsplit = 256;                // H tap split of the fragments (ladder7.hip walk7 HS)
};
// Groups of at most wmax units; a group's spare waves (if any) stage its pieces, else all its
// waves deal them, and each rendition's lead wave DMAs its V fragments.
bool plan7_graph(const Plan5In kinds[2], int wmax, int stages, int pb, bool by_rung, bool narrow, Plan7 &out);

} // namespace dts
