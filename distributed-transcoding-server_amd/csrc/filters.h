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

} // namespace dts
