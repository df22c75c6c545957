// ladder7.hip -- k_ladder7, the ladder kernel: 4:2:0 sources (8-bit planar, nv12,
// p010) to every rendition of a graph, both FIR passes on v_mfma_i32_16x16x64_i8,
// the source staged once per strip and the H outputs never leaving the VGPRs.
//
// Arithmetic: libswscale hScale8To15_c / hScale16To15 -> yuv2planeX_8_c /
// yuv2nv12cX_c / yuv2p010lX_c under SWS_BITEXACT|SWS_ACCURATE_RND (FFmpeg 4.4;
// bit-exact, DESIGN.md "Oracle"), the integer identities of k_ladder5 (ladder5.hip
// header) on signed-byte MFMA operands:
//
//  * one wave = one work unit: CT 16-column tiles of one rendition of one plane
//    kind (chroma: the same columns of U and V) of one frame, walked top to bottom
//    in granules of 16 source rows;
//  * H of a granule: per tile one MFMA per K block and tap part.  A = 16 source rows
//    x 64 columns (bytes xor 0x80), B = the tile's taps split into signed bytes
//    (c = HS hi + lo, plan6.cpp put6), held in VGPRs for the whole walk; p010: A =
//    the raw little-endian bytes, three chains (walk7 header below);
//  * the H result of a tile is, per lane, 4 consecutive source rows of one output
//    column -- a V A-operand dword once split into y >> 8 and (y & 255) ^ 0x80
//    bytes.  The last 4 VKB granules of every tile stay in a register ring (slot =
//    granule mod 4 VKB; the walk is unrolled by the ring length, so every slot is a
//    fixed register);
//  * V of a row block (16 output rows) runs after the granule that completes its
//    window: out^T = H^T C^T over the whole ring, the fragment laid out for where
//    each granule sits in the ring;
//  * stores: each lane holds 4 consecutive columns of one output row per tile;
//    permlane swaps transpose the tiles so a lane holds 4-16 consecutive bytes of its
//    row (nv12: U and V interleaved by v_perm), stored as whole row segments.
//
// Staging: a workgroup is a group of waves of every rendition whose K windows lie in
// one source strip [X0, X0 + 64 npc) of the plane(s) (plan6.cpp plan7_graph); per
// granule the group DMAs the strip's 16 rows into LDS once -- npc 1-KB pieces per
// plane, dealt round robin over all its waves -- and every wave reads its A operands
// there.  (Per-wave staging of every (tile, K block), the retired k_ladder6, moved
// ~5x the plane per frame through L2 and spent ~45 % of a wave's cycles issuing it:
// profiles/r02b_*.)
//
//  * LDS image of a piece: 16 rows x 64 bytes, lane-linear as the DMA writes it.
//    DMA lane l loads row l >> 2, 16-B chunk (l & 3) ^ sw(row), sw(r) = 2 ((r >> 3) & 1):
//    four consecutive lanes cover one row's 64 contiguous bytes.  The A read of lane
//    (m, g) -- row m, chunk c = xo / 16 + g of the strip -- is the ds_read_b128 at
//    piece (c >> 2), 16 (4 m + ((c & 3) ^ sw(m))), conflict-free for every xo (each
//    16-lane group of a ds_read_b128 meets the four chunk positions of each row
//    quad exactly once);
//  * kL7Stages granule stages: at granule q a wave waits for its own pieces of q
//    (counted vmcnt), the group barriers, then issues its pieces of q + 2 into the
//    stage granule q - 1 was read from (every wave is past those reads) and runs
//    H(q) and the row blocks firing at q;
//  * V fragments: the first wave of each rendition in the group DMAs them with its
//    pieces of the fire granule into the rendition's LDS slots; the barrier of that
//    granule publishes them to the other waves of the rendition;
//  * waves beyond the group's units (the workgroup has the widest group's size)
//    only stage pieces and keep the barrier count.
#include "dts_internal.h"
#include "ladder_mfma.h"

#ifndef DTS_L7_ABLATE
#define DTS_L7_ABLATE 0     // diagnostic builds only (wrong results): 1 no group barrier, 2 no A xor,
                            // 4 stage only the pieces left of the next strip's X0 (no halo re-reads),
                            // 8 no V (no row blocks, no stores), 16 no H (no A reads, MFMAs, epilogue),
                            // 32 V without its global stores, 64 V without exchange and stores,
                            // 128 V without its MFMAs (the ring's dwords exchanged and stored),
                            // 256 no V fragment DMAs, 512 every row block stored to its plane's row 0
#endif
#ifndef DTS_L7_DEFER
#define DTS_L7_DEFER 1      // row blocks run one granule after the one completing their window
#endif
#ifndef DTS_L7_SRC_AUX
#define DTS_L7_SRC_AUX 0    // cache-policy bits of the source staging loads (diagnostic A/B)
#endif
#ifndef DTS_L7_NS
#define DTS_L7_NS kL7Stages
#endif
#ifndef DTS_L7_PAIR
#define DTS_L7_PAIR (kL7Batch == 2)  // 1: stage 2 granules per batch (one barrier per 2 granules); plan with DTS_L7_PB=2
#endif
#ifndef DTS_L7_STAMP
#define DTS_L7_STAMP 0      // diagnostic builds only: per-variant, per-phase s_memtime sums (tools/stamp7.py)
#endif

namespace dts {

#if DTS_L7_STAMP
// [variant (16 = staging-only waves)][phase]: cycles summed over every wave; [v][6]: granules, [v][7]: waves
__device__ unsigned long long g_l7_stamp[kL7Variants + 1][8];
#define L7_STAMP(k)                                                        \
    do {                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();        \
        st_acc[k] += t_ - st_last;                                         \
        st_last = t_;                                                      \
    } while (0)
#define L7_STAMP_INIT                                                      \
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};                     \
    unsigned long long st_last = __builtin_amdgcn_s_memtime()
#define L7_STAMP_DONE(v, ng)                                               \
    do {                                                                   \
        L7_STAMP(5);                                                       \
        if ((threadIdx.x & 63) == 0) {                                     \
            for (int k_ = 0; k_ < 6; ++k_) atomicAdd(&g_l7_stamp[v][k_], st_acc[k_]); \
            atomicAdd(&g_l7_stamp[v][6], (unsigned long long)(ng));       \
            atomicAdd(&g_l7_stamp[v][7], 1ull);                            \
        }                                                                  \
    } while (0)
#else
#define L7_STAMP(k) (void)0
#define L7_STAMP_INIT (void)0
#define L7_STAMP_DONE(v, ng) (void)0
#endif

namespace {

constexpr int NS7 = DTS_L7_NS;
constexpr int PB7 = DTS_L7_PAIR ? 2 : 1;   // granules per staging batch
static_assert(NS7 >= 2 && NS7 <= 4, "stages (plan7_graph: V fragment slots for PB7 (NS7 + 1) granules)");

// s_waitcnt vmcnt(min(n, 15)) for a run-time n >= 0: waiting for fewer outstanding
// operations than were issued after the batch is never too short
__device__ __forceinline__ void vm_wait_rt7(int n)
{
#define DTS_W7I(k) __builtin_amdgcn_s_waitcnt((k) | (7 << 4) | (15 << 8))
#define DTS_W7(k) \
    case k: DTS_W7I(k); break;
    switch (min(max(n, 0), 15)) {
        DTS_W7(0) DTS_W7(1) DTS_W7(2) DTS_W7(3) DTS_W7(4) DTS_W7(5) DTS_W7(6) DTS_W7(7)
        DTS_W7(8) DTS_W7(9) DTS_W7(10) DTS_W7(11) DTS_W7(12) DTS_W7(13) DTS_W7(14)
    default: DTS_W7(15)
    }
#undef DTS_W7
#undef DTS_W7I
}

// every wave's pieces of the granule have landed (each wave waited for its own) and
// every wave is past its reads of the previous granule
__device__ __forceinline__ void group_barrier7()
{
    if (DTS_L7_ABLATE & 1)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The group's staging: this wave's share of the pieces of every granule, the counted
// wait and the barrier.  ops counts this wave's VMEM instructions (pieces, V fragment
// DMAs, stores); e[i] = ops after the batch of granule q + i (i < NS7 - 1).
struct Stage7 {
    uint64_t sb[2];                 // plane bases of this frame (chroma: U, V)
    uint32_t sp[2];                 // plane pitches
    int np, npc, ppp, npieces, w, nw, srcH1, ngran, stage_bytes, nown;
    uint32_t lcol;                  // this lane's byte in a piece row: X0 + 16 chunk
    int dr;                         // this lane's row in a piece
    int ops, e[NS7 - 1];

    // bpc: staged bytes per source column (Group7::bpc; a compile-time 1 for planar 8-bit
    // sources): the chroma of planar sources is two planes, every other staging one plane of
    // bpc npc pieces per granule
    __device__ __forceinline__ void init(const Group7 &G, const DevPlanes &S, int f, int wave, int waves, int lane,
                                         int bpc)
    {
        const bool il = bpc > 1;
        np = G.kind && !il ? 2 : 1;
        for (int p = 0; p < 2; ++p) {
            sb[p] = (G.kind ? S.data[1 + (il ? 0 : p)] : S.data[0]) + (uint64_t)f * (uint64_t)S.fstride;
            sp[p] = (uint32_t)(G.kind ? S.pitch[1 + (il ? 0 : p)] : S.pitch[0]);
        }
        npc = G.npc;
        ppp = bpc * npc;
        npieces = np * ppp;
        nown = min(ppp, ((G.xown - G.X0) * bpc + 63) >> 6);
        // the staging waves st0.. deal the pieces (Group7::st0)
        w = wave >= G.st0 ? wave - G.st0 : npieces;
        nw = waves - G.st0;
        srcH1 = G.srcH - 1;
        ngran = G.ngran;
        stage_bytes = PB7 * npieces * 1024;
        dr = lane >> 2;
        lcol = (uint32_t)(bpc * G.X0) + 16u * (uint32_t)((lane & 3) ^ (2 * ((dr >> 3) & 1)));
        ops = 0;
    }
    // this wave's pieces of batch b (granules PB7 b ..) into stage st (nothing past the plane)
    __device__ __forceinline__ void pieces(uint8_t *lds, int b, int st)
    {
#pragma unroll
        for (int h = 0; h < PB7; ++h) gran(lds, PB7 * b + h, st * stage_bytes + h * npieces * 1024);
    }
    __device__ __forceinline__ void gran(uint8_t *lds, int q, int at)
    {
        if (q >= ngran) return;
        const uint32_t row = (uint32_t)min(kL6Gran * q + dr, srcH1);
        uint8_t *dst = lds + at;
        for (int k = w; k < npieces; k += nw) {
            const int p = k >= ppp ? 1 : 0, i = k - p * ppp;
            if ((DTS_L7_ABLATE & 4) && i >= nown) continue;
            const uint64_t src = (p ? sb[1] : sb[0]) + (uint64_t)(row * (p ? sp[1] : sp[0])) + lcol + 64u * (uint32_t)i;
            __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)src,
                                             (__attribute__((address_space(3))) void *)(dst + 1024 * k), 16, 0,
                                             DTS_L7_SRC_AUX);
            ++ops;
        }
    }
    // granule q's batch has landed for this wave: everything issued after it may still fly
    __device__ __forceinline__ void wait_batch() { vm_wait_rt7(ops - e[0]); }
    // after the batch of granule q + NS7 - 1 was issued
    __device__ __forceinline__ void shift()
    {
#pragma unroll
        for (int i = 0; i + 1 < NS7 - 1; ++i) e[i] = e[i + 1];
        e[NS7 - 2] = ops;
    }
};

// The row block's bytes through the wave's 1-KB LDS exchange: lane (m, g) holds NB bytes
// of output row m at byte NB g of a 4 NB-byte segment; after the exchange lane 4 m + g
// does, so four consecutive lanes hold one row's segment (one cache access per row
// segment).  x[] is what vstore7 writes.  Chunk g of row m sits at chunk position
// g ^ ((m >> 2) & 3) of the row, so the 8 (16) lanes of a ds_write_b128 (b64) group
// meet distinct banks; the readers' four lanes of a row cover its four positions.
// nv12 chroma of two tiles: the two 32-byte tile rows make one 64-byte row (16-byte
// chunks, one store per lane).
template <int VAR, class UT>
__device__ __forceinline__ void xchg7(const UT &U, const uint32_t (&w)[Walk6<VAR>::T], uint8_t *scr, int m, int g,
                                      int lane, uint32_t (&x)[4])
{
    using W = Walk6<VAR>;
    __builtin_amdgcn_wave_barrier();
    const int d = 4 * m + (g ^ ((m >> 2) & 3));            // writer's chunk position
    const int r4 = lane >> 2, dr = 4 * r4 + ((lane & 3) ^ ((r4 >> 2) & 3));   // reader's
    if (W::NP == 1) {                                      // luma
        if (W::CT == 4) {
            uint32_t o[4];
            transpose4(w[0], w[1 % W::T], w[2 % W::T], w[3 % W::T], o);
            *reinterpret_cast<u32x4 *>(scr + 16 * d) = (u32x4){o[0], o[1], o[2], o[3]};
            const u32x4 r = *reinterpret_cast<const u32x4 *>(scr + 16 * dr);
            x[0] = r.x; x[1] = r.y; x[2] = r.z; x[3] = r.w;
        } else if (W::CT == 1) {                           // (p010 sources) 16-byte tile rows
            *reinterpret_cast<uint32_t *>(scr + 4 * d) = w[0];
            x[0] = *reinterpret_cast<const uint32_t *>(scr + 4 * dr);
            x[1] = x[2] = x[3] = 0;
        } else {
            uint32_t o[2];
            transpose2(w[0], w[1 % W::T], o);
            *reinterpret_cast<u32x2 *>(scr + 8 * d) = (u32x2){o[0], o[1]};
            const u32x2 r = *reinterpret_cast<const u32x2 *>(scr + 8 * dr);
            x[0] = r.x; x[1] = r.y; x[2] = x[3] = 0;
        }
    } else if (U.fmt == DTS_FMT_NV12 && W::CT == 2) {      // chroma, U V interleaved, 64 B per row
        // tile c's 8 bytes of row m are bytes 32 c + 8 g: 16-byte chunk 2 c + (g >> 1), half g & 1
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t u = w[c], v = w[2 + c];
            const int ch = (2 * c + (g >> 1)) ^ ((m >> 2) & 3);
            *reinterpret_cast<u32x2 *>(scr + 64 * m + 16 * ch + 8 * (g & 1)) =
                (u32x2){__builtin_amdgcn_perm(v, u, 0x05010400u), __builtin_amdgcn_perm(v, u, 0x07030602u)};
        }
        const u32x4 r = *reinterpret_cast<const u32x4 *>(scr + 16 * dr);
        x[0] = r.x; x[1] = r.y; x[2] = r.z; x[3] = r.w;
    } else if (U.fmt == DTS_FMT_NV12) {                    // chroma, U V interleaved, 32 B per tile row
#pragma unroll
        for (int c = 0; c < W::CT; ++c) {
            const uint32_t u = w[c], v = w[W::CT + c];
            *reinterpret_cast<u32x2 *>(scr + 512 * c + 8 * d) =
                (u32x2){__builtin_amdgcn_perm(v, u, 0x05010400u), __builtin_amdgcn_perm(v, u, 0x07030602u)};
        }
#pragma unroll
        for (int c = 0; c < W::CT; ++c) {
            const u32x2 r = *reinterpret_cast<const u32x2 *>(scr + 512 * c + 8 * dr);
            x[2 * c] = r.x; x[2 * c + 1] = r.y;
        }
        if (W::CT == 1) x[2] = x[3] = 0;
    } else {                                               // chroma, U and V planes
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            if (W::CT == 2) {
                uint32_t o[2];
                transpose2(w[2 * p], w[(2 * p + 1) % W::T], o);
                *reinterpret_cast<u32x2 *>(scr + 512 * p + 8 * d) = (u32x2){o[0], o[1]};
            } else {
                *reinterpret_cast<uint32_t *>(scr + 256 * p + 4 * d) = w[p % W::T];
            }
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            if (W::CT == 2) {
                const u32x2 r = *reinterpret_cast<const u32x2 *>(scr + 512 * p + 8 * dr);
                x[2 * p] = r.x; x[2 * p + 1] = r.y;
            } else {
                x[p] = *reinterpret_cast<const uint32_t *>(scr + 256 * p + 4 * dr);
            }
        }
        if (W::CT == 1) x[2] = x[3] = 0;
    }
    __builtin_amdgcn_wave_barrier();
}

// p010 renditions (yuv2p010lX / yuv2p010cX, LE 16-bit): lane (m, g) holds the 16-bit values
// of columns 4 g .. 4 g + 3 of one column tile (v[p][0..1]: plane p, two per dword); luma
// rows are 32 bytes per tile (8 per lane), chroma rows U V interleaved, 64 bytes (16 per
// lane); the same exchange as xchg7 gives four consecutive lanes one row's segment
template <int VAR, class UT>
__device__ __forceinline__ void xchg7p(const UT &U, const uint32_t (&v)[Walk6<VAR>::T][2], uint8_t *scr, int m,
                                       int g, int lane, uint32_t (&x)[4])
{
    using W = Walk6<VAR>;
    static_assert(W::CT == 1, "p010 renditions: one column tile per plane");
    __builtin_amdgcn_wave_barrier();
    const int d = 4 * m + (g ^ ((m >> 2) & 3));
    const int r4 = lane >> 2, dr = 4 * r4 + ((lane & 3) ^ ((r4 >> 2) & 3));
    if (W::NP == 1) {
        *reinterpret_cast<u32x2 *>(scr + 8 * d) = (u32x2){v[0][0], v[0][1]};
        const u32x2 r = *reinterpret_cast<const u32x2 *>(scr + 8 * dr);
        x[0] = r.x; x[1] = r.y; x[2] = x[3] = 0;
    } else {
        const uint32_t u0 = v[0][0], u1 = v[0][1], v0 = v[W::T - 1][0], v1 = v[W::T - 1][1];
        *reinterpret_cast<u32x4 *>(scr + 16 * d) =
            (u32x4){__builtin_amdgcn_perm(v0, u0, 0x05040100u), __builtin_amdgcn_perm(v0, u0, 0x07060302u),
                    __builtin_amdgcn_perm(v1, u1, 0x05040100u), __builtin_amdgcn_perm(v1, u1, 0x07060302u)};
        const u32x4 r = *reinterpret_cast<const u32x4 *>(scr + 16 * dr);
        x[0] = r.x; x[1] = r.y; x[2] = r.z; x[3] = r.w;
    }
    (void)U;
    __builtin_amdgcn_wave_barrier();
}

// the stores of row block j from x (xchg7); returns the store instructions issued (edge
// units' byte stores are not counted, which only makes the next source wait longer)
template <int VAR, class UT>
__device__ __forceinline__ int vstore7(const UT &U, int j, const uint32_t (&x)[4], const uint64_t (&ob)[2],
                                       const uint32_t (&op)[2], int lane)
{
    using W = Walk6<VAR>;
    const int y = (DTS_L7_ABLATE & 512) ? 0 : 16 * j + (lane >> 2), q4 = lane & 3;
    if (y < U.dstH) {
        if (W::CT == 1 && U.fmt == DTS_FMT_P010LE) {        // p010 renditions (xchg7p)
            if (W::NP == 1) {
                const uint32_t o[2] = {x[0], x[1]};
                const int at = 2 * U.col0 + 8 * q4;
                put_row6<8>(ob[0] + (uint64_t)y * op[0], at, 2 * U.dstW - at, o);
            } else {
                const uint32_t o[4] = {x[0], x[1], x[2], x[3]};
                const int at = 4 * U.col0 + 16 * q4;
                put_row6<16>(ob[0] + (uint64_t)y * op[0], at, 4 * U.dstW - at, o);
            }
        } else if (W::NP == 1) {
            if (W::CT == 4) {
                const uint32_t o[4] = {x[0], x[1], x[2], x[3]};
                put_row6<16>(ob[0] + (uint64_t)y * op[0], U.col0 + 16 * q4, U.dstW - U.col0 - 16 * q4, o);
            } else if (W::CT == 1) {
                const uint32_t o[1] = {x[0]};
                put_row6<4>(ob[0] + (uint64_t)y * op[0], U.col0 + 4 * q4, U.dstW - U.col0 - 4 * q4, o);
            } else {
                const uint32_t o[2] = {x[0], x[1]};
                put_row6<8>(ob[0] + (uint64_t)y * op[0], U.col0 + 8 * q4, U.dstW - U.col0 - 8 * q4, o);
            }
        } else if (U.fmt == DTS_FMT_NV12 && W::CT == 2) {
            const uint32_t o[4] = {x[0], x[1], x[2], x[3]};
            const int at = 2 * U.col0 + 16 * q4;
            put_row6<16>(ob[0] + (uint64_t)y * op[0], at, 2 * U.dstW - at, o);
        } else if (U.fmt == DTS_FMT_NV12) {
#pragma unroll
            for (int c = 0; c < W::CT; ++c) {
                const uint32_t o[2] = {x[2 * c], x[2 * c + 1]};
                const int at = 2 * U.col0 + 32 * c + 8 * q4;
                put_row6<8>(ob[0] + (uint64_t)y * op[0], at, 2 * U.dstW - at, o);
            }
        } else {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                if (W::CT == 2) {
                    const uint32_t o[2] = {x[2 * p], x[2 * p + 1]};
                    put_row6<8>(ob[p] + (uint64_t)y * op[p], U.col0 + 8 * q4, U.dstW - U.col0 - 8 * q4, o);
                } else {
                    const uint32_t o[1] = {x[p]};
                    put_row6<4>(ob[p] + (uint64_t)y * op[p], U.col0 + 4 * q4, U.dstW - U.col0 - 4 * q4, o);
                }
            }
        }
    }
    return W::NP == 1 ? 1 : (U.fmt == DTS_FMT_NV12 ? 1 : 2);
}

// V of one row block over the whole ring, as vcalc (ladder_mfma.h): 65536 hh + 256 (hl +
// lh) + ll as three chained accumulations; the bias enters as b1 << 16 (the chain's start)
// and b2 << 8 (added with the first shift), so a per-lane bias (the ordered dither of
// p010 sources: DIT) costs nothing.  8-bit: av_clip_uint8(v >> 19) of 4 columns, packed.
template <int VAR, bool DIT>
__device__ __forceinline__ void vcalc7(const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                       const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                       const v4i (&vdit)[2], uint32_t (&w)[Walk6<VAR>::T])
{
    using W = Walk6<VAR>;
    static_assert(kL5VBias == 12 << 16, "flat-dither V bias folded into the hh chain");
    const int b1 = DIT ? 0 : 12;                  // (128 + 64) << 12, or the dither's 128 << 12 in b2
    v4i acc[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] = (v4i){b1, b1, b1, b1};
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vh[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] = DIT ? (acc[t] << 8) + vdit[t / W::CT] : acc[t] << 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) {
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vl[kb], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vh[kb], acc[t], 0, 0, 0);
        }
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] <<= 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vl[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) {
        // the two 16-bit packs as one u16x2 (a v_perm of their low halves: no zero-extension of each)
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        const unsigned short lo = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][0], acc[t][1], 19);
        const unsigned short hi = __builtin_amdgcn_ashr_pk_u8_i32(acc[t][2], acc[t][3], 19);
        w[t] = __builtin_bit_cast(uint32_t, (u16x2){lo, hi});
    }
}

// the same chain for a p010 rendition: bias (1 << 16) + the ring's 128 << 12 = 9 << 16,
// av_clip_uintp2(v >> 17, 10) << 6, two 16-bit values per dword
template <int VAR>
__device__ __forceinline__ void vcalc7p(const v4i (&rh)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                        const v4i (&rl)[Walk6<VAR>::VKB][Walk6<VAR>::T],
                                        const v4i (&vh)[Walk6<VAR>::VKB], const v4i (&vl)[Walk6<VAR>::VKB],
                                        uint32_t (&w)[Walk6<VAR>::T][2])
{
    using W = Walk6<VAR>;
    v4i acc[W::T];
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] = (v4i){9, 9, 9, 9};
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vh[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] <<= 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) {
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rh[kb][t], vl[kb], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vh[kb], acc[t], 0, 0, 0);
        }
#pragma unroll
    for (int t = 0; t < W::T; ++t) acc[t] <<= 8;
#pragma unroll
    for (int kb = 0; kb < W::VKB; ++kb)
#pragma unroll
        for (int t = 0; t < W::T; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(rl[kb][t], vl[kb], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < W::T; ++t) {
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (uint32_t)min(max(acc[t][i] >> 17, 0), 1023) << 6;
        w[t][0] = __builtin_amdgcn_perm(o[1], o[0], 0x05040100u);
        w[t][1] = __builtin_amdgcn_perm(o[3], o[2], 0x05040100u);
    }
}

// a wave with no unit: stage its pieces, keep the group's barrier count
template <int SK>
__device__ __forceinline__ void idle7(const Group7 &G, const DevPlanes &S, int f, int wave, int waves)
{
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds7[];
    Stage7 Z;
    Z.init(G, S, f, wave, waves, (int)threadIdx.x & 63, SK == 0 ? 1 : G.bpc);
#pragma unroll
    for (int i = 0; i < NS7 - 1; ++i) {
        Z.pieces(lds7, i, i);
        Z.e[i] = Z.ops;
    }
    int sq = 0;
    L7_STAMP_INIT;
    const int nb = (G.ngran + PB7 - 1) / PB7;
    for (int b = 0; b < nb; ++b) {
        Z.wait_batch();
        L7_STAMP(0);
        group_barrier7();
        L7_STAMP(1);
        const int sn = sq == 0 ? NS7 - 1 : sq - 1;
        Z.pieces(lds7, b + NS7 - 1, sn);
        Z.shift();
        sq = sq + 1 == NS7 ? 0 : sq + 1;
        L7_STAMP(2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    L7_STAMP_DONE(kL7Variants, G.ngran);
}

// HS: the H taps' split in the fragments (plan6.cpp put6).  256: c = 256 hi + lo (signed
// bytes), the epilogue FFMIN(((hi << 8) + lo) >> 7, 32767).  128: c = 128 hi + lo, lo in
// [0, 127]; with x = src - 128, sum(src c) = 128 (sum(x hi) + 16384) + sum(x lo), so
//   y = sum(src c) >> 7 = sum(x hi) + ((sum(x lo) + (128 << 14)) >> 7)
// exactly (128 (...) is a multiple of 128): the lo MFMAs run first from the bias, one
// shift, and the hi MFMAs accumulate onto it -- y comes out of the matrix core and the
// epilogue is the saturating pack (FFMIN(y, 32767), y >= -32768 for 8-bit sources).
//
// SK: the source kind -- 0 planar 8-bit, 1 nv12 (chroma U V byte pairs, de-interleaved
// in the A reads), 2 p010 (16-bit samples, VAR | 16: one column tile per plane).  p010
// (input.c p010LEToY_c / p010LEToUV_c, swscale.c hScale16To15_c with sh = 9): the A
// operands are the samples' raw little-endian bytes masked to (s >> 2, (s & 3) << 6) and
// offset by 128, B the fragment triple of put6p (plan6.cpp); the three MFMA chains give
//   y = FFMIN(sum(s c) >> 9, 32767) = 2 A + ((M + ((L + K) >> 8)) >> 7)
// exactly (the floors nest), so the same saturating pack ends the H step.  8-bit outputs of
// p010 sources add the ordered dither ff_dither_8x8_128[y & 7][(x + off) & 7] << 12 (off 3
// for V) instead of the flat 64; p010 outputs (any source) are yuv2p010lX / cX:
// av_clip_uintp2((sum + (1 << 16)) >> 17, 10) << 6.
template <int VAR, bool RC, int HS, int SK>
__device__ __forceinline__ void walk7(const Ladder7Params &P, const Group7 &G, const Unit7 &U, const DevPlanes &S,
                                      int f, int wave, int waves)
{
    using W = Walk6<VAR>;
    constexpr int CT = W::CT, HKB = W::HKB, VKB = W::VKB, T = W::T, R = W::R;
    constexpr bool IL = SK == 1, P10 = SK == 2;
    static_assert(!P10 || (VAR & 16), "p010 walks are the 16-bit variants");
    constexpr int RKB = P10 ? 2 * HKB : HKB;        // MFMA K blocks per tile (p010: 32 samples each)
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds7[];
    const int lane = (int)threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    Stage7 Z;
    Z.init(G, S, f, wave, waves, lane, P10 ? (W::NP == 2 ? 4 : 2) : (W::NP == 2 && IL ? 2 : 1));
    // output planes: luma plane 0; nv12 chroma plane 1; yuv420p chroma planes 1 and 2
    uint64_t ob[2];
    uint32_t op[2];
    {
        const uint8_t *ka = (const uint8_t *)__builtin_amdgcn_kernarg_segment_ptr();
        const DevPlanes D = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder7Params, dst)) + U.rung);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            ob[p] = (U.kind ? D.data[1 + p] : D.data[0]) + (uint64_t)f * (uint64_t)D.fstride;
            op[p] = (uint32_t)(U.kind ? D.pitch[1 + p] : D.pitch[0]);
        }
    }
    const uint64_t fr = (uint64_t)(uintptr_t)P.frag + 16u * (uint32_t)lane;
    // H B operands of the walk (p010: bh = the M fragments, bl = L, ba = A of put6p)
    constexpr int BC = P10 ? RKB : HKB;
    v4i bh[CT][BC], bl[CT][BC], ba[P10 ? CT : 1][P10 ? RKB : 1];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int kb = 0; kb < BC; ++kb) {
            if (P10) {
                const uint64_t o = fr + (uint64_t)(U.hfrag + (uint32_t)(c * RKB + kb) * 2u) * 2048u;
                bl[c][kb] = *GP6(g_cv4i, o);
                bh[c][kb] = *GP6(g_cv4i, o + 1024);
                ba[P10 ? c : 0][P10 ? kb : 0] = *GP6(g_cv4i, o + 2048);
            } else {
                const uint64_t o = fr + (uint64_t)(U.hfrag + (uint32_t)(c * HKB + kb)) * 2048u;
                bh[c][kb] = *GP6(g_cv4i, o);
                bl[c][kb] = *GP6(g_cv4i, o + 1024);
            }
        }
    // p010 sources, 8-bit outputs: the ordered dither of the lane's 4 values (row y & 7 = m & 7,
    // column (4 g + i) & 7: the units start on 16-column boundaries), luma / U and V (offset 3),
    // as the middle term of the V chain ((d + 128) << 12 = 256 (16 (d + 128)))
    v4i vdit[2];
    if (P10) {
        static constexpr uint8_t kDit[8][8] = DTS_DITHER_8X8_128;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int i = 0; i < 4; ++i) vdit[p][i] = 16 * ((int)kDit[m & 7][(4 * g + i + 3 * p) & 7] + 128);
    }
    // A read offsets in a stage: tile t = (plane t / CT, column tile t % CT), K block kb;
    // B64 variants: the two 8-byte halves of the lane's 16 (windows 8-column aligned)
    constexpr bool B64 = l7_b64(VAR);
    constexpr int NH = B64 ? 2 : 1;
    uint32_t aoff[T][HKB][NH];
    // interleaved chroma (nv12; p010): the U and V operands of column tile c come from the
    // same 32 staged bytes per lane (two 16-B chunks); p010 luma: one 16-B chunk of raw
    // sample bytes per lane and K block
    constexpr bool il = W::NP == 2 && (IL || P10);
    constexpr int ICT = il || P10 ? CT : 1, IKB = il || P10 ? RKB : 1;
    uint32_t ioff[ICT][IKB][2];
    if (il || P10) {
        const uint32_t sw = 2u * (uint32_t)((m >> 3) & 1);
#pragma unroll
        for (int c = 0; c < ICT; ++c)
#pragma unroll
            for (int kb = 0; kb < IKB; ++kb)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // first staged byte of the lane's A chunk(s): nv12 2 (x0 + 64 kb + 16 g),
                    // p010 chroma 4 (x0 + 32 kb + 8 g), p010 luma 2 (x0 + 32 kb + 8 g)
                    const uint32_t b = IL ? 2u * ((uint32_t)U.xo[c] + 64u * (uint32_t)kb + 16u * (uint32_t)g)
                                          : (W::NP == 2 ? 4u : 2u) * ((uint32_t)U.xo[c] + 32u * (uint32_t)kb + 8u * (uint32_t)g);
                    const uint32_t cc = b / 16u + (uint32_t)h;
                    ioff[c][kb][h] = (cc >> 2) * 1024u + 16u * (4u * (uint32_t)m + ((cc & 3u) ^ sw));
                }
    }
    {
        const uint32_t sw = 2u * (uint32_t)((m >> 3) & 1);
#pragma unroll
        for (int t = 0; t < T; ++t)
#pragma unroll
            for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const uint32_t b = (uint32_t)U.xo[t % CT] + 64u * (uint32_t)kb + 16u * (uint32_t)g + 8u * (uint32_t)h;
                    const uint32_t c = b / 16u;
                    aoff[t][kb][h] = (il || P10) ? 0u : (uint32_t)((t / CT) * G.npc) * 1024u + (c >> 2) * 1024u +
                                     16u * (4u * (uint32_t)m + ((c & 3u) ^ sw)) + (B64 ? (b & 8u) : 0u);
                }
    }
    // V: the next row block to run and its fire granule (fg; fg1 the one after, loaded a
    // block ahead so no compare waits on a scalar load); the next one whose fragments
    // this wave DMAs (lead wave of the rendition) and its fire granule (fgf, fgf1)
    // The fire table rides in one VGPR (lane l: fire[l] | fire[64 + l] << 16) and is read
    // with v_readlane: a scalar load per row block would expose its latency at the next
    // LDS wait (SMEM and LDS share lgkmcnt).  Row blocks past 128 read memory.
    k_u32 *fire = GP6(k_u32, P.fire + U.fire);
    const int nrb = U.nrb;
    uint32_t vtab;
    {
        const int32_t *fp = P.fire + U.fire;
        const uint32_t lo = lane < nrb ? (uint32_t)fp[lane] : 0xffffu;
        const uint32_t hi = lane + 64 < nrb ? (uint32_t)fp[lane + 64] : 0xffffu;
        vtab = lo | (hi << 16);
    }
    // a fire entry: the granule (bits 0..9) and, for renditions stored per distinct V fragment
    // (Unit7::vdedup), the row block's fragment index (bits 10..15)
    auto fentry = [&](int i) -> int {
        if (i >= 128) return (int)fire[i];
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)vtab, i & 63);
        return (int)((i & 64 ? x >> 16 : x) & 0xffffu);
    };
    auto firev = [&](int i) -> int { return i >= nrb ? 0x7fffffff : (fentry(i) & 1023); };
    int j = 0, jf = 0;
    int fg = firev(0), fg1 = firev(1);
    int fgf = U.lead ? fg : 0x7fffffff, fgf1 = U.lead ? fg1 : 0x7fffffff;
    const v4i zero = {0, 0, 0, 0}, hbias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    // the ring: slot s of tile t is dword s % 4 of rh[s / 4][t] (hi bytes) and rl (lo bytes)
    v4i rh[VKB][T], rl[VKB][T];
#pragma unroll
    for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
        for (int t = 0; t < T; ++t) rh[kb][t] = rl[kb][t] = zero;
    uint8_t *fb = lds7 + U.flds;
    uint8_t *scr = lds7 + G.scr + 1024 * wave;
    const int FS = U.fs;
    int fsi = 0, fsu = 0;
    // the V fragments of the row blocks firing at granule <= upto (lead wave only)
    auto frags = [&](int upto) {
        while (fgf <= upto) {
            uint8_t *dst = fb + (uint32_t)fsi * (uint32_t)(VKB * 2048);
            const uint32_t fj = U.vdedup ? (uint32_t)fentry(jf) >> 10 : (uint32_t)jf;
            const uint64_t src = fr + (uint64_t)(U.vfrag + fj * (uint32_t)VKB) * 2048u;
            if (!(DTS_L7_ABLATE & 256)) {
                Z.ops += 2 * VKB;
#pragma unroll
                for (int h = 0; h < 2 * VKB; ++h)
                    __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(src + 1024u * h),
                                                     (__attribute__((address_space(3))) void *)(dst + 1024 * h), 16, 0, 0);
            }
            fsi = fsi + 1 == FS ? 0 : fsi + 1;
            ++jf;
            fgf = fgf1;
            fgf1 = firev(jf + 1);
        }
    };
    // the row blocks firing at granule qq (their window's last granule is in the ring)
    auto vfire = [&](int qq) {
        if (DTS_L7_ABLATE & 8) return;
        while (fg == qq) {
            v4i vh[VKB], vl[VKB];
            const uint8_t *fu = fb + (uint32_t)fsu * (uint32_t)(VKB * 2048) + 16u * (uint32_t)lane;
#pragma unroll
            for (int kb = 0; kb < VKB; ++kb) {
                vh[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb);
                vl[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb + 1024);
            }
            fsu = fsu + 1 == FS ? 0 : fsu + 1;
            uint32_t px[4];
            bool p010out = false;
            if constexpr (CT == 1 && P10) {
                if (U.fmt == DTS_FMT_P010LE) {              // p010 rendition
                    uint32_t w2[T][2];
                    vcalc7p<VAR>(rh, rl, vh, vl, w2);
                    xchg7p<VAR>(U, w2, scr, m, g, lane, px);
                    p010out = true;
                }
            }
            if (!p010out) {
                uint32_t w[T];
                if (DTS_L7_ABLATE & 128) {
#pragma unroll
                    for (int t = 0; t < T; ++t) w[t] = (uint32_t)(rh[0][t][0] ^ vh[0][t & 3]);
                } else {
                    vcalc7<VAR, P10>(rh, rl, vh, vl, vdit, w);
                }
                if (DTS_L7_ABLATE & 64) {
#pragma unroll
                    for (int t = 0; t < T; ++t) asm volatile("" ::"v"(w[t]));
                } else {
                    xchg7<VAR>(U, w, scr, m, g, lane, px);
                }
            }
            if (!(DTS_L7_ABLATE & 96)) Z.ops += vstore7<VAR>(U, j, px, ob, op, lane);
            ++j;
            fg = fg1;
            fg1 = firev(j + 1);
        }
    };
#pragma unroll
    for (int i = 0; i < NS7 - 1; ++i) {
        frags(PB7 * i + PB7 - 1);
        Z.pieces(lds7, i, i);
        Z.e[i] = Z.ops;
    }
    // unrolled by the ring length (8 covers both), so ring slot q % R is a fixed register
    // in each copy; stage q % NS7 is a run-time offset.  Per granule q: its A reads go out
    // first, then the DMA of granule q + NS7 - 1, then (DTS_L7_DEFER) the row blocks that
    // fired at q - 1 -- the ring still holds granules q - R .. q - 1 -- while the A reads
    // land, then H(q) into ring slot q % R.
    // UNR: the walk's unroll -- the ring length R (4 granules for the one-V-K-block walks, 8 for
    // two), or 8 for every walk (DTS_L7_UNROLL8, the round-3 shape: twice the code of the
    // one-K-block walks, whose copies compete for the CU pair's instruction cache)
#ifndef DTS_L7_UNROLL8
#define DTS_L7_UNROLL8 1
#endif
    constexpr int UNR = DTS_L7_UNROLL8 ? 8 : (R > 2 * PB7 ? R : 2 * PB7);
    static_assert(UNR % R == 0 && UNR % PB7 == 0, "ring and batch periods divide the unroll");
    const int ngran = G.ngran;
    int sq = 0;
    L7_STAMP_INIT;
    for (int q0 = 0; q0 < ngran; q0 += UNR) {
#pragma unroll
        for (int s = 0; s < UNR; ++s) {
            const int q = q0 + s;
            if (q >= ngran) break;
            if (s % PB7 == 0) {
                Z.wait_batch();
                L7_STAMP(0);
                group_barrier7();
                L7_STAMP(1);
            }
            v4i a[T][RKB];
            if (DTS_L7_ABLATE & 16) {
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int kb = 0; kb < RKB; ++kb) a[t][kb] = (v4i){0, 0, 0, 0};
            } else if (P10) {
                // raw sample bytes masked to (s >> 2, (s & 3) << 6) ^ 0x80 (one v_bitop3 per dword)
                const uint8_t *st = lds7 + sq * Z.stage_bytes + (s % PB7) * Z.npieces * 1024;
#pragma unroll
                for (int c = 0; c < CT; ++c)
#pragma unroll
                    for (int kb = 0; kb < RKB; ++kb) {
                        if (W::NP == 1) {
                            const v4i x = *reinterpret_cast<const v4i *>(st + ioff[c][kb][0]);
                            a[c][kb] = (x & (int)0xFFC0FFC0u) ^ (int)0x80808080u;
                        } else {
                            // U V 16-bit pairs: dword 2 q + h = [U lo, U hi, V lo, V hi] of sample 2 q + h
                            const v4i x = *reinterpret_cast<const v4i *>(st + ioff[c][kb][0]);
                            const v4i y = *reinterpret_cast<const v4i *>(st + ioff[c][kb][1]);
                            const uint32_t w8[8] = {(uint32_t)x.x, (uint32_t)x.y, (uint32_t)x.z, (uint32_t)x.w,
                                                    (uint32_t)y.x, (uint32_t)y.y, (uint32_t)y.z, (uint32_t)y.w};
#pragma unroll
                            for (int q4 = 0; q4 < 4; ++q4) {
                                const uint32_t u = __builtin_amdgcn_perm(w8[2 * q4 + 1], w8[2 * q4], 0x05040100u);
                                const uint32_t v = __builtin_amdgcn_perm(w8[2 * q4 + 1], w8[2 * q4], 0x07060302u);
                                a[c][kb][q4] = (int)((u & 0xFFC0FFC0u) ^ 0x80808080u);
                                a[CT + c][kb][q4] = (int)((v & 0xFFC0FFC0u) ^ 0x80808080u);
                            }
                        }
                    }
            } else if (il) {
                // nv12 chroma: even bytes are U, odd bytes V (yuv2nv12 order, input.c nv12ToUV_c)
                const uint8_t *st = lds7 + sq * Z.stage_bytes + (s % PB7) * Z.npieces * 1024;
#pragma unroll
                for (int c = 0; c < CT; ++c)
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb) {
                        const v4i x = *reinterpret_cast<const v4i *>(st + ioff[c][kb][0]);
                        const v4i y = *reinterpret_cast<const v4i *>(st + ioff[c][kb][1]);
                        const uint32_t w8[8] = {(uint32_t)x.x, (uint32_t)x.y, (uint32_t)x.z, (uint32_t)x.w,
                                                (uint32_t)y.x, (uint32_t)y.y, (uint32_t)y.z, (uint32_t)y.w};
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4) {
                            a[c][kb][q4] = (int)__builtin_amdgcn_perm(w8[2 * q4 + 1], w8[2 * q4], 0x06040200u);
                            a[CT + c][kb][q4] = (int)__builtin_amdgcn_perm(w8[2 * q4 + 1], w8[2 * q4], 0x07050301u);
                        }
                    }
            } else {
                const uint8_t *st = lds7 + sq * Z.stage_bytes + (s % PB7) * Z.npieces * 1024;
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb) {
                        if (B64) {
                            typedef int v2i __attribute__((ext_vector_type(2)));
                            const v2i x = *reinterpret_cast<const v2i *>(st + aoff[t][kb][0]);
                            const v2i y = *reinterpret_cast<const v2i *>(st + aoff[t][kb][NH - 1]);
                            a[t][kb] = (v4i){x.x, x.y, y.x, y.y};
                        } else {
                            a[t][kb] = *reinterpret_cast<const v4i *>(st + aoff[t][kb][0]);
                        }
                    }
            }
            // the next batch's pieces, right after the A reads
            if (s % PB7 == 0) {
                const int sn = sq == 0 ? NS7 - 1 : sq - 1, bn = q / PB7 + NS7 - 1;
                frags(PB7 * bn + PB7 - 1);
                Z.pieces(lds7, bn, sn);
                Z.shift();
            }
            L7_STAMP(2);
            if (DTS_L7_DEFER) vfire(q - 1);
            L7_STAMP(4);
            if (!(DTS_L7_ABLATE & 16)) {
                v4i ah[T], al[T];
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    ah[t] = zero;
                    al[t] = hbias;
                }
                if (P10) {
                    // L from K, >> 8, + M, >> 7, + A: y = FFMIN(sum(s c) >> 9, ...) before the pack
                    const v4i kp = {538968064, 538968064, 538968064, 538968064};   // 32896 << 14
#pragma unroll
                    for (int t = 0; t < T; ++t) al[t] = kp;
#pragma unroll
                    for (int kb = 0; kb < RKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bl[t % CT][kb], al[t], 0, 0, 0);
#pragma unroll
                    for (int t = 0; t < T; ++t) al[t] >>= 8;
#pragma unroll
                    for (int kb = 0; kb < RKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bh[t % CT][kb], al[t], 0, 0, 0);
#pragma unroll
                    for (int t = 0; t < T; ++t) ah[t] = al[t] >> 7;
#pragma unroll
                    for (int kb = 0; kb < RKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            ah[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], ba[P10 ? t % CT : 0][P10 ? kb : 0],
                                                                          ah[t], 0, 0, 0);
                } else if (HS == 128) {
                    v4i x[T][HKB];
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t) {
                            x[t][kb] = a[t][kb] ^ ((DTS_L7_ABLATE & 2) ? 0 : (int)0x80808080u);
                            al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[t][kb], bl[t % CT][kb], al[t], 0, 0, 0);
                        }
#pragma unroll
                    for (int t = 0; t < T; ++t) ah[t] = al[t] >> 7;
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            ah[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x[t][kb], bh[t % CT][kb], ah[t], 0, 0, 0);
                } else {
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t) {
                            const v4i x = a[t][kb] ^ ((DTS_L7_ABLATE & 2) ? 0 : (int)0x80808080u);
                            ah[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, bh[t % CT][kb], ah[t], 0, 0, 0);
                            al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, bl[t % CT][kb], al[t], 0, 0, 0);
                        }
                }
                const int rs = s % R;
#define WRING(t_, hv_, lv_)                                                                   \
    do {                                                                                      \
        rh[rs / 4][(t_)][rs % 4] = (int)(hv_);                                                \
        rl[rs / 4][(t_)][rs % 4] = (int)(lv_);                                                \
    } while (0)
                if ((HS == 128 || P10) && !RC) {
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        const uint32_t p0 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(ah[t].x, ah[t].y));
                        const uint32_t p1 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(ah[t].z, ah[t].w));
                        WRING(t, __builtin_amdgcn_perm(p1, p0, 0x07050301u), __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
                    }
                } else if (!RC) {
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        const uint32_t p0 = pack_h6(ah[t].x, al[t].x, ah[t].y, al[t].y);   // rows 4g, 4g+1
                        const uint32_t p1 = pack_h6(ah[t].z, al[t].z, ah[t].w, al[t].w);   // rows 4g+2, 4g+3
                        WRING(t, __builtin_amdgcn_perm(p1, p0, 0x07050301u), __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
                    }
                } else {
                    // range conversion of the 15-bit H output (swscale.c lum/chrRange{To,From}Jpeg_c:
                    // FFMIN(y, cap) * mul + add, >> sh, stored as int16)
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        int y[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int v = min((HS == 128 || P10) ? ah[t][i] : ((ah[t][i] << 8) + al[t][i]) >> 7, 32767);
                            y[i] = (min(v, U.rc_cap) * U.rc_mul + U.rc_add) >> U.rc_sh;
                        }
                        const uint32_t p0 = __builtin_amdgcn_perm((uint32_t)y[1], (uint32_t)y[0], 0x05040100u);
                        const uint32_t p1 = __builtin_amdgcn_perm((uint32_t)y[3], (uint32_t)y[2], 0x05040100u);
                        WRING(t, __builtin_amdgcn_perm(p1, p0, 0x07050301u), __builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
                    }
                }
            }
#undef WRING
            L7_STAMP(3);
            if (!DTS_L7_DEFER) vfire(q);
            L7_STAMP(4);
            if (s % PB7 == PB7 - 1) sq = sq + 1 == NS7 ? 0 : sq + 1;
        }
    }
    if (DTS_L7_DEFER) vfire(ngran - 1);
    // the pieces and fragments past the plane were not issued; drain the rest before the
    // workgroup's LDS goes away
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    L7_STAMP_DONE(VAR, ngran);
}

#ifndef DTS_L7_WPE
#define DTS_L7_WPE 0        // > 0: ask the compiler for at least this many waves per SIMD (register budget)
#endif

// RC: the graph converts the YUV range in the H epilogue (a separate instantiation, so
// the common kernel keeps its register allocation)
template <bool RC, int HS, int SK>
__global__ __launch_bounds__(64 * kL7MaxWaves)
#if DTS_L7_WPE > 0
__attribute__((amdgpu_waves_per_eu(DTS_L7_WPE)))
#endif
void k_ladder7(Ladder7Params P)
{
    // workgroup b: XCD b % 8, frame 8 fq + b % 8 of frame octet fq, k = b / 8.  Order 1 (the
    // default): k runs over every octet's luma groups, then over every octet's chroma groups;
    // order 0: each octet's groups in plan order (k / ngroups, k % ngroups); order 2: chroma first
    const int b = (int)blockIdx.x, k = b >> 3;
    int fq, gi;
    if (P.order == 0) {
        fq = k / P.ngroups;
        gi = k - fq * P.ngroups;
    } else if (P.order == 3) {              // diagnostic: luma then chroma per run of P.sup octets
        const int run = P.sup * P.ngroups, r = k / run, kr = k - r * run;
        const int nfq = (P.nframes + 7) >> 3, s0 = r * P.sup, ns = min(P.sup, nfq - s0);
        const int nl = P.nluma, nc = P.ngroups - nl;
        if (kr < ns * nl) {
            fq = s0 + kr / nl;
            gi = kr % nl;
        } else {
            const int k1 = kr - ns * nl;
            fq = s0 + k1 / nc;
            gi = nl + k1 % nc;
        }
    } else {
        const int nfq = (P.nframes + 7) >> 3;
        const int n0 = P.order == 1 ? P.nluma : P.ngroups - P.nluma, a0 = P.order == 1 ? 0 : P.nluma;
        const int n1 = P.ngroups - n0, a1 = P.order == 1 ? P.nluma : 0;
        if (k < nfq * n0) {
            fq = k / n0;
            gi = a0 + (k - fq * n0);
        } else {
            const int k1 = k - nfq * n0;
            fq = k1 / n1;
            gi = a1 + (k1 - fq * n1);
        }
    }
    const int f = 8 * fq + (b & 7);
    if (f >= P.nframes) return;
    const Group7 G = kld6(P.groups + gi);
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), waves = (int)blockDim.x >> 6;
    const uint8_t *ka = (const uint8_t *)__builtin_amdgcn_kernarg_segment_ptr();
    const DevPlanes S = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder7Params, src)));
    if (wave >= G.nwaves) {
        idle7<SK>(G, S, f, wave, waves);
        return;
    }
    const Unit7 U = kld6(P.units + G.u0 + wave);
#ifdef DTS_L7_ONLYVAR                       // disassembly studies of one variant's walk
    if constexpr ((SK == 2) == ((DTS_L7_ONLYVAR & 16) != 0)) {
        walk7<DTS_L7_ONLYVAR, RC, HS, SK>(P, G, U, S, f, wave, waves);
        return;
    }
#endif
    if constexpr (SK == 2) {                // p010 sources: the 16-bit one-K-block variants
        switch (U.variant) {
        case 16: walk7<16, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
        case 17: walk7<17, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
        default: walk7<20, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
        }
    } else {
    switch (U.variant) {
    case 0: walk7<0, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 1: walk7<1, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 2: walk7<2, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 3: walk7<3, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 4: walk7<4, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 5: walk7<5, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 6: walk7<6, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 7: walk7<7, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    case 8: walk7<8, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    default: walk7<12, RC, HS, SK>(P, G, U, S, f, wave, waves); break;
    }
    }
}

} // namespace

#if DTS_L7_STAMP
int ladder7_stamps(unsigned long long *out, bool reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l7_stamp), sizeof(g_l7_stamp)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[(kL7Variants + 1) * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_l7_stamp), z, sizeof z) != hipSuccess) return -1;
    }
    return (kL7Variants + 1) * 8;
}
#endif

// the staging geometry this build of k_ladder7 was compiled with: the planner sizes the
// stage buffers and the V fragment slots for exactly these, and refuses any other
void ladder7_compiled(int *stages, int *batch)
{
    *stages = NS7;
    *batch = PB7;
}

hipError_t launch_ladder7(const Ladder7Params &p, int grid, int waves, int lds_bytes, bool range_conv, int hsplit,
                          int src_kind, hipStream_t s)
{
    if (waves < 1 || waves > kL7MaxWaves || (hsplit != 128 && hsplit != 256)) return hipErrorInvalidValue;
    const dim3 g(grid), b(64 * waves);
    if (src_kind == kSrcP010) {          // p010 sources (the 15-bit converters too: dstBpc <= 14)
        if (range_conv)
            hipLaunchKernelGGL((k_ladder7<true, 256, 2>), g, b, lds_bytes, s, p);
        else
            hipLaunchKernelGGL((k_ladder7<false, 256, 2>), g, b, lds_bytes, s, p);
        return hipGetLastError();
    }
    if (src_kind == kSrcNV12) {          // nv12 sources
        if (range_conv && hsplit == 128)
            hipLaunchKernelGGL((k_ladder7<true, 128, 1>), g, b, lds_bytes, s, p);
        else if (range_conv)
            hipLaunchKernelGGL((k_ladder7<true, 256, 1>), g, b, lds_bytes, s, p);
        else if (hsplit == 128)
            hipLaunchKernelGGL((k_ladder7<false, 128, 1>), g, b, lds_bytes, s, p);
        else
            hipLaunchKernelGGL((k_ladder7<false, 256, 1>), g, b, lds_bytes, s, p);
        return hipGetLastError();
    }
    if (range_conv && hsplit == 128)
        hipLaunchKernelGGL((k_ladder7<true, 128, 0>), g, b, lds_bytes, s, p);
    else if (range_conv)
        hipLaunchKernelGGL((k_ladder7<true, 256, 0>), g, b, lds_bytes, s, p);
    else if (hsplit == 128)
        hipLaunchKernelGGL((k_ladder7<false, 128, 0>), g, b, lds_bytes, s, p);
    else
        hipLaunchKernelGGL((k_ladder7<false, 256, 0>), g, b, lds_bytes, s, p);
    return hipGetLastError();
}

} // namespace dts
