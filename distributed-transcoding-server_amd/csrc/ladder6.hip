// ladder6.hip -- k_ladder6, the v6 ladder kernel: 8-bit 4:2:0 planar sources
// to 8-bit renditions, both FIR passes on the matrix cores
// (v_mfma_i32_16x16x64_i8), the H outputs never leaving the VGPRs.
//
// Same arithmetic as libswscale hScale8To15_c -> yuv2planeX_8_c /
// yuv2nv12cX_c under SWS_BITEXACT|SWS_ACCURATE_RND (FFmpeg 4.4; bit-exact,
// DESIGN.md "Oracle"), and the same integer identities as k_ladder5
// (ladder5.hip header), organised so that nothing is shared between waves:
//
//  * one wave = one work unit: CT 16-column tiles of one rendition of one plane
//    kind (chroma: the same columns of U and V) of one frame, walked top to
//    bottom in granules of 16 source rows.  Workgroups are single waves; the
//    units of frame f all run on XCD f % 8 (workgroup ids go round robin over
//    the XCDs), so a frame's source rows are fetched from HBM into one L2 and
//    re-read from there by the other units of the frame;
//  * H of a granule: per tile one MFMA per K block and tap half.  A = 16 source
//    rows x 64 columns straight from memory (one 16-B load per lane, the bytes
//    x0 + 64 kb + 16 g .. + 15 of row m), xor 0x80; B = the tile's taps, held in
//    VGPRs for the whole walk (plan6.cpp K order);
//  * the H result of a tile is, per lane, 4 consecutive source rows of one
//    output column -- exactly a V A-operand dword once split into y >> 8 and
//    (y & 255) ^ 0x80 bytes.  The last 4 VKB granules of every tile stay in a
//    register ring (slot = granule mod 4 VKB; the walk is unrolled by the ring
//    length so every slot is a fixed register);
//  * V of a row block (16 output rows) runs right after the granule that
//    completes its window: out^T = H^T C^T over the whole ring, 4 MFMAs per K
//    block, the fragment laid out for where each granule sits in the ring;
//  * stores: each lane holds 4 consecutive columns of one output row per tile;
//    v_permlane32/16_swap transpose the tiles so a lane holds 16 (CT 4) or 8
//    consecutive bytes of its row (nv12: U and V interleaved by v_perm).
#include "dts_internal.h"

#ifndef DTS_L6_NS
#define DTS_L6_NS 2         // LDS stages per wave: source granules in flight (DMA'd NS granules ahead)
#endif
#ifndef DTS_L6_ABLATE
#define DTS_L6_ABLATE 0     // diagnostic builds only: 1 skip the source loads, 2 skip the V blocks, 8 load
                            // one (tile, K block) of source per granule and feed it to every tile,
                            // 4 skip the V stores
#endif
#ifndef DTS_L6_LDSPAD
#define DTS_L6_LDSPAD 0     // diagnostic builds only: extra LDS per wave (fewer waves per CU)
#endif
#ifndef DTS_L6_WPE
#define DTS_L6_WPE 0        // > 0: ask the compiler for at least this many waves per SIMD
#endif

#include "ladder_mfma.h"

#ifndef DTS_L6_STAMP
#define DTS_L6_STAMP 0      // diagnostic builds only: per-variant, per-phase s_memtime sums (tools/stamp6.py)
#endif

namespace dts {

#if DTS_L6_STAMP
// [variant][phase]: cycles summed over every wave; [variant][6]: granules, [variant][7]: waves
__device__ unsigned long long g_l6_stamp[kL6Variants][8];
#define L6_STAMP(k)                                                        \
    do {                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();        \
        st_acc[k] += t_ - st_last;                                         \
        st_last = t_;                                                      \
    } while (0)
#else
#define L6_STAMP(k) (void)0
#endif

namespace {

template <int VAR>
__device__ __forceinline__ void walk6(const Ladder6Params &P, const Unit6 &U, int f)
{
    using W = Walk6<VAR>;
    constexpr int CT = W::CT, NP = W::NP, HKB = W::HKB, VKB = W::VKB, T = W::T, R = W::R;
    const int lane = (int)threadIdx.x, m = lane & 15, g = lane >> 4;
    // source planes of this frame (luma: plane 0; chroma: planes 1 and 2)
    // (the plane tables are read from the kernarg segment by s_load: indexing the by-value
    // parameter with a run-time index would copy it to scratch)
    const uint8_t *ka = (const uint8_t *)__builtin_amdgcn_kernarg_segment_ptr();
    const DevPlanes S = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder6Params, src)));
    uint64_t sb[NP];
    uint32_t sp[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        sb[p] = (U.kind ? S.data[1 + p] : S.data[0]) + (uint64_t)f * (uint64_t)S.fstride;
        sp[p] = (uint32_t)(U.kind ? S.pitch[1 + p] : S.pitch[0]);
    }
    // output planes: luma plane 0; nv12 chroma plane 1; yuv420p chroma planes 1 and 2
    uint64_t ob[2];
    uint32_t op[2];
    {
        const DevPlanes D = kld6(reinterpret_cast<const DevPlanes *>(ka + offsetof(Ladder6Params, dst)) + U.rung);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            ob[p] = (U.kind ? D.data[1 + p] : D.data[0]) + (uint64_t)f * (uint64_t)D.fstride;
            op[p] = (uint32_t)(U.kind ? D.pitch[1 + p] : D.pitch[0]);
        }
    }
    (void)P;
    const uint64_t fr = (uint64_t)(uintptr_t)P.frag + 16u * (uint32_t)lane;
    // H B operands of the walk
    v4i bh[CT][HKB], bl[CT][HKB];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int kb = 0; kb < HKB; ++kb) {
            const uint64_t o = fr + (uint64_t)(U.hfrag + (uint32_t)(c * HKB + kb)) * 2048u;
            bh[c][kb] = *GP6(g_cv4i, o);
            bl[c][kb] = *GP6(g_cv4i, o + 1024);
        }
    // V: the next row block to run and its fire granule; the next one whose fragments are
    // to be DMA'd and its fire granule
    k_u32 *fire = GP6(k_u32, P.fire + U.fire);
    int j = 0, jf = 0;
    int fg = U.nrb > 0 ? (int)fire[0] : 0x7fffffff, fgf = fg;
    v4i vh[VKB], vl[VKB];
    const v4i zero = {0, 0, 0, 0}, hbias = {kL5Bias, kL5Bias, kL5Bias, kL5Bias};
    // the ring: slot s of tile t is dword s % 4 of rh[s / 4][t] (hi bytes) and rl (lo bytes)
    v4i rh[VKB][T], rl[VKB][T];
#pragma unroll
    for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
        for (int t = 0; t < T; ++t) rh[kb][t] = rl[kb][t] = zero;
    const int ngran = U.ngran, srcH1 = U.srcH - 1;
#if DTS_L6_STAMP
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    // A operands: the 16 rows x 64 bytes of every (plane, tile, K block) reach this wave's
    // LDS by LDS-DMA, NS granules ahead (stage q % NS).  DMA lane l loads row l >> 2, chunk
    // (l & 3) ^ ((l >> 4) & 3) of the 64 bytes: four lanes cover one row's 64 contiguous
    // bytes (one cache access instead of four), and the A read of lane (m, g) -- row m,
    // chunk g -- is a conflict-free ds_read_b128 at 16 (4 m + (g ^ ((m >> 2) & 3))).
    constexpr int NS = DTS_L6_NS, ND = T * HKB;
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds6[];
    const int dr = lane >> 2, dch = (lane & 3) ^ ((dr >> 2) & 3);
    uint32_t dcol[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) dcol[c] = (uint32_t)U.x0[c] + 16u * (uint32_t)dch;
    const uint32_t roff = 16u * (uint32_t)(4 * m + (g ^ ((m >> 2) & 3)));
    // V fragment slots after the stages: row block j's fragments in slot j % fs, DMA'd right
    // after the source of its fire granule, so the source wait covers them too
    uint8_t *fb = lds6 + NS * ND * 1024;
    const int FS = U.fs;
    int fsi = 0, fsu = 0;
    int ops = 0;                                           // VMEM instructions issued so far
    int oend[NS];                                          // ops after the batch of granule q (slot q % NS)
    auto frags = [&](int upto) {
        while (fgf <= upto) {
            ops += 2 * VKB;
            uint8_t *dst = fb + (uint32_t)fsi * (uint32_t)(VKB * 2048);
            const uint64_t src = fr + (uint64_t)(U.vfrag + (uint32_t)(jf * VKB)) * 2048u;
#pragma unroll
            for (int h = 0; h < 2 * VKB; ++h)
                __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(src + 1024u * h),
                                                 (__attribute__((address_space(3))) void *)(dst + 1024 * h), 16, 0, 0);
            fsi = fsi + 1 == FS ? 0 : fsi + 1;
            ++jf;
            fgf = jf < U.nrb ? (int)fire[jf] : 0x7fffffff;
        }
    };
    // one batch: the fragments of the row blocks firing at granule q, then granule q's source
    auto dma = [&](int q) {
        frags(q);
        if (DTS_L6_ABLATE & 1) return;
        const uint32_t row = (uint32_t)min(kL6Gran * q + dr, srcH1);
        uint8_t *st = lds6 + (uint32_t)(q % NS) * (uint32_t)(ND * 1024);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const uint64_t rp = sb[p] + (uint64_t)(row * sp[p]);
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
                    if (!(DTS_L6_ABLATE & 8) || (p * CT + c) * HKB + kb == 0)
                    {
                        __builtin_amdgcn_global_load_lds(
                            (const void *)(uintptr_t)(rp + dcol[c] + 64u * kb),
                            (__attribute__((address_space(3))) void *)(st + 1024 * ((p * CT + c) * HKB + kb)), 16, 0, 0);
                        ++ops;
                    }
        }
    };
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) {
        dma(i);
        oend[i] = ops;
    }
    // the walk is unrolled by the ring length, so ring slot q % R and stage q % NS are
    // fixed registers / offsets in each copy; granules past the plane (to a whole ring
    // period) are computed and never used
    static_assert(R % NS == 0, "the stages cycle within a ring period");
    const int ngp = (ngran + R - 1) / R * R;
    for (int q0 = 0; q0 < ngp; q0 += R) {
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const int q = q0 + s;
            // granule q + NS - 1 into the stage granule q - 1 was read from (its ds_reads
            // completed before its MFMAs); past the plane: clamped rows, unused, which keeps
            // the count uniform
            L6_STAMP(4);
            dma(q + NS - 1);
            oend[(s + NS - 1) % NS] = ops;
            L6_STAMP(0);
            // granule q's batch (its source and the fragments of the row blocks firing at
            // q) has landed: every VMEM instruction issued after it may still be in flight
            vm_wait_n6<(NS - 1) * ((DTS_L6_ABLATE & (1 | 8)) ? (DTS_L6_ABLATE & 1 ? 0 : 1) : ND)>(ops - oend[s % NS]);
            L6_STAMP(1);
            {
                const uint8_t *st = lds6 + (s % NS) * (ND * 1024) + roff;
                v4i a[T][HKB];
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int kb = 0; kb < HKB; ++kb)
                        a[t][kb] = *reinterpret_cast<const v4i *>(st + ((DTS_L6_ABLATE & 8) ? 0 : 1024 * (t * HKB + kb))) ^
                                   (int)0x80808080u;
                v4i ah[T], al[T];
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    ah[t] = zero;
                    al[t] = hbias;
                }
#pragma unroll
                for (int kb = 0; kb < HKB; ++kb)
#pragma unroll
                    for (int t = 0; t < T; ++t) {
                        ah[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bh[t % CT][kb], ah[t], 0, 0, 0);
                        al[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t][kb], bl[t % CT][kb], al[t], 0, 0, 0);
                    }
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const uint32_t p0 = pack_h6(ah[t].x, al[t].x, ah[t].y, al[t].y);   // rows 4g, 4g+1
                    const uint32_t p1 = pack_h6(ah[t].z, al[t].z, ah[t].w, al[t].w);   // rows 4g+2, 4g+3
                    rh[s / 4][t][s % 4] = (int)__builtin_amdgcn_perm(p1, p0, 0x07050301u);
                    rl[s / 4][t][s % 4] = (int)(__builtin_amdgcn_perm(p1, p0, 0x06040200u) ^ 0x80808080u);
                }
            }
            L6_STAMP(2);
            while (fg == q) {
                {
                    const uint8_t *fu = fb + (uint32_t)fsu * (uint32_t)(VKB * 2048) + 16u * (uint32_t)lane;
#pragma unroll
                    for (int kb = 0; kb < VKB; ++kb) {
                        vh[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb);
                        vl[kb] = *reinterpret_cast<const v4i *>(fu + 2048 * kb + 1024);
                    }
                    fsu = fsu + 1 == FS ? 0 : fsu + 1;
                }
                if (!(DTS_L6_ABLATE & 2)) {
                    ops += vblock<VAR>(U, j, rh, rl, vh, vl, ob, op, m, g, fb + FS * VKB * 2048);
                } else {
#pragma unroll
                    for (int kb = 0; kb < VKB; ++kb)
#pragma unroll
                        for (int t = 0; t < T; ++t)
                            asm volatile("" ::"v"(rh[kb][t]), "v"(rl[kb][t]), "v"(vh[kb]), "v"(vl[kb]));
                }
                ++j;
                fg = j < U.nrb ? (int)fire[j] : 0x7fffffff;
                L6_STAMP(3);
            }
        }
    }
    // the DMAs past the plane still write this workgroup's LDS: drain them before the
    // wave (and its LDS allocation) ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if DTS_L6_STAMP
    L6_STAMP(5);
    if (lane == 0) {
        for (int k = 0; k < 6; ++k) atomicAdd(&g_l6_stamp[VAR][k], st_acc[k]);
        atomicAdd(&g_l6_stamp[VAR][6], (unsigned long long)ngp);
        atomicAdd(&g_l6_stamp[VAR][7], 1ull);
    }
#endif
}

__global__ __launch_bounds__(64)
#if DTS_L6_WPE > 0
__attribute__((amdgpu_waves_per_eu(DTS_L6_WPE)))
#endif
void k_ladder6(Ladder6Params P)
{
    // workgroup b: XCD b % 8; frame 8 (k / nunits) + b % 8, unit k % nunits (k = b / 8)
    const int b = (int)blockIdx.x, k = b >> 3;
    const int fq = k / P.nunits;
    const int f = 8 * fq + (b & 7);
    if (f >= P.nframes) return;
    const Unit6 U = kld6(P.units + (k - fq * P.nunits));
    switch (U.variant) {
    case 0: walk6<0>(P, U, f); break;
    case 1: walk6<1>(P, U, f); break;
    case 2: walk6<2>(P, U, f); break;
    case 3: walk6<3>(P, U, f); break;
    case 4: walk6<4>(P, U, f); break;
    case 5: walk6<5>(P, U, f); break;
    case 6: walk6<6>(P, U, f); break;
    default: walk6<7>(P, U, f); break;
    }
}

} // namespace

#if DTS_L6_STAMP
int ladder6_stamps(unsigned long long *out, bool reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l6_stamp), sizeof(g_l6_stamp)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[kL6Variants * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_l6_stamp), z, sizeof z) != hipSuccess) return -1;
    }
    return kL6Variants * 8;
}
#endif

static_assert(DTS_L6_NS <= kL6Stages, "the planner sizes the fragment slots for kL6Stages granules");

int ladder6_lds_bytes(const Unit6 &u)
{
    const int v = u.variant;
    return DTS_L6_NS * l6_ct(v) * l6_np(v) * l6_hkb(v) * 1024 + u.fs * l6_vkb(v) * 2048 + 1024 +   // + store scratch
           DTS_L6_LDSPAD;
}

hipError_t launch_ladder6(const Ladder6Params &p, int grid, int lds_bytes, hipStream_t s)
{
    hipLaunchKernelGGL(k_ladder6, dim3(grid), dim3(64), lds_bytes, s, p);
    return hipGetLastError();
}

} // namespace dts
