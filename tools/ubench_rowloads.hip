// ubench_rowloads.hip -- does a lane-per-row 16-B load pattern stream as fast
// as a coalesced one?  The H pass of k_ladder4 gives each lane one source row
// pair and loads the row window straight into VGPRs (global_load_dwordx4,
// consecutive instructions sweep the window).  This times that shape against
// the coalesced shape over the same bytes.
//
//   tile  = 128 rows x W bytes of a 3840-byte-pitch plane
//   rowpl : lane l loads rows 2l and 2l+1, W/16 dwordx4 each (the v4 H shape)
//   coal  : lanes sweep the tile row-major, 16 B per lane (coalesced)
// Each workgroup (4 waves) takes 4 adjacent tiles of one 128-row band; the
// grid covers every frame of a ring larger than the Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_rowloads.hip -o tools/ubench_rowloads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kPitch = 3840, kRows = 2160;

template <int W>
__global__ void __launch_bounds__(256) rowpl(const uint8_t *__restrict__ src, long long fstride, int tiles_x,
                                             unsigned *__restrict__ out)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int per_frame = tiles_x / 4 * (kRows / 128);
    const int f = blockIdx.x / per_frame, r = blockIdx.x % per_frame;
    const int band = r / (tiles_x / 4), tx = (r % (tiles_x / 4)) * 4 + wave;
    const uint8_t *base = src + (long long)f * fstride + (long long)(band * 128 + 2 * lane) * kPitch + tx * W;
    uint4 v[2][W / 16];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int k = 0; k < W / 16; ++k) v[q][k] = *reinterpret_cast<const uint4 *>(base + q * kPitch + 16 * k);
    unsigned acc = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int k = 0; k < W / 16; ++k) acc += v[q][k].x ^ v[q][k].y ^ v[q][k].z ^ v[q][k].w;
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int W>
__global__ void __launch_bounds__(256) coal(const uint8_t *__restrict__ src, long long fstride, int tiles_x,
                                            unsigned *__restrict__ out)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int per_frame = tiles_x / 4 * (kRows / 128);
    const int f = blockIdx.x / per_frame, r = blockIdx.x % per_frame;
    const int band = r / (tiles_x / 4), tx = (r % (tiles_x / 4)) * 4 + wave;
    const uint8_t *base = src + (long long)f * fstride + (long long)(band * 128) * kPitch + tx * W;
    constexpr int chunks = 128 * W / 16;
    uint4 v[chunks / 64];
#pragma unroll
    for (int k = 0; k < chunks / 64; ++k) {
        const int c = lane + 64 * k, row = c / (W / 16), col = c % (W / 16);
        v[k] = *reinterpret_cast<const uint4 *>(base + (long long)row * kPitch + 16 * col);
    }
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < chunks / 64; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int W>
static void run(const uint8_t *src, long long fstride, int nframes, unsigned *out)
{
    const int tiles_x = kPitch / W / 4 * 4;
    const int blocks = nframes * (tiles_x / 4) * (kRows / 128);
    const double bytes = (double)blocks * 4 * 128 * W;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int variant = 0; variant < 2; ++variant) {
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
            CHK(hipEventRecord(a));
            if (variant == 0)
                hipLaunchKernelGGL(rowpl<W>, dim3(blocks), dim3(256), 0, 0, src, fstride, tiles_x, out);
            else
                hipLaunchKernelGGL(coal<W>, dim3(blocks), dim3(256), 0, 0, src, fstride, tiles_x, out);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (it > 0 && ms < best) best = ms;
        }
        std::printf("W=%3d %-6s %8.3f ms  %7.1f GB/s\n", W, variant ? "coal" : "rowpl", best, bytes / best / 1e6);
    }
}

int main()
{
    const int nframes = 96;
    const long long fstride = (long long)kPitch * kRows;
    uint8_t *src = nullptr;
    unsigned *out = nullptr;
    CHK(hipMalloc(&src, fstride * nframes));
    CHK(hipMalloc(&out, 1 << 24));
    CHK(hipMemset(src, 1, fstride * nframes));
    run<32>(src, fstride, nframes, out);
    run<64>(src, fstride, nframes, out);
    run<128>(src, fstride, nframes, out);
    return 0;
}
