// fetch_micro.hip -- calibrates rocprofv3 FETCH_SIZE on gfx950 for the access widths the encode
// kernels use (tools only).  The guide (MI355X_MICROARCH.md, HBM section)
// calibrates 16-B-per-lane streaming reads only (FETCH_SIZE = 1/2 of the bytes); the c4 (8-channel
// 24-bit) analysis and pack stage their PCM with 4-B LDS-DMA (global_load_lds_dword), and the
// channel-half split reads half of every 24-B interchannel row.  Each kernel below reads a known
// byte count from a buffer far larger than the 256 MiB Infinity Cache; run it under
//   rocprofv3 --pmc FETCH_SIZE      and      rocprofv3 --kernel-trace --stats
// and divide FETCH_SIZE x 1024 by the "bytes" the program prints per kernel (tools/fetch_calib.py).
//
//   m0 g16    global_load_dwordx4, 16 B/lane, contiguous       (the guide's calibrated case)
//   m1 dma16  global_load_lds_dwordx4, 16 B/lane, contiguous
//   m2 dma4   global_load_lds_dword, 4 B/lane, contiguous      (stage_dma, unsplit)
//   m3 g4     global_load_dword, 4 B/lane, contiguous
//   m4 half0  dma4, half 0 of every 6-dword row only           (one channel half alone: 1/2 the bytes)
//   m5 split  dma4, both halves, item 2f+h on block 2f+h       (halves on different XCDs)
//   m6 xcdq   dma4, both halves via per-XCD queues             (k_analyze's xcd_ticket placement)
//   m7 pair   dma4, both halves in ONE workgroup, same frame   (the halves' lines fetched together)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr uint32_t kFrameBytes = 4096u * 24u;  // c4: 4096 interchannel samples x 8 ch x 3 B
constexpr uint32_t kFrameDw = kFrameBytes / 4u;
constexpr uint32_t kHalfDw = kFrameDw / 2u;
constexpr uint32_t kDrh = 3u;  // dwords of one channel half of a 6-dword row

template <int SZ>
__device__ __forceinline__ void dma(const void *g, void *lds) {
    if constexpr (SZ == 16)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                         (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    else
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                         (__attribute__((address_space(3))) void *)lds, 4, 0, 0);
}

// dword x of half h of a frame: row x / 3, dword x % 3 of that row's half
__device__ __forceinline__ uint32_t half_dw(uint32_t x, uint32_t h) {
    const uint32_t r = (uint32_t)((float)x * (1.0f / 3.0f)), k = x - r * kDrh;
    return r * 2u * kDrh + h * kDrh + k;
}

__device__ __forceinline__ void read_half(const uint32_t *f, uint32_t h, uint32_t *stg, uint32_t wave, uint32_t nw,
                                          uint32_t l) {
    for (uint32_t x0 = 64u * wave; x0 < kHalfDw; x0 += 64u * nw) dma<4>(f + half_dw(x0 + l, h), stg + (x0 & 4095u));
}

template <int M>
__global__ void __launch_bounds__(256) k_fetch(const uint8_t *buf, uint32_t n_frames, uint32_t *q, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint32_t stg[4096 + 1024];
    const uint32_t tid = threadIdx.x, l = tid & 63u, wave = tid >> 6, nw = blockDim.x >> 6;
    uint32_t acc = 0;
    if constexpr (M == 0 || M == 1 || M == 2 || M == 3) {
        const uint32_t f = blockIdx.x;
        if (f >= n_frames) return;
        const uint8_t *p = buf + (uint64_t)f * kFrameBytes;
        if constexpr (M == 0) {
            for (uint32_t o = 16u * tid; o < kFrameBytes; o += 16u * blockDim.x) {
                const uint4 v = *(const uint4 *)(p + o);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        } else if constexpr (M == 1) {
            for (uint32_t o = 1024u * wave; o < kFrameBytes; o += 1024u * nw) dma<16>(p + o + 16u * l, stg + ((o >> 2) & 4095u));
        } else if constexpr (M == 2) {
            for (uint32_t o = 256u * wave; o < kFrameBytes; o += 256u * nw) dma<4>(p + o + 4u * l, stg + ((o >> 2) & 4095u));
        } else {
            for (uint32_t o = 4u * tid; o < kFrameBytes; o += 4u * blockDim.x) acc ^= *(const uint32_t *)(p + o);
        }
    } else if constexpr (M == 4) {
        const uint32_t f = blockIdx.x;
        if (f >= n_frames) return;
        read_half((const uint32_t *)(buf + (uint64_t)f * kFrameBytes), 0u, stg, wave, nw, l);
    } else if constexpr (M == 5) {
        const uint32_t it = blockIdx.x;
        if (it >= 2u * n_frames) return;
        read_half((const uint32_t *)(buf + (uint64_t)(it >> 1) * kFrameBytes), it & 1u, stg, wave, nw, l);
    } else if constexpr (M == 6) {
        // persistent: XCD x hands out the items of frames [x n / 8, (x + 1) n / 8) in order
        __shared__ uint32_t item;
        for (;;) {
            if (tid == 0) {
                uint32_t x;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
                x &= 7u;
                uint32_t got = 0xFFFFFFFFu;
                for (uint32_t i = 0; i < 8u && got == 0xFFFFFFFFu; i++) {
                    const uint32_t y = (x + i) & 7u;
                    const uint32_t f0 = (uint32_t)(((uint64_t)n_frames * y) >> 3);
                    const uint32_t f1 = (uint32_t)(((uint64_t)n_frames * (y + 1u)) >> 3);
                    if (f1 == f0) continue;
                    const uint32_t t = atomicAdd(&q[y], 1u);
                    if (t < 2u * (f1 - f0)) got = 2u * f0 + t;
                }
                item = got;
            }
            __syncthreads();
            const uint32_t it = item;
            __syncthreads();
            if (it == 0xFFFFFFFFu) break;
            read_half((const uint32_t *)(buf + (uint64_t)(it >> 1) * kFrameBytes), it & 1u, stg, wave, nw, l);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else {
        const uint32_t f = blockIdx.x;
        if (f >= n_frames) return;
        // waves 0-1 half 0, waves 2-3 half 1, interleaved in time
        read_half((const uint32_t *)(buf + (uint64_t)f * kFrameBytes), wave & 1u, stg, wave >> 1, nw >> 1, l);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc ^= stg[tid];
    if (acc == 0x9e3779b9u) sink[blockIdx.x & 1023u] = acc;  // keeps the reads alive, ~never stores
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

template <int M>
static int run(const char *name, const uint8_t *buf, uint32_t nf, uint32_t *q, uint32_t *sink, int reps) {
    const uint64_t half_modes = (M >= 4 && M <= 7) ? 1 : 0;
    const uint64_t bytes = (M == 4) ? (uint64_t)nf * kFrameBytes / 2 : (uint64_t)nf * kFrameBytes;
    const uint32_t grid = (M == 5) ? 2u * nf : (M == 6 ? 2048u : nf);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; r++) {
        CK(hipMemset(q, 0, 64));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_fetch<M>, dim3(grid), dim3(256), 0, 0, buf, nf, q, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        sum += ms;
    }
    printf("{\"mode\": %d, \"name\": \"%s\", \"kernel\": \"k_fetch<%d>\", \"bytes\": %llu, \"split\": %llu, "
           "\"best_ms\": %.4f, \"avg_ms\": %.4f, \"gbs_best\": %.1f}\n",
           M, name, M, (unsigned long long)bytes, (unsigned long long)half_modes, best, sum / reps,
           bytes / (best * 1e-3) / 1e9);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 0;
}

int main(int argc, char **argv) {
    const uint32_t nf = argc > 1 ? (uint32_t)atoi(argv[1]) : 32768u;  // 3.2 GB: past the 256 MiB L3
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    uint8_t *buf;
    uint32_t *q, *sink;
    CK(hipMalloc(&buf, (uint64_t)nf * kFrameBytes));
    CK(hipMalloc(&q, 64));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 0x5a, (uint64_t)nf * kFrameBytes));
    CK(hipDeviceSynchronize());
    if (run<0>("g16", buf, nf, q, sink, reps) || run<1>("dma16", buf, nf, q, sink, reps) ||
        run<2>("dma4", buf, nf, q, sink, reps) || run<3>("g4", buf, nf, q, sink, reps) ||
        run<4>("half0", buf, nf, q, sink, reps) || run<5>("split", buf, nf, q, sink, reps) ||
        run<6>("xcdq", buf, nf, q, sink, reps) || run<7>("pair", buf, nf, q, sink, reps))
        return 1;
    CK(hipFree(buf));
    CK(hipFree(q));
    CK(hipFree(sink));
    return 0;
}
