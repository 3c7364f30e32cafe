// md5_lab.hip -- why does the per-stream MD5 run 2x slower beside the encode kernels? (tools only)
//
// The MD5 kernel (one lane per stream, as k_md5_streams) is timed alone and beside "hog" kernels
// that each reproduce ONE property of the encode kernels, launched on a second stream:
//   valu_small : VALU-bound integer work, 4 waves/SIMD, a 64-instruction loop body (fits any I-cache)
//   valu_big   : the same work with a ~48 KiB straight-line loop body (instruction-cache pressure,
//                like k_analyze's 55 KiB)
//   mem        : LDS-DMA streaming of 1 GiB, contiguous 16 KiB pieces (HBM / TA pressure)
// MD5 variants: data = 0 streams in HBM (the product's 64-KiB-apart scattered 16-B loads),
//               1 cache-resident (every stream reads the same 64 KiB), 2 no loads (message from state).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
constexpr int SH[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9, 14, 20, 5, 9, 14, 20,
                        5, 9, 14, 20, 5, 9, 14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                        6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

__device__ __forceinline__ void compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f, g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl(a + f + K[i] + m[g], SH[i]);
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

typedef uint32_t v4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void load_block(const uint8_t *p, uint32_t (&m)[16]) {
    const v4 *q = (const v4 *)p;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const v4 v = q[i];
        m[4 * i] = v.x; m[4 * i + 1] = v.y; m[4 * i + 2] = v.z; m[4 * i + 3] = v.w;
    }
}

// DATA 0: stream s at base + s * stride; 1: every stream reads base[0 .. 64 KiB); 2: no loads
template <int DATA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8)))
k_md5(const uint8_t *base, uint64_t stride, uint64_t nblocks, uint32_t n, uint32_t *out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint8_t *p = DATA == 0 ? base + (uint64_t)s * stride : base + (s & 63) * 64;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u + s};
    uint32_t m[2][16];
    if (DATA == 2) {
        for (int i = 0; i < 16; i++) m[0][i] = m[1][i] = s * 0x9e3779b9u + i;
    } else {
        load_block(p, m[0]);
        load_block(p + 64 * (1 % nblocks), m[1]);
    }
    for (uint64_t b = 0; b + 2 <= nblocks; b += 2) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            compress(st, m[k]);
            if (DATA == 2) {
                m[k][0] ^= st[0];
            } else {
                uint64_t nb = b + k + 2;
                if (DATA == 1) nb &= 1023;
                if (nb < nblocks) load_block(p + 64 * nb, m[k]);
            }
        }
    }
    out[s] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// DATA 3: coalesced LDS-DMA ring.  Two waves per workgroup, 64 streams per wave.  Chunk c of a
// stream = its blocks 2c, 2c+1 (128 B, one cache line).  LDS-DMA instruction i of a chunk moves
// 8 streams x 128 B (8 lines instead of 64): lane j -> stream 8i + j/8, LDS slot u = j % 8 of that
// stream's 128-B row, holding piece p = (u - (stream>>1)) & 7, so that the 16 lanes of a
// ds_read_b128 quarter hit 16 distinct 16-B bank groups.  R chunks in flight per wave.
template <int R>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(7, 8)))
k_md5_lds(const uint8_t *base, uint64_t stride, uint64_t nblocks, uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2][R][8192];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t g0 = blockIdx.x * 128 + w * 64;
    const uint32_t s = g0 + l;
    const uint64_t nchunks = nblocks / 2;
    uint8_t *ring = &lds[w][0][0];
    auto issue = [&](uint64_t c) {
        uint8_t *dst = ring + (c % R) * 8192;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t sl = 8 * i + (l >> 3), u = l & 7, p = (u - (sl >> 1)) & 7;
            const uint8_t *src = base + (uint64_t)(g0 + sl) * stride + 128 * c + 16 * p;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + 1024 * i), 16, 0, 0);
        }
    };
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u + s};
    for (int c = 0; c < R; c++) issue(c);
    const uint32_t row = 1024 * (l >> 3) + 128 * (l & 7);
    for (uint64_t c = 0; c < nchunks; c++) {
        // chunk c landed when at most the R - 1 younger chunks' 8 DMAs each are outstanding
        if constexpr (R == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        const uint8_t *buf = ring + (c % R) * 8192 + row;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            uint32_t m[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t p = 4 * k + q;
                const v4 v = *(const v4 *)(buf + 16 * ((p + (l >> 1)) & 7));
                m[4 * q] = v.x; m[4 * q + 1] = v.y; m[4 * q + 2] = v.z; m[4 * q + 3] = v.w;
            }
            compress(st, m);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(c + R < nchunks ? c + R : nchunks - 1);  // a redundant refill keeps vmcnt counting uniform
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[s] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// DATA 6/7: the same LDS ring filled by a third, loader-only wave: the two compute waves never
// issue a DMA (an LDS-DMA instruction costs its issuing wave ~60-180 cycles); per chunk one
// barrier says "chunk c landed" and one says "chunk c read into registers".
__device__ __forceinline__ void bar_raw() { asm volatile("s_barrier" ::: "memory"); }
template <int R>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(7, 8)))
k_md5_ldr(const uint8_t *base, uint64_t stride, uint64_t nblocks, uint32_t n, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[R][2][8192];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint64_t nchunks = nblocks / 2;
    if (w == 2) {
        auto issue = [&](uint64_t c) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint8_t *dst = &lds[c % R][h][0];
                const uint32_t g0 = blockIdx.x * 128 + h * 64;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t sl = 8 * i + (l >> 3), u = l & 7, p = (u - (sl >> 1)) & 7;
                    const uint8_t *src = base + (uint64_t)(g0 + sl) * stride + 128 * c + 16 * p;
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                                     (__attribute__((address_space(3))) void *)(dst + 1024 * i), 16, 0, 0);
                }
            }
        };
        for (int c = 0; c < R; c++) issue(c);
        for (uint64_t c = 0; c < nchunks; c++) {
            if constexpr (R == 3) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            else if constexpr (R == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
            bar_raw();  // A: chunk c landed
            bar_raw();  // B: chunk c read
            issue(c + R < nchunks ? c + R : nchunks - 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    const uint32_t s = blockIdx.x * 128 + w * 64 + l;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u + s};
    const uint32_t row = 1024 * (l >> 3) + 128 * (l & 7);
    for (uint64_t c = 0; c < nchunks; c++) {
        bar_raw();  // A
        const uint8_t *buf = &lds[c % R][w][0] + row;
        uint32_t m[2][16];
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t p = 4 * k + q;
                const v4 v = *(const v4 *)(buf + 16 * ((p + (l >> 1)) & 7));
                m[k][4 * q] = v.x; m[k][4 * q + 1] = v.y; m[k][4 * q + 2] = v.z; m[k][4 * q + 3] = v.w;
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar_raw();  // B
        compress(st, m[0]);
        compress(st, m[1]);
    }
    out[s] = st[0] ^ st[1] ^ st[2] ^ st[3];
}

// ---- hogs -------------------------------------------------------------------------------------
#define OP4(i) asm volatile("v_add3_u32 %0, %0, %1, 3\n v_xad_u32 %1, %1, %2, %0\n v_bitop3_b32 %2, %2, %3, %0 bitop3:0xe4\n v_alignbit_b32 %3, %3, %2, 7" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
#define OP16(i) OP4(i##0) OP4(i##1) OP4(i##2) OP4(i##3)
#define OP64(i) OP16(i##0) OP16(i##1) OP16(i##2) OP16(i##3)
#define OP256(i) OP64(i##0) OP64(i##1) OP64(i##2) OP64(i##3)
// 4 independent chains per lane x 4 ops each: 16 instructions per OP4

template <int BIG>
__global__ void __launch_bounds__(256) k_valu(uint32_t *out, int iters) {
    uint32_t x0 = threadIdx.x, x1 = blockIdx.x, x2 = 7, x3 = 9;
    for (int it = 0; it < iters; it++) {
        if (BIG) {
            // 4 x 256 x 4 = 4096 instructions x 8 B ~ 32 KiB ... x2 below ~ 64 KiB
            OP256(1) OP256(2) OP256(3) OP256(1)
            OP256(2) OP256(3) OP256(1) OP256(2)
        } else {
            OP4(1) OP4(2) OP4(3) OP4(1)
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
}

// persistent LDS-DMA streamer: each workgroup pulls 16 KiB pieces (like a C2 frame) into LDS
__global__ void __launch_bounds__(256) k_mem(const uint8_t *src, uint64_t pieces, uint32_t *out, uint32_t *ticket) {
    __shared__ uint32_t lds[4096];
    uint32_t acc = 0;
    for (;;) {
        __shared__ uint32_t tk;
        if (threadIdx.x == 0) tk = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t t = tk;
        __syncthreads();
        if (t >= pieces) break;
        const uint8_t *p = src + (uint64_t)t * 16384;
        // 16 KiB = 4 waves x 4 x (64 lanes x 16 B)
        const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t off = (w * 4 + k) * 1024;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(p + off + l * 16),
                                             (__attribute__((address_space(3))) void *)(lds + off / 4), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        acc += lds[threadIdx.x * 16 + (t & 15)];
        __syncthreads();
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 16384u;  // streams
    const uint64_t nblocks = argc > 2 ? (uint64_t)atoll(argv[2]) : 1024;  // 64-B blocks per stream
    const uint64_t stride = nblocks * 64;
    const uint64_t bytes = (uint64_t)n * stride;
    uint8_t *d;
    uint32_t *o, *tk;
    CK(hipMalloc(&d, bytes < (1ull << 30) ? (1ull << 30) : bytes));
    CK(hipMalloc(&o, 64u << 20));
    CK(hipMalloc(&tk, 4));
    CK(hipMemset(d, 0x5a, bytes < (1ull << 30) ? (1ull << 30) : bytes));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t a0, a1, b0, b1;
    CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1)); CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t hog_wgs = cus * 4;  // 4 x 256-thread workgroups per CU = 4 waves per SIMD
    const int small_iters = argc > 3 ? atoi(argv[3]) : 6000, big_iters = small_iters / 512;
    const uint64_t pieces = (1ull << 30) / 16384;
    printf("CUs %d, MD5: %u streams x %llu blocks; hog grid %u x 256\n", cus, n, (unsigned long long)nblocks, hog_wgs);
    auto md5 = [&](int data) {
        dim3 g((n + 255) / 256), b(256);
        if (data == 0) hipLaunchKernelGGL(k_md5<0>, g, b, 0, sa, d, stride, nblocks, n, o);
        if (data == 1) hipLaunchKernelGGL(k_md5<1>, g, b, 0, sa, d, stride, nblocks, n, o);
        if (data == 2) hipLaunchKernelGGL(k_md5<2>, g, b, 0, sa, d, stride, nblocks, n, o);
        if (data == 3) hipLaunchKernelGGL(k_md5_lds<2>, dim3(n / 128), dim3(128), 0, sa, d, stride, nblocks, n, o);
        if (data == 4) hipLaunchKernelGGL(k_md5_lds<3>, dim3(n / 128), dim3(128), 0, sa, d, stride, nblocks, n, o);
        if (data == 5) hipLaunchKernelGGL(k_md5_lds<4>, dim3(n / 128), dim3(128), 0, sa, d, stride, nblocks, n, o);
        if (data == 6) hipLaunchKernelGGL(k_md5_ldr<3>, dim3(n / 128), dim3(192), 0, sa, d, stride, nblocks, n, o);
        if (data == 7) hipLaunchKernelGGL(k_md5_ldr<4>, dim3(n / 128), dim3(192), 0, sa, d, stride, nblocks, n, o);
    };
    auto hog = [&](int h) {
        if (h == 1) hipLaunchKernelGGL(k_valu<0>, dim3(hog_wgs), dim3(256), 0, sb, o + (8u << 20), small_iters);
        if (h == 2) hipLaunchKernelGGL(k_valu<1>, dim3(hog_wgs), dim3(256), 0, sb, o + (8u << 20), big_iters);
        if (h == 3) {
            hipMemsetAsync(tk, 0, 4, sb);
            hipLaunchKernelGGL(k_mem, dim3(cus * 4), dim3(256), 0, sb, d, pieces, o + (8u << 20), tk);
        }
    };
    const char *dn[8] = {"hbm", "cached", "noload", "lds_r2", "lds_r3", "lds_r4", "ldr_r3", "ldr_r4"}, *hn[4] = {"alone", "valu_small", "valu_big", "mem"};
    float hog_alone[4] = {0, 0, 0, 0};
    for (int h = 1; h < 4; h++) {
        for (int r = 0; r < 3; r++) {
            CK(hipEventRecord(b0, sb)); hog(h); CK(hipEventRecord(b1, sb)); CK(hipStreamSynchronize(sb));
            CK(hipEventElapsedTime(&hog_alone[h], b0, b1));
        }
        printf("hog %-10s alone %.3f ms\n", hn[h], hog_alone[h]);
    }
    for (int data = 0; data < 8; data++) {
        if (data == 1 || data == 2 || data == 3) continue;
        for (int h = 0; h < 4; h++) {
            float ma = 0, hb = 0;
            for (int r = 0; r < 3; r++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a0, sa)); md5(data); CK(hipEventRecord(a1, sa));
                if (h) { CK(hipEventRecord(b0, sb)); hog(h); CK(hipEventRecord(b1, sb)); }
                CK(hipDeviceSynchronize());
                CK(hipEventElapsedTime(&ma, a0, a1));
                if (h) CK(hipEventElapsedTime(&hb, b0, b1));
            }
            printf("md5 %-7s beside %-10s md5 %.3f ms = %.3f us/block | hog %.3f ms (alone %.3f)\n", dn[data], hn[h], ma,
                   ma * 1e3 / nblocks, hb, hog_alone[h]);
        }
    }
    return 0;
}
