// md5_micro.hip -- latency experiment for the per-stream MD5 (tools only).
// Variants: 0 = one stream per lane (as k_md5_streams), 1 = two interleaved
// streams per lane, 2 = rotate via shifts instead of v_alignbit, 3 = 16 active lanes,
// 4 = H round as v_xad_u32 (3 dependent ops per step instead of 4).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>

constexpr uint32_t K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
constexpr int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9, 14, 20, 5, 9, 14, 20,
                       5, 9, 14, 20, 5, 9, 14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                       6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

template <int ROT>
__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
    if (ROT == 0) return __builtin_amdgcn_alignbit(x, x, 32 - s);
    return (x << s) | (x >> (32 - s));
}

template <int ROT>
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
        b = b + rotl<ROT>(a + f + K[i] + m[g], S[i]);
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

__device__ __forceinline__ uint32_t xad(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ void compress_xad(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t x, g;
        if (i < 16) { g = i; x = ((b & c) | (~b & d)) + (a + K[i] + m[g]); }
        else if (i < 32) { g = (5 * i + 1) & 15; x = ((d & b) | (~d & c)) + (a + K[i] + m[g]); }
        else if (i < 48) { g = (3 * i + 5) & 15; x = xad(b, c ^ d, a + K[i] + m[g]); }
        else { g = (7 * i) & 15; x = (c ^ (b | ~d)) + (a + K[i] + m[g]); }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl<0>(x, S[i]);
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

template <int V>
__global__ void __launch_bounds__(64) k_md5(const uint32_t *data, uint64_t words_per_stream, uint32_t n, uint32_t *out) {
    const uint32_t s = blockIdx.x * 64 + threadIdx.x;
    if (V == 1) {
        if (s >= n / 2) return;
        const uint32_t *p = data + (uint64_t)s * words_per_stream, *q = data + (uint64_t)(s + n / 2) * words_per_stream;
        uint32_t st[4] = {1, 2, 3, 4}, su[4] = {5, 6, 7, 8};
        for (uint64_t b = 0; b < words_per_stream / 16; b++) {
            uint32_t m[16], mm[16];
            for (int i = 0; i < 16; i++) { m[i] = p[b * 16 + i]; mm[i] = q[b * 16 + i]; }
            compress<0>(st, m);
            compress<0>(su, mm);
        }
        out[s] = st[0] ^ st[1] ^ st[2] ^ st[3];
        out[s + n / 2] = su[0] ^ su[1] ^ su[2] ^ su[3];
    } else if (V == 3) {
        // 16 active lanes per wave (lanes 16..63 idle): does a partial exec mask issue faster?
        const uint32_t lane = threadIdx.x;
        const uint32_t s3 = blockIdx.x * 16 + lane;
        if (lane >= 16 || s3 >= n) return;
        const uint32_t *p = data + (uint64_t)s3 * words_per_stream;
        uint32_t st[4] = {1, 2, 3, 4};
        for (uint64_t b = 0; b < words_per_stream / 16; b++) {
            uint32_t m[16];
            for (int i = 0; i < 16; i++) m[i] = p[b * 16 + i];
            compress<0>(st, m);
        }
        out[s3] = st[0] ^ st[1] ^ st[2] ^ st[3];
    } else {
        if (s >= n) return;
        const uint32_t *p = data + (uint64_t)s * words_per_stream;
        uint32_t st[4] = {1, 2, 3, 4};
        for (uint64_t b = 0; b < words_per_stream / 16; b++) {
            uint32_t m[16];
            for (int i = 0; i < 16; i++) m[i] = p[b * 16 + i];
            if (V == 4) compress_xad(st, m); else compress<V == 2 ? 1 : 0>(st, m);
        }
        out[s] = st[0] ^ st[1] ^ st[2] ^ st[3];
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096u;
    const uint64_t words = 128 * 1024 / 4;  // 128 KiB per stream
    uint32_t *d, *o;
    hipMalloc(&d, n * words * 4);
    hipMalloc(&o, n * 4);
    hipMemset(d, 1, n * words * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int v = 0; v < 5; v++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            uint32_t grid = v == 3 ? n / 16 : (v == 1 ? n / 2 : n) / 64;
            if (v == 0) hipLaunchKernelGGL(k_md5<0>, dim3(grid), dim3(64), 0, 0, d, words, n, o);
            if (v == 1) hipLaunchKernelGGL(k_md5<1>, dim3(grid), dim3(64), 0, 0, d, words, n, o);
            if (v == 2) hipLaunchKernelGGL(k_md5<2>, dim3(grid), dim3(64), 0, 0, d, words, n, o);
            if (v == 3) hipLaunchKernelGGL(k_md5<3>, dim3(grid), dim3(64), 0, 0, d, words, n, o);
            if (v == 4) hipLaunchKernelGGL(k_md5<4>, dim3(grid), dim3(64), 0, 0, d, words, n, o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) printf("variant %d: %.3f ms (%u streams x %llu KiB), %.1f ns per block per stream\n", v, ms, n,
                                 (unsigned long long)(words * 4 / 1024), ms * 1e6 / (words / 16));
        }
    }
    return 0;
}
