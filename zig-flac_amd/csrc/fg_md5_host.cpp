// fg_md5_host.cpp -- host MD5 (see fg_md5_host.hpp).
#include "fg_md5_host.hpp"

#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace fg {
namespace {

inline uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

#define H5F(b, c, d) ((d) ^ ((b) & ((c) ^ (d))))
#define H5G(b, c, d) ((c) ^ ((d) & ((b) ^ (c))))
#define H5H(b, c, d) ((b) ^ (c) ^ (d))
#define H5I(b, c, d) ((c) ^ ((b) | ~(d)))
#define H5STEP(F, a, b, c, d, x, k, s) a = b + rol(a + F(b, c, d) + (x) + (k), s)

void compress(uint32_t st[4], const uint8_t *blk, size_t nblocks) {
    uint32_t a0 = st[0], b0 = st[1], c0 = st[2], d0 = st[3];
    for (size_t n = 0; n < nblocks; n++, blk += 64) {
        uint32_t X[16];
        memcpy(X, blk, 64);  // little-endian host (x86-64)
        uint32_t a = a0, b = b0, c = c0, d = d0;
        H5STEP(H5F, a, b, c, d, X[0], 0xd76aa478, 7);   H5STEP(H5F, d, a, b, c, X[1], 0xe8c7b756, 12);
        H5STEP(H5F, c, d, a, b, X[2], 0x242070db, 17);  H5STEP(H5F, b, c, d, a, X[3], 0xc1bdceee, 22);
        H5STEP(H5F, a, b, c, d, X[4], 0xf57c0faf, 7);   H5STEP(H5F, d, a, b, c, X[5], 0x4787c62a, 12);
        H5STEP(H5F, c, d, a, b, X[6], 0xa8304613, 17);  H5STEP(H5F, b, c, d, a, X[7], 0xfd469501, 22);
        H5STEP(H5F, a, b, c, d, X[8], 0x698098d8, 7);   H5STEP(H5F, d, a, b, c, X[9], 0x8b44f7af, 12);
        H5STEP(H5F, c, d, a, b, X[10], 0xffff5bb1, 17); H5STEP(H5F, b, c, d, a, X[11], 0x895cd7be, 22);
        H5STEP(H5F, a, b, c, d, X[12], 0x6b901122, 7);  H5STEP(H5F, d, a, b, c, X[13], 0xfd987193, 12);
        H5STEP(H5F, c, d, a, b, X[14], 0xa679438e, 17); H5STEP(H5F, b, c, d, a, X[15], 0x49b40821, 22);
        H5STEP(H5G, a, b, c, d, X[1], 0xf61e2562, 5);   H5STEP(H5G, d, a, b, c, X[6], 0xc040b340, 9);
        H5STEP(H5G, c, d, a, b, X[11], 0x265e5a51, 14); H5STEP(H5G, b, c, d, a, X[0], 0xe9b6c7aa, 20);
        H5STEP(H5G, a, b, c, d, X[5], 0xd62f105d, 5);   H5STEP(H5G, d, a, b, c, X[10], 0x02441453, 9);
        H5STEP(H5G, c, d, a, b, X[15], 0xd8a1e681, 14); H5STEP(H5G, b, c, d, a, X[4], 0xe7d3fbc8, 20);
        H5STEP(H5G, a, b, c, d, X[9], 0x21e1cde6, 5);   H5STEP(H5G, d, a, b, c, X[14], 0xc33707d6, 9);
        H5STEP(H5G, c, d, a, b, X[3], 0xf4d50d87, 14);  H5STEP(H5G, b, c, d, a, X[8], 0x455a14ed, 20);
        H5STEP(H5G, a, b, c, d, X[13], 0xa9e3e905, 5);  H5STEP(H5G, d, a, b, c, X[2], 0xfcefa3f8, 9);
        H5STEP(H5G, c, d, a, b, X[7], 0x676f02d9, 14);  H5STEP(H5G, b, c, d, a, X[12], 0x8d2a4c8a, 20);
        H5STEP(H5H, a, b, c, d, X[5], 0xfffa3942, 4);   H5STEP(H5H, d, a, b, c, X[8], 0x8771f681, 11);
        H5STEP(H5H, c, d, a, b, X[11], 0x6d9d6122, 16); H5STEP(H5H, b, c, d, a, X[14], 0xfde5380c, 23);
        H5STEP(H5H, a, b, c, d, X[1], 0xa4beea44, 4);   H5STEP(H5H, d, a, b, c, X[4], 0x4bdecfa9, 11);
        H5STEP(H5H, c, d, a, b, X[7], 0xf6bb4b60, 16);  H5STEP(H5H, b, c, d, a, X[10], 0xbebfbc70, 23);
        H5STEP(H5H, a, b, c, d, X[13], 0x289b7ec6, 4);  H5STEP(H5H, d, a, b, c, X[0], 0xeaa127fa, 11);
        H5STEP(H5H, c, d, a, b, X[3], 0xd4ef3085, 16);  H5STEP(H5H, b, c, d, a, X[6], 0x04881d05, 23);
        H5STEP(H5H, a, b, c, d, X[9], 0xd9d4d039, 4);   H5STEP(H5H, d, a, b, c, X[12], 0xe6db99e5, 11);
        H5STEP(H5H, c, d, a, b, X[15], 0x1fa27cf8, 16); H5STEP(H5H, b, c, d, a, X[2], 0xc4ac5665, 23);
        H5STEP(H5I, a, b, c, d, X[0], 0xf4292244, 6);   H5STEP(H5I, d, a, b, c, X[7], 0x432aff97, 10);
        H5STEP(H5I, c, d, a, b, X[14], 0xab9423a7, 15); H5STEP(H5I, b, c, d, a, X[5], 0xfc93a039, 21);
        H5STEP(H5I, a, b, c, d, X[12], 0x655b59c3, 6);  H5STEP(H5I, d, a, b, c, X[3], 0x8f0ccc92, 10);
        H5STEP(H5I, c, d, a, b, X[10], 0xffeff47d, 15); H5STEP(H5I, b, c, d, a, X[1], 0x85845dd1, 21);
        H5STEP(H5I, a, b, c, d, X[8], 0x6fa87e4f, 6);   H5STEP(H5I, d, a, b, c, X[15], 0xfe2ce6e0, 10);
        H5STEP(H5I, c, d, a, b, X[6], 0xa3014314, 15);  H5STEP(H5I, b, c, d, a, X[13], 0x4e0811a1, 21);
        H5STEP(H5I, a, b, c, d, X[4], 0xf7537e82, 6);   H5STEP(H5I, d, a, b, c, X[11], 0xbd3af235, 10);
        H5STEP(H5I, c, d, a, b, X[2], 0x2ad7d2bb, 15);  H5STEP(H5I, b, c, d, a, X[9], 0xeb86d391, 21);
        a0 += a;
        b0 += b;
        c0 += c;
        d0 += d;
    }
    st[0] = a0;
    st[1] = b0;
    st[2] = c0;
    st[3] = d0;
}

// N independent messages, nblocks blocks each, one step of every chain after the other: the
// chains are independent, so an out-of-order core overlaps them (one MD5 chain is latency-bound
// on ~4 dependent ALU ops per step and leaves most execution ports idle).
template <int N>
void compress_n(uint32_t *const st[N], const uint8_t *const blk0[N], size_t nblocks) {
    uint32_t a0[N], b0[N], c0[N], d0[N];
    const uint8_t *blk[N];
    for (int j = 0; j < N; j++) {
        a0[j] = st[j][0]; b0[j] = st[j][1]; c0[j] = st[j][2]; d0[j] = st[j][3];
        blk[j] = blk0[j];
    }
    for (size_t n = 0; n < nblocks; n++) {
        uint32_t X[N][16], a[N], b[N], c[N], d[N];
        for (int j = 0; j < N; j++) {
            memcpy(X[j], blk[j], 64);
            blk[j] += 64;
            a[j] = a0[j]; b[j] = b0[j]; c[j] = c0[j]; d[j] = d0[j];
        }
#define H5N(F, A, B, C, D, i, k, s) \
    for (int j = 0; j < N; j++) H5STEP(F, A[j], B[j], C[j], D[j], X[j][i], k, s);
        H5N(H5F, a, b, c, d, 0, 0xd76aa478, 7)   H5N(H5F, d, a, b, c, 1, 0xe8c7b756, 12)
        H5N(H5F, c, d, a, b, 2, 0x242070db, 17)  H5N(H5F, b, c, d, a, 3, 0xc1bdceee, 22)
        H5N(H5F, a, b, c, d, 4, 0xf57c0faf, 7)   H5N(H5F, d, a, b, c, 5, 0x4787c62a, 12)
        H5N(H5F, c, d, a, b, 6, 0xa8304613, 17)  H5N(H5F, b, c, d, a, 7, 0xfd469501, 22)
        H5N(H5F, a, b, c, d, 8, 0x698098d8, 7)   H5N(H5F, d, a, b, c, 9, 0x8b44f7af, 12)
        H5N(H5F, c, d, a, b, 10, 0xffff5bb1, 17) H5N(H5F, b, c, d, a, 11, 0x895cd7be, 22)
        H5N(H5F, a, b, c, d, 12, 0x6b901122, 7)  H5N(H5F, d, a, b, c, 13, 0xfd987193, 12)
        H5N(H5F, c, d, a, b, 14, 0xa679438e, 17) H5N(H5F, b, c, d, a, 15, 0x49b40821, 22)
        H5N(H5G, a, b, c, d, 1, 0xf61e2562, 5)   H5N(H5G, d, a, b, c, 6, 0xc040b340, 9)
        H5N(H5G, c, d, a, b, 11, 0x265e5a51, 14) H5N(H5G, b, c, d, a, 0, 0xe9b6c7aa, 20)
        H5N(H5G, a, b, c, d, 5, 0xd62f105d, 5)   H5N(H5G, d, a, b, c, 10, 0x02441453, 9)
        H5N(H5G, c, d, a, b, 15, 0xd8a1e681, 14) H5N(H5G, b, c, d, a, 4, 0xe7d3fbc8, 20)
        H5N(H5G, a, b, c, d, 9, 0x21e1cde6, 5)   H5N(H5G, d, a, b, c, 14, 0xc33707d6, 9)
        H5N(H5G, c, d, a, b, 3, 0xf4d50d87, 14)  H5N(H5G, b, c, d, a, 8, 0x455a14ed, 20)
        H5N(H5G, a, b, c, d, 13, 0xa9e3e905, 5)  H5N(H5G, d, a, b, c, 2, 0xfcefa3f8, 9)
        H5N(H5G, c, d, a, b, 7, 0x676f02d9, 14)  H5N(H5G, b, c, d, a, 12, 0x8d2a4c8a, 20)
        H5N(H5H, a, b, c, d, 5, 0xfffa3942, 4)   H5N(H5H, d, a, b, c, 8, 0x8771f681, 11)
        H5N(H5H, c, d, a, b, 11, 0x6d9d6122, 16) H5N(H5H, b, c, d, a, 14, 0xfde5380c, 23)
        H5N(H5H, a, b, c, d, 1, 0xa4beea44, 4)   H5N(H5H, d, a, b, c, 4, 0x4bdecfa9, 11)
        H5N(H5H, c, d, a, b, 7, 0xf6bb4b60, 16)  H5N(H5H, b, c, d, a, 10, 0xbebfbc70, 23)
        H5N(H5H, a, b, c, d, 13, 0x289b7ec6, 4)  H5N(H5H, d, a, b, c, 0, 0xeaa127fa, 11)
        H5N(H5H, c, d, a, b, 3, 0xd4ef3085, 16)  H5N(H5H, b, c, d, a, 6, 0x04881d05, 23)
        H5N(H5H, a, b, c, d, 9, 0xd9d4d039, 4)   H5N(H5H, d, a, b, c, 12, 0xe6db99e5, 11)
        H5N(H5H, c, d, a, b, 15, 0x1fa27cf8, 16) H5N(H5H, b, c, d, a, 2, 0xc4ac5665, 23)
        H5N(H5I, a, b, c, d, 0, 0xf4292244, 6)   H5N(H5I, d, a, b, c, 7, 0x432aff97, 10)
        H5N(H5I, c, d, a, b, 14, 0xab9423a7, 15) H5N(H5I, b, c, d, a, 5, 0xfc93a039, 21)
        H5N(H5I, a, b, c, d, 12, 0x655b59c3, 6)  H5N(H5I, d, a, b, c, 3, 0x8f0ccc92, 10)
        H5N(H5I, c, d, a, b, 10, 0xffeff47d, 15) H5N(H5I, b, c, d, a, 1, 0x85845dd1, 21)
        H5N(H5I, a, b, c, d, 8, 0x6fa87e4f, 6)   H5N(H5I, d, a, b, c, 15, 0xfe2ce6e0, 10)
        H5N(H5I, c, d, a, b, 6, 0xa3014314, 15)  H5N(H5I, b, c, d, a, 13, 0x4e0811a1, 21)
        H5N(H5I, a, b, c, d, 4, 0xf7537e82, 6)   H5N(H5I, d, a, b, c, 11, 0xbd3af235, 10)
        H5N(H5I, c, d, a, b, 2, 0x2ad7d2bb, 15)  H5N(H5I, b, c, d, a, 9, 0xeb86d391, 21)
#undef H5N
        for (int j = 0; j < N; j++) {
            a0[j] += a[j]; b0[j] += b[j]; c0[j] += c[j]; d0[j] += d[j];
        }
    }
    for (int j = 0; j < N; j++) {
        st[j][0] = a0[j]; st[j][1] = b0[j]; st[j][2] = c0[j]; st[j][3] = d0[j];
    }
}

// Up to 16 independent chains in the 16 dword lanes of AVX-512 registers (lane j = chain j): one
// step of all of them is five vector instructions (vpternlogd computes F/G/H/I in one), so a core
// advances 16 chains at the latency of one -- the scalar interleave above runs out of issue width
// at about four.  Message words reach their lanes by a 16 x 16 dword transpose of the chains' next
// blocks.  Chains j >= n read a zero block and are not stored.  Compiled for AVX-512F only (the
// rest of the library stays baseline x86-64); avx512_on() picks it at run time.
#define M5X_F(b, c, d) _mm512_ternarylogic_epi32(b, c, d, 0xCA)  // b ? c : d
#define M5X_G(b, c, d) _mm512_ternarylogic_epi32(d, b, c, 0xCA)  // d ? b : c
#define M5X_H(b, c, d) _mm512_ternarylogic_epi32(b, c, d, 0x96)  // b ^ c ^ d
#define M5X_I(b, c, d) _mm512_ternarylogic_epi32(b, c, d, 0x39)  // c ^ (b | ~d)
#define M5X_STEP(F, a, b, c, d, x, k, s)                                                                     \
    a = _mm512_add_epi32(b, _mm512_rol_epi32(_mm512_add_epi32(_mm512_add_epi32(a, F(b, c, d)),               \
                                                              _mm512_add_epi32(x, _mm512_set1_epi32((int)(k)))), s))

__attribute__((target("avx512f"))) static inline void m5x_transpose(__m512i (&m)[16]) {
    __m512i t[16];
    for (int i = 0; i < 16; i += 2) {
        t[i] = _mm512_unpacklo_epi32(m[i], m[i + 1]);
        t[i + 1] = _mm512_unpackhi_epi32(m[i], m[i + 1]);
    }
    for (int i = 0; i < 16; i += 4) {
        m[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
        m[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
        m[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
        m[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    for (int i = 0; i < 4; i++) {
        t[i] = _mm512_shuffle_i32x4(m[i], m[i + 4], 0x88);
        t[i + 4] = _mm512_shuffle_i32x4(m[i], m[i + 4], 0xDD);
        t[i + 8] = _mm512_shuffle_i32x4(m[i + 8], m[i + 12], 0x88);
        t[i + 12] = _mm512_shuffle_i32x4(m[i + 8], m[i + 12], 0xDD);
    }
    for (int i = 0; i < 4; i++) {
        m[i] = _mm512_shuffle_i32x4(t[i], t[i + 8], 0x88);
        m[i + 8] = _mm512_shuffle_i32x4(t[i], t[i + 8], 0xDD);
        m[i + 4] = _mm512_shuffle_i32x4(t[i + 4], t[i + 12], 0x88);
        m[i + 12] = _mm512_shuffle_i32x4(t[i + 4], t[i + 12], 0xDD);
    }
}

__attribute__((target("avx512f"))) void compress_x16(uint32_t *const st[], const uint8_t *const blk0[], int n,
                                                      size_t nblocks) {
    alignas(64) static const uint8_t zero[64] = {};
    alignas(64) uint32_t sa[16], sb[16], sc[16], sd[16];
    const uint8_t *blk[16];
    for (int j = 0; j < 16; j++) {
        const bool on = j < n;
        sa[j] = on ? st[j][0] : 0u; sb[j] = on ? st[j][1] : 0u; sc[j] = on ? st[j][2] : 0u; sd[j] = on ? st[j][3] : 0u;
        blk[j] = on ? blk0[j] : zero;
    }
    __m512i a0 = _mm512_load_si512(sa), b0 = _mm512_load_si512(sb), c0 = _mm512_load_si512(sc), d0 = _mm512_load_si512(sd);
    for (size_t nb = 0; nb < nblocks; nb++) {
        __m512i X[16];
        for (int j = 0; j < 16; j++) {
            X[j] = _mm512_loadu_si512((const void *)blk[j]);
            if (j < n) blk[j] += 64;
        }
        // rows (chains) -> columns (message words): afterwards X[w] lane j = word w of chain j
        m5x_transpose(X);
        const __m512i *W = X;
        __m512i a = a0, b = b0, c = c0, d = d0;
        M5X_STEP(M5X_F, a, b, c, d, W[0], 0xd76aa478, 7);   M5X_STEP(M5X_F, d, a, b, c, W[1], 0xe8c7b756, 12);
        M5X_STEP(M5X_F, c, d, a, b, W[2], 0x242070db, 17);  M5X_STEP(M5X_F, b, c, d, a, W[3], 0xc1bdceee, 22);
        M5X_STEP(M5X_F, a, b, c, d, W[4], 0xf57c0faf, 7);   M5X_STEP(M5X_F, d, a, b, c, W[5], 0x4787c62a, 12);
        M5X_STEP(M5X_F, c, d, a, b, W[6], 0xa8304613, 17);  M5X_STEP(M5X_F, b, c, d, a, W[7], 0xfd469501, 22);
        M5X_STEP(M5X_F, a, b, c, d, W[8], 0x698098d8, 7);   M5X_STEP(M5X_F, d, a, b, c, W[9], 0x8b44f7af, 12);
        M5X_STEP(M5X_F, c, d, a, b, W[10], 0xffff5bb1, 17); M5X_STEP(M5X_F, b, c, d, a, W[11], 0x895cd7be, 22);
        M5X_STEP(M5X_F, a, b, c, d, W[12], 0x6b901122, 7);  M5X_STEP(M5X_F, d, a, b, c, W[13], 0xfd987193, 12);
        M5X_STEP(M5X_F, c, d, a, b, W[14], 0xa679438e, 17); M5X_STEP(M5X_F, b, c, d, a, W[15], 0x49b40821, 22);
        M5X_STEP(M5X_G, a, b, c, d, W[1], 0xf61e2562, 5);   M5X_STEP(M5X_G, d, a, b, c, W[6], 0xc040b340, 9);
        M5X_STEP(M5X_G, c, d, a, b, W[11], 0x265e5a51, 14); M5X_STEP(M5X_G, b, c, d, a, W[0], 0xe9b6c7aa, 20);
        M5X_STEP(M5X_G, a, b, c, d, W[5], 0xd62f105d, 5);   M5X_STEP(M5X_G, d, a, b, c, W[10], 0x02441453, 9);
        M5X_STEP(M5X_G, c, d, a, b, W[15], 0xd8a1e681, 14); M5X_STEP(M5X_G, b, c, d, a, W[4], 0xe7d3fbc8, 20);
        M5X_STEP(M5X_G, a, b, c, d, W[9], 0x21e1cde6, 5);   M5X_STEP(M5X_G, d, a, b, c, W[14], 0xc33707d6, 9);
        M5X_STEP(M5X_G, c, d, a, b, W[3], 0xf4d50d87, 14);  M5X_STEP(M5X_G, b, c, d, a, W[8], 0x455a14ed, 20);
        M5X_STEP(M5X_G, a, b, c, d, W[13], 0xa9e3e905, 5);  M5X_STEP(M5X_G, d, a, b, c, W[2], 0xfcefa3f8, 9);
        M5X_STEP(M5X_G, c, d, a, b, W[7], 0x676f02d9, 14);  M5X_STEP(M5X_G, b, c, d, a, W[12], 0x8d2a4c8a, 20);
        M5X_STEP(M5X_H, a, b, c, d, W[5], 0xfffa3942, 4);   M5X_STEP(M5X_H, d, a, b, c, W[8], 0x8771f681, 11);
        M5X_STEP(M5X_H, c, d, a, b, W[11], 0x6d9d6122, 16); M5X_STEP(M5X_H, b, c, d, a, W[14], 0xfde5380c, 23);
        M5X_STEP(M5X_H, a, b, c, d, W[1], 0xa4beea44, 4);   M5X_STEP(M5X_H, d, a, b, c, W[4], 0x4bdecfa9, 11);
        M5X_STEP(M5X_H, c, d, a, b, W[7], 0xf6bb4b60, 16);  M5X_STEP(M5X_H, b, c, d, a, W[10], 0xbebfbc70, 23);
        M5X_STEP(M5X_H, a, b, c, d, W[13], 0x289b7ec6, 4);  M5X_STEP(M5X_H, d, a, b, c, W[0], 0xeaa127fa, 11);
        M5X_STEP(M5X_H, c, d, a, b, W[3], 0xd4ef3085, 16);  M5X_STEP(M5X_H, b, c, d, a, W[6], 0x04881d05, 23);
        M5X_STEP(M5X_H, a, b, c, d, W[9], 0xd9d4d039, 4);   M5X_STEP(M5X_H, d, a, b, c, W[12], 0xe6db99e5, 11);
        M5X_STEP(M5X_H, c, d, a, b, W[15], 0x1fa27cf8, 16); M5X_STEP(M5X_H, b, c, d, a, W[2], 0xc4ac5665, 23);
        M5X_STEP(M5X_I, a, b, c, d, W[0], 0xf4292244, 6);   M5X_STEP(M5X_I, d, a, b, c, W[7], 0x432aff97, 10);
        M5X_STEP(M5X_I, c, d, a, b, W[14], 0xab9423a7, 15); M5X_STEP(M5X_I, b, c, d, a, W[5], 0xfc93a039, 21);
        M5X_STEP(M5X_I, a, b, c, d, W[12], 0x655b59c3, 6);  M5X_STEP(M5X_I, d, a, b, c, W[3], 0x8f0ccc92, 10);
        M5X_STEP(M5X_I, c, d, a, b, W[10], 0xffeff47d, 15); M5X_STEP(M5X_I, b, c, d, a, W[1], 0x85845dd1, 21);
        M5X_STEP(M5X_I, a, b, c, d, W[8], 0x6fa87e4f, 6);   M5X_STEP(M5X_I, d, a, b, c, W[15], 0xfe2ce6e0, 10);
        M5X_STEP(M5X_I, c, d, a, b, W[6], 0xa3014314, 15);  M5X_STEP(M5X_I, b, c, d, a, W[13], 0x4e0811a1, 21);
        M5X_STEP(M5X_I, a, b, c, d, W[4], 0xf7537e82, 6);   M5X_STEP(M5X_I, d, a, b, c, W[11], 0xbd3af235, 10);
        M5X_STEP(M5X_I, c, d, a, b, W[2], 0x2ad7d2bb, 15);  M5X_STEP(M5X_I, b, c, d, a, W[9], 0xeb86d391, 21);
        a0 = _mm512_add_epi32(a0, a);
        b0 = _mm512_add_epi32(b0, b);
        c0 = _mm512_add_epi32(c0, c);
        d0 = _mm512_add_epi32(d0, d);
    }
    _mm512_store_si512(sa, a0);
    _mm512_store_si512(sb, b0);
    _mm512_store_si512(sc, c0);
    _mm512_store_si512(sd, d0);
    for (int j = 0; j < n; j++) {
        st[j][0] = sa[j]; st[j][1] = sb[j]; st[j][2] = sc[j]; st[j][3] = sd[j];
    }
}

// the host supports AVX-512F (checked once); FLACGPU_MD5_AVX512=0 turns the vector path off
bool avx512_on() {
    static const bool on = [] {
        const char *e = std::getenv("FLACGPU_MD5_AVX512");
        if (e && e[0] == '0') return false;
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") != 0;
    }();
    return on;
}

// The process-wide hashing pool (Md5Pool below): a job is one whole-buffer update of a HostMd5.
struct Md5Job {
    HostMd5 *h;
    const uint8_t *p;  // the job's next full block
    size_t nb;         // full blocks left
    const uint8_t *tail;
    size_t tail_len;
    bool done = false;
    size_t *left = nullptr;  // a batch's count of unfinished jobs (run_many)
};

}  // namespace

// The pool size from the CPU facts.  One process per GPU (torchrun sets LOCAL_WORLD_SIZE): the
// node's ranks share the CPUs, so each rank's pool takes its 1/LOCAL_WORLD_SIZE -- but only when
// this process sees the whole machine (affinity mask = every online CPU, no cgroup quota).  A mask
// or quota narrower than that is already this rank's share (numactl, SLURM --cpu-bind, a per-rank
// cgroup) and is used as it is.
int md5_pool_share_of(int quota_cpus, int aff, int online, const char *local_world) {
    int n = (quota_cpus > 0 && quota_cpus < aff) ? quota_cpus : aff;
    const bool whole_machine = quota_cpus <= 0 && aff >= online;
    if (local_world && whole_machine) {
        const int lw = std::atoi(local_world);
        if (lw > 1) n = std::max(1, n / lw);
    }
    return n;
}

namespace {

class Md5Pool {
  public:
    static Md5Pool &get() {
        // never destroyed: its detached workers wait on its condition variable until the process
        // ends (a static object's destructor would destroy it under them at exit)
        static Md5Pool *pool = new Md5Pool;
        return *pool;
    }
    // hash `len` bytes into h on a pool worker, interleaved with other callers' jobs; blocks
    void run(HostMd5 *h, const uint8_t *p, size_t len) {
        // the partial block in h first (on the caller: at most 63 bytes of copying)
        if (h->fill && len) {
            const size_t take = len < 64u - h->fill ? len : 64u - h->fill;
            h->update(p, take);
            p += take;
            len -= take;
        }
        // short updates, no workers, or a forked child (the pool's threads live only in the
        // process that created them): the caller hashes its own chain
        if (h->fill || len < 64u * 64u || workers_ == 0 || getpid() != owner_) {
            h->update(p, len);
            return;
        }
        Md5Job job;
        job.h = h;
        job.p = p;
        job.nb = len / 64u;
        job.tail = p + job.nb * 64u;
        job.tail_len = len - job.nb * 64u;
        h->bytes += job.nb * 64u;
        {
            std::unique_lock<std::mutex> lk(m_);
            q_.push_back(&job);
            cv_.notify_one();
            done_cv_.wait(lk, [&] { return job.done; });
        }
        h->update(job.tail, job.tail_len);
    }
    // n updates at once (independent chains): the long ones are queued together, so the workers
    // interleave up to eight of them per core; the short ones are hashed on the caller meanwhile
    void run_many(HostMd5 *const *hs, const uint8_t *const *ps, const size_t *lens, size_t n) {
        if (workers_ == 0 || getpid() != owner_) {
            for (size_t i = 0; i < n; i++) hs[i]->update(ps[i], lens[i]);
            return;
        }
        struct Part {
            HostMd5 *h;
            const uint8_t *p;
            size_t len;
        };
        std::vector<Md5Job> jobs;
        std::vector<Part> own;
        jobs.reserve(n);  // the queue holds pointers into it
        size_t left = 0;
        for (size_t i = 0; i < n; i++) {
            HostMd5 *h = hs[i];
            const uint8_t *p = ps[i];
            size_t len = lens[i];
            if (h->fill && len) {
                const size_t take = len < 64u - h->fill ? len : 64u - h->fill;
                h->update(p, take);
                p += take;
                len -= take;
            }
            if (h->fill || len < 64u * 64u) {
                own.push_back({h, p, len});
                continue;
            }
            Md5Job j;
            j.h = h;
            j.p = p;
            j.nb = len / 64u;
            j.tail = p + j.nb * 64u;
            j.tail_len = len - j.nb * 64u;
            j.left = &left;
            h->bytes += j.nb * 64u;
            jobs.push_back(j);
        }
        if (!jobs.empty()) {
            std::lock_guard<std::mutex> lk(m_);
            left = jobs.size();
            for (auto &j : jobs) q_.push_back(&j);
            cv_.notify_all();
        }
        for (auto &o : own) o.h->update(o.p, o.len);
        if (!jobs.empty()) {
            std::unique_lock<std::mutex> lk(m_);
            done_cv_.wait(lk, [&] { return left == 0; });
        }
        for (auto &j : jobs) j.h->update(j.tail, j.tail_len);
    }
    int workers() const { return workers_; }
    // chains held by workers or queued (other callers hashing right now)
    bool busy() {
        std::lock_guard<std::mutex> lk(m_);
        return active_ > 0 || !q_.empty();
    }

  private:
    // up to four chains interleaved per worker: a core's throughput is flat past ~4 chains and
    // falls at 8 (the interleaved states no longer fit the x86-64 registers: 8 workers x 8 chains
    // 3.4 GB/s, x 4 chains 4.5 GB/s, tools/md5_pool_rate.py).  More chains than 4 x workers are
    // time-sliced: a worker that finishes a chunk while chains wait puts its own back at the
    // queue's tail, so every chain advances in turn and the batch ends as one round, not with a
    // tail round of the last few chains (r4ze measured that tail: 64 files on 15 workers)
    // With AVX-512 a worker whose share is kVecMin or more chains takes up to 16 into the lanes of
    // compress_x16, whose per-worker throughput keeps rising to 16 chains; below that the scalar
    // interleave is faster per chain (EPYC 9575F, r5i: one vector chain 0.42 GB/s, scalar 0.78;
    // per worker at 4 chains 1.71 vector vs 2.30 scalar GB/s, at 16 chains 6.8 vector vs 2.30
    // time-sliced scalar)
    static constexpr size_t kVecMin = 6;
    static size_t max_chains(size_t share) { return (avx512_on() && share >= kVecMin) ? 16 : 4; }
    static constexpr size_t kChunk = 256;  // blocks per chain between queue checks
    // The process's CPU share: the cgroup v2 quota where one is set (it is not visible in the
    // affinity mask), else the affinity mask.  Not OMP_NUM_THREADS: launchers such as torchrun
    // set it to 1 per process, which would put every file's chain on one worker.
    static int cpu_share() {
        int quota_cpus = 0;
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {};
            long long period = 0;
            if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
                const long long quota = atoll(q);
                if (quota > 0) quota_cpus = (int)((quota + period - 1) / period);
            }
            fclose(f);
        }
        cpu_set_t set;
        const int aff = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
        const long online = sysconf(_SC_NPROCESSORS_ONLN);
        return md5_pool_share_of(quota_cpus, aff, online > 0 ? (int)online : aff, std::getenv("LOCAL_WORLD_SIZE"));
    }
    Md5Pool() : owner_(getpid()) {
        int n = 0;
        if (const char *e = std::getenv("FLACGPU_MD5_THREADS")) n = std::atoi(e);  // < 0: no pool (A/B)
        if (n == 0) n = cpu_share();  // the callers mostly wait on the GPU
        if (n > 64) n = 64;
        if (n < 0) n = 0;  // every caller hashes its own chain
        for (int i = 0; i < n; i++) {
            try {
                std::thread([this] { loop(); }).detach();
                workers_++;
            } catch (...) {
                break;
            }
        }
    }
    void loop() {
        std::vector<Md5Job *> act;
        for (;;) {
            {
                // an idle worker takes one message; a busy one adds more only while no worker is
                // idle (so a few files spread over the workers, many files share them), and only
                // up to its even share of the chains in flight (so 32 files on 16 workers run two
                // chains each rather than four on a few workers and one on the rest)
                std::unique_lock<std::mutex> lk(m_);
                if (act.empty()) {
                    idle_++;
                    cv_.wait(lk, [&] { return !q_.empty(); });
                    idle_--;
                }
                const size_t chains = active_ + q_.size();
                const size_t even = std::max<size_t>(1, (chains + workers_ - 1) / workers_);
                const size_t share = std::min<size_t>(max_chains(even), even);
                while (act.size() < share && !q_.empty() && (act.empty() || idle_ == 0)) {
                    act.push_back(q_.front());
                    q_.pop_front();
                    active_++;
                }
            }
            size_t nb = kChunk;
            for (auto *j : act) nb = j->nb < nb ? j->nb : nb;
            uint32_t *st[16];
            const uint8_t *bp[16];
            for (size_t i = 0; i < act.size(); i++) {
                st[i] = act[i]->h->h;
                bp[i] = act[i]->p;
            }
            if (act.size() > 4) {  // only taken with the AVX-512 path (max_chains)
                compress_x16(st, bp, (int)act.size(), nb);
            } else {
                switch (act.size()) {
                case 1: compress_n<1>(st, bp, nb); break;
                case 2: compress_n<2>(st, bp, nb); break;
                case 3: compress_n<3>(st, bp, nb); break;
                default: compress_n<4>(st, bp, nb); break;
                }
            }
            bool finished = false;
            for (auto *j : act) {
                j->p += nb * 64u;
                j->nb -= nb;
                finished |= j->nb == 0;
            }
            if (finished) {
                std::lock_guard<std::mutex> lk(m_);
                for (auto *j : act)
                    if (j->nb == 0) {
                        j->done = true;
                        active_--;
                        if (j->left) --*j->left;
                    }
                done_cv_.notify_all();
                act.erase(std::remove_if(act.begin(), act.end(), [](Md5Job *j) { return j->done; }), act.end());
            }
            if (!act.empty()) {
                // chains waiting for a worker: yield this worker's to the queue's tail (time slicing)
                std::lock_guard<std::mutex> lk(m_);
                if (!q_.empty()) {
                    for (auto *j : act) q_.push_back(j);
                    active_ -= act.size();
                    act.clear();
                }
            }
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<Md5Job *> q_;
    int workers_ = 0, idle_ = 0;
    size_t active_ = 0;  // chains held by the workers
    const pid_t owner_;  // the process whose workers these are
};

}  // namespace

void md5_pool_update(HostMd5 *h, const void *data, size_t len) { Md5Pool::get().run(h, (const uint8_t *)data, len); }

void md5_pool_update_many(HostMd5 *const *hs, const uint8_t *const *data, const size_t *lens, size_t n) {
    Md5Pool::get().run_many(hs, data, lens, n);
}

int md5_pool_workers() { return Md5Pool::get().workers(); }

bool md5_avx512() { return avx512_on(); }

// Host MD5 rates on this machine: rate[i] = bytes/s per pool worker with pts[i] chains each
// (pts = 1, 2, 3, 4 for the scalar interleave; 1, 4, 8, 16 with the AVX-512 path), measured by
// running the pool itself on pts[i] x workers chains of 256 KiB (one buffer that stays in the
// caches: the pool's chains stream from memory, but MD5 at ~1 GB/s per chain is far below what a
// core can fetch), so SMT siblings, the workers' placement and wake-up costs are in the figure;
// best of three per point, ~5-15 ms in all.  Without a pool: one chain on the caller.
bool md5_measure_rates(double rate[4], uint32_t pts[4]) {
    // chain j hashes 256 KiB slice j mod 128 of a 32-MiB buffer: streaming reads, as a real
    // file's chain does, not one cache-resident block re-read by every chain
    constexpr size_t kLen = 256 * 1024, kSlices = 128;
    static uint8_t *buf = [] {
        uint8_t *b = new uint8_t[kLen * kSlices];
        uint32_t x = 0x12345678u;
        for (size_t i = 0; i < kLen * kSlices; i++) {
            x = x * 1664525u + 1013904223u;
            b[i] = (uint8_t)(x >> 24);
        }
        return b;
    }();
    Md5Pool &pool = Md5Pool::get();
    const int W = pool.workers();
    const bool vec = avx512_on();  // points past four chains per worker use the vector path
    bool contended = false;
    for (int i = 0; i < 4; i++) pts[i] = vec ? (i == 0 ? 1u : 4u << (i - 1)) : (uint32_t)(i + 1);
    for (int i = 0; i < 4; i++) {
        const size_t n = W > 0 ? (size_t)pts[i] * W : 1;
        std::vector<HostMd5> hs(n);
        std::vector<HostMd5 *> hp(n);
        std::vector<const uint8_t *> ps(n);
        std::vector<size_t> lens(n, kLen);
        for (size_t j = 0; j < n; j++) {
            hp[j] = &hs[j];
            ps[j] = buf + (j % kSlices) * kLen;
        }
        double best = 0;
        for (int rep = 0; rep < 3; rep++) {
            // another caller's chains on the pool would share its workers with this sample: wait
            // (up to 50 ms) for the pool to drain; a sample that still overlaps them is reported
            // as contended (flacgpu_md5_rates.measured = 3)
            if (W > 0) {
                for (int t = 0; t < 50 && pool.busy(); t++) std::this_thread::sleep_for(std::chrono::milliseconds(1));
                contended |= pool.busy();
            }
            const auto t0 = std::chrono::steady_clock::now();
            if (W > 0) pool.run_many(hp.data(), ps.data(), lens.data(), n);
            else hs[0].update(buf, kLen);
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt > 0) best = std::max(best, (double)n * kLen / dt / (W > 0 ? W : 1));
        }
        rate[i] = best;
        if (W == 0) {
            for (int j = 1; j < 4; j++) rate[j] = best;
            break;
        }
    }
    return contended;
}

void HostMd5::reset() {
    h[0] = 0x67452301u;
    h[1] = 0xefcdab89u;
    h[2] = 0x98badcfeu;
    h[3] = 0x10325476u;
    bytes = 0;
    fill = 0;
}

void HostMd5::update(const void *data, size_t len) {
    const uint8_t *p = (const uint8_t *)data;
    bytes += len;
    if (fill) {
        const size_t take = len < 64u - fill ? len : 64u - fill;
        memcpy(buf + fill, p, take);
        fill += (uint32_t)take;
        p += take;
        len -= take;
        if (fill < 64) return;
        compress(h, buf, 1);
        fill = 0;
    }
    const size_t nb = len / 64;
    compress(h, p, nb);
    p += nb * 64;
    len -= nb * 64;
    memcpy(buf, p, len);
    fill = (uint32_t)len;
}

void HostMd5::final(uint8_t digest[16]) {
    uint8_t tail[128] = {};
    memcpy(tail, buf, fill);
    tail[fill] = 0x80;
    const size_t nb = fill < 56 ? 1 : 2;
    const uint64_t bits = bytes * 8;
    for (int i = 0; i < 8; i++) tail[nb * 64 - 8 + i] = (uint8_t)(bits >> (8 * i));
    compress(h, tail, nb);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) digest[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
    reset();
}

}  // namespace fg
