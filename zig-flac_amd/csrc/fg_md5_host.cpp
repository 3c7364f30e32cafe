// fg_md5_host.cpp -- host MD5 (see fg_md5_host.hpp).
#include "fg_md5_host.hpp"

#include <string.h>

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

}  // namespace

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
