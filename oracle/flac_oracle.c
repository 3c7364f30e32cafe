/*
 * flac_oracle.c -- scalar CPU restatement of toastori/zig-flac's per-block
 * encode path.  TEST INFRASTRUCTURE ONLY (see flac_oracle.h for the rules and
 * the parity-pinning status).  Paths are relative to /root/reference/.
 *
 * This file deliberately follows the reference's control flow and integer
 * semantics one function at a time (including its quirks, SURVEY.md
 * Appendix A); it is not optimised.
 */
#include "flac_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MAX_BLOCK 65535u
#define INVALID_U64 UINT64_MAX

/* ===================================================================== */
/* CRC-8/SMBUS: std.hash.crc.Crc8Smbus used by frame_writer.zig:138.       */
/* poly 0x07, init 0, no reflection, no xorout (published check 0xF4).      */
/* ===================================================================== */
uint8_t oracle_crc8(const uint8_t *p, size_t n) {
    uint8_t crc = 0;
    for (size_t i = 0; i < n; i++) {
        crc ^= p[i];
        for (int b = 0; b < 8; b++) crc = (uint8_t)((crc & 0x80) ? (crc << 1) ^ 0x07 : (crc << 1));
    }
    return crc;
}

/* CRC-16/UMTS (crc16.zig:15-57; the PCLMUL fold and the std table fallback
 * are the same function): poly 0x8005, init 0, MSB first (check 0xFEE8).
 * oracle_crc16_bitwise is the definition, one bit per step; oracle_crc16 computes the same
 * value eight bytes per step from eight 256-entry tables (slicing-by-8), so the CPU-baseline
 * build does not time a bit-serial loop where the reference folds with PCLMUL
 * (tests/test_oracle_kat.py checks the two against each other).                         */
uint16_t oracle_crc16_bitwise(uint16_t crc, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) {
        crc ^= (uint16_t)(p[i] << 8);
        for (int b = 0; b < 8; b++)
            crc = (uint16_t)((crc & 0x8000) ? (crc << 1) ^ 0x8005 : (crc << 1));
    }
    return crc;
}

/* T[k][v]: the register contribution of byte value v followed by k zero bytes */
static uint16_t crc16_tab[8][256];
__attribute__((constructor)) static void crc16_tab_init(void) {
    for (int v = 0; v < 256; v++) {
        uint8_t b = (uint8_t)v;
        crc16_tab[0][v] = oracle_crc16_bitwise(0, &b, 1);
    }
    for (int k = 1; k < 8; k++)
        for (int v = 0; v < 256; v++) {
            const uint16_t t = crc16_tab[k - 1][v];
            crc16_tab[k][v] = (uint16_t)((t << 8) ^ crc16_tab[0][t >> 8]);
        }
}

uint16_t oracle_crc16(uint16_t crc, const uint8_t *p, size_t n) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint8_t b0 = (uint8_t)(p[i] ^ (crc >> 8)), b1 = (uint8_t)(p[i + 1] ^ (crc & 0xff));
        crc = (uint16_t)(crc16_tab[7][b0] ^ crc16_tab[6][b1] ^ crc16_tab[5][p[i + 2]] ^ crc16_tab[4][p[i + 3]] ^
                         crc16_tab[3][p[i + 4]] ^ crc16_tab[2][p[i + 5]] ^ crc16_tab[1][p[i + 6]] ^
                         crc16_tab[0][p[i + 7]]);
    }
    for (; i < n; i++) crc = (uint16_t)((crc << 8) ^ crc16_tab[0][(crc >> 8) ^ p[i]]);
    return crc;
}

/* ===================================================================== */
/* MD5 (md5.zig:3-35 = Zig std.crypto.hash.Md5 or OpenSSL MD5_*): RFC 1321 */
/* ===================================================================== */
static const uint32_t MD5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t MD5_S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                  5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                  4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                  6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static uint32_t rol32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

/* RFC 1321 section 3.4: 64 steps in four rounds of 16, each round's loop fully unrolled so
 * the step's constant, shift and message word index are immediates (the branch-per-step form
 * hashed at 311 MB/s against OpenSSL's 498 on the same core; the CPU baseline times this). */
#define MD5_ROUND(FN, G)                                                   \
    _Pragma("GCC unroll 16") for (int j = 0; j < 16; j++) {                \
        const int i = r0 + j;                                              \
        const uint32_t f = FN, t = d;                                      \
        d = cc;                                                            \
        cc = b;                                                            \
        b = b + rol32(a + f + MD5_K[i] + m[(G) & 15], MD5_S[i]);            \
        a = t;                                                             \
    }
static void md5_block(oracle_md5_ctx *c, const uint8_t *blk) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) |
               ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = c->a, b = c->b, cc = c->c, d = c->d;
    int r0 = 0;
    MD5_ROUND((b & cc) | (~b & d), i)
    r0 = 16;
    MD5_ROUND((d & b) | (~d & cc), 5 * i + 1)
    r0 = 32;
    MD5_ROUND(b ^ cc ^ d, 3 * i + 5)
    r0 = 48;
    MD5_ROUND(cc ^ (b | ~d), 7 * i)
    c->a += a; c->b += b; c->c += cc; c->d += d;
}
#undef MD5_ROUND

void oracle_md5_init(oracle_md5_ctx *c) {
    c->a = 0x67452301; c->b = 0xefcdab89; c->c = 0x98badcfe; c->d = 0x10325476;
    c->len = 0; c->fill = 0;
}

void oracle_md5_update(oracle_md5_ctx *c, const void *vp, size_t n) {
    const uint8_t *p = (const uint8_t *)vp;
    c->len += n;
    while (n > 0) {
        if (c->fill == 0 && n >= 64) { md5_block(c, p); p += 64; n -= 64; continue; }
        size_t take = 64 - c->fill;
        if (take > n) take = n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += (uint32_t)take; p += take; n -= take;
        if (c->fill == 64) { md5_block(c, c->buf); c->fill = 0; }
    }
}

void oracle_md5_final(oracle_md5_ctx *c, uint8_t out[16]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80;
    oracle_md5_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->fill != 56) oracle_md5_update(c, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (8 * i));
    oracle_md5_update(c, lb, 8);
    uint32_t w[4] = {c->a, c->b, c->c, c->d};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

void oracle_md5(const void *p, size_t n, uint8_t out[16]) {
    oracle_md5_ctx c;
    oracle_md5_init(&c);
    oracle_md5_update(&c, p, n);
    oracle_md5_final(&c, out);
}

/* ===================================================================== */
/* FrameWriter bit packer (frame_writer.zig:40-125): 64-bit MSB-first      */
/* accumulator, stored as big-endian u64 words.  writeBits ORs the value   */
/* UNMASKED into the accumulator (frame_writer.zig:44-58).                 */
/* ===================================================================== */
typedef struct {
    uint64_t accu;
    uint64_t *words;
    size_t cap_words;
    size_t end;
    unsigned remain; /* remain_bits, starts at 64 */
    int overflow;
} bw_t;

static void bw_store(bw_t *w, uint64_t v) {
    if (w->end < w->cap_words) w->words[w->end] = v;
    else w->overflow = 1;
    w->end++;
}

/* writeBits (frame_writer.zig:40-59) */
static void bw_bits(bw_t *w, unsigned bits, uint64_t value) {
    if (bits == 0) return;
    if (bits <= w->remain) {
        w->accu = (bits == 64) ? 0 : (w->accu << bits);
        w->accu |= value;
        w->remain -= bits;
    } else {
        unsigned shift = bits - w->remain;
        w->accu = (w->remain == 64) ? 0 : (w->accu << w->remain);
        w->accu |= value >> shift;
        bw_store(w, w->accu);
        w->accu = value;
        w->remain = 64 - shift;
    }
}

/* writeBitsSigned (frame_writer.zig:62-65) */
static void bw_bits_signed(bw_t *w, unsigned size, uint64_t value) {
    if (size == 0) return;
    uint64_t mask = UINT64_MAX >> (64 - size);
    bw_bits(w, size, value & mask);
}

/* writeZeros (frame_writer.zig:68-101) */
static void bw_zeros(bw_t *w, uint64_t bits) {
    if (bits == 0) return;
    uint64_t remain = bits;
    if (w->remain != 64) {
        unsigned first = (w->remain < bits) ? w->remain : (unsigned)bits;
        w->accu = (first == 64) ? 0 : (w->accu << first);
        w->remain -= first;
        remain -= first;
        if (w->remain == 0) {
            bw_store(w, w->accu);
            w->remain = 64;
        }
        if (remain == 0) return;
    }
    while (remain >= 64) {
        bw_store(w, 0);
        remain -= 64;
    }
    if (remain != 0) {
        w->accu = 0;
        w->remain = (unsigned)(64 - remain);
    }
}

static void be64(uint8_t *dst, uint64_t v) {
    for (int i = 0; i < 8; i++) dst[i] = (uint8_t)(v >> (56 - 8 * i));
}

/* writeCrc8 (frame_writer.zig:128-141): CRC-8 over the header bytes. */
static void bw_crc8(bw_t *w) {
    uint8_t bytes[16];
    unsigned byte_end = 8 - w->remain / 8;
    uint64_t accu_aligned = (w->remain == 64) ? w->accu : (w->accu << w->remain);
    size_t nb;
    if (w->end == 0) {
        be64(bytes, accu_aligned);
        nb = byte_end;
    } else { /* end == 1 (frame_writer.zig:132); end > 1 is unreachable */
        be64(bytes, w->words[0]);
        be64(bytes + 8, accu_aligned);
        nb = 8 + byte_end;
    }
    bw_bits(w, 8, oracle_crc8(bytes, nb));
}

/* ===================================================================== */
/* Rice (rice.zig)                                                         */
/* ===================================================================== */
#define RICE_MAX_ORDER 8
#define RICE_MAX_PART 256
#define MAX_PARAM_4BIT 14u
#define MAX_PARAM_5BIT 30u

/* calcZigzag (rice.zig:281-284), u32 result */
static uint32_t zigzag(int32_t v) {
    return v < 0 ? (uint32_t)(0u - (uint32_t)v) * 2u - 1u : (uint32_t)v * 2u;
}

static unsigned bitlen64(uint64_t x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }
static unsigned log2_floor(uint64_t x) { return 63u - (unsigned)__builtin_clzll(x); }

/* flacCalcPartSize (rice.zig:402-405): (1+p)*len + (p==0 ? 2S : (S>>(p-1)) -% len/2),
 * all in wrapping u64. */
uint64_t oracle_rice_part_size(uint64_t len, uint32_t param, uint64_t abs_sum) {
    uint64_t lin = (uint64_t)(1 + param) * len;
    if (param == 0) return lin + (abs_sum << 1);
    return lin + ((abs_sum >> (param - 1)) - (len >> 1));
}

typedef struct {
    uint8_t method;
    uint8_t part_order;
    uint8_t params[RICE_MAX_PART];
} rice_cfg;

/* calcSums (rice.zig:288-340) */
static void rice_sums(const int32_t *res, uint32_t n, unsigned P, unsigned order,
                      uint64_t sums[RICE_MAX_ORDER + 1][RICE_MAX_PART],
                      uint64_t maxs[RICE_MAX_ORDER + 1][RICE_MAX_PART]) {
    uint32_t ps = n >> P, pc = 1u << P;
    for (uint32_t part = 0; part < pc; part++) {
        uint64_t s = 0, m = 0;
        uint32_t lo = part * ps, hi = lo + ps;
        if (part == 0) lo = order; /* res[pred_order..part_size] (rice.zig:308) */
        for (uint32_t i = lo; i < hi; i++) {
            int32_t r = res[i];
            s += (uint64_t)(r < 0 ? (uint32_t)(0u - (uint32_t)r) : (uint32_t)r);
            m |= zigzag(r);
        }
        sums[P][part] = s;
        maxs[P][part] = bitlen64(m);
    }
    if (P == 0) return;
    for (int i = (int)P - 1; i >= 0; i--)
        for (uint32_t j = 0; j < (1u << i); j++) {
            sums[i][j] = sums[i + 1][2 * j] + sums[i + 1][2 * j + 1];
            uint64_t a = maxs[i + 1][2 * j], b = maxs[i + 1][2 * j + 1];
            maxs[i][j] = a > b ? a : b;
        }
}

/* calcOptimalParams (rice.zig:343-395) */
static uint64_t rice_optimal(unsigned o, uint32_t n, unsigned max_param, unsigned order,
                             const uint64_t *sums, uint64_t *maxs, rice_cfg *cfg) {
    uint32_t pc = 1u << o;
    cfg->part_order = (uint8_t)o;
    cfg->method = 0;
    uint64_t first_len = (uint64_t)(n >> o) - order;
    uint64_t ps = n >> o;
    uint64_t first_max = maxs[0];
    for (uint32_t j = 0; j < pc; j++) {
        cfg->params[j] = (uint8_t)(0x80 | maxs[j]);        /* Param.makeEscape */
        maxs[j] = (maxs[j] <= 31) ? 5 + maxs[j] * ps : INVALID_U64; /* isValidEscape */
    }
    maxs[0] -= first_max * order;
    for (unsigned p = 0; p < max_param; p++) {
        uint64_t size = oracle_rice_part_size(first_len, p, sums[0]);
        if (size < maxs[0]) { cfg->params[0] = (uint8_t)p; maxs[0] = size; }
        for (uint32_t j = 1; j < pc; j++) {
            size = oracle_rice_part_size(ps, p, sums[j]);
            if (size < maxs[j]) { cfg->params[j] = (uint8_t)p; maxs[j] = size; }
        }
    }
    if (max_param > MAX_PARAM_4BIT)
        for (uint32_t j = 0; j < pc; j++)
            if (!(cfg->params[j] & 0x80) && cfg->params[j] > MAX_PARAM_4BIT) cfg->method = 1;
    uint64_t bits = 0;
    for (uint32_t j = 0; j < pc; j++) bits += maxs[j];
    return bits + (uint64_t)(4 + cfg->method) * pc;
}

/* calcParams + calcParamEstimate (rice.zig:87-107,248-279).
 * One divergence, applied identically in the GPU path: the reference's
 * partition-order cap can leave partition 0 shorter than the predictor order
 * (block size a power of two <= 512 with order 3); the reference then slices
 * res[3..2] (rice.zig:308) -- undefined behaviour in ReleaseFast, a panic in
 * safe builds.  We lower the order until partition 0 holds the warm-up. */
static uint64_t rice_params(const int32_t *res, uint32_t n, unsigned max_part_order,
                            unsigned max_param_cfg, unsigned bps, unsigned order, rice_cfg *out,
                            int *clamped) {
    unsigned limited = order ? log2_floor(n) - log2_floor(order) : 15;
    unsigned ctz = (unsigned)__builtin_ctz(n);
    unsigned P = max_part_order;
    if (ctz < P) P = ctz;
    if (limited < P) P = limited;
    *clamped = 0;
    while (P > 0 && (n >> P) < order) { P--; *clamped = 1; }
    unsigned max_param = bps > 16 ? MAX_PARAM_5BIT : MAX_PARAM_4BIT;
    if (max_param_cfg < max_param) max_param = max_param_cfg;

    static __thread uint64_t sums[RICE_MAX_ORDER + 1][RICE_MAX_PART];
    static __thread uint64_t maxs[RICE_MAX_ORDER + 1][RICE_MAX_PART];
    rice_sums(res, n, P, order, sums, maxs);
    uint64_t best = INVALID_U64;
    rice_cfg cfg;
    for (unsigned o = 0; o <= P; o++) {
        uint64_t bc = rice_optimal(o, n, max_param, order, sums[o], maxs[o], &cfg);
        if (bc <= best) { best = bc; *out = cfg; }
    }
    return best;
}

/* ===================================================================== */
/* Fixed predictor (fixed.zig)                                             */
/* ===================================================================== */

/* bestOrder (fixed.zig:85-167).  s[] widened to i64.  Returns -1 for null. */
int oracle_best_order(const int64_t *s, uint32_t n, int wide, uint64_t totals[5]) {
    uint64_t tot[5] = {0, 0, 0, 0, 0}, orall[5] = {0, 0, 0, 0, 0};
    int64_t prev[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < 4 && i < n; i++) { /* warm-up loop (fixed.zig:102-127) */
        int64_t e0 = s[i];
        int64_t e1 = i < 1 ? 0 : e0 - prev[0];
        int64_t e2 = i < 2 ? 0 : e1 - prev[1];
        int64_t e3 = i < 3 ? 0 : e2 - prev[2];
        uint64_t a0 = (uint64_t)llabs(e0), a1 = (uint64_t)llabs(e1), a2 = (uint64_t)llabs(e2),
                 a3 = (uint64_t)llabs(e3);
        prev[0] = e0; prev[1] = e1; prev[2] = e2; prev[3] = e3;
        tot[0] += a0; tot[1] += a1; tot[2] += a2; tot[3] += a3;
        orall[0] |= a0; orall[1] |= a1; orall[2] |= a2; orall[3] |= a3;
    }
    for (uint32_t i = 4; i < n; i++) { /* main loop (fixed.zig:129-158) */
        int64_t e0 = s[i];
        int64_t e1 = e0 - prev[0];
        int64_t e2 = e1 - prev[1];
        int64_t e3 = e2 - prev[2];
        int64_t e4 = e3 - prev[3];
        uint64_t a0 = (uint64_t)llabs(e0), a1 = (uint64_t)llabs(e1), a2 = (uint64_t)llabs(e2),
                 a3 = (uint64_t)llabs(e3), a4 = (uint64_t)llabs(e4);
        prev[0] = e0; prev[1] = e1; prev[2] = e2; prev[3] = e3;
        tot[0] += a0; tot[1] += a1; tot[2] += a2; tot[3] += a3; tot[4] += a4;
        orall[0] |= a0; orall[1] |= a1; orall[2] |= a2; orall[3] |= a3; orall[4] |= a4;
    }
    if (wide)
        for (int k = 0; k < 5; k++)
            if (orall[k] > 0x7fffffffULL) tot[k] = INVALID_U64; /* fixed.zig:160-162 */
    int best = 0; /* std.mem.indexOfMin: first minimum */
    for (int k = 1; k < 5; k++)
        if (tot[k] < tot[best]) best = k;
    if (totals) memcpy(totals, tot, sizeof(tot));
    if (wide && tot[best] == INVALID_U64) return -1;
    return best;
}

/* calcResiduals (fixed.zig:30-76,169-201): COEFF_SCALAR stencil, wrapping
 * i32 (narrow) or i64 truncated to the low 32 bits (wide).  e[0..k) unused. */
/* COEFF_SCALAR = {}, {1}, {-1, 2}, {1, -3, 3}, {-1, 4, -6, 4}: the residual is x_i minus them
 * applied to x_{i-k} .. x_{i-1}, expanded below per order */
static void calc_residuals(const int64_t *s, uint32_t n, unsigned k, int wide, int32_t *e) {
    /* one branch-free loop per (order, width) with the stencil as immediates, so the compiler
     * vectorises it as the reference does (calcResidualVec, fixed.zig:169-201) */
    uint32_t i = 0;
    for (; i < k && i < n; i++) e[i] = 0;
    /* X(j) = sample i - j in the loop's width (i >= k here, so every X(j), j <= k, is in range) */
#define X(j) ((T)s[i - (j)])
#define RES_LOOP(T_, EXPR)                                                  \
    {                                                                       \
        typedef T_ T;                                                       \
        for (; i < n; i++) e[i] = (int32_t)(uint32_t)(EXPR);                \
    }
    if (wide) {
        switch (k) {
        case 0: RES_LOOP(uint64_t, X(0)) break;
        case 1: RES_LOOP(uint64_t, X(0) - X(1)) break;
        case 2: RES_LOOP(uint64_t, X(0) - 2 * X(1) + X(2)) break;
        case 3: RES_LOOP(uint64_t, X(0) - 3 * X(1) + 3 * X(2) - X(3)) break;
        default: RES_LOOP(uint64_t, X(0) - 4 * X(1) + 6 * X(2) - 4 * X(3) + X(4)) break;
        }
    } else {
        switch (k) {
        case 0: RES_LOOP(uint32_t, X(0)) break;
        case 1: RES_LOOP(uint32_t, X(0) - X(1)) break;
        case 2: RES_LOOP(uint32_t, X(0) - 2 * X(1) + X(2)) break;
        case 3: RES_LOOP(uint32_t, X(0) - 3 * X(1) + 3 * X(2) - X(3)) break;
        default: RES_LOOP(uint32_t, X(0) - 4 * X(1) + 6 * X(2) - 4 * X(3) + X(4)) break;
        }
    }
#undef RES_LOOP
#undef X
}

/* ===================================================================== */
/* LPC -- build-defined extension.  The reference has no LPC (readme.md:27 */
/* lists it as in progress; Prediction = {fixed, none}, encoder.zig:629-640;*/
/* the `linear` subframe is commented out, encoder.zig:694-699), so this is */
/* the contract the gfx950 kernels share with this restatement bit for bit: */
/*  0. LPC is searched on i32 samples only (a 32-bit stereo side that     */
/*     still needs 33 bits after its waste shift keeps its fixed choice);  */
/*  1. window w(i) = (i+1)(n-i): integer, Welch-shaped, never zero;        */
/*  2. xw(i) = (x(i) w(i)) >> sh (arithmetic), sh = max(0, bitlen(max|x|)  */
/*     + bitlen(floor((n+1)^2/4)) - 25), so |xw| <= 2^25;                 */
/*  3. R[lag] = sum_i xw(i) xw(i-lag) exactly in i64 (order-free);          */
/*  4. Levinson-Durbin in IEEE double, the operation order below, no FMA;  */
/*  5. quantisation to 15-bit coefficients: shift = 14 - e where           */
/*     max|a| = f 2^e, f in [0.5,1); shift > 15 -> 15; shift < 0 -> order  */
/*     unusable; round half away from zero with error feedback;            */
/*  6. residual e(i) = x(i) - ((sum_t c_t x(i-1-t)) >> shift) in i64; an   */
/*     order with a coded residual outside [-2^30, 2^30) is unusable (its  */
/*     zigzag code then fits 31 bits, so an escape is always possible);    */
/*  7. order selection by the Levinson-Durbin error (as libFLAC without    */
/*     its exhaustive search): among orders 1..Q (Q < n) whose coefficients */
/*     quantise, the lowest q with the smallest                             */
/*       key(q) = l2(err_q) * (n / 2) + q (bps' + 15)   (IEEE double, this  */
/*     operation order; err_q = the LD error after order q; l2(x) = (e-1) + */
/*     (2f-1) for x = f 2^e, f in [0.5,1): a piecewise-linear log2 made of  */
/*     exact IEEE operations; err_q <= 0 -> key = -1e300);                  */
/*  8. that one order gets the fixed path's Rice search with q warm-ups;    */
/*     subframe total = rice + q (bps' + 15) + 9; it replaces the fixed/    */
/*     verbatim choice only if strictly smaller (totals incl. warm-ups)     */
/* ===================================================================== */
#define LPC_XW_BITS 25u

int oracle_lpc_autocorr(const int64_t *x, uint32_t n, unsigned max_lag, int64_t *R) {
    uint64_t m = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t a = (uint64_t)(x[i] < 0 ? -x[i] : x[i]);
        if (a > m) m = a;
    }
    uint64_t wmax = ((uint64_t)(n + 1) * (uint64_t)(n + 1)) / 4u;
    int sh = (int)bitlen64(m) + (int)bitlen64(wmax) - (int)LPC_XW_BITS;
    if (sh < 0) sh = 0;
    int64_t *xw = (int64_t *)malloc((n ? n : 1) * sizeof(int64_t));
    for (uint32_t i = 0; i < n; i++) {
        int64_t w = (int64_t)(i + 1) * (int64_t)(n - i);
        xw[i] = (x[i] * w) >> sh;
    }
    for (unsigned lag = 0; lag <= max_lag; lag++) {
        int64_t acc = 0;
        for (uint32_t i = lag; i < n; i++) acc += xw[i] * xw[i - lag];
        R[lag] = acc;
    }
    free(xw);
    return sh;
}

/* Levinson-Durbin; errs[m] (if non-NULL) = the prediction error after order m + 1 */
int oracle_lpc_levinson_err(const int64_t *R, unsigned max_order, double *coefs, double *errs) {
    double r[ORACLE_LPC_MAX_ORDER + 1], a[ORACLE_LPC_MAX_ORDER], tmp[ORACLE_LPC_MAX_ORDER];
    for (unsigned i = 0; i <= max_order; i++) r[i] = (double)R[i];
    if (!(r[0] > 0.0)) return 0;
    double err = r[0];
    unsigned valid = 0;
    for (unsigned m = 0; m < max_order; m++) {
        double acc = r[m + 1];
        for (unsigned t = 0; t < m; t++) {
            double p = a[t] * r[m - t];
            acc = acc - p;
        }
        double k = acc / err;
        for (unsigned t = 0; t < m; t++) {
            double p = k * a[m - 1 - t];
            tmp[t] = a[t] - p;
        }
        for (unsigned t = 0; t < m; t++) a[t] = tmp[t];
        a[m] = k;
        for (unsigned t = 0; t <= m; t++) coefs[m * ORACLE_LPC_MAX_ORDER + t] = a[t];
        valid = m + 1;
        double kk = k * k;
        err = err * (1.0 - kk);
        if (errs) errs[m] = err;
        if (!(err > 0.0)) break;
    }
    return (int)valid;
}

int oracle_lpc_levinson(const int64_t *R, unsigned max_order, double *coefs) {
    return oracle_lpc_levinson_err(R, max_order, coefs, NULL);
}

/* order-selection key of contract step 7 */
double oracle_lpc_order_key(double err, unsigned q, uint32_t n, unsigned bps) {
    if (!(err > 0.0)) return -1e300;
    int e;
    const double f = frexp(err, &e);
    const double l2 = (double)(e - 1) + (2.0 * f - 1.0);
    return l2 * (0.5 * (double)n) + (double)(q * (bps + ORACLE_LPC_PRECISION));
}

int oracle_lpc_quantize(const double *a, unsigned order, unsigned precision, int32_t *q, int *shift) {
    double cmax = 0.0;
    for (unsigned t = 0; t < order; t++) {
        double v = a[t] < 0.0 ? -a[t] : a[t];
        if (v > cmax) cmax = v;
    }
    if (!(cmax > 0.0)) return -1;
    int e;
    frexp(cmax, &e);
    int sh = (int)precision - 1 - e;
    if (sh > 15) sh = 15;
    if (sh < 0) return -1;
    const double scale = (double)(1u << sh);
    const int64_t qmax = ((int64_t)1 << (precision - 1)) - 1, qmin = -((int64_t)1 << (precision - 1));
    double carry = 0.0;
    for (unsigned t = 0; t < order; t++) {
        double v = a[t] * scale;
        v = v + carry;
        int64_t qi = v >= 0.0 ? (int64_t)floor(v + 0.5) : -(int64_t)floor(-v + 0.5);
        if (qi > qmax) qi = qmax;
        if (qi < qmin) qi = qmin;
        carry = v - (double)qi;
        q[t] = (int32_t)qi;
    }
    *shift = sh;
    return 0;
}

/* residuals of one quantised predictor; returns -1 if any leaves [-2^30, 2^30) */
static int lpc_residuals(const int64_t *s, uint32_t n, unsigned order, const int32_t *c, int shift, int32_t *e) {
    for (uint32_t i = 0; i < order && i < n; i++) e[i] = 0;
    for (uint32_t i = order; i < n; i++) {
        int64_t acc = 0;
        for (unsigned t = 0; t < order; t++) acc += (int64_t)c[t] * s[i - 1 - t];
        int64_t v = s[i] - (acc >> shift);
        if (v < -(INT64_C(1) << 30) || v >= (INT64_C(1) << 30)) return -1;
        e[i] = (int32_t)v;
    }
    return 0;
}

/* ===================================================================== */
/* Encoder decisions (encoder.zig)                                         */
/* ===================================================================== */
typedef struct {
    oracle_subframe rec;
    const int64_t *samples; /* shifted samples used for verbatim/warm-ups */
    int32_t *residuals;
} sub_t;

/* calcWasteBits (encoder.zig:556-570), applied to a widened copy. */
static unsigned calc_waste(int64_t *s, uint32_t n, unsigned bps) {
    uint64_t orv = 0;
    for (uint32_t i = 0; i < n; i++) orv |= (uint64_t)s[i];
    unsigned w = orv == 0 ? bps : (unsigned)__builtin_ctzll(orv);
    if (w != 0 && w != bps)
        for (uint32_t i = 0; i < n; i++) s[i] = (int64_t)(int32_t)(s[i] >> w); /* @intCast into i32 plane */
    return w;
}

/* Analysis mode, NOT the contract (tools/lpc_ratio.py only): every order 1..Q whose coefficients
 * quantise gets the Rice search and the smallest total wins (an exhaustive order search, what
 * libFLAC's -e does), to measure what step 7's single order costs in compression. */
static int g_lpc_exhaustive = 0;
void oracle_set_lpc_exhaustive(int on) { g_lpc_exhaustive = on != 0; }

/* LPC order search (build-defined, contract above).  Replaces the current
 * choice when an order's total is strictly smaller. */
static void lpc_search(sub_t *sub, const int64_t *s, uint32_t n, const oracle_config *cfg, unsigned bps,
                       unsigned Q) {
    oracle_subframe *r = &sub->rec;
    for (uint32_t i = 0; i < n; i++)
        if (s[i] != (int64_t)(int32_t)s[i]) return; /* 33-bit side: no LPC (contract step 0) */
    int64_t R[ORACLE_LPC_MAX_ORDER + 1];
    static __thread double coefs[ORACLE_LPC_MAX_ORDER * ORACLE_LPC_MAX_ORDER];
    double errs[ORACLE_LPC_MAX_ORDER];
    oracle_lpc_autocorr(s, n, Q, R);
    int valid = oracle_lpc_levinson_err(R, Q, coefs, errs);
    /* step 7: the order with the smallest key (lowest q on ties) among those that quantise */
    unsigned qs = 0;
    double best_key = 0.0;
    int32_t cs[ORACLE_LPC_MAX_ORDER];
    int shs = 0;
    for (unsigned q = 1; q <= (unsigned)valid; q++) {
        int32_t c[ORACLE_LPC_MAX_ORDER];
        int shift;
        if (oracle_lpc_quantize(coefs + (q - 1) * ORACLE_LPC_MAX_ORDER, q, ORACLE_LPC_PRECISION, c, &shift)) continue;
        const double key = oracle_lpc_order_key(errs[q - 1], q, n, bps);
        if (qs == 0 || key < best_key) {
            qs = q;
            best_key = key;
            memcpy(cs, c, q * sizeof(int32_t));
            shs = shift;
        }
    }
    if (qs == 0) return;
    int32_t *e = (int32_t *)malloc(n * sizeof(int32_t));
    /* step 8: the selected order only (analysis mode: every order that quantises) */
    const unsigned q0 = g_lpc_exhaustive ? 1u : qs, q1 = g_lpc_exhaustive ? (unsigned)valid : qs;
    for (unsigned q = q0; q <= q1; q++) {
        int32_t cq[ORACLE_LPC_MAX_ORDER];
        int shq = shs;
        if (q != qs) {
            if (oracle_lpc_quantize(coefs + (q - 1) * ORACLE_LPC_MAX_ORDER, q, ORACLE_LPC_PRECISION, cq, &shq)) continue;
        } else {
            memcpy(cq, cs, q * sizeof(int32_t));
        }
        const int32_t *c = cq;
        const int shift = shq;
        if (lpc_residuals(s, n, q, c, shift, e)) continue;
        rice_cfg rc;
        memset(&rc, 0, sizeof(rc));
        int clamped = 0;
        uint64_t rice = rice_params(e, n, cfg->max_rice_part_order, cfg->max_rice_param, bps, q, &rc, &clamped);
        uint64_t total = rice + (uint64_t)q * (bps + ORACLE_LPC_PRECISION) + 9u;
        if (total < r->estimate) {
            r->type = OR_LPC;
            r->estimate = total;
            r->order = (uint8_t)q;
            r->part_order = rc.part_order;
            r->method = rc.method;
            r->ub_clamped = (uint8_t)clamped;
            memcpy(r->params, rc.params, sizeof(rc.params));
            r->lpc_precision = ORACLE_LPC_PRECISION;
            r->lpc_shift = (int8_t)shift;
            memset(r->lpc_coefs, 0, sizeof(r->lpc_coefs));
            memcpy(r->lpc_coefs, c, q * sizeof(int32_t));
            memcpy(sub->residuals, e, n * sizeof(int32_t));
        }
    }
    free(e);
}

static void choose_fixed(sub_t *sub, const int64_t *s, uint32_t n, int32_t *res, const oracle_config *cfg,
                         unsigned bps, int i64_samples);

/* chooseSubframeEncoding (encoder.zig:482-554).  `i64_samples` marks the
 * SampleVariant.wide side channel (32-bit stereo, waste 0). */
static void choose_subframe(sub_t *sub, int64_t *s, uint32_t n, int32_t *res, const oracle_config *cfg,
                            unsigned bit_depth, unsigned waste, int i64_samples) {
    oracle_subframe *r = &sub->rec;
    memset(r, 0, sizeof(*r));
    sub->samples = s;
    sub->residuals = res;
    r->waste = (uint8_t)waste;
    r->bits = (uint8_t)bit_depth;
    unsigned bps = bit_depth - waste;
    if (bps == 0) { r->type = OR_CONSTANT; r->estimate = 0; r->constant = 0; return; }
    int all_eq = 1;
    for (uint32_t i = 1; i < n; i++)
        if (s[i] != s[0]) { all_eq = 0; break; }
    if (all_eq) { r->type = OR_CONSTANT; r->estimate = bps; r->constant = s[0]; return; }
    r->type = OR_VERBATIM;
    r->estimate = (uint64_t)n * bps;
    const unsigned lpc_q = cfg->prediction;
    if (n > 4) choose_fixed(sub, s, n, res, cfg, bps, i64_samples);
    /* LPC mode (build-defined extension) */
    if (lpc_q && n > lpc_q && n <= 4096) lpc_search(sub, s, n, cfg, bps, lpc_q);
}

/* The fixed-predictor part of chooseSubframeEncoding (encoder.zig:514-550). */
static void choose_fixed(sub_t *sub, const int64_t *s, uint32_t n, int32_t *res, const oracle_config *cfg,
                         unsigned bps, int i64_samples) {
    oracle_subframe *r = &sub->rec;
    const unsigned lpc_q = cfg->prediction;
    int wide = !(bps < 28 && !i64_samples);
    r->wide = (uint8_t)wide;
    int k = oracle_best_order(s, n, wide, NULL);
    if (k < 0) return; /* wide overflow -> verbatim (encoder.zig:520) */
    calc_residuals(s, n, (unsigned)k, wide, res);
    rice_cfg rc;
    memset(&rc, 0, sizeof(rc));
    int clamped = 0;
    uint64_t fixed_size = rice_params(res, n, cfg->max_rice_part_order, cfg->max_rice_param, bps, (unsigned)k,
                                      &rc, &clamped);
    /* LPC mode (build-defined): estimates are whole payloads, warm-ups included */
    if (lpc_q) fixed_size += (uint64_t)k * bps;
    if (fixed_size < r->estimate) { /* strict (encoder.zig:538) */
        r->type = OR_FIXED;
        r->estimate = fixed_size;
        r->order = (uint8_t)k;
        r->part_order = rc.part_order;
        r->method = rc.method;
        r->ub_clamped = (uint8_t)clamped;
        memcpy(r->params, rc.params, sizeof(rc.params));
    }
}

/* ===================================================================== */
/* Frame header + subframe writers (frame_writer.zig:151-372)              */
/* ===================================================================== */
static void write_header(bw_t *w, uint64_t frame_number, unsigned bit_depth, unsigned channel_code,
                         uint32_t block_size, uint32_t sample_rate) {
    bw_bits(w, 16, 0xFFF8); /* fixed blocking (frame_writer.zig:163) */
    int unc_bs = 0;         /* 0 none, 8 byte, 16 half */
    unsigned ctz = (unsigned)__builtin_ctz(block_size);
    if ((block_size & (block_size - 1)) == 0 && ctz <= 15 && ctz >= 8) {
        bw_bits(w, 4, ctz);
    } else if (block_size == 192) {
        bw_bits(w, 4, 1);
    } else if ((block_size >> ctz) == 144 && ctz <= 5 && ctz >= 2) { /* never true (odd part) */
        bw_bits(w, 4, ctz);
    } else if (block_size < 0x100) {
        bw_bits(w, 4, 6);
        unc_bs = 8;
    } else {
        bw_bits(w, 4, 7);
        unc_bs = 16;
    }
    int unc_sr = 0; /* 0 none, 4 byte, 1 half, 10 half_tenth */
    unsigned rc;
    switch (sample_rate) {
    case 0: rc = 0; break;
    case 88200: rc = 1; break;
    case 176400: rc = 2; break;
    case 192000: rc = 3; break;
    case 8000: rc = 4; break;
    case 16000: rc = 5; break;
    case 22050: rc = 6; break;
    case 24000: rc = 7; break;
    case 32000: rc = 8; break;
    case 44100: rc = 9; break;
    case 48000: rc = 10; break;
    case 96000: rc = 11; break;
    default:
        if (sample_rate <= 255) { unc_sr = 4; rc = 12; }
        else if (sample_rate <= 65535) { unc_sr = 1; rc = 13; }
        else { unc_sr = 10; rc = 14; }
    }
    bw_bits(w, 4, rc);
    bw_bits(w, 4, channel_code);
    unsigned bc = bit_depth == 8 ? 2 : bit_depth == 16 ? 8 : bit_depth == 24 ? 12 : bit_depth == 32 ? 14 : 0;
    bw_bits(w, 4, bc);
    if (frame_number <= 0x7F) {
        bw_bits(w, 8, frame_number);
    } else {
        uint64_t buffer = 0, number = frame_number, first_byte_max = 0x3F;
        unsigned i = 0;
        while (number > first_byte_max) {
            buffer |= (0x80 + (number & 0x3F)) << (8 * i);
            i++;
            number >>= 6;
            first_byte_max >>= 1;
        }
        buffer |= (((uint64_t)0xFE << (6 - i)) | number) << (8 * i);
        buffer &= (1ULL << 56) - 1; /* u56 */
        bw_bits_signed(w, 8 * (i + 1), buffer);
    }
    if (unc_bs) bw_bits(w, (unsigned)unc_bs, block_size - 1);
    if (unc_sr == 4) bw_bits(w, 8, block_size); /* writes block size, unmasked (frame_writer.zig:260) */
    else if (unc_sr) bw_bits(w, 16, block_size / (unsigned)unc_sr);
    bw_crc8(w);
}

int oracle_utf8_number(uint64_t v, uint8_t out[8]) {
    uint64_t words[4] = {0, 0, 0, 0};
    bw_t w = {0, words, 4, 0, 64, 0};
    if (v <= 0x7F) { out[0] = (uint8_t)v; return 1; }
    uint64_t buffer = 0, number = v, first_byte_max = 0x3F;
    unsigned i = 0;
    while (number > first_byte_max) {
        buffer |= (0x80 + (number & 0x3F)) << (8 * i);
        i++;
        number >>= 6;
        first_byte_max >>= 1;
    }
    buffer |= (((uint64_t)0xFE << (6 - i)) | number) << (8 * i);
    bw_bits_signed(&w, 8 * (i + 1), buffer & ((1ULL << 56) - 1));
    uint64_t a = w.accu << w.remain;
    for (unsigned b = 0; b <= i; b++) out[b] = (uint8_t)(a >> (56 - 8 * b));
    return (int)i + 1;
}

/* writeChannelSubframe (encoder.zig:287-310) + FrameWriter.write*Subframe */
static void write_subframe(bw_t *w, const sub_t *sub, uint32_t n) {
    const oracle_subframe *r = &sub->rec;
    unsigned waste = r->waste, bps = r->bits - waste;
    if (r->type == OR_CONSTANT) { /* frame_writer.zig:269-279: never the wasted flag */
        bw_bits(w, 8, 0);
        uint64_t v = (uint64_t)r->constant << waste;
        bw_bits_signed(w, bps + waste, waste >= 64 ? 0 : v);
        return;
    }
    if (r->type == OR_VERBATIM) { /* frame_writer.zig:282-301 */
        if (waste == 0) bw_bits(w, 8, 0x02);
        else { bw_bits(w, 8, 0x03); bw_bits(w, waste, 1); }
        for (uint32_t i = 0; i < n; i++) bw_bits_signed(w, bps, (uint64_t)sub->samples[i]);
        return;
    }
    /* FIXED (frame_writer.zig:303-361); LPC (build-defined, FLAC subframe syntax:
     * type 0b1xxxxx = order-1, warm-ups, 4-bit precision-1, 5-bit signed shift,
     * coefficients, then the same residual coding) */
    unsigned order = r->order, method = r->method;
    unsigned param_len = 4 + method;
    uint32_t pc = 1u << r->part_order;
    unsigned tcode = r->type == OR_LPC ? (0x20u | (order - 1u)) : (8u | order);
    if (waste == 0) bw_bits(w, 8, tcode << 1);
    else { bw_bits(w, 8, (tcode << 1) | 1); bw_bits(w, waste, 1); }
    for (unsigned i = 0; i < order; i++) bw_bits_signed(w, bps, (uint64_t)sub->samples[i]);
    if (r->type == OR_LPC) {
        bw_bits(w, 4, r->lpc_precision - 1u);
        bw_bits_signed(w, 5, (uint64_t)(int64_t)r->lpc_shift);
        for (unsigned i = 0; i < order; i++) bw_bits_signed(w, r->lpc_precision, (uint64_t)(int64_t)r->lpc_coefs[i]);
    }
    bw_bits(w, 6, (method << 4) | r->part_order);
    const int32_t *rem = sub->residuals + order;
    uint32_t part_len = (n >> r->part_order) - order;
    for (uint32_t j = 0; j < pc; j++) {
        uint8_t p = r->params[j];
        if (p & 0x80) {
            unsigned eb = p & 0x7F;
            bw_bits(w, param_len, 0x0F | (method << 4));
            bw_bits(w, 5, eb);
            if (eb != 0)
                for (uint32_t i = 0; i < part_len; i++) bw_bits_signed(w, eb, (uint64_t)(uint32_t)rem[i]);
        } else {
            bw_bits(w, param_len, p);
            uint64_t mask = 1ULL << p; /* writeRicePart (frame_writer.zig:363-372) */
            for (uint32_t i = 0; i < part_len; i++) {
                uint32_t zz = zigzag(rem[i]);
                bw_zeros(w, zz >> p);
                bw_bits(w, p + 1, mask | (zz & ((1u << p) - 1u)));
            }
        }
        rem += part_len;
        part_len = n >> r->part_order;
    }
}

size_t oracle_max_frame_bytes(uint32_t block_size, uint32_t bit_depth, uint32_t channels) {
    /* maxFrameBytes (encoder.zig:583-595); the reference passes
     * compute_waste_bits (always true) as the stereo flag (encoder.zig:59). */
    size_t header_max = 2 + 7 + 2 + 2 + 1, sub_hdr = 8;
    size_t bps = channels == 2 ? bit_depth + 1 : bit_depth;
    size_t bytes_per = (bps + 7) / 8;
    return header_max + sub_hdr * channels + (size_t)block_size * bytes_per * (channels + 1) + 2;
}

/* Encoder.writeFrame + processChannels (encoder.zig:234-284,313-477). */
long oracle_encode_frame(const oracle_config *cfg, const int32_t *const *planes, uint32_t n,
                         uint64_t frame_number, uint8_t *out, size_t cap, oracle_frame_record *rec) {
    unsigned ch = cfg->channels, bd = cfg->bits_per_sample;
    if (n == 0 || n > MAX_BLOCK || ch < 1 || ch > 8) return -1;
    if (bd != 8 && bd != 16 && bd != 24 && bd != 32) return -1;

    size_t max_bytes = oracle_max_frame_bytes(n, bd, ch) + 64;
    size_t cap_words = (max_bytes + 7) / 8 + 4;
    uint64_t *words = (uint64_t *)calloc(cap_words, 8);
    int64_t *S[8];
    int32_t *R[8];
    for (unsigned c = 0; c < 8; c++) {
        S[c] = (int64_t *)calloc(n, sizeof(int64_t));
        R[c] = (int32_t *)calloc(n, sizeof(int32_t));
    }
    sub_t subs[8];
    const sub_t *order_out[8];
    unsigned n_out = 0, channel_code;
    memset(rec, 0, sizeof(*rec));

    if (ch == 2 && cfg->stereo_decorrelation) {
        /* Mid / side from the UN-shifted L/R (encoder.zig:329-350). */
        for (uint32_t i = 0; i < n; i++) {
            int64_t L = planes[0][i], Rr = planes[1][i];
            S[0][i] = L;
            S[1][i] = Rr;
            if (bd == 32) {
                S[2][i] = (int64_t)(int32_t)((L + Rr) >> 1);
                S[3][i] = L - Rr; /* samples64 */
            } else {
                S[2][i] = (int32_t)((uint32_t)(int32_t)L + (uint32_t)(int32_t)Rr) >> 1;
                S[3][i] = (int32_t)((uint32_t)(int32_t)L - (uint32_t)(int32_t)Rr);
            }
        }
        uint64_t est[4];
        for (unsigned c = 0; c < 3; c++) { /* left, right, mid */
            unsigned w = calc_waste(S[c], n, bd);
            choose_subframe(&subs[c], S[c], n, R[c], cfg, bd, w, 0);
            est[c] = subs[c].rec.estimate;
        }
        { /* side (encoder.zig:398-439) */
            unsigned w = calc_waste(S[3], n, bd + 1);
            int i64s = (bd == 32 && w == 0);
            choose_subframe(&subs[3], S[3], n, R[3], cfg, bd + 1, w, i64s);
            est[3] = subs[3].rec.estimate;
        }
        uint64_t sum[4] = {est[0] + est[1], est[0] + est[3], est[3] + est[1], est[2] + est[3]};
        unsigned best = 0;
        for (unsigned i = 1; i < 4; i++)
            if (sum[i] < sum[best]) best = i;
        static const unsigned pairs[4][2] = {{0, 1}, {0, 3}, {3, 1}, {2, 3}};
        channel_code = best == 0 ? 1 : best + 7;
        order_out[0] = &subs[pairs[best][0]];
        order_out[1] = &subs[pairs[best][1]];
        n_out = 2;
        rec->n_cand = 4;
        for (unsigned c = 0; c < 4; c++) rec->cand[c] = subs[c].rec;
    } else {
        for (unsigned c = 0; c < ch; c++) { /* encoder.zig:456-475 */
            for (uint32_t i = 0; i < n; i++) S[c][i] = planes[c][i];
            unsigned w = calc_waste(S[c], n, bd);
            choose_subframe(&subs[c], S[c], n, R[c], cfg, bd, w, 0);
            order_out[c] = &subs[c];
            rec->cand[c] = subs[c].rec;
        }
        n_out = ch;
        rec->n_cand = (uint8_t)ch;
        channel_code = ch - 1;
    }

    bw_t w = {0, words, cap_words, 0, 64, 0};
    write_header(&w, frame_number, bd, channel_code, n, cfg->sample_rate);
    for (unsigned i = 0; i < n_out; i++) {
        write_subframe(&w, order_out[i], n);
        rec->written[i] = order_out[i]->rec;
    }
    /* writeCrc16 -> flushAllNoBitEndReset (frame_writer.zig:111-125,144-148) */
    size_t byte_count = w.end * 8;
    if (w.remain != 64) {
        bw_store(&w, w.accu << w.remain);
        byte_count += 8 - w.remain / 8;
    }
    long result = -2;
    if (!w.overflow && byte_count + 2 <= cap) {
        for (size_t i = 0; i < (byte_count + 7) / 8; i++) {
            uint8_t tmp[8];
            be64(tmp, words[i]);
            size_t take = byte_count - i * 8 < 8 ? byte_count - i * 8 : 8;
            memcpy(out + i * 8, tmp, take);
        }
        uint16_t crc = oracle_crc16(0, out, byte_count);
        out[byte_count] = (uint8_t)(crc >> 8);
        out[byte_count + 1] = (uint8_t)crc;
        result = (long)(byte_count + 2);
    }
    rec->channel_code = (uint8_t)channel_code;
    rec->n_sub = (uint8_t)n_out;
    rec->frame_bytes = result > 0 ? (uint32_t)result : 0;
    free(words);
    for (unsigned c = 0; c < 8; c++) { free(S[c]); free(R[c]); }
    return result;
}

/* ===================================================================== */
/* PCM unpack (wav_reader.zig:44-91,172-249)                               */
/* ===================================================================== */
void oracle_unpack_pcm(const uint8_t *bytes, uint32_t B, uint32_t channels, uint32_t bit_depth, uint32_t n,
                       int32_t *const *planes) {
    uint32_t start = 4 - B;
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t c = 0; c < channels; c++) {
            uint32_t v = 0;
            for (uint32_t b = start; b < 4; b++) v |= (uint32_t)bytes[(i * channels + c) * B + (b - start)] << (8 * b);
            int32_t s = (int32_t)v;
            if (bit_depth != 32) s >>= (32 - bit_depth); /* sign extend (wav_reader.zig:81-88) */
            planes[c][i] = s;
        }
}

/* ===================================================================== */
/* Stream / file drivers (wav2flac.zig:10-97, metadata.zig, encoder.zig)    */
/* ===================================================================== */
void oracle_streaminfo_init(oracle_streaminfo *si) {
    memset(si, 0, sizeof(*si));
    si->min_frame_size = 0xFFFFFF;
    si->max_frame_size = 0;
}

void oracle_streaminfo_update(oracle_streaminfo *si, uint32_t sz) {
    if (sz > si->max_frame_size) si->max_frame_size = sz; /* else-if quirk (metadata.zig:35-40) */
    else if (sz < si->min_frame_size) si->min_frame_size = sz;
}

void oracle_streaminfo_bytes(const oracle_streaminfo *si, uint8_t o[34]) {
    o[0] = (uint8_t)(si->min_block_size >> 8); o[1] = (uint8_t)si->min_block_size;
    o[2] = (uint8_t)(si->max_block_size >> 8); o[3] = (uint8_t)si->max_block_size;
    o[4] = (uint8_t)(si->min_frame_size >> 16); o[5] = (uint8_t)(si->min_frame_size >> 8); o[6] = (uint8_t)si->min_frame_size;
    o[7] = (uint8_t)(si->max_frame_size >> 16); o[8] = (uint8_t)(si->max_frame_size >> 8); o[9] = (uint8_t)si->max_frame_size;
    uint32_t sr = si->sample_rate << 4;
    o[10] = (uint8_t)(sr >> 16); o[11] = (uint8_t)(sr >> 8);
    o[12] = (uint8_t)sr | (uint8_t)((si->channels - 1) << 1) | (uint8_t)((si->bit_depth - 1) >> 4);
    uint64_t ts = si->interchannel_samples << 24;
    uint8_t t[8];
    be64(t, ts);
    t[0] |= (uint8_t)((si->bit_depth - 1) << 4);
    memcpy(o + 13, t, 5);
    memcpy(o + 18, si->md5, 16);
}

long oracle_encode_stream(const oracle_config *cfg, const uint8_t *pcm, uint32_t B, uint64_t n_samples,
                          uint64_t first_frame, uint8_t *out, size_t cap, uint32_t *frame_bytes,
                          uint8_t md5_out[16]) {
    uint32_t ch = cfg->channels, bs = cfg->block_size;
    int32_t *planes[8];
    for (unsigned c = 0; c < 8; c++) planes[c] = (int32_t *)calloc(bs, sizeof(int32_t));
    oracle_md5_ctx md5;
    oracle_md5_init(&md5);
    size_t pos = 0;
    uint64_t f = 0;
    long rc = 0;
    oracle_frame_record rec;
    for (uint64_t done = 0; done < n_samples; f++) {
        uint32_t n = (uint32_t)((n_samples - done) < bs ? (n_samples - done) : bs);
        const uint8_t *src = pcm + done * ch * B;
        oracle_md5_update(&md5, src, (size_t)n * ch * B);
        oracle_unpack_pcm(src, B, ch, cfg->bits_per_sample, n, planes);
        long fb = oracle_encode_frame(cfg, (const int32_t *const *)planes, n, first_frame + f, out + pos,
                                      cap - pos, &rec);
        if (fb < 0) { rc = fb; break; }
        if (frame_bytes) frame_bytes[f] = (uint32_t)fb;
        pos += (size_t)fb;
        done += n;
    }
    if (md5_out) oracle_md5_final(&md5, md5_out);
    for (unsigned c = 0; c < 8; c++) free(planes[c]);
    return rc < 0 ? rc : (long)pos;
}

long oracle_encode_file(const oracle_config *cfg, const uint8_t *pcm, uint32_t B, uint64_t n_samples,
                        uint8_t *out, size_t cap) {
    static const char vendor[] = "toastori FLAC 0.0.0"; /* encoder.zig:212 */
    size_t vlen = sizeof(vendor) - 1;
    size_t hdr = 42 + 4 + 4 + vlen + 4; /* skipHeader (42 B) + VORBIS_COMMENT */
    if (cap < hdr) return -2;
    uint64_t nframes = (n_samples + cfg->block_size - 1) / cfg->block_size;
    uint32_t *fb = (uint32_t *)calloc(nframes ? nframes : 1, sizeof(uint32_t));
    oracle_streaminfo si;
    oracle_streaminfo_init(&si);
    long body = oracle_encode_stream(cfg, pcm, B, n_samples, 0, out + hdr, cap - hdr, fb, si.md5);
    if (body < 0) { free(fb); return body; }
    for (uint64_t f = 0; f < nframes; f++) oracle_streaminfo_update(&si, fb[f]);
    free(fb);
    si.interchannel_samples = n_samples;
    si.sample_rate = cfg->sample_rate;
    si.channels = cfg->channels;
    si.bit_depth = cfg->bits_per_sample;
    si.min_block_size = si.max_block_size = cfg->block_size; /* wav_reader.zig:106-107 */
    uint8_t *o = out;
    memcpy(o, "fLaC", 4);
    o[4] = 0x00; /* BlockHeader{StreamInfo, last=false}: packed u8, type in low 7 bits */
    o[5] = 0; o[6] = 0; o[7] = 34;
    oracle_streaminfo_bytes(&si, o + 8);
    o += 42;
    o[0] = 0x80 | 4; /* VorbisComment, last=true (encoder.zig:211-226) */
    uint32_t blen = (uint32_t)(vlen + 8);
    o[1] = (uint8_t)(blen >> 16); o[2] = (uint8_t)(blen >> 8); o[3] = (uint8_t)blen;
    o[4] = (uint8_t)vlen; o[5] = (uint8_t)(vlen >> 8); o[6] = (uint8_t)(vlen >> 16); o[7] = (uint8_t)(vlen >> 24);
    memcpy(o + 8, vendor, vlen);
    memset(o + 8 + vlen, 0, 4);
    return (long)(hdr + (size_t)body);
}
