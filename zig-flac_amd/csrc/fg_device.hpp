// fg_device.hpp -- device helpers and the frame-encode kernel template (gfx950).
//
// One workgroup encodes one frame at a time (persistent loop over frames);
// one 64-lane wave owns one candidate subframe (stereo: L, R, M, S; otherwise
// one wave per channel) and each lane owns 64 consecutive samples held in
// VGPRs.  The kernel restates toastori/zig-flac's Encoder.writeFrame
// (src/lib/encoder.zig:234-284): mid/side (encoder.zig:329-350), wasted bits
// (:556-570), subframe choice (:482-554), fixed-order analysis and residuals
// (fixed.zig:30-201), Rice partition/parameter search (rice.zig:87-107,
// 248-405), bit packing (frame_writer.zig:40-372) and CRC-8/CRC-16
// (frame_writer.zig:128-148, crc16.zig).  No MFMA: there is no dense
// contraction on this path.  Cross-lane work uses DPP (row = 16 lanes) and
// v_readlane, never LDS permutes.  Instantiated per sample width in
// fg_enc_b{1,2,3,4}.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "fg_common.hpp"
#include "fg_layout.hpp"

namespace fg {

// compile-time value tag for uniform dispatch (one branch around a loop, not one per element)
template <uint32_t V>
using ic = std::integral_constant<uint32_t, V>;
// type tag (C++17 has no std::type_identity)
template <typename T>
struct tyt {
    using type = T;
};

// ------------------------------------------------------------------------
// wave64 helpers
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
// A value the optimiser cannot see through: values derived from it are recomputed
// where used instead of being hoisted out of the persistent loop and held in VGPRs.
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

// v_sad_u32: |a - b| (unsigned) + acc
__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t acc) {
    uint32_t d;
    asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(acc));
    return d;
}

// a + b that the optimiser cannot reassociate: a long `acc += x_j` chain over an
// unrolled loop is otherwise rebuilt as an add tree that keeps every x_j live.
__device__ __forceinline__ uint32_t add_chain(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}

enum : int {
    DPP_XOR1 = 0xB1,     // quad_perm [1,0,3,2]
    DPP_XOR2 = 0x4E,     // quad_perm [2,3,0,1]
    DPP_SHR1 = 0x111,    // row_shr:1
    DPP_SHR2 = 0x112,
    DPP_SHR4 = 0x114,
    DPP_SHR8 = 0x118,
    DPP_WSHR1 = 0x138,   // wave_shr:1
    DPP_MIRROR = 0x140,  // row_mirror
    DPP_HMIRROR = 0x141, // row_half_mirror
    DPP_BCAST15 = 0x142, // row_bcast:15
    DPP_BCAST31 = 0x143, // row_bcast:31
};

// lanes whose DPP source is invalid (or whose row is masked off) read 0
template <int CTRL, int RM = 0xF, int BM = 0xF, bool BC = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, BM, BC);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    return (uint64_t)dpp<CTRL>((uint32_t)v) | ((uint64_t)dpp<CTRL>((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int lane) {
    return (uint64_t)rdl((uint32_t)v, lane) | ((uint64_t)rdl((uint32_t)(v >> 32), lane) << 32);
}

// Row (16-lane) reductions: after the 4 steps every lane holds its row's result.
// The intermediate steps are the lane-group results for groups of 2, 4, 8 lanes.
template <typename T>
__device__ __forceinline__ T dppT(T v, int which);
#define FG_ROW_REDUCE(NAME, T, OP, DPPF)                       \
    __device__ __forceinline__ T NAME(T v) {                   \
        v = OP(v, DPPF<DPP_XOR1>(v));                          \
        v = OP(v, DPPF<DPP_XOR2>(v));                          \
        v = OP(v, DPPF<DPP_HMIRROR>(v));                       \
        v = OP(v, DPPF<DPP_MIRROR>(v));                        \
        return v;                                              \
    }
#define FG_ADD(a, b) ((a) + (b))
#define FG_OR(a, b) ((a) | (b))
#define FG_XOR(a, b) ((a) ^ (b))
// (a function, not a ternary: `b` is a DPP read, and a ternary evaluating it twice had the compiler
// redo the read under the compare's exec mask, where a source lane that is switched off reads 0 --
// the row maximum survived only in the lane that held it, and wave_max32 read lanes 0/16/32/48)
// (#ifndef: tests/hip/wave_ops.hip builds the pre-fix ternary on purpose, to show its test catches it)
#ifndef FG_MAX
#define FG_MAX(a, b) max((a), (b))
#endif
// LKEEP for 24-bit LPC frames (c3): the fast pass's residuals kept for the exact pass (A/B switch)
#ifndef FG_LKEEP24
#define FG_LKEEP24 1
#endif
FG_ROW_REDUCE(row_sum32, uint32_t, FG_ADD, dpp)
FG_ROW_REDUCE(row_sum64, uint64_t, FG_ADD, dpp64)
FG_ROW_REDUCE(row_or32, uint32_t, FG_OR, dpp)
FG_ROW_REDUCE(row_or64, uint64_t, FG_OR, dpp64)
FG_ROW_REDUCE(row_xor32, uint32_t, FG_XOR, dpp)
FG_ROW_REDUCE(row_max32, uint32_t, FG_MAX, dpp)

// wave-uniform results (SGPR) from the four row results
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
    v = row_sum32(v);
    return rdl(v, 0) + rdl(v, 16) + rdl(v, 32) + rdl(v, 48);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    v = row_sum64(v);
    return rdl64(v, 0) + rdl64(v, 16) + rdl64(v, 32) + rdl64(v, 48);
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
    v = row_or32(v);
    return rdl(v, 0) | rdl(v, 16) | rdl(v, 32) | rdl(v, 48);
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    v = row_or64(v);
    return rdl64(v, 0) | rdl64(v, 16) | rdl64(v, 32) | rdl64(v, 48);
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t v) {
    v = row_max32(v);
    return max(max(rdl(v, 0), rdl(v, 16)), max(rdl(v, 32), rdl(v, 48)));
}
__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {
    v = row_xor32(v);
    return rdl(v, 0) ^ rdl(v, 16) ^ rdl(v, 32) ^ rdl(v, 48);
}
// inclusive prefix sum over the wave (Hillis-Steele in rows, then row carries)
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    x += dpp<DPP_SHR1>(x);
    x += dpp<DPP_SHR2>(x);
    x += dpp<DPP_SHR4>(x);
    x += dpp<DPP_SHR8>(x);
    x += dpp<DPP_BCAST15, 0xA, 0xF, false>(x);
    x += dpp<DPP_BCAST31, 0xC, 0xF, false>(x);
    return x;
}
// lane l gets lane l-1's value, lane 0 gets 0
__device__ __forceinline__ uint32_t shr1_32(uint32_t v) { return dpp<DPP_WSHR1>(v); }
__device__ __forceinline__ int32_t shr1(int32_t v) { return (int32_t)shr1_32((uint32_t)v); }
__device__ __forceinline__ int64_t shr1(int64_t v) { return (int64_t)dpp64<DPP_WSHR1>((uint64_t)v); }

__device__ __forceinline__ uint32_t bitlen32(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }
__device__ __forceinline__ uint32_t bitlen64(uint64_t x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }
__device__ __forceinline__ uint32_t zigzag32(int32_t r) { return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31); }

// ------------------------------------------------------------------------
// Rice partition decision (rice.zig:343-405) in closed form.
// f(0) = len + 2S; f(p) = (1+p)*len + (S >> (p-1)) - floor(len/2), p >= 1.
// f is convex in p, so the lowest argmin over 0..maxp-1 -- the
// parameter the reference's strict "<" scan keeps -- is the first p whose
// forward difference is >= 0:  p = 0 if S <= ceil(len/2), else p = m + 1 for
// the smallest m with (S >> m) <= 2*len, clamped to maxp - 1.  The escape
// code (5 + width*len, invalid above 31 bits) is the initial candidate and
// wins ties (strict "<" on the rice side).  Returns param (0x80|width = escape).
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rice_choose(uint64_t S, uint32_t len, uint32_t width, uint32_t maxp,
                                                uint32_t *cost) {
    uint32_t p;
    if (S <= (uint64_t)((len + 1u) >> 1)) {
        p = 0;
    } else {
        const uint64_t two = 2ull * len;
        uint32_t m = 0;
        if (S > two) {
            m = bitlen64(S) - bitlen64(two);
            if ((S >> m) > two) m++;
        }
        p = m + 1u;
    }
    if (p > maxp - 1u) p = maxp - 1u;
    const uint64_t f = (p == 0) ? (uint64_t)len + (S << 1)
                                : (uint64_t)(1u + p) * len + ((S >> (p - 1u)) - (uint64_t)(len >> 1));
    const uint64_t esc = (width <= 31u) ? 5ull + (uint64_t)width * len : ~0ull;
    if (f < esc) {
        *cost = (uint32_t)f;
        return p;
    }
    *cost = (uint32_t)esc;
    return 0x80u | width;
}

// The same decision for a partition sum known to fit 32 bits (16-bit input, partitions of
// <= 2048 samples: |e| <= 2^20).  Every intermediate then fits 32 bits: f(p) uses
// S >> (p-1) <= 2*len unless p was clamped to maxp-1 >= 13, where S >> 13 < 2^19.
__device__ __forceinline__ uint32_t rice_choose(uint32_t S, uint32_t len, uint32_t width, uint32_t maxp,
                                                uint32_t *cost) {
    uint32_t p;
    if (S <= ((len + 1u) >> 1)) {
        p = 0;
    } else {
        const uint32_t two = 2u * len;
        uint32_t m = 0;
        if (S > two) {
            m = bitlen32(S) - bitlen32(two);
            if ((S >> m) > two) m++;
        }
        p = m + 1u;
    }
    if (p > maxp - 1u) p = maxp - 1u;
    const uint32_t f = (p == 0) ? len + (S << 1) : (1u + p) * len + ((S >> (p - 1u)) - (len >> 1));
    const uint32_t esc = (width <= 31u) ? 5u + width * len : ~0u;
    if (f < esc) {
        *cost = f;
        return p;
    }
    *cost = esc;
    return 0x80u | width;
}

// CRC-16/UMTS (crc16.zig: poly 0x8005, init 0) without tables.  P = z^16 + z^15 + z^2 + 1 = (z + 1)(z^15 + z + 1), so a residue
// mod P is the pair (residue mod Q = z^15 + z + 1, residue mod z + 1 = the parity of the
// message bits), recombined by CRT: r = A ^ (parity(A) != p ? Q : 0) (Q has three terms, so
// adding it flips the parity and keeps A mod Q).  Mod Q, z^15 = z + 1 folds 14 bits per
// shift/XOR step, so the per-lane CRC chain is VALU only -- no table gathers, whose random
// indices cost 2-3 LDS bank-conflict cycles each.  Frame words are big-endian (first byte in bits
// 31..24), so a word is the next 32 coefficients of the message polynomial.
__device__ __forceinline__ uint32_t q_fold(uint32_t t) {  // t < 2^32 -> same residue, < 2^18
    const uint32_t h = t >> 15;
    return (t & 0x7FFFu) ^ h ^ (h << 1);
}
// s * z^32 + W mod Q (z^32 = z^4 + z^2 mod Q); s < 2^18 in and out, not fully reduced
__device__ __forceinline__ uint32_t q_word(uint32_t s, uint32_t W) { return q_fold(W ^ (s << 4) ^ (s << 2)); }
// a * e mod Q, a and e < 2^15 (fully reduced): 15 terms accumulated in one register (once per
// frame per lane: few live registers matter more than the chain), one fold
__device__ __forceinline__ uint32_t q_mul(uint32_t a, uint32_t e) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 15; i++) r ^= (e << i) & (uint32_t)(-(int32_t)((a >> i) & 1u));
    return q_fold(r);
}
// (residue mod Q in bits 0..14, message parity in bit 16) -> CRC-16 register value
__device__ __forceinline__ uint32_t crc_from_q(uint32_t qp) {
    const uint32_t A = qp & 0x7FFFu;
    return A ^ (((__builtin_popcount(A) ^ (qp >> 16)) & 1u) ? 0x8003u : 0u);
}
// one lane's share of a frame CRC: words [va, va + n) of img (negative indices read as zero: the
// front padding of an init-0 CRC), times e = z^(16 + 32 * words after them) mod Q; parity in bit 16.
__device__ __forceinline__ uint32_t crc_lane_q(const uint32_t *img, int32_t va, uint32_t n, uint32_t e) {
    uint32_t s = 0, px = 0;
    // the padding words before the image leave an init-0 chain at 0: start past them instead of
    // testing every index (the test put each load under its own exec mask)
    for (uint32_t i = va < 0 ? (uint32_t)(-va) : 0u; i < n; i++) {
        const uint32_t w = img[va + (int32_t)i];
        s = q_word(s, w);
        px ^= w;
    }
    return q_mul(q_fold(s), e) | ((__builtin_popcount(px) & 1u) << 16);
}
// crc16.zig's byte step without a table: T[t] = t * z^16 mod P = (t << 1) ^ (t << 2) ^ (parity(t) ? Q : 0)
__device__ __forceinline__ uint32_t crc_byte_v(uint32_t crc, uint32_t b) {
    const uint32_t t = ((crc >> 8) ^ b) & 255u;
    return ((crc << 8) ^ (t << 1) ^ (t << 2) ^ ((__builtin_popcount(t) & 1u) ? 0x8003u : 0u)) & 0xFFFFu;
}
// a * b mod P for a, b < 2^16 without tables: the carry-less product mod Q plus its parity
__device__ __forceinline__ uint32_t crc_mulmod_v(uint32_t a, uint32_t b) {
    uint32_t t[16];
#pragma unroll
    for (int i = 0; i < 16; i++) t[i] = (b << i) & (uint32_t)(-(int32_t)((a >> i) & 1u));
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; i++) t[i] ^= t[i + w];
    return crc_from_q(q_fold(q_fold(t[0])) | ((__builtin_popcount(t[0]) & 1u) << 16));
}

// OR two words into LDS at byte address addr (4-aligned) and addr + 4.  Inline asm: the
// address is an absolute LDS address, so no base add per code; the ORs are ordered before
// any read of the image by the s_waitcnt lgkmcnt(0) of the next barrier.
__device__ __forceinline__ void lds_or2(uint32_t addr, uint32_t hi, uint32_t lo) {
    asm volatile("ds_or_b32 %0, %1\n\tds_or_b32 %0, %2 offset:4" ::"v"(addr), "v"(hi), "v"(lo) : "memory");
}

// Frame image (big-endian words, bit 0 of the frame = bit 31 of word 0) -> out[D, D + fbytes),
// realigned to the byte offset D: 16 bytes per thread and store, edge units byte-masked.
// lo > 0: the first lo bytes are left unwritten (out[D + lo, D + fbytes) only).
__device__ __forceinline__ void store_frame16(const uint32_t *img, uint8_t *out, uint64_t D, uint32_t fbytes,
                                              uint32_t tid, uint32_t NT, uint32_t lo = 0) {
    const uint64_t E = D + fbytes;
    const uint32_t sa = (uint32_t)(D & 3u);
    const uint64_t qD = D >> 2;
    const uint64_t DL = D + lo;
    // the unit's image words m0 - 1 .. m0 + 3 lie in the two 16-B-aligned blocks at m0 + r - 4 and
    // m0 + r (r = qD & 3, uniform): two conflict-free ds_read_b128 per unit instead of five
    // ds_read_b32 at a 4-word lane stride (4-way bank conflicts)
    const uint32_t r = (uint32_t)(qD & 3u);
    for (uint64_t u = (DL >> 4) + tid; u < ((E + 15u) >> 4); u += NT) {
        const int32_t m0 = (int32_t)(4u * u - qD);  // image word of the unit's first word (>= -3)
        const int32_t a1 = m0 + (int32_t)r;           // >= 0, a multiple of 4
        const uint4 q1 = *(const uint4 *)(img + a1);
        const uint4 q0 = a1 >= 4 ? *(const uint4 *)(img + a1 - 4) : make_uint4(0, 0, 0, 0);
        const uint32_t w8[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        uint32_t wv[5];  // image words m0 - 1 .. m0 + 3 = w8[3 - r .. 7 - r]
#pragma unroll
        for (int c = 0; c < 5; c++)
            wv[c] = r == 0 ? w8[3 + c] : r == 1 ? w8[2 + c] : r == 2 ? w8[1 + c] : w8[c];
        uint32_t v[4];
        uint32_t prev = m0 >= 1 ? wv[0] : 0u;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t lo = m0 + c >= 0 ? wv[c + 1] : 0u;
            v[c] = __builtin_bswap32(sa ? __builtin_amdgcn_alignbyte(prev, lo, sa) : lo);
            prev = lo;
        }
        const uint64_t b0 = 16u * u;
        if (b0 >= DL && b0 + 16u <= E) {
            *(uint4 *)(out + b0) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) {
                    const uint64_t bb = b0 + 4u * c + b;
                    if (bb >= DL && bb < E) out[bb] = (uint8_t)(v[c] >> (8 * b));
                }
        }
    }
}

// OR `len` (<= 33) bits of v at bit position pos of the big-endian word image.
__device__ __forceinline__ void put_bits(uint32_t *img, uint32_t pos, uint64_t v, uint32_t len) {
    if (len == 0) return;
    const uint32_t wi = pos >> 5, o = pos & 31u;
    const uint64_t t = v << (64u - o - len);
    atomicOr(&img[wi], (uint32_t)(t >> 32));
    if (o + len > 32u) atomicOr(&img[wi + 1], (uint32_t)t);
}

// Branch-free variant: always two ORs (the second may OR 0); len == 0 writes nothing.
__device__ __forceinline__ void put_or2(uint32_t *img, uint32_t pos, uint64_t v, uint32_t len) {
    const uint32_t wi = pos >> 5, o = pos & 31u;
    const uint64_t t = len ? (v << (64u - o - len)) : 0ull;
    atomicOr(&img[wi], (uint32_t)(t >> 32));
    atomicOr(&img[wi + 1], (uint32_t)t);
}

// Sequential writer for the few per-subframe header fields: every field ORed into
// the image at its bit position.
struct AtomicWriter {
    uint32_t *img;
    uint32_t pos;
    __device__ __forceinline__ void init(uint32_t *im, uint32_t bitpos) {
        img = im;
        pos = bitpos;
    }
    __device__ __forceinline__ void put(uint64_t v, uint32_t len) {
        put_bits(img, pos, v, len);
        pos += len;
    }
    __device__ __forceinline__ void zeros(uint32_t q) { pos += q; }
    __device__ __forceinline__ void finish() {}
};

// ------------------------------------------------------------------------
// Frame header (frame_writer.zig:151-265) on one lane, emulating the
// reference's 64-bit accumulator exactly (writeBits ORs its value unmasked;
// only the uncommon-sample-rate field can overflow, frame_writer.zig:260).
// ------------------------------------------------------------------------
struct HdrWriter {
    uint64_t accu = 0;
    uint64_t w0 = 0;
    uint32_t remain = 64;
    uint32_t end = 0;
    __device__ void bits(uint32_t n, uint64_t v) {
        if (n == 0) return;
        if (n <= remain) {
            accu = (n == 64) ? 0 : (accu << n);
            accu |= v;
            remain -= n;
        } else {
            const uint32_t sh = n - remain;
            accu = (remain == 64) ? 0 : (accu << remain);
            accu |= v >> sh;
            w0 = accu;  // end is at most 1 inside a header
            end++;
            accu = v;
            remain = 64 - sh;
        }
    }
};

__device__ __forceinline__ uint32_t crc8_byte(uint32_t c, uint32_t b) {
    c ^= b;
#pragma unroll
    for (int i = 0; i < 8; i++) c = (c & 0x80u) ? ((c << 1) ^ 0x07u) & 0xFFu : (c << 1) & 0xFFu;
    return c;
}

// Writes the header (with its CRC-8) into the zeroed image; returns its bytes.
__device__ __noinline__ uint32_t write_frame_header(uint32_t *img, uint64_t frame_number, uint32_t bits,
                                                    uint32_t channel_code, uint32_t block_size,
                                                    uint32_t sample_rate) {
    HdrWriter h;
    h.bits(16, 0xFFF8);
    uint32_t unc_bs = 0;
    const uint32_t ctz = (uint32_t)__builtin_ctz(block_size);
    if ((block_size & (block_size - 1u)) == 0 && ctz <= 15 && ctz >= 8) {
        h.bits(4, ctz);
    } else if (block_size == 192) {
        h.bits(4, 1);
    } else if ((block_size >> ctz) == 144 && ctz <= 5 && ctz >= 2) {
        h.bits(4, ctz);  // unreachable (odd part of 144*2^v is 9), kept for fidelity
    } else if (block_size < 0x100) {
        h.bits(4, 6);
        unc_bs = 8;
    } else {
        h.bits(4, 7);
        unc_bs = 16;
    }
    uint32_t unc_sr = 0, rc;
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
    h.bits(4, rc);
    h.bits(4, channel_code);
    h.bits(4, bits == 8 ? 2u : bits == 16 ? 8u : bits == 24 ? 12u : 14u);
    if (frame_number <= 0x7F) {
        h.bits(8, frame_number);
    } else {  // UTF-8 coded frame number (frame_writer.zig:235-251)
        uint64_t buf = 0, num = frame_number, fbm = 0x3F;
        uint32_t i = 0;
        while (num > fbm) {
            buf |= (0x80ull + (num & 0x3F)) << (8 * i);
            i++;
            num >>= 6;
            fbm >>= 1;
        }
        buf |= ((0xFEull << (6 - i)) | num) << (8 * i);
        const uint32_t nb = 8 * (i + 1);
        h.bits(nb, buf & (~0ull >> (64 - nb)));
    }
    if (unc_bs) h.bits(unc_bs, block_size - 1u);
    if (unc_sr == 4) h.bits(8, block_size);  // the reference writes the block size here (unmasked)
    else if (unc_sr) h.bits(16, block_size / unc_sr);
    // writeCrc8 (frame_writer.zig:128-141): stored word w0 (if any), then the accumulator
    const uint32_t byte_end = 8u - h.remain / 8u;
    const uint64_t a_al = (h.remain == 64) ? h.accu : (h.accu << h.remain);
    const uint32_t nb = (h.end == 1 ? 8u : 0u) + byte_end;
    uint32_t c = 0;
    for (uint32_t q = 0; q < nb; q++) {
        const uint64_t src = (h.end == 1 && q < 8) ? h.w0 : a_al;
        const uint32_t qq = (h.end == 1 && q >= 8) ? q - 8 : q;
        const uint32_t byte = (uint32_t)(src >> (56 - 8 * qq)) & 255u;
        c = crc8_byte(c, byte);
        atomicOr(&img[q >> 2], byte << (24 - 8 * (q & 3)));
    }
    atomicOr(&img[nb >> 2], c << (24 - 8 * (nb & 3)));
    return nb + 1;
}

// ------------------------------------------------------------------------
// Residual helpers
// ------------------------------------------------------------------------
template <int CLS>
struct Cls {
    using S = typename std::conditional<CLS == 32, int64_t, int32_t>::type;
    using Sum = typename std::conditional<CLS == 16, uint32_t, uint64_t>::type;
};

template <int B>
__device__ __forceinline__ int32_t ld_sample(const uint8_t *p) {
    if constexpr (B == 1) return (int32_t)(*(const int8_t *)p);
    else if constexpr (B == 2) return (int32_t)(*(const int16_t *)p);
    else if constexpr (B == 3)
        return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8)) | ((int32_t)(*(const int8_t *)(p + 2)) << 16);
    else return *(const int32_t *)p;
}

struct CandRes {
    uint32_t type, waste, bd, order, porder, method;
    int32_t lsh;  // LPC quantisation shift
    uint64_t est;
    int64_t cval;
    // every field is wave-uniform: pinned to SGPRs (readfirstlane) before the LPC search, whose
    // register peak otherwise spilled the VGPR copies the merges of divergent-looking control flow
    // had made of them (c3: 12 dwords of scratch stores per lane and frame)
    __device__ __forceinline__ void make_uniform() {
        auto u32 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
        auto u64 = [&](uint64_t v) { return (uint64_t)u32((uint32_t)v) | ((uint64_t)u32((uint32_t)(v >> 32)) << 32); };
        type = u32(type); waste = u32(waste); bd = u32(bd); order = u32(order); porder = u32(porder);
        method = u32(method); lsh = (int32_t)u32((uint32_t)lsh); est = u64(est); cval = (int64_t)u64((uint64_t)cval);
    }
};

#ifdef FG_STAMPS
#define STAMP(i)                                           \
    do {                                                   \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        ph_[i] += t_ - tprev_;                             \
        tprev_ = t_;                                       \
    } while (0)
#else
#define STAMP(i) \
    do {         \
    } while (0)
#endif

// LDS-DMA (global_load_lds_dword / _dwordx4) issued from inline asm.  Issued through the
// builtin, the compiler's wait-count pass cannot tell the DMA's LDS destination from the LDS
// the kernel reads next (one extern array), so it put an s_waitcnt vmcnt(0) before the first
// LDS access after every DMA: each wave waited for the next frame's PCM right after issuing it,
// and the double-buffered prefetch hid nothing.  Hidden from that pass, the DMA is waited for
// only where the kernels say so (an explicit s_waitcnt vmcnt before the data is read); the
// compiler's own vmcnt waits stay correct, only conservative (in-order completion).  M0 (the
// LDS base of the wave's piece) is saved and restored around the instruction.
#ifndef FG_DMA_ASM
#define FG_DMA_ASM 1
#endif
template <int SZ>
__device__ __forceinline__ void lds_dma(const void *g, void *lds) {
#if FG_DMA_ASM
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)lds);
    uint32_t sv;
    if constexpr (SZ == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(sv) : "s"(m), "v"(g) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(sv) : "s"(m), "v"(g) : "memory");
#else
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)lds, SZ, 0, 0);
#endif
}

// LDS-DMA one full frame into the staging area.  Interleaved 16-bit stereo layout
// (fg_layout.hpp): 16 instructions of 1 KiB, lane i of instruction k filling byte 16i of
// block k from 16-B group i >> 2 of chunk 4k + (i & 3).  Padded layouts: each
// wave-instruction moves <= 64 dwords of one 64-sample chunk (M0 = that chunk's base).
// drh != 0: channel half `half` only -- the staged chunk holds drh of every 2 drh source dwords
// of each interchannel row (cw = the half row's dwords x 64), see k_analyze's split mode.
__device__ __forceinline__ void stage_dma(const uint8_t *pcm, uint64_t off, uint32_t *stg, uint32_t cw, uint32_t cst,
                                          uint32_t wave, uint32_t NW, uint32_t l, bool ilv = false, uint32_t drh = 0,
                                          uint32_t half = 0) {
    const uint32_t *src = (const uint32_t *)(pcm + off);
    if (ilv) {
        for (uint32_t k = wave; k < 16u; k += NW)
            lds_dma<16>(src + (4u * k + (l & 3u)) * 64u + 4u * (l >> 2), stg + 272u * k);
        return;
    }
    if (drh) {
        const float inv = 1.0f / (float)drh;  // x / drh exactly for x < 2^10, drh <= 4
        for (uint32_t ch = wave; ch < 64u; ch += NW) {
            for (uint32_t x0 = 0; x0 < cw; x0 += 64u) {
                const uint32_t x = x0 + l, r = (uint32_t)((float)x * inv), k = x - r * drh;
                if (x < cw)
                    lds_dma<4>(src + ch * 2u * cw + r * 2u * drh + half * drh + k, stg + ch * cst + x0);
            }
        }
        return;
    }
    for (uint32_t ch = wave; ch < 64u; ch += NW) {
        for (uint32_t x0 = 0; x0 < cw; x0 += 64u) {
            if (x0 + l < cw)
                lds_dma<4>(src + ch * cw + x0 + l, stg + ch * cst + x0);
        }
    }
}


// Workgroup barrier for LDS hand-offs only: __syncthreads() would also wait for vmcnt(0),
// i.e. drain the next frame's PCM DMA and this frame's output stores at every barrier.
__device__ __forceinline__ void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Frame-queue tickets (EncodeArgs::work_ctr, one set of kCtrSet u32 per overlapped range):
// [0] analysis full, [1] analysis tail, [2] pack full, [3] pack tail, [8..15] the split
// analysis's per-XCD queues, [16..23] the split pack's.  Each stage zeroes the other stage's tickets at its start (the
// launches of one set are ordered), so no memset precedes a launch.
__device__ __forceinline__ void reset_analysis_tickets(uint32_t *ctr, uint32_t tid) {
    if (blockIdx.x == 0 && tid < 16u && (tid < 2u || tid >= 8u)) ctr[tid] = 0u;
}

// XCD-aware queue of channel-half work items (split analysis, item = 2 frame + half): XCD x
// owns frames [x n / 8, (x + 1) n / 8) and hands out their items in order from its own counter,
// so the two halves of a frame -- which fetch the same cache lines of its interleaved rows --
// go to workgroups of one XCD at about the same time and the second fetch hits that XCD's L2.
// An exhausted queue passes on to the next XCD's.  Placement is read from the hardware
// (HW_REG_XCC_ID) and is used for speed only: every item is handed out exactly once whatever
// the placement.  Returns 0xFFFFFFFF when every queue is empty.
__device__ __forceinline__ uint32_t xcd_ticket(uint32_t *q, uint32_t n_frames) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 7u;
    for (uint32_t i = 0; i < 8u; i++) {
        const uint32_t y = (x + i) & 7u;
        const uint32_t f0 = (uint32_t)(((uint64_t)n_frames * y) >> 3);
        const uint32_t f1 = (uint32_t)(((uint64_t)n_frames * (y + 1u)) >> 3);
        if (f1 == f0) continue;
        const uint32_t t = atomicAdd(&q[y], 1u);
        if (t < 2u * (f1 - f0)) return 2u * f0 + t;
    }
    return 0xFFFFFFFFu;
}

// Stage one frame's interleaved PCM synchronously (tail frames zero-filled).
template <bool FULL>
__device__ __forceinline__ void stage_sync(const uint8_t *pcm, uint64_t off, uint32_t n, uint32_t CB, uint32_t *stg,
                                           uint32_t cw, uint32_t cst, uint32_t wave, uint32_t NW, uint32_t l,
                                           bool ilv = false) {
    const uint32_t in_bytes = n * CB;
    const uint32_t *src = (const uint32_t *)(pcm + off);
    const uint32_t nchunks = FULL ? 64u : (n + 63u) >> 6;
    for (uint32_t ch = wave; ch < nchunks; ch += NW) {
        for (uint32_t x = l; x < cw; x += 64) {
            const uint32_t wd = ch * cw + x;
            uint32_t v = 0;
            if (FULL || 4u * wd + 4u <= in_bytes) {
                v = src[wd];
            } else if (4u * wd < in_bytes) {
                const uint8_t *sb = (const uint8_t *)src + 4u * wd;
                for (uint32_t q = 0; 4u * wd + q < in_bytes; q++) v |= (uint32_t)sb[q] << (8 * q);
            }
            // interleaved 16-bit stereo layout: dword x of chunk ch at 272 (ch >> 2) + 16 (x >> 2) + 4 (ch & 3) + (x & 3)
            if (ilv) stg[272u * (ch >> 2) + 16u * (x >> 2) + 4u * (ch & 3u) + (x & 3u)] = v;
            else stg[ch * cst + x] = v;
        }
    }
}

// Lane l loads samples [64l, 64l+64) of candidate `cand` from the staging area:
// stereo 0 L, 1 R, 2 mid, 3 side (encoder.zig:329-350, from the un-shifted
// L/R), otherwise channel `cand`.  Samples past n read as 0.  The candidate
// switch is hoisted out of the sample loops so each loop is branch-free.
template <int B, int CLS, bool FULL, int NC>
__device__ __forceinline__ void load_candidate(const uint32_t *stg, uint32_t cst, uint32_t l, uint32_t n, bool stereo,
                                               uint32_t cand, uint32_t C, typename Cls<CLS>::S (&s)[64]) {
    using ST = typename Cls<CLS>::S;
    const uint32_t *lw = stg + l * cst;
    const uint32_t kind = stereo ? cand : 0u;  // 0 plain channel, 1 R, 2 mid, 3 side
    const uint32_t chan = stereo ? (cand == 1 ? 1u : 0u) : cand;
    // Groups of 16 samples with a scheduling barrier between them: without it the
    // scheduler hoists every LDS read ahead of the unpacking and holds the raw words
    // and the samples live together (2x the registers).
    auto fill = [&](auto getL, auto getR) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            if (kind <= 1) {
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    int64_t x = getL(j, chan);
                    if (!FULL && l * 64u + j >= n) x = 0;
                    s[j] = (ST)x;
                }
            } else if (kind == 2) {  // mid (encoder.zig:337,347)
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    int64_t x = (getL(j, 0u) + getR(j)) >> 1;
                    if (!FULL && l * 64u + j >= n) x = 0;
                    s[j] = (ST)x;
                }
            } else {  // side; 33-bit at 32 bps (samples64, encoder.zig:338)
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    int64_t x = getL(j, 0u) - getR(j);
                    if (!FULL && l * 64u + j >= n) x = 0;
                    s[j] = (ST)x;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    if constexpr (NC == 2 && B == 4) {
        // (L,R) dword pair per sample (8-B pad: conflict-free ds_read_b64)
        const uint2 *p2 = (const uint2 *)lw;
        fill([&](int j, uint32_t c) -> int64_t { return (int32_t)(c ? p2[j].y : p2[j].x); },
             [&](int j) -> int64_t { return (int32_t)p2[j].y; });
    } else if constexpr (NC == 2 && B == 2) {
        // (L,R) packed in one dword per sample, read as explicit ds_read_b128 from the
        // interleaved layout (group t of this lane's chunk at 16 t dwords past its base)
        const uint4 *q4 = (const uint4 *)(stg + 272u * (l >> 2) + 4u * (l & 3u));
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint32_t raw[16];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint4 v = q4[4 * (4 * g + t)];
                raw[4 * t] = v.x; raw[4 * t + 1] = v.y; raw[4 * t + 2] = v.z; raw[4 * t + 3] = v.w;
            }
            auto put = [&](auto f) {
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    int32_t x = f((int32_t)(raw[jj] << 16) >> 16, (int32_t)raw[jj] >> 16);
                    if (!FULL && l * 64u + j >= n) x = 0;
                    s[j] = (ST)x;
                }
            };
            if (kind == 0 && chan == 0) put([](int32_t L, int32_t) { return L; });
            else if (kind <= 1) put([](int32_t, int32_t R) { return R; });
            else if (kind == 2) {
                // mid: L + R from the two sign-extended halves in one SDWA add, then >> 1 (the
                // compiler's packed-16-bit form took ~13 issue slots per sample pair, this 3 per sample)
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    uint32_t sum;
                    asm("v_add_u32_sdwa %0, sext(%1), sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1"
                        : "=v"(sum) : "v"(raw[jj]));
                    int32_t x = (int32_t)sum >> 1;
                    if (!FULL && l * 64u + j >= n) x = 0;
                    s[j] = (ST)x;
                }
            } else put([](int32_t L, int32_t R) { return L - R; });
            __builtin_amdgcn_sched_barrier(0);
        }
    } else if constexpr (B == 3) {
        // 24-bit: the two dwords around the sample (a ds_read2_b32) and v_alignbyte, instead of
        // three byte loads per sample
        const uint32_t CB = C * 3u;
        auto ld24 = [&](uint32_t off) -> int64_t {
            const uint32_t w = off >> 2, o = off & 3u;
            const uint32_t v = __builtin_amdgcn_alignbyte(lw[w + 1u], lw[w], o);
            return (int32_t)(v << 8) >> 8;
        };
        fill([&](int j, uint32_t c) -> int64_t { return ld24((uint32_t)j * CB + 3u * c); },
             [&](int j) -> int64_t { return ld24((uint32_t)j * CB + 3u); });
    } else {
        const uint8_t *base = (const uint8_t *)lw;
        const uint32_t CB = C * B;
        fill([&](int j, uint32_t c) -> int64_t { return ld_sample<B>(base + j * CB + c * B); },
             [&](int j) -> int64_t { return ld_sample<B>(base + j * CB + B); });
    }
}

// Samples of candidate `cand` for the LPC search, as i32 after the waste shift w: the
// build-defined LPC works on i32 samples, so a 32-bit stereo side that still needs 33
// bits after its shift skips LPC.  Returns false on a lane holding such a sample.
template <int B, int CLS, bool FULL, int NC>
__device__ __forceinline__ bool load_lpc_samples(const uint32_t *stg, uint32_t cst, uint32_t l, uint32_t n,
                                                 bool stereo, uint32_t cand, uint32_t C, uint32_t w,
                                                 int32_t (&x)[64]) {
    if constexpr (CLS != 32) {
        load_candidate<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, x);
        if (w != 0) {
#pragma unroll
            for (int j = 0; j < 64; j++) x[j] >>= w;
        }
        return true;
    } else {
        const uint32_t *lw = stg + l * cst;
        const uint32_t kind = stereo ? cand : 0u;
        const uint32_t chan = stereo ? (cand == 1 ? 1u : 0u) : cand;
        bool fits = true;
#pragma unroll
        for (int g = 0; g < 4; g++) {
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                const int j = 16 * g + jj;
                int64_t L, Rr;
                if constexpr (NC == 2) {
                    const uint2 v = ((const uint2 *)lw)[j];
                    L = (int32_t)(chan ? v.y : v.x);
                    Rr = (int32_t)v.y;
                    if (kind >= 2) L = (int32_t)v.x;
                } else {
                    const uint8_t *base = (const uint8_t *)lw;
                    L = ld_sample<4>(base + j * C * 4u + chan * 4u);
                    Rr = 0;
                }
                int64_t v = kind <= 1 ? L : (kind == 2 ? (L + Rr) >> 1 : L - Rr);
                if (!FULL && l * 64u + j >= n) v = 0;
                v >>= w;
                fits &= v == (int64_t)(int32_t)v;
                x[j] = (int32_t)v;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        return fits;
    }
}

// 32-bit input (CLS 32): samples held compactly as their low 32 bits plus one mask bit per
// sample (bit j of hb = bit 32 of sample j, i.e. the sign of the 33-bit side of
// encoder.zig:330-339; for every other candidate the sign of a value that fits i32).  Half
// the registers of an i64 array: the 32-bit kernels held 128 VGPRs of samples and spilled.
// The i64 value is rebuilt only where exact 64-bit arithmetic is needed (bestOrder's wide
// mode, fixed.zig:85-167); residuals truncated to i32 (fixed.zig:69-74) follow from the low
// words alone, since a sample and its low word agree mod 2^32.
__device__ __forceinline__ int64_t wide_value(int32_t lo, uint64_t hb, int j) {
    const uint32_t hi = ((hb >> j) & 1ull) ? 0xFFFFFFFFu : 0u;
    return (int64_t)(((uint64_t)hi << 32) | (uint64_t)(uint32_t)lo);
}
template <int B, bool FULL, int NC>
__device__ __forceinline__ void load_candidate32(const uint32_t *stg, uint32_t cst, uint32_t l, uint32_t n, bool stereo,
                                                 uint32_t cand, uint32_t C, int32_t (&s)[64], uint64_t &hb) {
    const uint32_t *lw = stg + l * cst;
    const uint32_t kind = stereo ? cand : 0u;  // 0 plain channel, 1 R, 2 mid, 3 side
    const uint32_t chan = stereo ? (cand == 1 ? 1u : 0u) : cand;
    hb = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
            const int j = 16 * g + jj;
            int64_t L, Rr;
            if constexpr (NC == 2) {
                const uint2 v = ((const uint2 *)lw)[j];
                L = (int32_t)(chan ? v.y : v.x);
                Rr = (int32_t)v.y;
                if (kind >= 2) L = (int32_t)v.x;
            } else {
                const uint8_t *base = (const uint8_t *)lw;
                L = ld_sample<4>(base + j * C * 4u + chan * 4u);
                Rr = 0;
            }
            int64_t v = kind <= 1 ? L : (kind == 2 ? (L + Rr) >> 1 : L - Rr);
            if (!FULL && l * 64u + j >= n) v = 0;
            s[j] = (int32_t)v;
            hb |= (uint64_t)((v >> 32) & 1) << j;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}
// the waste shift (encoder.zig:556-570) of the compact form: v >> w for 0 < w < bd (<= 33);
// the result fits i32, so its mask bits become the signs
__device__ __forceinline__ void shift32(int32_t (&s)[64], uint64_t &hb, uint32_t w) {
    uint64_t nb = 0;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const uint32_t hi = ((hb >> j) & 1ull) ? 0xFFFFFFFFu : 0u;
        const uint32_t v = w < 32u ? __builtin_amdgcn_alignbit(hi, (uint32_t)s[j], w) : hi;
        s[j] = (int32_t)v;
        nb |= (uint64_t)(v >> 31) << j;
    }
    hb = nb;
}

// Fixed-predictor residual of order K from sample x and history q1..q4
// (fixed.zig:12-18 COEFF_SCALAR stencil): wrapping i32 (narrow, fixed.zig:63-68)
// or exact i64 truncated to i32 (wide, fixed.zig:69-74).
template <int K, typename ST>
__device__ __forceinline__ ST fixed_residual(ST x, ST q1, ST q2, ST q3, ST q4) {
    using UT = typename std::conditional<sizeof(ST) == 4, uint32_t, uint64_t>::type;
    const UT ux = (UT)x, u1 = (UT)q1, u2 = (UT)q2, u3 = (UT)q3, u4 = (UT)q4;
    UT r;
    if constexpr (K == 0) r = ux;
    else if constexpr (K == 1) r = ux - u1;
    else if constexpr (K == 2) r = (ux + u2) - 2u * u1;
    else if constexpr (K == 3) r = (ux - u3) + 3u * (u2 - u1);
    else r = (ux + u4) - 4u * (u1 + u3) + 6u * u2;
    return (ST)(int32_t)(uint32_t)r;
}

// Residuals of a compile-time order K, read-only over s: f(j, warm, r) sees
// every residual (lane 0's first K samples are warm-ups).  Used where the
// residuals are consumed on the fly, so the five instantiations behind a
// uniform switch share no live state but the caller's accumulators.
// The residual is formed by the difference chain e_{q+1}[i] = e_q[i] - e_q[i-1] (K full-rate
// subtractions per sample, carried differences d_q = e_q[i-1]) rather than the K-th stencil
// (x + u4 - 4(u1 + u3) + 6 u2 and the like: two-slot shift-adds and multiplies on gfx950); both
// are the same polynomial, so the low 32 bits -- all fixed.zig:63-74 keeps -- agree.
template <int K, typename ST, typename F>
__device__ __forceinline__ void residuals_k(const ST (&s)[64], ST h1, ST h2, ST h3, ST h4, uint32_t l, F &&f) {
    const uint32_t u1 = (uint32_t)h1, u2 = (uint32_t)h2, u3 = (uint32_t)h3, u4 = (uint32_t)h4;
    // d_q = e_q at the previous sample (the lane's history: the previous lane's last four)
    uint32_t d0 = u1, d1 = u1 - u2, d2 = u1 - 2u * u2 + u3, d3 = u1 - 3u * u2 + 3u * u3 - u4;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const uint32_t e0 = (uint32_t)s[j];
        uint32_t e = e0;
        if constexpr (K >= 1) {
            const uint32_t e1 = e0 - d0;
            d0 = e0;
            e = e1;
            if constexpr (K >= 2) {
                const uint32_t e2 = e1 - d1;
                d1 = e1;
                e = e2;
                if constexpr (K >= 3) {
                    const uint32_t e3 = e2 - d2;
                    d2 = e2;
                    e = e3;
                    if constexpr (K >= 4) {
                        e = e3 - d3;
                        d3 = e3;
                    }
                }
            }
        }
        f(j, (j < K) && (l == 0), (ST)(int32_t)e);
    }
}
#define FG_DISPATCH_K(k, CALL)                        \
    switch (k) {                                      \
        case 0: { constexpr int K = 0; CALL; } break; \
        case 1: { constexpr int K = 1; CALL; } break; \
        case 2: { constexpr int K = 2; CALL; } break; \
        case 3: { constexpr int K = 3; CALL; } break; \
        default: { constexpr int K = 4; CALL; } break; \
    }

// Fixed-predictor residuals in place, s[j] := e_k (lane 0 keeps its k warm-up
// samples; history h1..h4 = the 4 samples before the lane's chunk), for a runtime
// (wave-uniform) order k: the difference chain
// e_{q+1}[i] = e_q[i] - e_q[i-1] for q < 4, then a uniform select.  One code
// path instead of five keeps the register allocation of the callers compact.
// Narrow: wrapping u32 (== the stencil mod 2^32); wide: exact i64 truncated to
// i32 (fixed.zig:69-74).
template <typename ST, typename F>
__device__ __forceinline__ void residuals_generic(ST (&s)[64], ST h1, ST h2, ST h3, ST h4, uint32_t l, uint32_t k,
                                                  F &&f) {
    using UT = typename std::conditional<sizeof(ST) == 4, uint32_t, uint64_t>::type;
    const UT u1 = (UT)h1, u2 = (UT)h2, u3 = (UT)h3, u4 = (UT)h4;
    UT p0 = u1, p1 = u1 - u2, p2 = u1 - 2u * u2 + u3, p3 = u1 - 3u * u2 + 3u * u3 - u4;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const UT e0 = (UT)s[j], e1 = e0 - p0, e2 = e1 - p1, e3 = e2 - p2, e4 = e3 - p3;
        p0 = e0; p1 = e1; p2 = e2; p3 = e3;
        const UT e = k == 0 ? e0 : k == 1 ? e1 : k == 2 ? e2 : k == 3 ? e3 : e4;
        const ST r = (ST)(int32_t)(uint32_t)e;
        const bool warm = (j < 4) && (l == 0) && ((uint32_t)j < k);
        if (!warm) s[j] = r;
        f(j, warm, r);
    }
}

// ------------------------------------------------------------------------
// LPC (build-defined extension: the reference has no LPC, readme.md:27,
// encoder.zig:629-640,694-699).  The contract is stated once in
// oracle/flac_oracle.c ("LPC -- build-defined extension") and followed here
// operation for operation: integer Welch window (i+1)(n-i), windowed samples
// scaled to <= 25 bits, exact i64 autocorrelation, Levinson-Durbin in IEEE
// double in a fixed order (the library is built with -ffp-contract=off),
// 15-bit coefficients with error feedback, residuals in i64.
// ------------------------------------------------------------------------

// R[0..W] of the lane-distributed samples s (lane l owns [64l, 64l+64); zero past n).
template <int W, typename ST>
__device__ __forceinline__ void lpc_autocorr(const ST (&s)[64], uint32_t n, uint32_t l, int64_t (&R)[W + 1]) {
    uint64_t ov = 0;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const int64_t x = (int64_t)s[j];
        ov |= (uint64_t)(x < 0 ? -x : x);
    }
    const uint32_t mb = bitlen64(wave_or64(ov));
    const uint32_t wb = bitlen32(((n + 1u) * (n + 1u)) >> 2);
    const int32_t shv = (int32_t)(mb + wb) - 25;
    const uint32_t sh = shv > 0 ? (uint32_t)shv : 0u;
    auto xw = [&](int j) -> int32_t {
        const uint32_t i = l * 64u + (uint32_t)j;
        const int32_t w = i < n ? (int32_t)((i + 1u) * (n - i)) : 0;
        int64_t p;
        if constexpr (sizeof(ST) == 4) p = (int64_t)(int32_t)s[j] * (int64_t)w;
        else p = (int64_t)s[j] * (int64_t)w;
        return (int32_t)(p >> sh);
    };
    int32_t hx[W];
#pragma unroll
    for (int t = 0; t < W; t++) hx[t] = shr1(xw(63 - t));  // the previous lane's last W
    int64_t acc[W + 1];
#pragma unroll
    for (int g = 0; g <= W; g++) acc[g] = 0;
    int32_t xv[64];
#pragma unroll
    for (int j = 0; j < 64; j++) {
        xv[j] = xw(j);
#pragma unroll
        for (int g = 0; g <= W; g++) {
            const int32_t y = (j - g >= 0) ? xv[(j - g) >= 0 ? (j - g) : 0] : hx[(g - j - 1) >= 0 ? (g - j - 1) : 0];
            acc[g] += (int64_t)xv[j] * (int64_t)y;
        }
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g <= W; g++) R[g] = (int64_t)wave_sum64((uint64_t)acc[g]);
}

// Levinson-Durbin + quantisation of every order 1..Q: tab[(q-1)*13 + t] = coefficient t of
// order q (0 past q), tab[(q-1)*13 + 12] = its shift, or -1 if the order is unusable.  The
// recursion is serial and runs on every lane; lane m keeps the coefficients of order m+1 and
// the LD error after it as they are produced and quantises them itself afterwards (each
// order's error-feedback chain is independent), so the quantisation costs one order's chain,
// not all of them in series.  Returns the selected order (contract step 7: the lowest q with
// the smallest key l2(err_q) * n/2 + q (bps' + 15) among the orders that quantise), 0 if none.
template <int W>
__device__ __forceinline__ uint32_t lpc_coefs(const int64_t (&R)[W + 1], uint32_t Q, int32_t *tab, uint32_t lane,
                                              uint32_t n, uint32_t bps) {
#pragma clang fp contract(off)
    double r[W + 1], a[W], mine[W], myerr = 0.0;
#pragma unroll
    for (int i = 0; i <= W; i++) r[i] = (double)R[i];
#pragma unroll
    for (int t = 0; t < W; t++) mine[t] = 0.0;
    bool have = false;  // this lane's order (lane + 1) was reached
    if (r[0] > 0.0) {
        double err = r[0];
        bool live = true;  // uniform: order m+1 is computed while live (stops at Q or when err <= 0)
#pragma unroll
        for (int m = 0; m < W; m++) {
            live = live && (uint32_t)m < Q;
            if (!live) continue;
            double acc = r[m + 1];
#pragma unroll
            for (int t = 0; t < m; t++) {
                const double p = a[t] * r[m - t];
                acc = acc - p;
            }
            const double k = acc / err;
            // a[t] -= k a[m-1-t] for t < m, in symmetric pairs (t, m-1-t) so that only two new
            // values are live at a time (each element's operations and rounding unchanged)
#pragma unroll
            for (int t = 0; t < m / 2; t++) {
                const double lo = a[t] - k * a[m - 1 - t];
                const double hi = a[m - 1 - t] - k * a[t];
                a[t] = lo;
                a[m - 1 - t] = hi;
            }
            if (m & 1) a[m / 2] = a[m / 2] - k * a[m / 2];
            a[m] = k;
            const bool me = lane == (uint32_t)m;
            have = have || me;
#pragma unroll
            for (int t = 0; t <= m; t++) mine[t] = me ? a[t] : mine[t];
            const double kk = k * k;
            err = err * (1.0 - kk);
            myerr = me ? err : myerr;
            live = err > 0.0;
        }
    }
    // quantise order lane+1 (oracle_lpc_quantize); lanes past W or past the recursion keep -1
    const uint32_t m = lane;
    int32_t shq = -1;
    int32_t qc[W];
#pragma unroll
    for (int t = 0; t < W; t++) qc[t] = 0;
    if (have) {
        double cmax = 0.0;
#pragma unroll
        for (int t = 0; t < W; t++) {
            const double v = mine[t] < 0.0 ? -mine[t] : mine[t];
            cmax = ((uint32_t)t <= m && v > cmax) ? v : cmax;
        }
        if (cmax > 0.0) {
            int e;
            (void)frexp(cmax, &e);
            shq = kLpcPrec - 1 - e;
            if (shq > 15) shq = 15;
            if (shq >= 0) {
                const double scale = (double)(1u << shq);
                const int64_t qmax = (1ll << (kLpcPrec - 1)) - 1, qmin = -(1ll << (kLpcPrec - 1));
                double carry = 0.0;
#pragma unroll
                for (int t = 0; t < W; t++) {
                    if ((uint32_t)t <= m) {
                        double v = mine[t] * scale;
                        v = v + carry;
                        int64_t qi = v >= 0.0 ? (int64_t)floor(v + 0.5) : -(int64_t)floor(-v + 0.5);
                        qi = qi > qmax ? qmax : (qi < qmin ? qmin : qi);
                        carry = v - (double)qi;
                        qc[t] = (int32_t)qi;
                    }
                }
            }
        }
    }
    if (lane < (uint32_t)kLpcMax) {
#pragma unroll
        for (int t = 0; t < kLpcMax; t++) tab[m * 13u + t] = (t < W) ? qc[t < W ? t : 0] : 0;
        tab[m * 13u + 12u] = shq;
    }
    // selection key of order lane + 1 (oracle_lpc_order_key), as an integer with the same order
    double key = -1e300;
    if (myerr > 0.0) {
        int e;
        const double f = frexp(myerr, &e);
        const double l2 = (double)(e - 1) + (2.0 * f - 1.0);
        key = l2 * (0.5 * (double)n) + (double)((lane + 1u) * (bps + (uint32_t)kLpcPrec));
    }
    const int64_t kb = __builtin_bit_cast(int64_t, key);
    const uint64_t ko = (uint64_t)(kb < 0 ? ~kb : (kb | INT64_MIN));  // monotone in key
    const bool ok = have && shq >= 0 && lane < Q;
    uint32_t qsel = 0;
    uint64_t kbest = 0;
#pragma unroll
    for (int t = 0; t < W; t++) {  // ascending order, strict "<": the lowest order wins ties
        const uint32_t okt = (uint32_t)__builtin_amdgcn_readlane((int)ok, t);
        const uint64_t kt = rdl64(ko, t);
        if (okt && (qsel == 0 || kt < kbest)) {
            qsel = (uint32_t)t + 1u;
            kbest = kt;
        }
    }
    return qsel;
}

// Prediction sum_t c[t] * x[j-1-t] over the lane's samples and the previous lane's
// last W samples hs[] (hs[t] = sample 64l-1-t); c[t] = 0 past the order.
template <int W, typename ST>
__device__ __forceinline__ int64_t lpc_pred(const ST (&s)[64], const ST (&hs)[W], const int32_t (&c)[W], int j) {
    int64_t acc = 0;
#pragma unroll
    for (int t = 0; t < W; t++) {
        const int idx = j - 1 - t;
        const ST x = idx >= 0 ? s[idx >= 0 ? idx : 0] : hs[(-idx - 1) >= 0 ? (-idx - 1) : 0];
        if constexpr (sizeof(ST) == 4) acc += (int64_t)c[t] * (int64_t)(int32_t)x;
        else acc += (int64_t)c[t] * (int64_t)x;
    }
    return acc;
}

// LPC residuals read-only over s: f(j, warm, e) with e the exact i64 residual.
template <int W, typename ST, typename F>
__device__ __forceinline__ void residuals_lpc(const ST (&s)[64], const ST (&hs)[W], const int32_t (&c)[W],
                                              uint32_t shift, uint32_t q, uint32_t l, F &&f) {
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const int64_t e = (int64_t)s[j] - (lpc_pred<W, ST>(s, hs, c, j) >> shift);
        const bool warm = (j < W) && (l == 0) && ((uint32_t)j < q);
        f(j, warm, e);
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bound the scheduler's hoisting
    }
}

// LPC residuals in place (descending, so every prediction reads original samples);
// lane 0 keeps its q warm-up samples.
template <int W, typename ST>
__device__ __forceinline__ void residuals_lpc_inplace(ST (&s)[64], const ST (&hs)[W], const int32_t (&c)[W],
                                                      uint32_t shift, uint32_t q, uint32_t l) {
#pragma unroll
    for (int j = 63; j >= 0; j--) {
        const int64_t e = (int64_t)s[j] - (lpc_pred<W, ST>(s, hs, c, j) >> shift);
        const bool warm = (j < W) && (l == 0) && ((uint32_t)j < q);
        if (!warm) s[j] = (ST)(int32_t)e;
        if ((j & 7) == 0) __builtin_amdgcn_sched_barrier(0);
    }
}

// Fast LPC residual pass (full frames, order <= W taps; c[t] = 0 past the order): the
// prediction's low word P_lo = bits [shift+31 : shift] of the i64 sum, e = x - P_lo mod 2^32
// (exact when the caller's magnitude bound holds).  Per 16-sample group g: S += |e|,
// T |= e ^ (e >> 31) (= zz >> 1), N |= e (bit 31: some e < 0); lane 0's first `nwarm`
// samples (warm-ups) are left out.
template <int W, int LPWX, bool KEEP = false>
__device__ __forceinline__ void lpc_fast_pass(int32_t (&x)[64], const int32_t (&hs)[LPWX], const int32_t (&c)[LPWX],
                                              uint32_t shift, uint32_t nwarm, uint64_t (&S)[4], uint32_t (&T)[4],
                                              uint32_t (&N)[4]) {
    // KEEP: descending, each residual's low word written over its sample (a prediction reads only
    // the samples below it, none of them overwritten yet), so the caller holds the residuals for
    // the exact-bits pass instead of recomputing them
#pragma unroll
    for (int jj = 0; jj < 64; jj++) {
        const int j = KEEP ? 63 - jj : jj;
        int64_t acc = 0;
#pragma unroll
        for (int t = 0; t < W; t++) {
            const int idx = j - 1 - t;
            const int32_t xv = idx >= 0 ? x[idx >= 0 ? idx : 0] : hs[(-idx - 1) >= 0 ? (-idx - 1) : 0];
            acc += (int64_t)c[t] * (int64_t)xv;
        }
        const uint32_t plo = __builtin_amdgcn_alignbit((uint32_t)((uint64_t)acc >> 32), (uint32_t)acc, shift);
        uint32_t e = (uint32_t)x[j] - plo;
        if (KEEP) x[j] = (int32_t)e;
        const uint32_t sg = (uint32_t)((int32_t)e >> 31);
        uint32_t t = e ^ sg;
        uint32_t av = t - sg;
        if (j < LPWX) {
            const bool warm = (uint32_t)j < nwarm;
            e = warm ? 0u : e;
            t = warm ? 0u : t;
            av = warm ? 0u : av;
        }
        S[j >> 4] += av;
        T[j >> 4] |= t;
        N[j >> 4] |= e;
        if ((jj & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bound the scheduler's hoisting
    }
}

// ------------------------------------------------------------------------
// Kernel 1: frame analysis.  One workgroup per frame (persistent loop), one
// wave per candidate subframe.  Decides every candidate exactly as
// Encoder.writeFrame does (encoder.zig:234-284, 482-570), measures the exact
// bits of each candidate's lane segments (pass A of frame_writer.zig:269-372),
// takes the stereo decision (encoder.zig:441-452), and writes the frame
// descriptor + exact frame size.  No frame bytes are produced here.
//   B    : bytes per PCM sample (1..4, == bits/8)
//   CLS  : 16 (bits <= 16), 24 (bits == 24) or 32 (bits == 32)
//   FULL : every frame of the launch has n == 4096 (lane-owned partitions,
//          LDS-DMA prefetch); otherwise any 1 <= n <= 4096 (tail frames)
//   MAXT : 256 (<= 4 candidate waves) or 512
//   NC   : channel count if fixed at compile time (1 or 2), 0 = runtime
// ------------------------------------------------------------------------
#ifndef FG_MINW
#define FG_MINW 4
#endif
#ifndef FG_PACK_MINW
#define FG_PACK_MINW 4
#endif

#ifndef FG_BO_FUSED
#define FG_BO_FUSED 1
#endif
#ifndef FG_JOB_LDS
#define FG_JOB_LDS 1  // the next job records in an LDS ring instead of registers
#endif
#include "fg_fused.hpp"
#include "fg_rice16.hpp"

template <int B, int CLS, bool FULL, int MAXT, int NC, int LPW, bool FP = false>
// FP  : fused single-pass encode (full 16-bit stereo frames only, fg_fused.hpp): the workgroup
//       packs the frame it analysed; frames come from the ticket queue one at a time (no
//       prefetch) and the staging is single-buffered (it becomes the frame image)
// i64 samples (32-bit input), the tail kernels' LDS tables and the LPC search need
// the larger register budget (2 waves/SIMD); the rest fits 128 VGPRs (4 waves/SIMD).
//   LPW  : 0 = fixed prediction only (the reference); 8 / 12 = LPC taps held in
//          registers (orders up to LPW, build-defined extension)
// 24-bit LPC full frames: three waves per SIMD (168 VGPRs, more scratch, single-buffered staging
// so three workgroups fit the LDS) beat two with double buffering: c3 analysis 5.56 -> 4.80 ms
// (the 32-bit variant spills too much at 168: c5 8.7 -> 10.7 ms, so it stays at two).
__global__ void __launch_bounds__(MAXT, ((MAXT == 256 && CLS != 32 && FULL && LPW == 0) ? FG_MINW
                                          : ((FULL && LPW > 0 && CLS == 24) ? FG_C3_W : 2)))
    k_analyze(EncodeArgs a) {
    if (a.enc_prio) __builtin_amdgcn_s_setprio(1);
    using ST = typename Cls<CLS>::S;
    // LPC residuals may reach 2^30 in magnitude: 16-sample sums need 64 bits
    using SumT = typename std::conditional<LPW == 0, typename Cls<CLS>::Sum, uint64_t>::type;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const uint32_t tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
    // the wave index is wave-uniform: keep it (and everything derived from it) in SGPRs
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)), l0 = lane_id();
    const uint32_t C = NC ? (uint32_t)NC : a.channels;
    const uint32_t cw = 16u * C * B;           // dwords per 64-sample chunk
    const uint32_t cst = cw + stage_pad(C, B);  // LDS chunk stride (dwords)
    const bool dbuf = FULL && a.stage_dbuf != 0;
    static_assert(!FP || (B == 2 && CLS == 16 && FULL && MAXT == 256 && NC == 2 && LPW == 0), "fused: C2 only");
    const AnaLayout LY = ana_layout(C, B, NW, FULL, dbuf, LPW > 0, FP ? a.image_bytes : 0u);
    uint8_t *par = smem + LY.par + wave * LY.par_stride;
    uint32_t *recs = (uint32_t *)(smem + LY.rec);
    uint32_t *misc = (uint32_t *)(smem + LY.misc);
    const bool stereo = a.stereo != 0;
    const uint32_t cand = wave;
    const uint32_t bd = a.bits + ((stereo && cand == 3) ? 1u : 0u);
#ifdef FG_STAMPS
    uint64_t ph_[16] = {};
    uint64_t tprev_ = __builtin_amdgcn_s_memtime();
#endif

    // Persistent loop over a dynamic frame queue: workgroup b starts with frame b, then takes
    // gridDim.x + (an atomic ticket) -- slower CUs (e.g. sharing SIMDs with the MD5 waves)
    // simply take fewer frames.  With double buffering the next frame's PCM is DMA'd into
    // the idle staging buffer while this one is analysed.
    // The queue runs two frames ahead (as in k_pack): the job record of frame i+2 is loaded
    // while frame i is analysed, so issuing frame i+1's DMA never waits on a global load.
    uint32_t *ctr = a.work_ctr + (FULL ? 0u : 1u);
    if (blockIdx.x == 0 && tid == 0) a.work_ctr[2] = a.work_ctr[3] = 0u;  // the pack kernel's queues
    if (blockIdx.x == 0 && tid < 8u) a.work_ctr[16u + tid] = 0u;  // ... and its per-XCD split queues
    // Channel halves (a.ch_split, full frames of 4+ independent channels staged single-buffered):
    // a work item is (frame, half); the half's C channels are dwords [half drh, half drh + drh)
    // of every 2 drh-dword interchannel row, so two or three workgroups share a CU where one
    // whole 96-KiB frame would fill its LDS.  The frame-level fields are completed by
    // k_frame_totals after the launch.  The items come from the per-XCD queues (xcd_ticket).
    const uint32_t ssh = (FULL && a.ch_split) ? 1u : 0u;
    const bool xq = ssh && a.xcd_queue;
    // jit (xcd_queue bit 1): the item's ticket is taken right before its DMA, not two items
    // ahead, so the two halves of a frame -- consecutive items of one XCD's queue -- are staged
    // about one ticket interval apart and the second fetch finds the first's lines in that
    // XCD's L2 (taken ahead, the stagings are up to an item's duration apart: ~30 MB of other
    // traffic through a 4-MB L2 in between)
    const bool jit = NC != 1 && NC != 2 && xq && !dbuf && (a.xcd_queue & 2u);  // (split: 4+ channels only)
    uint32_t *xqc = a.work_ctr + 8;
    const uint32_t drh = ssh ? C * (uint32_t)B / 4u : 0u;
    const uint32_t n_items = a.n_jobs << ssh;
    if (tid == 0) {
        if (FP) {
            // fused: every frame from the queue, taken when its processing starts (a workgroup
            // never holds a frame it has not started: the look-back waits only on running ones)
            misc[22] = atomicAdd(ctr, 1u);
        } else if (xq) {
            misc[22] = xcd_ticket(xqc, a.n_jobs);
            misc[21] = jit ? 0xFFFFFFFFu : xcd_ticket(xqc, a.n_jobs);
        } else {
            misc[22] = blockIdx.x;
            misc[21] = gridDim.x + atomicAdd(ctr, 1u);
        }
    }
    __syncthreads();
    uint32_t jidx = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]), buf = 0;
    uint32_t nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[21]);
    FrameJob job{}, jn{};
    if (jidx < n_items) job = a.jobs[jidx >> ssh];
    // FG_JOB_LDS: the next two job records ride in an LDS ring (misc[52..63], two 6-dword slots)
    // filled by LDS-DMA from wave 0, instead of being held in registers through the frame; slot
    // `ri` holds the next frame's, the other the one after it
    constexpr bool JL = FG_JOB_LDS && !FP;
    uint32_t *jring = misc + 52;
    uint32_t ri = 0;
    auto job_dma = [&](uint32_t idx, uint32_t slot) {
        if (wave == 0 && l0 < 6u) lds_dma<4>((const uint32_t *)(a.jobs + (idx >> ssh)) + l0, jring + 6u * slot);
    };
    auto job_lds = [&](uint32_t slot) -> FrameJob {
        FrameJob j;
        const uint32_t *r = jring + 6u * slot;
        j.pcm_off = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r[0]) |
                    ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r[1]) << 32);
        j.number = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r[2]) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r[3]) << 32);
        j.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)r[4]);
        j.slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)r[5]);
        return j;
    };
    if (nxt < n_items) {
        if constexpr (JL) job_dma(nxt, 0u);
        else jn = a.jobs[nxt >> ssh];
    }
    if (dbuf && jidx < n_items) stage_dma(a.pcm, job.pcm_off, (uint32_t *)(smem + LY.stage0), cw, cst, wave, NW, l0, NC == 2 && B == 2, drh, jidx & ssh);
    // The ticket of the frame after next is taken at the END of the frame before (behind its
    // descriptor stores, which the top of the next frame waits for anyway) and published at the
    // estimate barrier (step 9).  Taken after the DMA of the next frame's PCM, the wait for the
    // atomic's value also waited for that DMA.
    uint32_t tk = 0;
    if (!FP && !jit && tid == 0) tk = xq ? xcd_ticket(xqc, a.n_jobs) : gridDim.x + atomicAdd(ctr, 1u);
    while (jidx < n_items) {
        const uint32_t l = opaque(l0);  // keeps lane-derived addresses from being hoisted out of the loop
        const uint32_t half = jidx & ssh;
        STAMP(8);
        const uint32_t n = FULL ? (uint32_t)kBlock : job.n;
        uint32_t *stg = (uint32_t *)(smem + (buf ? LY.stage1 : LY.stage0));

        // ---- 1. the frame's interleaved PCM in LDS (64 padded chunks of 64 samples)
        if (dbuf) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (FULL) {
            // one buffer (the frame is too large for two): every wave issues all its LDS-DMA
            // loads at once and waits once -- not one load-store round trip per dword
            stage_dma(a.pcm, job.pcm_off, stg, cw, cst, wave, NW, l, NC == 2 && B == 2, drh, half);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            stage_sync<FULL>(a.pcm, job.pcm_off, n, C * B, stg, cw, cst, wave, NW, l, NC == 2 && B == 2);
        }
        STAMP(9);
        __syncthreads();
        STAMP(10);
        if (dbuf && nxt < n_items) {
            const uint64_t noff = JL ? job_lds(ri).pcm_off : jn.pcm_off;
            stage_dma(a.pcm, noff, (uint32_t *)(smem + (buf ? LY.stage0 : LY.stage1)), cw, cst, wave, NW, l, NC == 2 && B == 2, drh, nxt & ssh);
        }
        STAMP(0);

        // ---- 2. each wave loads its candidate: lane l owns samples [64l, 64l+64)
        // (32-bit input: low words + the bit-32 mask, see load_candidate32)
        using SS = typename std::conditional<CLS == 32, int32_t, ST>::type;
        SS s[64];
        uint64_t hb = 0;
        if constexpr (CLS == 32) load_candidate32<B, FULL, NC>(stg, cst, l, n, stereo, cand, C, s, hb);
        else load_candidate<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, s);
        STAMP(1);

        // ---- 3. wasted bits (encoder.zig:556-570)
        CandRes R;
        R.bd = bd;
        R.order = R.porder = R.method = 0;
        R.lsh = 0;
        R.cval = 0;
        {
            uint64_t o;
            if constexpr (CLS != 32) {
                uint32_t o32 = 0;
#pragma unroll
                for (int j = 0; j < 64; j++) o32 |= (uint32_t)s[j];
                o = wave_or32(o32);
            } else {
                uint32_t o32 = 0;
#pragma unroll
                for (int j = 0; j < 64; j++) o32 |= (uint32_t)s[j];
                o = wave_or64((uint64_t)o32 | (hb ? 0xFFFFFFFF00000000ull : 0ull));
            }
            const uint32_t w = (o == 0) ? bd : (uint32_t)__builtin_ctzll(o);
            if (w != 0 && w != bd) {
                if constexpr (CLS == 32) {
                    shift32(s, hb, w);
                } else {
#pragma unroll
                    for (int j = 0; j < 64; j++) s[j] >>= w;
                }
            }
            R.waste = w;
        }
        const uint32_t bps = bd - R.waste;

        // history: the 4 samples before this lane's chunk (lane 0 gets zeros; its i<k terms are masked)
        // (32-bit input: hl* the low words for the truncated residuals, h* the exact values)
        const SS hl1 = shr1(s[63]), hl2 = shr1(s[62]), hl3 = shr1(s[61]), hl4 = shr1(s[60]);
        ST h1, h2, h3, h4;
        if constexpr (CLS == 32) {
            const uint64_t hbp = (uint64_t)shr1_32((uint32_t)(hb >> 32)) << 32;  // the previous lane's bits 32..63
            h1 = wide_value(hl1, hbp, 63);
            h2 = wide_value(hl2, hbp, 62);
            h3 = wide_value(hl3, hbp, 61);
            h4 = wide_value(hl4, hbp, 60);
        } else {
            h1 = hl1; h2 = hl2; h3 = hl3; h4 = hl4;
        }

        // ---- 4. CONSTANT / VERBATIM defaults (encoder.zig:493-514)
        // Full 16-bit frames (FUSED below): no separate all-equal pass -- bestOrder's order-1 sum
        // T[1] = sum_{i >= 1} |x[i] - x[i-1]| (exact) is zero iff every sample equals x[0], so the
        // CONSTANT decision is taken from it after step 5 (a constant frame runs bestOrder for
        // nothing; 128 VALU slots per wave-frame saved on every other frame)
        constexpr bool EQ_FROM_T1 = FULL && CLS == 16 && FG_BO_FUSED;
        bool try_fixed = false;
        ST x0c = 0;
        if (bps == 0) {
            R.type = 0;
            R.est = 0;
        } else if (EQ_FROM_T1) {
            x0c = (ST)rdl((uint32_t)s[0], 0);
            R.type = 1;
            R.est = (uint64_t)n * bps;
            try_fixed = true;
        } else {
            ST x0;
            if constexpr (CLS != 32) x0 = (ST)rdl((uint32_t)s[0], 0);
            else x0 = wide_value((int32_t)rdl((uint32_t)s[0], 0), (uint64_t)(rdl((uint32_t)hb, 0) & 1u), 0);
            bool eq = true;
            if constexpr (CLS != 32) {
                // all equal to x0 <=> max == min == x0: v_max3/v_min3 over the samples instead of a
                // compare per sample feeding a serial scalar AND chain (samples past n count as x0)
                int32_t mx = (int32_t)x0, mn = (int32_t)x0;
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const int32_t v = (!FULL && l * 64u + j >= n) ? (int32_t)x0 : (int32_t)s[j];
                    mx = max(mx, v);
                    mn = min(mn, v);
                }
                eq = (mx == (int32_t)x0) && (mn == (int32_t)x0);
            } else {
                // the low words by max / min as above, the bit-32 mask against x0's sign
                const uint32_t x0l = (uint32_t)x0;
                uint32_t mx = x0l, mn = x0l;
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const uint32_t v = (!FULL && l * 64u + j >= n) ? x0l : (uint32_t)s[j];
                    mx = max(mx, v);
                    mn = min(mn, v);
                }
                const uint32_t nv = FULL ? 64u : (n > l * 64u ? min(n - l * 64u, 64u) : 0u);
                const uint64_t vm = nv >= 64u ? ~0ull : ((1ull << nv) - 1ull);
                const uint64_t hx = x0 < 0 ? ~0ull : 0ull;
                eq = mx == x0l && mn == x0l && ((hb ^ hx) & vm) == 0ull;
            }
            if (__all(eq)) {
                R.type = 0;
                R.est = bps;
                R.cval = (int64_t)x0;
            } else {
                R.type = 1;
                R.est = (uint64_t)n * bps;
                try_fixed = FULL || n > 4;
            }
        }
        STAMP(2);

        uint32_t k = 0;
        // Full 16-bit frames: bestOrder accumulates |e_q| per 16-sample group (the finest Rice
        // partitions) for every order, so the chosen order's partition sums come out of it and
        // the second residual pass only ORs zigzags (the escape widths).
#ifndef FG_DESC_SUB
#define FG_DESC_SUB 1  // two-channel builds: SubDesc fixed fields in one six-lane store (r4s: WRITE 0.68 -> 0.50 GB)
#endif
#ifndef FG_DESC_FRAME
#define FG_DESC_FRAME 0  // two-channel builds: FrameDesc in one eight-lane store (r4s: no WRITE gain, off)
#endif
        constexpr bool FUSED = FULL && CLS == 16 && FG_BO_FUSED;
        uint32_t tg[5][4];
        if (try_fixed) {
            // ---- 5. bestOrder (fixed.zig:85-167)
            uint64_t T[5];
            if constexpr (FUSED) {
                const uint32_t KB = 0x7FFFFFFFu;
                const uint32_t u1 = (uint32_t)h1, u2 = (uint32_t)h2, u3 = (uint32_t)h3, u4 = (uint32_t)h4;
                uint32_t pb0 = u1 + KB;
                uint32_t pb1 = (u1 - u2) + KB;
                uint32_t pb2 = (u1 - 2u * u2 + u3) + KB;
                uint32_t pb3 = (u1 - 3u * u2 + 3u * u3 - u4) + KB;
#pragma unroll
                for (int q = 0; q < 5; q++)
#pragma unroll
                    for (int g = 0; g < 4; g++) tg[q][g] = 0;
                // orders 3 and 4 of group 0 leave the registers when the group ends: to this wave's
                // Rice parameter area (free until step 7) for the S8 pick, and into uniform partial
                // sums for T -- two VGPRs fewer at the loop's end, where the compiler spilled one
                // per frame (scratch writes)
#define FG_ROWS64(v) ((uint64_t)rdl(v, 0) + rdl(v, 16) + rdl(v, 32) + rdl(v, 48))
                uint32_t *stash = (uint32_t *)par;
                uint64_t part3 = 0, part4 = 0;
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const int g = j >> 4;
                    const uint32_t b0 = (uint32_t)s[j] + KB;
                    const uint32_t n0 = sad_u32(b0, KB, tg[0][g]);
                    const uint32_t n1 = sad_u32(b0, pb0, tg[1][g]);
                    const uint32_t b1 = (pb0 ^ KB) + b0;
                    const uint32_t n2 = sad_u32(b1, pb1, tg[2][g]);
                    const uint32_t b2 = (pb1 ^ KB) + b1;
                    const uint32_t n3 = sad_u32(b2, pb2, tg[3][g]);
                    const uint32_t b3 = (pb2 ^ KB) + b2;
                    const uint32_t n4 = sad_u32(b3, pb3, tg[4][g]);
                    if (j < 4) {  // lane 0: e_q[i] for i < q does not count (fixed.zig:102-127)
                        const bool z = (l == 0);
                        tg[0][g] = n0;
                        tg[1][g] = !(z && j < 1) ? n1 : tg[1][g];
                        tg[2][g] = !(z && j < 2) ? n2 : tg[2][g];
                        tg[3][g] = !(z && j < 3) ? n3 : tg[3][g];
                        tg[4][g] = !z ? n4 : tg[4][g];
                    } else {
                        tg[0][g] = n0; tg[1][g] = n1; tg[2][g] = n2; tg[3][g] = n3; tg[4][g] = n4;
                    }
                    pb0 = b0; pb1 = b1; pb2 = b2; pb3 = b3;
                    if (!FP && j == 15) {
                        stash[l] = tg[3][0];
                        stash[64u + l] = tg[4][0];
                        part3 = FG_ROWS64(row_sum32(tg[3][0]));
                        part4 = FG_ROWS64(row_sum32(tg[4][0]));
                        tg[3][0] = tg[4][0] = 0;
                    }
                }
                // per lane <= 64 * 2^21: row sums (16 lanes) stay below 2^32
#pragma unroll
                for (int q = 0; q < 5; q++) {
                    const uint32_t r = row_sum32(tg[q][0] + tg[q][1] + tg[q][2] + tg[q][3]);
                    T[q] = FG_ROWS64(r);
                }
                T[3] += part3;
                T[4] += part4;
#undef FG_ROWS64
            } else if constexpr (CLS != 32) {
                // biased differences b = e + 0x7FFFFFFF keep unsigned order == signed order:
                // |e_{q+1}| = v_sad_u32(b_q, b_q[prev]) and b_{q+1} = (b_q[prev] ^ 0x7FFFFFFF) + b_q
                const uint32_t KB = 0x7FFFFFFFu;
                const uint32_t u1 = (uint32_t)h1, u2 = (uint32_t)h2, u3 = (uint32_t)h3, u4 = (uint32_t)h4;
                uint32_t pb0 = u1 + KB;
                uint32_t pb1 = (u1 - u2) + KB;
                uint32_t pb2 = (u1 - 2u * u2 + u3) + KB;
                uint32_t pb3 = (u1 - 3u * u2 + 3u * u3 - u4) + KB;
                uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
                uint64_t T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0;
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const bool valid = FULL || (l * 64u + j < n);
                    const uint32_t b0 = (uint32_t)s[j] + KB;
                    const uint32_t n0 = sad_u32(b0, KB, t0);
                    const uint32_t n1 = sad_u32(b0, pb0, t1);
                    const uint32_t b1 = (pb0 ^ KB) + b0;
                    const uint32_t n2 = sad_u32(b1, pb1, t2);
                    const uint32_t b2 = (pb1 ^ KB) + b1;
                    const uint32_t n3 = sad_u32(b2, pb2, t3);
                    const uint32_t b3 = (pb2 ^ KB) + b2;
                    const uint32_t n4 = sad_u32(b3, pb3, t4);
                    if (j < 4) {  // lane 0: e_q[i] for i < q does not count (fixed.zig:102-127)
                        const bool z = (l == 0);
                        t0 = valid ? n0 : t0;
                        t1 = (valid && !(z && j < 1)) ? n1 : t1;
                        t2 = (valid && !(z && j < 2)) ? n2 : t2;
                        t3 = (valid && !(z && j < 3)) ? n3 : t3;
                        t4 = (valid && !z) ? n4 : t4;
                    } else if (!FULL) {
                        t0 = valid ? n0 : t0; t1 = valid ? n1 : t1; t2 = valid ? n2 : t2;
                        t3 = valid ? n3 : t3; t4 = valid ? n4 : t4;
                    } else {
                        t0 = n0; t1 = n1; t2 = n2; t3 = n3; t4 = n4;
                    }
                    pb0 = b0; pb1 = b1; pb2 = b2; pb3 = b3;
                    if (CLS == 24 && (j & 7) == 7) {  // 8 terms of <= 2^28 fit in u32; widen
                        T0 += t0; T1 += t1; T2 += t2; T3 += t3; T4 += t4;
                        t0 = t1 = t2 = t3 = t4 = 0;
                    }
                }
                if constexpr (CLS == 16) {
                    // per lane <= 64 * 2^20: row sums (16 lanes) stay below 2^32
                    const uint32_t r0 = row_sum32(t0), r1 = row_sum32(t1), r2 = row_sum32(t2), r3 = row_sum32(t3),
                                   r4 = row_sum32(t4);
#define FG_ROWS64(v) ((uint64_t)rdl(v, 0) + rdl(v, 16) + rdl(v, 32) + rdl(v, 48))
                    T[0] = FG_ROWS64(r0); T[1] = FG_ROWS64(r1); T[2] = FG_ROWS64(r2); T[3] = FG_ROWS64(r3);
                    T[4] = FG_ROWS64(r4);
#undef FG_ROWS64
                } else {
                    T0 += t0; T1 += t1; T2 += t2; T3 += t3; T4 += t4;
                    T[0] = wave_sum64(T0); T[1] = wave_sum64(T1); T[2] = wave_sum64(T2); T[3] = wave_sum64(T3);
                    T[4] = wave_sum64(T4);
                }
            } else {
                // 32-bit input.  Full frames first try the differences in u32: the low words are
                // exact mod 2^32 and the biased words b_q = e_q + 0x7FFFFFFF (b_{q+1} = (b_q[prev] ^
                // 0x7FFFFFFF) + b_q, as in the narrow path) are the exact e_q + 0x7FFFFFFF while e_q
                // lies in [-2^31 + 1, 2^31 - 1]; then |e_{q+1}| = v_sad_u32(b_q, b_q[prev]) is exact.
                // Certificate, from each order's range of b over the wave's counted samples: if
                // e_0 fits i32 (the side: bit 32 == bit 31) and is never -2^31, and max b_q - min b_q
                // <= 2^31 - 1 for q = 0..3, every e_{q+1} lies in [-(2^31 - 1), 2^31 - 1] -- so all
                // five orders are valid (fixed.zig:160-162) and every total exact.  Otherwise the
                // totals are redone in i64 below.  c5 stamps: this phase was 15 % of an analysis
                // wave's time on i64 arithmetic (r5q).
                bool done = false;
                if constexpr (FULL) {
                    uint32_t nf = 0;  // the side's 33-bit samples: bit 32 != bit 31 somewhere
                    if (stereo && cand == 3) {
#pragma unroll
                        for (int j = 0; j < 64; j++) nf |= ((uint32_t)(hb >> j) ^ ((uint32_t)s[j] >> 31)) & 1u;
                    }
                    if (__builtin_expect(!__any(nf != 0u), 1)) {  // (expect: the fast path laid out inline)
                        const uint32_t KB = 0x7FFFFFFFu;
                        const uint32_t u1 = (uint32_t)h1, u2 = (uint32_t)h2, u3 = (uint32_t)h3, u4 = (uint32_t)h4;
                        uint32_t pb0 = u1 + KB;
                        uint32_t pb1 = (u1 - u2) + KB;
                        uint32_t pb2 = (u1 - 2u * u2 + u3) + KB;
                        uint32_t pb3 = (u1 - 3u * u2 + 3u * u3 - u4) + KB;
                        uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
                        uint32_t mx0 = 0, mx1 = 0, mx2 = 0, mx3 = 0, mn0 = ~0u, mn1 = ~0u, mn2 = ~0u, mn3 = ~0u;
                        uint64_t A0 = 0, A1 = 0, A2 = 0, A3 = 0, A4 = 0;
#pragma unroll
                        for (int j = 0; j < 64; j++) {
                            const uint32_t b0 = (uint32_t)s[j] + KB;
                            const uint32_t b1 = (pb0 ^ KB) + b0;
                            const uint32_t b2 = (pb1 ^ KB) + b1;
                            const uint32_t b3 = (pb2 ^ KB) + b2;
                            const uint32_t n0 = sad_u32(b0, KB, t0), n1 = sad_u32(b0, pb0, t1), n2 = sad_u32(b1, pb1, t2),
                                           n3 = sad_u32(b2, pb2, t3), n4 = sad_u32(b3, pb3, t4);
                            if (j < 4) {  // lane 0: e_q[i] for i < q neither counts (fixed.zig:102-127) nor bounds
                                const bool z = (l == 0);
                                t0 = n0;
                                t1 = (z && j < 1) ? t1 : n1;
                                t2 = (z && j < 2) ? t2 : n2;
                                t3 = (z && j < 3) ? t3 : n3;
                                t4 = z ? t4 : n4;
                                mx0 = max(mx0, b0); mn0 = min(mn0, b0);
                                mx1 = max(mx1, (z && j < 1) ? 0u : b1); mn1 = min(mn1, (z && j < 1) ? ~0u : b1);
                                mx2 = max(mx2, (z && j < 2) ? 0u : b2); mn2 = min(mn2, (z && j < 2) ? ~0u : b2);
                                mx3 = max(mx3, (z && j < 3) ? 0u : b3); mn3 = min(mn3, (z && j < 3) ? ~0u : b3);
                            } else {
                                t0 = n0; t1 = n1; t2 = n2; t3 = n3; t4 = n4;
                                mx0 = max(mx0, b0); mn0 = min(mn0, b0);
                                mx1 = max(mx1, b1); mn1 = min(mn1, b1);
                                mx2 = max(mx2, b2); mn2 = min(mn2, b2);
                                mx3 = max(mx3, b3); mn3 = min(mn3, b3);
                            }
                            if (j & 1) {  // two terms <= 2^31 - 1 fit u32 (certified below)
                                A0 += t0; A1 += t1; A2 += t2; A3 += t3; A4 += t4;
                                t0 = t1 = t2 = t3 = t4 = 0;
                                // serial accumulations (reassociated trees hold every pair sum / bound live)
                                asm volatile("" : "+v"(A0), "+v"(A1), "+v"(A2), "+v"(A3), "+v"(A4));
                                asm volatile("" : "+v"(mx0), "+v"(mx1), "+v"(mx2), "+v"(mx3));
                                asm volatile("" : "+v"(mn0), "+v"(mn1), "+v"(mn2), "+v"(mn3));
                            }
                            pb0 = b0; pb1 = b1; pb2 = b2; pb3 = b3;
                            if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // no hoisting of later samples' b0
                        }
                        const uint32_t M0 = wave_max32(mx0), M1 = wave_max32(mx1), M2 = wave_max32(mx2),
                                       M3 = wave_max32(mx3);
                        const uint32_t m0 = ~wave_max32(~mn0), m1 = ~wave_max32(~mn1), m2 = ~wave_max32(~mn2),
                                       m3 = ~wave_max32(~mn3);
                        if (__builtin_expect(M0 != ~0u && M0 - m0 <= KB && M1 - m1 <= KB && M2 - m2 <= KB && M3 - m3 <= KB, 1)) {
                            T[0] = wave_sum64(A0); T[1] = wave_sum64(A1); T[2] = wave_sum64(A2);
                            T[3] = wave_sum64(A3); T[4] = wave_sum64(A4);
                            done = true;
                        }
                    }
                }
                if (__builtin_expect(!done, 0)) {  // the exact totals
                    STAMP(15);  // (stamps build: bestOrder's time before a fallback)
                    // wide path (i64): an order is invalid if any |e| exceeds i32 (fixed.zig:160-162);
                    // applying the check for bps' < 28 too is a no-op there, so one path serves both
                    int64_t p0 = h1, p1 = h1 - h2, p2 = h1 - 2 * h2 + h3, p3 = h1 - 3 * h2 + 3 * h3 - h4;
                    uint64_t A0 = 0, A1 = 0, A2 = 0, A3 = 0, A4 = 0, O0 = 0, O1 = 0, O2 = 0, O3 = 0, O4 = 0;
#pragma unroll
                    for (int j = 0; j < 64; j++) {
                        const bool valid = FULL || (l * 64u + j < n);
                        const bool z = (l == 0);
                        const int64_t e0 = wide_value(s[j], hb, j), e1 = e0 - p0, e2 = e1 - p1, e3 = e2 - p2,
                                      e4 = e3 - p3;
                        const uint64_t a0 = (uint64_t)(e0 < 0 ? -e0 : e0), a1 = (uint64_t)(e1 < 0 ? -e1 : e1),
                                       a2 = (uint64_t)(e2 < 0 ? -e2 : e2), a3 = (uint64_t)(e3 < 0 ? -e3 : e3),
                                       a4 = (uint64_t)(e4 < 0 ? -e4 : e4);
                        const bool v0 = valid, v1 = valid && !(z && j < 1), v2 = valid && !(z && j < 2),
                                   v3 = valid && !(z && j < 3), v4 = valid && !(z && j < 4);
                        A0 += v0 ? a0 : 0; O0 |= v0 ? a0 : 0;
                        A1 += v1 ? a1 : 0; O1 |= v1 ? a1 : 0;
                        A2 += v2 ? a2 : 0; O2 |= v2 ? a2 : 0;
                        A3 += v3 ? a3 : 0; O3 |= v3 ? a3 : 0;
                        A4 += v4 ? a4 : 0; O4 |= v4 ? a4 : 0;
                        p0 = e0; p1 = e1; p2 = e2; p3 = e3;
                        // keep the ten accumulations serial: reassociated into trees they would hold all
                        // 64 terms of each live at once (hundreds of VGPRs, spilled)
                        asm volatile("" : "+v"(A0), "+v"(A1), "+v"(A2), "+v"(A3), "+v"(A4));
                        asm volatile("" : "+v"(O0), "+v"(O1), "+v"(O2), "+v"(O3), "+v"(O4));
                    }
                    T[0] = wave_or64(O0) > 0x7FFFFFFFull ? ~0ull : wave_sum64(A0);
                    T[1] = wave_or64(O1) > 0x7FFFFFFFull ? ~0ull : wave_sum64(A1);
                    T[2] = wave_or64(O2) > 0x7FFFFFFFull ? ~0ull : wave_sum64(A2);
                    T[3] = wave_or64(O3) > 0x7FFFFFFFull ? ~0ull : wave_sum64(A3);
                    T[4] = wave_or64(O4) > 0x7FFFFFFFull ? ~0ull : wave_sum64(A4);
                }
            }
            k = 0;
#pragma unroll
            for (int q = 1; q < 5; q++)
                if (T[q] < T[k]) k = q;  // first minimum (fixed.zig:164)
            if (CLS == 32 && T[k] == ~0ull) try_fixed = false;  // null -> VERBATIM (encoder.zig:520)
            if (EQ_FROM_T1 && T[1] == 0) {  // all samples equal x[0]: CONSTANT (encoder.zig:497-503)
                R.type = 0;
                R.est = bps;
                R.cval = (int64_t)x0c;
                try_fixed = false;
            }
        }
        STAMP(3);

        // ---- 6/7. finest-level partition sums (rice.zig:288-340) and the parameter search for
        // every partition order (rice.zig:248-279,343-405) of one residual set with kw warm-up
        // samples -- shared by the fixed predictor and (build-defined) the LPC orders.
        const uint32_t capp = bps > 16 ? 30u : 14u;
        const uint32_t maxp = capp < a.max_param ? capp : a.max_param;
        // P16: fg_rice16.hpp's power-of-two search for 16-bit fixed prediction on full frames
        // (parameter rows at (1 << o), PO = 0).  Measured slower here (tools/ab.sh r4f: analysis
        // 4.57 vs 4.45 ms per 262144 frames), so off: every path keeps the
        // search below with rows at (1 << o) - 1 (PO = 1)
        constexpr bool P16 = false && FULL && CLS == 16 && LPW == 0 && !FP;
        constexpr uint32_t PO = P16 ? 0u : 1u;
        uint64_t *psum = nullptr;
        uint32_t *pmax = nullptr;
        if constexpr (!FULL) {
            psum = (uint64_t *)(smem + LY.psum) + wave * 256u;
            pmax = (uint32_t *)(smem + LY.pmax) + wave * 256u;
        }
        // caps of rice.calcParams (rice.zig:97-103).  The while-clamp only changes the reference's
        // result where it would slice res[kw..ps] with ps < kw (UB there).  Full frames: n = 4096
        // and kw <= 12 leave the configured order.
        auto part_cap = [&](uint32_t kw) -> uint32_t {
            uint32_t P = a.max_part_order;
            if constexpr (!FULL) {
                const uint32_t lim = kw ? (31u - __builtin_clz(n)) - (31u - __builtin_clz(kw)) : 15u;
                const uint32_t ctzn = (uint32_t)__builtin_ctz(n);
                if (ctzn < P) P = ctzn;
                if (lim < P) P = lim;
                while (P > 0 && (n >> P) < kw) P--;
            }
            return P;
        };
        auto zero_parts = [&]() {
            if constexpr (!FULL) {
                for (uint32_t i = l; i < 256u; i += 64) {
                    psum[i] = 0;
                    pmax[i] = 0;
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        };
        // residual r at lane position j -> finest-level sums (full: 4 lane-owned partitions of 16)
        auto part_acc = [&](SumT (&S8)[4], uint32_t (&O8)[4], uint32_t ps, int j, bool warm, int32_t r) {
            const uint32_t zz = zigzag32(r);
            const uint32_t av = (zz >> 1) + (zz & 1u);  // |r|
            if constexpr (FULL) {
                S8[j >> 4] += warm ? 0u : av;
                O8[j >> 4] |= warm ? 0u : zz;
                if constexpr (CLS == 32) asm volatile("" : "+v"(S8[j >> 4]));  // serial 64-bit sums
            } else {
                const uint32_t i = l * 64u + j;
                if (!warm && i < n) {
                    const uint32_t pid = i / ps;
                    atomicAdd((unsigned long long *)&psum[pid], (unsigned long long)av);
                    atomicOr(&pmax[pid], zz);
                }
            }
        };
        // SWT: tyt<uint32_t> where every partition below order 0 sums < 2^32 (|e| <= 2^20), else tyt<uint64_t>
        auto rice_search = [&](auto SWT, const auto (&S8)[4], const uint32_t (&O8)[4], uint32_t kw, uint32_t P,
                               uint8_t *pb, uint32_t &best_o, uint32_t &best_m) -> uint64_t {
            uint64_t tots[9];
            uint32_t fives[9];
            if constexpr (P16) {
                // 16-bit fixed prediction: power-of-two cost model, parameters at pb[(1 << o) + j]
                // (fg_rice16.hpp)
                const uint32_t S32[4] = {(uint32_t)S8[0], (uint32_t)S8[1], (uint32_t)S8[2], (uint32_t)S8[3]};
                const uint32_t W8[4] = {bitlen32(O8[0]), bitlen32(O8[1]), bitlen32(O8[2]), bitlen32(O8[3])};
                return rice_search16(S32, W8, kw, P, maxp, pb, l, best_o, best_m);
            } else if constexpr (FULL) {
                uint32_t W8[4];
#pragma unroll
                for (int q = 0; q < 4; q++) W8[q] = bitlen32(O8[q]);
                using SW = typename decltype(SWT)::type;
                const SW S7a = (SW)S8[0] + (SW)S8[1], S7b = (SW)S8[2] + (SW)S8[3];
                const uint32_t W7a = max(W8[0], W8[1]), W7b = max(W8[2], W8[3]);
                const SW S6 = S7a + S7b;
                const uint32_t W6 = max(W7a, W7b);
                // levels 5..2: partitions of 2/4/8/16 lanes -> DPP butterflies (every lane of the
                // group ends up with the group value); levels 1, 0: the four row values (uniform)
                SW Sl[4];
                uint32_t Wl[4];
                {
                    SW Sg = S6;
                    uint32_t Wg = W6;
                    if constexpr (sizeof(SW) == 4) {
                        Sg += dpp<DPP_XOR1>(Sg); Wg = max(Wg, dpp<DPP_XOR1>(Wg)); Sl[0] = Sg; Wl[0] = Wg;
                        Sg += dpp<DPP_XOR2>(Sg); Wg = max(Wg, dpp<DPP_XOR2>(Wg)); Sl[1] = Sg; Wl[1] = Wg;
                        Sg += dpp<DPP_HMIRROR>(Sg); Wg = max(Wg, dpp<DPP_HMIRROR>(Wg)); Sl[2] = Sg; Wl[2] = Wg;
                        Sg += dpp<DPP_MIRROR>(Sg); Wg = max(Wg, dpp<DPP_MIRROR>(Wg)); Sl[3] = Sg; Wl[3] = Wg;
                    } else {
                        Sg += dpp64<DPP_XOR1>(Sg); Wg = max(Wg, dpp<DPP_XOR1>(Wg)); Sl[0] = Sg; Wl[0] = Wg;
                        Sg += dpp64<DPP_XOR2>(Sg); Wg = max(Wg, dpp<DPP_XOR2>(Wg)); Sl[1] = Sg; Wl[1] = Wg;
                        Sg += dpp64<DPP_HMIRROR>(Sg); Wg = max(Wg, dpp<DPP_HMIRROR>(Wg)); Sl[2] = Sg; Wl[2] = Wg;
                        Sg += dpp64<DPP_MIRROR>(Sg); Wg = max(Wg, dpp<DPP_MIRROR>(Wg)); Sl[3] = Sg; Wl[3] = Wg;
                    }
                }
                uint64_t r0, r1, r2, r3;  // row sums (uniform); order 0 may reach 2^32
                if constexpr (sizeof(SW) == 4) {
                    r0 = rdl(Sl[3], 0); r1 = rdl(Sl[3], 16); r2 = rdl(Sl[3], 32); r3 = rdl(Sl[3], 48);
                } else {
                    r0 = rdl64(Sl[3], 0); r1 = rdl64(Sl[3], 16); r2 = rdl64(Sl[3], 32); r3 = rdl64(Sl[3], 48);
                }
                const uint32_t m0 = rdl(Wl[3], 0), m1 = rdl(Wl[3], 16), m2 = rdl(Wl[3], 32), m3 = rdl(Wl[3], 48);
                {
                    // Orders 5..2 (32 + 16 + 8 + 4 partitions of 2..16 lanes each): one partition per
                    // lane -- lanes 0-31 order 5, 32-47 order 4, 48-55 order 3, 56-59 order 2 --
                    // instead of every lane evaluating all four orders (three closed-form Rice
                    // decisions, ~130 issue slots, fewer per wave-frame).  A group's sum sits in every
                    // lane of the group; the lane the partition reads it from is chosen so the source
                    // sets are disjoint (order 5: odd lanes; 4: 2 mod 4; 3: 4 mod 8; 2: 8 mod 16), so
                    // each source lane exposes one level and one ds_bpermute moves them all.
                    const uint32_t lvl = l < 32u ? 0u : (l < 48u ? 1u : (l < 56u ? 2u : 3u));
                    const uint32_t jp = l - (l < 32u ? 0u : (l < 48u ? 32u : (l < 56u ? 48u : 56u)));
                    const uint32_t tz = (uint32_t)__builtin_ctz(l | 16u);
                    const SW Se = tz == 0u ? Sl[0] : (tz == 1u ? Sl[1] : (tz == 2u ? Sl[2] : Sl[3]));
                    const uint32_t We = tz == 0u ? Wl[0] : (tz == 1u ? Wl[1] : (tz == 2u ? Wl[2] : Wl[3]));
                    const int src4 = (int)(((jp << (lvl + 1u)) + (1u << lvl)) << 2);
                    SW Sx;
                    if constexpr (sizeof(SW) == 4) {
                        Sx = (SW)__builtin_amdgcn_ds_bpermute(src4, (int)Se);
                    } else {
                        Sx = (SW)(uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)(uint32_t)Se) |
                             ((SW)(uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)(uint32_t)((uint64_t)Se >> 32)) << 32);
                    }
                    const uint32_t Wx = (uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)We);
                    const uint32_t oo = 5u - lvl;
                    const uint32_t len = (128u << lvl) - (jp == 0u ? kw : 0u);
                    uint32_t cc;
                    const uint32_t p = rice_choose(Sx, len, Wx, maxp, &cc);
                    const bool act = l < 60u;
                    if (act) pb[(1u << oo) - 1u + jp] = (uint8_t)p;
                    const uint64_t fb = __ballot(act && p < 0x80u && p > 14u);
                    const uint32_t rA = row_sum32(l < 56u ? cc : 0u), rB = row_sum32((l >= 56u && act) ? cc : 0u);
                    tots[5] = (uint64_t)rdl(rA, 0) + rdl(rA, 16);
                    tots[4] = rdl(rA, 32);
                    tots[3] = rdl(rA, 48);
                    tots[2] = rdl(rB, 48);
                    fives[5] = (maxp > 14u && (fb & 0xFFFFFFFFull)) ? 1u : 0u;
                    fives[4] = (maxp > 14u && ((fb >> 32) & 0xFFFFull)) ? 1u : 0u;
                    fives[3] = (maxp > 14u && ((fb >> 48) & 0xFFull)) ? 1u : 0u;
                    fives[2] = (maxp > 14u && ((fb >> 56) & 0xFull)) ? 1u : 0u;
                }
#pragma unroll
                for (int o = 0; o < 9; o++) {
                    if (true) {  // every order unconditionally: straight-line code the scheduler can interleave (o > P is never selected)
                        uint32_t cost = 0, c;
                        bool five = false;
                        if (o >= 6) {
                            const int per = 1 << (o - 6);
#pragma unroll
                            for (int q = 0; q < per; q++) {
                                SW S;
                                uint32_t W;
                                if (o == 8) { S = S8[q]; W = W8[q]; }
                                else if (o == 7) { S = q ? S7b : S7a; W = q ? W7b : W7a; }
                                else { S = S6; W = W6; }
                                const uint32_t j = l * per + q;
                                const uint32_t len = (4096u >> o) - (j == 0 ? kw : 0u);
                                const uint32_t p = rice_choose(S, len, W, maxp, &c);
                                cost += c;
                                five |= (p < 0x80u && p > 14u);
                                pb[(1u << o) - 1u + j] = (uint8_t)p;
                            }
                            tots[o] = wave_sum32(cost);
                        } else if (o >= 2) {
                            // orders 5..2: computed once for all four below the loop head
                        } else {
                            // uniform: order 1 = rows {0,1} and {2,3}; order 0 = all rows
                            const uint32_t len0 = (4096u >> o) - kw, len1 = 4096u >> o;
                            uint32_t c0, c1 = 0, p1 = 0;
                            const uint32_t p0 = (o == 1) ? rice_choose(r0 + r1, len0, max(m0, m1), maxp, &c0)
                                                         : rice_choose(r0 + r1 + r2 + r3, len0,
                                                                       max(max(m0, m1), max(m2, m3)), maxp, &c0);
                            if (o == 1) p1 = rice_choose(r2 + r3, len1, max(m2, m3), maxp, &c1);
                            if (l == 0) {
                                pb[(1u << o) - 1u] = (uint8_t)p0;
                                if (o == 1) pb[2] = (uint8_t)p1;
                            }
                            five = (p0 < 0x80u && p0 > 14u) || (o == 1 && p1 < 0x80u && p1 > 14u);
                            tots[o] = (uint64_t)c0 + c1;
                        }
                        if (o < 2 || o > 5) fives[o] = (maxp > 14u && __any(five)) ? 1u : 0u;
                    }
                }
            } else {
                uint64_t *cs = psum;
                uint32_t *cm = pmax;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
                for (int o = 8; o >= 0; o--) {
                    if ((uint32_t)o <= P) {
                        const uint32_t np = 1u << o, len_full = n >> o;
                        uint32_t cost = 0;
                        bool five = false;
                        for (uint32_t j = l; j < np; j += 64) {
                            const uint32_t len = len_full - (j == 0 ? kw : 0u);
                            uint32_t c;
                            const uint32_t p = rice_choose(cs[j], len, bitlen32(cm[j]), maxp, &c);
                            cost += c;
                            five |= (p < 0x80u && p > 14u);
                            pb[np - 1u + j] = (uint8_t)p;
                        }
                        tots[o] = wave_sum32(cost);
                        fives[o] = (maxp > 14u && __any(five)) ? 1u : 0u;
                        if (o > 0) {
                            // next coarser level in place: each pass reads entries 2j, 2j+1 (all
                            // lanes, before any write of the pass) and writes entry j < 2j; later
                            // passes read only entries above those written so far
                            for (uint32_t j = l; j < (np >> 1); j += 64) {
                                const uint64_t s2 = cs[2 * j] + cs[2 * j + 1];
                                const uint32_t m2 = cm[2 * j] | cm[2 * j + 1];
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                                cs[j] = s2;
                                cm[j] = m2;
                            }
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        }
                    }
                }
            }
            uint64_t best = ~0ull;
            best_o = 0;
            best_m = 0;
#pragma unroll
            for (int o = 0; o < 9; o++) {
                const uint64_t tot = tots[o] + ((uint64_t)(4u + fives[o]) << o);
                if ((uint32_t)o <= P && tot <= best) {  // ascending, "<=": the higher order wins ties
                    best = tot;                           // (rice.zig:271)
                    best_o = (uint32_t)o;
                    best_m = fives[o];
                }
            }
            return best;
        };

        // 16-bit fixed prediction: every partition below order 0 sums < 2^32 (|e| <= 2^20)
        using SWD = typename std::conditional<(CLS == 16 && LPW == 0), uint32_t, uint64_t>::type;
        // LPC mode (build-defined): estimates are whole payloads, warm-ups included
        const bool lpc_on = LPW > 0 && a.lpc_order != 0;
        uint32_t cur = 0;  // parameter buffer holding the current choice (LPC: 2 per wave)
        if (try_fixed) {
            // ---- 6. residuals (read-only over s) and the finest-level partition sums
            SumT S8[4] = {0, 0, 0, 0};
            uint32_t O8[4] = {0, 0, 0, 0};
            const uint32_t P = part_cap(k);
            const uint32_t ps = n >> P;
            zero_parts();
            if constexpr (FUSED) {
#pragma unroll
                for (int g = 0; g < 4; g++)
                    S8[g] = k == 0 ? tg[0][g] : k == 1 ? tg[1][g] : k == 2 ? tg[2][g] : k == 3 ? tg[3][g] : tg[4][g];
                if (!FP && k >= 3) S8[0] = ((const uint32_t *)par)[(k == 3 ? 0u : 64u) + l];  // stashed above
                // escape widths: bitlen(OR of zigzags) == bitlen(largest zigzag) = bitlen(max(2 max e,
                // -2 min e - 1)) -- a running max/min per group (v_max3 / v_min3 over sample pairs:
                // 2 issue slots a sample) instead of a zigzag and an OR per sample (4-5)
                int32_t mx[4] = {0, 0, 0, 0}, mn[4] = {0, 0, 0, 0};
                auto acc = [&](int j, bool warm, SS r) {
                    const int32_t v = warm ? 0 : (int32_t)r;
                    mx[j >> 4] = max(mx[j >> 4], v);
                    mn[j >> 4] = min(mn[j >> 4], v);
                };
                FG_DISPATCH_K(k, (residuals_k<K, SS>(s, hl1, hl2, hl3, hl4, l, acc)))
#pragma unroll
                for (int g = 0; g < 4; g++) O8[g] = (uint32_t)max(2 * mx[g], -2 * mn[g] - 1);
            } else {
                auto acc = [&](int j, bool warm, SS r) { part_acc(S8, O8, ps, j, warm, (int32_t)r); };
                FG_DISPATCH_K(k, (residuals_k<K, SS>(s, hl1, hl2, hl3, hl4, l, acc)))
            }
            STAMP(4);

            // ---- 7. parameter search
            uint32_t best_o, best_m;
            uint64_t best = rice_search(tyt<SWD>{}, S8, O8, k, P, par, best_o, best_m);
            if (lpc_on) best += (uint64_t)k * bps;

            // ---- 8. FIXED iff its estimate < the verbatim estimate (encoder.zig:538)
            if (best < R.est) {
                R.type = 2;
                R.est = best;
                R.order = k;
                R.porder = best_o;
                R.method = best_m;
            }
        }
        int32_t *ltab = nullptr;
        // LKEEP (full 32-bit frames, c5): the fast LPC pass leaves the residuals in its sample
        // registers and, when LPC wins, the exact data bits of the lane's segment are taken from
        // them right after the parameter search (lseg), so step 10 neither reloads the samples nor
        // recomputes 64 q-tap predictions per lane -- for the two written candidates that pass
        // sat on the frame's critical path (15 % of a c5 analysis wave's time, r4n stamps)
        constexpr bool LKEEP = FULL && LPW > 0 && (CLS == 32 || (CLS == 24 && FG_LKEEP24));
        uint32_t lseg = 0;
        bool lkept = false;
        if constexpr (LPW > 0) {
            // ---- 8b. LPC order search (oracle/flac_oracle.c lpc_search): every order 1..Q with
            // usable coefficients; total = rice + q (bps' + 15) + 9; strictly smaller replaces
            ltab = (int32_t *)(smem + LY.lpc) + wave * (uint32_t)kLpcTab;
            const uint32_t Q = a.lpc_order;
            R.make_uniform();
            if (lpc_on && R.type != 0 && n > Q) {
                STAMP(11);  // (stamps build: the fixed predictor's search ends here)
                bool fits;
                uint32_t qsel = 0;  // the order selected by its LD error (contract step 7)
                // the samples are reloaded from the staging here: a memory clobber keeps the compiler
                // from proving this load equal to step 2's (same LDS words, same waste shift) and
                // holding those 64 registers live through steps 5-8, where they spilled
                asm volatile("" ::: "memory");
                {
                    int32_t x[64];
                    fits = __all(load_lpc_samples<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, R.waste, x));
                    if (fits) {
                        int64_t Rac[LPW + 1];
                        lpc_autocorr<LPW, int32_t>(x, n, l, Rac);
                        STAMP(12);
                        __builtin_amdgcn_sched_barrier(0);
                        qsel = lpc_coefs<LPW>(Rac, Q, ltab, l, n, bps);
                        STAMP(13);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (fits) {
                    // the samples again (not held through Levinson-Durbin: register pressure)
                    int32_t x[64];
                    (void)load_lpc_samples<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, R.waste, x);
                    int32_t hs[LPW];
#pragma unroll
                    for (int t = 0; t < LPW; t++) hs[t] = shr1(x[63 - t]);
                    // fast path bound (full frames): |x| <= xmax for every sample of the wave
                    uint32_t xmax = 0;
                    if constexpr (FULL) {
                        uint32_t xm = 0;
#pragma unroll
                        for (int j = 0; j < 64; j++) xm = max(xm, (uint32_t)(x[j] < 0 ? -(int64_t)x[j] : x[j]));
                        xmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_max32(xm));
                    }
                    // contract step 8: the selected order only (`continue` ends the search)
                    for (uint32_t q = qsel; q != 0; q = 0) {
                        const int32_t shq = __builtin_amdgcn_readfirstlane(ltab[(q - 1u) * 13u + 12u]);
                        if (shq < 0) continue;
                        int32_t c[LPW];
                        uint64_t csum = 0;
#pragma unroll
                        for (int t = 0; t < LPW; t++) {
                            c[t] = __builtin_amdgcn_readfirstlane(ltab[(q - 1u) * 13u + t]);
                            csum += (uint64_t)(c[t] < 0 ? -c[t] : c[t]);
                        }
                        if constexpr (FULL) {
                            // Fast path: |P| <= (csum * xmax >> shq) + 1 for the prediction P = acc >> shq,
                            // so |e| = |x - P| < 3 * 2^30 when the test holds.  Then the low words
                            // suffice: e_lo = x - P_lo (mod 2^32) and e is usable (e in [-2^30, 2^30))
                            // iff e_lo ^ (e_lo >> 31) < 2^30 -- no 64-bit residual, no per-sample check.
                            if ((uint64_t)xmax + ((csum * xmax) >> shq) + 1u < (3ull << 30)) {
                                uint64_t S8[4] = {0, 0, 0, 0};
                                uint32_t T8[4] = {0, 0, 0, 0}, N8[4] = {0, 0, 0, 0};
                                const uint32_t nw = l == 0 ? q : 0u;
                                if (q <= 4u) lpc_fast_pass<4, LPW, LKEEP>(x, hs, c, (uint32_t)shq, nw, S8, T8, N8);
                                else if (LPW <= 8 || q <= 8u) lpc_fast_pass<(LPW < 8 ? LPW : 8), LPW, LKEEP>(x, hs, c, (uint32_t)shq, nw, S8, T8, N8);
                                else lpc_fast_pass<LPW, LPW, LKEEP>(x, hs, c, (uint32_t)shq, nw, S8, T8, N8);
                                const uint32_t tall = (uint32_t)__builtin_amdgcn_readfirstlane(
                                    (int)wave_or32(T8[0] | T8[1] | T8[2] | T8[3]));
                                STAMP(14);
                                if (tall >= (1u << 30)) continue;  // some residual outside [-2^30, 2^30)
                                // OR of the zigzags' bit lengths: zz = 2t + sign
                                uint32_t O8[4];
#pragma unroll
                                for (int g = 0; g < 4; g++) O8[g] = T8[g] ? ((T8[g] << 1) | 1u) : (N8[g] >> 31);
                                const uint32_t P = part_cap(q);
                                uint8_t *pb = par + (cur ^ 1u) * 512u;
                                uint32_t best_o, best_m;
                                uint64_t rb;
                                if (tall < (1u << 20)) {  // |e| <= 2^20: 32-bit partition sums
                                    const uint32_t S32[4] = {(uint32_t)S8[0], (uint32_t)S8[1], (uint32_t)S8[2], (uint32_t)S8[3]};
                                    rb = rice_search(tyt<uint32_t>{}, S32, O8, q, P, pb, best_o, best_m);
                                } else {
                                    rb = rice_search(tyt<uint64_t>{}, S8, O8, q, P, pb, best_o, best_m);
                                }
                                const uint64_t tot = rb + (uint64_t)q * (bps + (uint32_t)kLpcPrec) + 9u;
                                if (tot < R.est) {
                                    R.type = 3;
                                    R.est = tot;
                                    R.order = q;
                                    R.porder = best_o;
                                    R.method = best_m;
                                    R.lsh = shq;
                                    cur ^= 1u;
                                    if constexpr (LKEEP) {
                                        // step 10's data bits (frame_writer.zig:299-372) from the residuals
                                        // in x: per 16-sample group the quotients, cnt (1 + p) or an escape's
                                        // cnt * width, and the partition headers the lane opens
                                        const uint32_t sh = 12u - best_o, psz = 4096u >> best_o;
                                        const uint32_t plen = 4u + best_m;
                                        const uint8_t *pp = par + cur * 512u + ((1u << best_o) - PO);
                                        uint32_t pq[4], qa[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                                        for (int g = 0; g < 4; g++) pq[g] = pp[(l * 64u + 16u * g) >> sh];
                                        if (__all(pq[0] != 0u && pq[1] != 0u && pq[2] != 0u && pq[3] != 0u)) {
                                            uint32_t sm[4];
#pragma unroll
                                            for (int g = 0; g < 4; g++) sm[g] = (pq[g] - 1u) & 31u;
#pragma unroll
                                            for (int j = 0; j < 64; j++) {
                                                const int32_t e = x[j];
                                                const uint32_t t = (uint32_t)(e ^ (e >> 31));
                                                const bool warm = j < LPW && l == 0 && (uint32_t)j < q;
                                                qa[j >> 4] = add_chain(qa[j >> 4], warm ? 0u : (t >> sm[j >> 4]));
                                            }
                                        } else {
#pragma unroll
                                            for (int j = 0; j < 64; j++) {
                                                const uint32_t zz = zigzag32(x[j]);
                                                const bool warm = j < LPW && l == 0 && (uint32_t)j < q;
                                                qa[j >> 4] = add_chain(qa[j >> 4], warm ? 0u : (zz >> (pq[j >> 4] & 31u)));
                                            }
                                        }
                                        uint32_t sg = 0;
#pragma unroll
                                        for (int g = 0; g < 4; g++) {
                                            const uint32_t pg = pq[g], i = l * 64u + 16u * g;
                                            const bool esc = (pg & 0x80u) != 0;
                                            const uint32_t cnt = 16u - ((g == 0 && l == 0) ? q : 0u);
                                            sg += esc ? cnt * (pg & 0x7Fu) : qa[g] + cnt * (1u + pg);
                                            if (i != 0 && (i & (psz - 1u)) == 0) sg += plen + (esc ? 5u : 0u);
                                        }
                                        lseg = sg;
                                        lkept = true;
                                    }
                                }
                                continue;
                            }
                        }
                        SumT S8[4] = {0, 0, 0, 0};
                        uint32_t O8[4] = {0, 0, 0, 0};
                        const uint32_t P = part_cap(q);
                        const uint32_t ps = n >> P;
                        zero_parts();
                        uint32_t bad = 0;
                        auto acc = [&](int j, bool warm, int64_t e) {
                            // usable only if every coded residual's zigzag fits 31 bits
                            const bool valid = !warm && (FULL || l * 64u + (uint32_t)j < n);
                            bad |= (valid && (uint64_t)(e + (1ll << 30)) >= (1ull << 31)) ? 1u : 0u;
                            part_acc(S8, O8, ps, j, warm, (int32_t)e);
                        };
                        residuals_lpc<LPW, int32_t>(x, hs, c, (uint32_t)shq, q, l, acc);
                        if (__any(bad)) continue;
                        uint8_t *pb = par + (cur ^ 1u) * 512u;
                        uint32_t best_o, best_m;
                        const uint64_t rb = rice_search(tyt<SumT>{}, S8, O8, q, P, pb, best_o, best_m);
                        const uint64_t tot = rb + (uint64_t)q * (bps + (uint32_t)kLpcPrec) + 9u;
                        if (tot < R.est) {
                            R.type = 3;
                            R.est = tot;
                            R.order = q;
                            R.porder = best_o;
                            R.method = best_m;
                            R.lsh = shq;
                            cur ^= 1u;
                        }
                    }
                }
            }
        }
        STAMP(5);

        // ---- 9. publish the estimate; stereo decision (encoder.zig:441-452) or independent
        // channels (:456-475)
        if (l == 0) {
            uint32_t *rc = recs + cand * 16u;
            rc[6] = (uint32_t)R.est; rc[7] = (uint32_t)(R.est >> 32);
        }
        if (!FP && tid == 0) misc[20] = tk;
        bar_lds();
        // the job record of the frame after next (DMA'd at the top of the next frame)
        uint32_t nn = 0;
        FrameJob jnn{};
        if constexpr (!FP) {
            nn = jit ? 0xFFFFFFFFu : (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[20]);
            if (nn < n_items) {
                if constexpr (JL) job_dma(nn, ri ^ 1u);  // lands before the next frame's top barrier
                else jnn = a.jobs[nn >> ssh];
            }
        }
        uint32_t channel_code, n_out;
        int my_slot;
        if (stereo) {
            uint64_t e[4];
#pragma unroll
            for (int c = 0; c < 4; c++) e[c] = (uint64_t)recs[c * 16 + 6] | ((uint64_t)recs[c * 16 + 7] << 32);
            const uint64_t sum[4] = {e[0] + e[1], e[0] + e[3], e[3] + e[1], e[2] + e[3]};
            uint32_t b = 0;
#pragma unroll
            for (int i = 1; i < 4; i++)
                if (sum[i] < sum[b]) b = i;  // first minimum
            channel_code = b == 0 ? 1u : b + 7u;
            // written pairs (encoder.zig:263-268): LR {0,1}, LS {0,3}, SR {3,1}, MS {2,3}
            const uint32_t c0 = (b == 0 || b == 1) ? 0u : (b == 2 ? 3u : 2u);
            const uint32_t c1 = (b == 0 || b == 2) ? 1u : 3u;
            my_slot = (cand == c0) ? 0 : ((cand == c1) ? 1 : -1);
            n_out = 2;
        } else {
            // channel halves: this workgroup holds channels [half C, half C + C) of 2C
            channel_code = (C << ssh) - 1u;
            n_out = C << ssh;
            my_slot = (int)(cand + half * C);
        }

        if (tid == 0) {  // frame header (frame_writer.zig:151-265) while the other waves measure
            uint32_t *hw = misc + 32;
            hw[0] = hw[1] = hw[2] = hw[3] = 0;
            misc[18] = write_frame_header(hw, job.number, a.bits, channel_code, n, a.sample_rate);
        }

        // ---- 10. exact bits of each lane's segment of the written subframes (pass A of
        // frame_writer.zig:269-372).  FIXED: the residuals were not kept through the search
        // (register pressure), so the samples are reloaded from the staged PCM.
        uint32_t seg = 0;
        if (my_slot >= 0) {
            if (R.type == 0) {
                seg = (l == 0) ? 8u + bd : 0u;
            } else if (R.type == 1) {
                const uint32_t cnt = FULL ? 64u : (n > l * 64u ? min(64u, n - l * 64u) : 0u);
                seg = cnt * bps + ((l == 0) ? 8u + R.waste : 0u);
            } else {
                k = R.order;
                // ---- 9a. exact bits of the lane's segment (frame_writer.zig:299-372).  The
                // residuals were not kept through the search (register pressure): reload the
                // samples from the staged PCM and recompute them.
                const uint32_t o = R.porder, param_len = 4u + R.method, w = R.waste;
                const uint8_t *pp = par + cur * 512u + ((1u << o) - PO);
                // residuals of the chosen predictor, recomputed from the staged PCM: fixed order k
                // (fixed.zig:30-76) or the chosen LPC order from the coefficient table
                auto pass = [&](auto &&f) {
                    if (LPW > 0 && R.type == 3) {
                        if constexpr (LPW > 0) {
                            int32_t x[64];
                            (void)load_lpc_samples<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, w, x);
                            int32_t hs[LPW];
#pragma unroll
                            for (int q = 0; q < LPW; q++) hs[q] = shr1(x[63 - q]);
                            int32_t c[LPW];
#pragma unroll
                            for (int q = 0; q < LPW; q++)
                                c[q] = __builtin_amdgcn_readfirstlane(ltab[(k - 1u) * 13u + q]);
                            // taps bucketed by order (c[t] = 0 past it), as in the order search
                            auto lpc = [&](auto WT) {
                                constexpr int W = decltype(WT)::value;
                                int32_t hsw[W], cw[W];
#pragma unroll
                                for (int q = 0; q < W; q++) {
                                    hsw[q] = hs[q];
                                    cw[q] = c[q];
                                }
                                residuals_lpc<W, int32_t>(x, hsw, cw, (uint32_t)R.lsh, k, l,
                                                          [&](int j, bool warm, int64_t e) { f(j, warm, (ST)(int32_t)e); });
                            };
                            if (k <= 4u) lpc(ic<4>{});
                            else if (LPW <= 8 || k <= 8u) lpc(ic<(LPW < 8 ? LPW : 8)>{});
                            else lpc(ic<LPW>{});
                        }
                    } else {
                        SS t[64];
                        if constexpr (CLS == 32) {
                            uint64_t hbt;
                            load_candidate32<B, FULL, NC>(stg, cst, l, n, stereo, cand, C, t, hbt);
                            if (w != 0) shift32(t, hbt, w);
                        } else {
                            load_candidate<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, t);
                            if (w != 0) {
#pragma unroll
                                for (int j = 0; j < 64; j++) t[j] >>= w;
                            }
                        }
                        const SS g1 = shr1(t[63]), g2 = shr1(t[62]), g3 = shr1(t[61]), g4 = shr1(t[60]);
                        FG_DISPATCH_K(k, (residuals_k<K, SS>(t, g1, g2, g3, g4, l, f)))
                    }
                };
                if (LKEEP && lkept && R.type == 3) {
                    seg = lseg;  // from the order search's registers (LKEEP above)
                } else if constexpr (FULL) {
                    const uint32_t sh = 12u - o, psz = 4096u >> o;
                    uint32_t pq[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) pq[q] = pp[(l * 64u + 16u * q) >> sh];
                    // per 16-sample group (one Rice parameter each): sum of the quotients only;
                    // the unary stop bits and low bits (cnt * (1 + p)), an escape group's
                    // cnt * width and the partition headers are added once per group
                    uint32_t qa[4] = {0u, 0u, 0u, 0u};
                    if (__all(pq[0] != 0u && pq[1] != 0u && pq[2] != 0u && pq[3] != 0u)) {
                        // no Rice parameter 0 in the wave (escape groups' quotients are unused): the
                        // quotient zz >> p = (2t + sign) >> p = t >> (p - 1) with t = e ^ (e >> 31),
                        // two issue slots less per sample than forming the zigzag
                        uint32_t sm[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) sm[q] = (pq[q] - 1u) & 31u;
                        auto len_t = [&](int j, bool warm, ST r) {
                            const int32_t e = (int32_t)r;
                            const uint32_t t = (uint32_t)(e ^ (e >> 31));
                            qa[j >> 4] = add_chain(qa[j >> 4], warm ? 0u : (t >> sm[j >> 4]));
                        };
                        pass(len_t);
                    } else {
                        auto len_a = [&](int j, bool warm, ST r) {
                            const uint32_t zz = zigzag32((int32_t)r);
                            qa[j >> 4] = add_chain(qa[j >> 4], warm ? 0u : (zz >> (pq[j >> 4] & 31u)));
                        };
                        pass(len_a);
                    }
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        const uint32_t p = pq[g], i = l * 64u + 16u * g;
                        const bool esc = (p & 0x80u) != 0;
                        const uint32_t cnt = 16u - ((g == 0 && l == 0) ? k : 0u);  // warm-ups: lane 0, j < k
                        seg += esc ? cnt * (p & 0x7Fu) : qa[g] + cnt * (1u + p);
                        if (i != 0 && (i & (psz - 1u)) == 0) seg += param_len + (esc ? 5u : 0u);
                    }
                } else {
                    const uint32_t psz = n >> o;
                    auto len_a = [&](int j, bool warm, ST r) {
                        const uint32_t i = l * 64u + j;
                        if (i < n && !warm) {
                            const uint32_t p = pp[i / psz];
                            const bool esc = (p & 0x80u) != 0;
                            if (i != 0 && (i % psz) == 0) seg += param_len + (esc ? 5u : 0u);
                            const uint32_t zz = zigzag32((int32_t)r);
                            seg += esc ? (p & 0x7Fu) : (zz >> p) + 1u + p;
                        }
                    };
                    pass(len_a);
                }
                // the subframe header (lane 0), added after the pass: not held live through it
                if (l == 0) {
                    const uint32_t p0 = pp[0];
                    seg += 8u + w + k * bps + 6u + param_len + ((p0 & 0x80u) ? 5u : 0u);
                    if (R.type == 3) seg += 4u + 5u + k * (uint32_t)kLpcPrec;  // precision, shift, coefficients
                }
            }
        }
        const uint32_t sub_bits = wave_sum32(seg);
        if (l == 0 && my_slot >= 0) misc[40 + my_slot] = sub_bits;
        STAMP(7);

        // ---- 11. the frame descriptor (fused: the written subframes' fields in LDS, see below)
        uint8_t *fd = a.desc + (uint64_t)job.slot * a.desc_stride;
        const uint8_t *pp = par + cur * 512u + ((1u << R.porder) - PO);
        if (FP && my_slot >= 0) {
            uint32_t *lbits = (uint32_t *)(smem + LY.lbits);
            lbits[64u * (uint32_t)my_slot + l] = seg;
            if (l == 0) {
                misc[44 + my_slot] = cand;
                misc[46 + my_slot] = R.type | (R.waste << 8) | (R.bd << 16) | (R.order << 24);
                misc[48 + my_slot] = R.porder | (R.method << 8);
                misc[50 + 2 * my_slot] = (uint32_t)R.cval;
                misc[51 + 2 * my_slot] = (uint32_t)((uint64_t)R.cval >> 32);
            }
        }
        if (!FP && my_slot >= 0) {
            SubDesc *sd = (SubDesc *)(fd + sizeof(FrameDesc)) + my_slot;  // (split: the global channel)
            // the fixed fields (type .. lpc_shift, bits, lpc_prec, cval: bytes 0..23) as six dwords
            // from lanes 0..5 -- one store instruction, one 32-B write, where eleven one-lane
            // stores of 1-8 bytes were eleven partial-line writes per subframe (two-channel
            // builds; the four-channel build spills twice as much with it, so it keeps the
            // one-lane stores)
            if constexpr (NC == 2 && FG_DESC_SUB) {
                if (l < 6u) {
                    const uint32_t w0 = R.type | (R.waste << 8) | (R.bd << 16) | (R.order << 24);
                    const uint32_t w1 = R.porder | (R.method << 8) | (cand << 16) | ((uint32_t)(uint8_t)(int8_t)R.lsh << 24);
                    const uint64_t cv = (uint64_t)R.cval;
                    const uint32_t v = l == 0 ? w0 : l == 1 ? w1 : l == 2 ? sub_bits : l == 3 ? (uint32_t)kLpcPrec
                                     : l == 4 ? (uint32_t)cv : (uint32_t)(cv >> 32);
                    ((uint32_t *)sd)[l] = v;
                }
            } else if (l == 0) {
                sd->type = (uint8_t)R.type;
                sd->waste = (uint8_t)R.waste;
                sd->bd = (uint8_t)R.bd;
                sd->order = (uint8_t)R.order;
                sd->porder = (uint8_t)R.porder;
                sd->method = (uint8_t)R.method;
                sd->cand = (uint8_t)(cand + half * C);  // the channel (split: of the whole frame)
                sd->bits = sub_bits;
                sd->cval = R.cval;
                sd->lpc_shift = (int8_t)R.lsh;
                sd->lpc_prec = (uint32_t)kLpcPrec;
            }
            if constexpr (LPW > 0) {
                if (R.type == 3 && l < (uint32_t)kLpcMax) sd->coef[l] = (int16_t)ltab[(R.order - 1u) * 13u + l];
            }
            sd->lane_bits[l] = seg;
            if (R.type >= 2) {
                const uint32_t np = 1u << R.porder;
                for (uint32_t j = l; j < np; j += 64) sd->params[j] = pp[j];
            }
        }
        if (FP) bar_lds();  // every written wave's sub_bits and fields (LDS only)
        else __syncthreads();  // every written wave's sub_bits
        if (FP && tid == 0) {
            uint32_t total = 8u * misc[18];
            for (uint32_t c = 0; c < n_out; c++) total += misc[40 + c];
            misc[17] = total;
            const uint32_t fbytes = ((total + 7u) >> 3) + 2u;
            if (fbytes + 16u > a.image_bytes) atomicOr(a.err, 1u);  // the image bound
            a.frame_bytes[job.slot] = fbytes;
            st_publish(a.status, job.slot, kStAgg | fbytes);  // before any wait (fg_fused.hpp)
        }
        if (!FP && NC == 2 && FG_DESC_FRAME && wave == 0) {
            // the FrameDesc (32 B) from lanes 0..7 in one store (two-channel builds, as above)
            const uint32_t *hw = misc + 32;
            const uint32_t hb = misc[18];
            uint32_t total = 8u * hb;
            for (uint32_t c = 0; c < n_out; c++) total += misc[40 + c];
            if (l < 8u) {
                const uint32_t v = l == 0 ? hb : l == 1 ? total : l == 2 ? channel_code : l == 3 ? n_out : hw[(l - 4u) & 3u];
                ((uint32_t *)fd)[l] = v;
            }
            if (l == 0) {
                const uint32_t fbytes = ((total + 7u) >> 3) + 2u;
                if (fbytes + 16u > a.image_bytes) atomicOr(a.err, 1u);  // the pack kernel's image bound
                a.frame_bytes[job.slot] = fbytes;
                if (a.status) st_publish(a.status, job.slot, kStAgg | fbytes);  // fused launch follows
                misc[17] = fbytes;
            }
        } else if (!FP && tid == 0 && half == 0) {
            const uint32_t *hw = misc + 32;
            const uint32_t hb = misc[18];
            FrameDesc *f = (FrameDesc *)fd;
            f->hdr_bytes = hb;
            f->channel_code = channel_code;
            f->n_out = n_out;
            f->hdr[0] = hw[0]; f->hdr[1] = hw[1]; f->hdr[2] = hw[2]; f->hdr[3] = hw[3];
            if (!ssh) {  // (split: k_frame_totals sums both halves' subframes)
                uint32_t total = 8u * hb;
                for (uint32_t c = 0; c < n_out; c++) total += misc[40 + c];
                f->total_bits = total;
                const uint32_t fbytes = ((total + 7u) >> 3) + 2u;
                if (fbytes + 16u > a.image_bytes) atomicOr(a.err, 1u);  // the pack kernel's image bound
                a.frame_bytes[job.slot] = fbytes;
                if (a.status) st_publish(a.status, job.slot, kStAgg | fbytes);  // fused launch follows
                misc[17] = fbytes;
            }
        }

        // ---- 12. optional decision records (parity tests)
        if (a.records) {
            FrameRec *fr = a.records + job.slot;
            SubRec *sr = &fr->cand[cand + half * C];
            if (l == 0) {
                sr->type = (uint8_t)R.type;
                sr->waste = (uint8_t)R.waste;
                sr->bits = (uint8_t)R.bd;
                sr->order = (uint8_t)R.order;
                sr->part_order = (uint8_t)R.porder;
                sr->method = (uint8_t)R.method;
                sr->written = my_slot >= 0 ? 1 : 0;
                sr->pad = 0;
                sr->pad2 = 0;
                sr->estimate = R.est;
                sr->constant = R.cval;
                sr->lpc_precision = R.type == 3 ? (uint8_t)kLpcPrec : 0;
                sr->lpc_shift = R.type == 3 ? (int8_t)R.lsh : 0;
            }
            if (l < 32u) {
                int32_t cv = 0;
                if constexpr (LPW > 0) {
                    if (R.type == 3 && l < (uint32_t)kLpcMax) cv = ltab[(R.order - 1u) * 13u + l];
                }
                sr->lpc_coefs[l] = cv;
            }
            const uint32_t np = 1u << R.porder;
            for (uint32_t j = l; j < 256u; j += 64) sr->params[j] = (R.type >= 2 && j < np) ? pp[j] : 0;
            if (tid == 0 && half == 0) {
                fr->channel_code = channel_code;
                fr->n_cand = NW << ssh;
                if (!ssh) fr->frame_bytes = FP ? ((misc[17] + 7u) >> 3) + 2u : misc[17];  // (split: k_frame_totals)
                fr->pad = 0;
            }
        }
        // params / records / scratch are reused by the next frame: with double-buffered staging
        // nothing touches LDS between here and the next frame's top barrier, which then orders
        // this frame's last reads before the next frame's writes; synchronous staging writes the
        // staging buffer before that barrier, so it needs its own
        if constexpr (FP) {
            // ---- 13. fused: pack the frame from the staged PCM (fg_fused.hpp), then the next ticket
            bar_lds();  // records read misc[17]
            fused_pack(a, stg, misc, (const uint32_t *)(smem + LY.lbits), smem + LY.par, LY.par_stride, job.slot,
                       misc[17], tid, wave, l);
            if (tid == 0) misc[22] = atomicAdd(ctr, 1u);
            __syncthreads();  // the image is read by the stores; the next frame's DMA overwrites it
            jidx = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]);
            if (jidx < n_items) job = a.jobs[jidx];
            STAMP(6);
            continue;
        }
        if (!dbuf) __syncthreads();
        if (jit) {
            // the next item's ticket now (single-buffered split staging: nothing is in flight)
            if (tid == 0) misc[22] = xcd_ticket(xqc, a.n_jobs);
            __syncthreads();
            jidx = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]);
            if (jidx < n_items) job = a.jobs[jidx >> ssh];
            buf ^= 1u;
            STAMP(6);
            continue;
        }
        if (tid == 0) tk = xq ? xcd_ticket(xqc, a.n_jobs) : gridDim.x + atomicAdd(ctr, 1u);
        STAMP(6);
        if constexpr (JL) {
            if (nxt < n_items) job = job_lds(ri);  // DMA'd a frame ago, waited at this frame's top
            ri ^= 1u;
        } else {
            job = jn;
            jn = jnn;
        }
        jidx = nxt; nxt = nn;
        buf ^= 1u;
    }  // persistent frame loop
#ifdef FG_STAMPS
    if (l0 == 0 && a.stamps)
        for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], (unsigned long long)ph_[i]);
#endif
}

// ------------------------------------------------------------------------
// Kernel 3: frame packing.  One workgroup per frame (persistent loop), one
// wave per written subframe.  Recomputes the chosen subframe's samples and
// residuals from the PCM (cheaper than storing them), packs the frame into an
// LDS image with every lane writing its own bit segment at the offset the
// analysis kernel measured (frame_writer.zig:269-372), appends the CRC-16
// (frame_writer.zig:111-125,144-148) and stores the frame at its final byte
// offset in the output bitstream.
// ------------------------------------------------------------------------
template <int B, int CLS, bool FULL, int MAXT, int NC, int LPW>
__global__ void __launch_bounds__(MAXT, ((CLS != 32 && FULL && LPW == 0) ? FG_PACK_MINW : 2)) k_pack(EncodeArgs a) {
    constexpr int KW = LPW > 4 ? LPW : 4;  // most warm-up samples of any predictor
    using ST = typename Cls<CLS>::S;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const uint32_t tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)), l0 = lane_id();
    const uint32_t C = NC ? (uint32_t)NC : a.channels;
    const uint32_t cw = 16u * C * B;
    const uint32_t cst = cw + stage_pad(C, B);
    const bool dbuf = FULL && a.pack_dbuf != 0;
    const PackLayout LY = pack_layout(C, B, a.image_bytes, dbuf);
    uint32_t *misc = (uint32_t *)(smem + LY.misc);
    const bool stereo = a.stereo != 0;

    // Persistent loop over a dynamic frame queue, two frames ahead: while frame i is packed, the
    // PCM of frame i+1 arrives in the idle buffer by LDS-DMA and the job record of frame i+2 is
    // loaded, so neither the staging nor the DMA issue waits on a global round trip.
    uint32_t *ctr = a.work_ctr + (FULL ? 2u : 3u);
    reset_analysis_tickets(a.work_ctr, tid);  // the analysis kernel's queues
    if (tid == 0) misc[21] = gridDim.x + atomicAdd(ctr, 1u);
    __syncthreads();
    uint32_t jidx = blockIdx.x, buf = 0;
    uint32_t nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[21]);
    FrameJob job{}, jn{};
    if (jidx < a.n_jobs) job = a.jobs[jidx];
    if (nxt < a.n_jobs) jn = a.jobs[nxt];
    if (dbuf && jidx < a.n_jobs) stage_dma(a.pcm, job.pcm_off, (uint32_t *)(smem + LY.buf0), cw, cst, wave, NW, l0, NC == 2 && B == 2);
#ifdef FG_STAMPS
    uint64_t ph_[16] = {};
    uint64_t tprev_ = __builtin_amdgcn_s_memtime();
#endif
    while (jidx < a.n_jobs) {
        const uint32_t l = opaque(l0);  // keeps lane-derived addresses from being hoisted out of the loop
        if (tid == 0) misc[20] = gridDim.x + atomicAdd(ctr, 1u);
        uint32_t *stg = (uint32_t *)(smem + (buf ? LY.buf1 : LY.buf0));
        uint32_t *img = stg;  // the image reuses the staging buffer once the samples are in VGPRs
        const uint32_t n = FULL ? (uint32_t)kBlock : job.n;
        // single-buffered full frames: the frame's DMA first, so the descriptor's dependent loads
        // below run under it (the previous frame's last barrier freed the buffer)
        if constexpr (FULL) {
            if (!dbuf) stage_dma(a.pcm, job.pcm_off, stg, cw, cst, wave, NW, l, NC == 2 && B == 2);
        }
        const uint8_t *fd = a.desc + (uint64_t)job.slot * a.desc_stride;
        const FrameDesc *F = (const FrameDesc *)fd;
        const SubDesc *sd = (const SubDesc *)(fd + sizeof(FrameDesc)) + wave;
        const uint32_t total_bits = F->total_bits;
        const uint32_t fbytes = ((total_bits + 7u) >> 3) + 2u;
        const uint64_t D = a.offsets[job.slot];
        // CRC fold geometry and its shift constants, loaded early (used after the packing)
        const uint32_t Lb = (total_bits + 7u) >> 3;
        const uint32_t W4 = Lb >> 2;
        const uint32_t H = ((W4 + 2u * NT - 1u) / (2u * NT)) | 1u;
        const uint32_t hq = min(H, a.crc_hmax) - 1u;
        const uint32_t crc_jw = a.crc_join[hq], crc_pw = a.crc_pow[hq * NT + tid];
        const bool skip = fbytes + 16u > a.image_bytes || D + fbytes > a.out_cap;  // uniform
        const uint32_t type = sd->type, w = sd->waste, bd = sd->bd, k = sd->order, o = sd->porder,
                       method = sd->method, cand = sd->cand;
        // full frames: the Rice parameters of the lane's four 16-sample groups, loaded now so the
        // packing never waits on a global read (partitions hold >= 16 samples: no group straddles)
        uint32_t pq4[4] = {0, 0, 0, 0};
        if constexpr (FULL) {
#pragma unroll
            for (int q = 0; q < 4; q++) pq4[q] = sd->params[(l0 * 64u + 16u * q) >> (12u - o)];
        }

        // ---- 1. PCM -> LDS (already in flight with double buffering), candidate samples -> VGPRs
        STAMP(7);
        if (dbuf || FULL) {
            // (one buffer: every wave issued all its LDS-DMA loads at the top and waits once)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            stage_sync<FULL>(a.pcm, job.pcm_off, n, C * B, stg, cw, cst, wave, NW, l, NC == 2 && B == 2);
        }
        STAMP(8);
        __syncthreads();
        STAMP(0);
        const uint32_t nn = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[20]);
        // the job record of the frame after next before the DMA: waiting for it then never
        // waits for the DMA (vmcnt completes in order)
        FrameJob jnn{};
        if (nn < a.n_jobs) jnn = a.jobs[nn];
        if (dbuf && nxt < a.n_jobs)
            stage_dma(a.pcm, jn.pcm_off, (uint32_t *)(smem + (buf ? LY.buf0 : LY.buf1)), cw, cst, wave, NW, l, NC == 2 && B == 2);
        if (skip) {
            if (tid == 0) atomicOr(a.err, fbytes + 16u > a.image_bytes ? 1u : 2u);
            __syncthreads();
            jidx = nxt; job = jn; nxt = nn; jn = jnn; buf ^= dbuf ? 1u : 0u;
            continue;
        }
        ST s[64];
        load_candidate<B, CLS, FULL, NC>(stg, cst, l, n, stereo, cand, C, s);  // (unused for CONSTANT)
        STAMP(9);
        // lane offsets from the measured segment lengths (uniform prefix of earlier subframes)
        const uint32_t seg = sd->lane_bits[l];
        // subframes before this wave's: every subframe's bits in one load (lane t: subframe t)
        const uint32_t sbits = l < NW ? ((const SubDesc *)(fd + sizeof(FrameDesc)) + l)->bits : 0u;
        uint32_t sub_start = 8u * F->hdr_bytes;
        for (uint32_t t = 0; t < wave; t++) sub_start += rdl(sbits, (int)t);
        const uint32_t lane_off = wave_incl_scan32(seg) - seg;
        STAMP(10);
        bar_lds();  // staging dead: zero the image
        STAMP(1);
        const uint32_t Wz = (fbytes + 3u) / 4u + 2u;
        for (uint32_t i = tid; i < Wz; i += NT) img[i] = 0;
        bar_lds();
        STAMP(2);
        if (tid < 4) {
            const uint32_t hv = F->hdr[tid];
            if (hv) atomicOr(&img[tid], hv);
        }

        // ---- 2. waste shift and residuals (fixed.zig:30-81)
        const uint32_t bps = bd - w;
        if (type != 0 && w != 0) {
#pragma unroll
            for (int j = 0; j < 64; j++) s[j] >>= w;
        }
        if (type == 2) {
            // one uniform switch around the lane loop (residuals_k keeps its own history
            // registers, so writing s[j] from the callback is safe)
            const ST h1 = shr1(s[63]), h2 = shr1(s[62]), h3 = shr1(s[61]), h4 = shr1(s[60]);
            auto none = [](int, bool, ST) {};
            residuals_generic<ST>(s, h1, h2, h3, h4, l, k, none);
        }
        if constexpr (LPW > 0) {
            if (type == 3) {  // LPC (build-defined): coefficients from the descriptor
                ST hs[LPW];
#pragma unroll
                for (int t = 0; t < LPW; t++) hs[t] = shr1(s[63 - t]);
                int32_t c[LPW];
#pragma unroll
                for (int t = 0; t < LPW; t++) c[t] = (t < kLpcMax) ? __builtin_amdgcn_readfirstlane((int32_t)sd->coef[t < kLpcMax ? t : 0]) : 0;
                // taps bucketed by order (c[t] = 0 past it), as in the analysis kernel
                auto lpc = [&](auto WT) {
                    constexpr int W = decltype(WT)::value;
                    ST hsw[W];
                    int32_t cw[W];
#pragma unroll
                    for (int t = 0; t < W; t++) {
                        hsw[t] = hs[t];
                        cw[t] = c[t];
                    }
                    residuals_lpc_inplace<W, ST>(s, hsw, cw, (uint32_t)(int32_t)sd->lpc_shift, k, l);
                };
                if (k <= 4u) lpc(ic<4>{});
                else if (LPW <= 8 || k <= 8u) lpc(ic<(LPW < 8 ? LPW : 8)>{});
                else lpc(ic<LPW>{});
            }
        }

        STAMP(3);
        // ---- 3. pack: each lane writes its contiguous bit segment (frame_writer.zig:269-372).
        // Every field is ORed into the zeroed image at its bit position; the per-sample
        // code is branch-free (escape/rice/warm-up/partition header selected per lane).
        {
            uint32_t pos = sub_start + lane_off;
            const uint64_t mask = ~0ull >> (64 - (bps ? bps : 1u));
            if (l == 0) {
                AtomicWriter bw;
                bw.init(img, pos);
                if (type == 0) {  // writeConstantSubframe: header 0x00, value << waste in bd bits, no wasted flag
                    bw.put(0, 8);
                    bw.put(((uint64_t)sd->cval << w) & (~0ull >> (64 - bd)), bd);
                } else {
                    // type code: VERBATIM 1, FIXED 8|k, LPC 0x20|(k-1) (build-defined)
                    const uint32_t tc = (type == 1) ? 1u : (type == 2 ? (8u | k) : (0x20u | (k - 1u)));
                    bw.put((tc << 1) | (w ? 1u : 0u), 8);
                    if (w) bw.put(1, w);
                    if (type >= 2) {
#pragma unroll
                        for (int j = 0; j < KW; j++)  // warm-up samples
                            if ((uint32_t)j < k) bw.put((uint64_t)(int64_t)s[j] & mask, bps);
                        if (type == 3) {
                            const uint32_t prec = sd->lpc_prec;
                            bw.put(prec - 1u, 4);
                            bw.put((uint32_t)(int32_t)sd->lpc_shift & 31u, 5);
                            for (uint32_t t = 0; t < k; t++)
                                bw.put((uint64_t)(int64_t)sd->coef[t] & (~0ull >> (64 - prec)), prec);
                        }
                        bw.put((method << 4) | o, 6);
                        const uint32_t p0 = sd->params[0];
                        if (p0 & 0x80u) {
                            bw.put(0x0Fu | (method << 4), 4u + method);
                            bw.put(p0 & 0x7Fu, 5);
                        } else {
                            bw.put(p0, 4u + method);
                        }
                    }
                }
                pos = bw.pos;
            }
            if (type == 1) {
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const bool ok = FULL || l * 64u + j < n;
                    put_or2(img, pos, (uint64_t)(int64_t)s[j] & mask, ok ? bps : 0u);
                    pos += ok ? bps : 0u;
                }
            } else if (type >= 2) {
                const uint32_t param_len = 4u + method;
                const uint32_t esc_code = (0x0Fu | (method << 4)) << 5;
                const uint8_t *pp = sd->params;
                // one residual: rice (q zeros, 1, p low bits) or escape (raw w-bit two's complement)
                auto code = [&](int32_t r, uint32_t p, bool skip) {
                    const bool esc = (p & 0x80u) != 0;
                    const uint32_t wb = p & 0x7Fu;
                    const uint32_t zz = zigzag32(r);
                    const uint32_t pr = esc ? 0u : p;
                    const uint32_t qz = (esc || skip) ? 0u : (zz >> pr);
                    const uint64_t v = esc ? ((uint64_t)(uint32_t)r & (~0ull >> (64 - (wb ? wb : 1u))))
                                           : (uint64_t)((1u << pr) | (zz & ((1u << pr) - 1u)));
                    const uint32_t len = skip ? 0u : (esc ? wb : pr + 1u);
                    pos += qz;
                    put_or2(img, pos, v, len);
                    pos += len;
                };
                auto part_header = [&](uint32_t p, bool on) {
                    const bool esc = (p & 0x80u) != 0;
                    const uint32_t hl = on ? param_len + (esc ? 5u : 0u) : 0u;
                    put_or2(img, pos, esc ? (esc_code | (p & 0x7Fu)) : p, hl);
                    pos += hl;
                };
                if constexpr (FULL) {
                    // per 16-sample group (one partition each: partitions hold >= 16 samples) the
                    // code shape is lane-constant: rice = q zeros then (1 << p) | low p bits in
                    // p + 1 bits, escape = the raw wb-bit value; warm-ups code as nothing.  Codes
                    // are ORed at absolute LDS bit addresses pa (word address (pa >> 5) * 4).
                    const uint32_t psz = 4096u >> o;
                    const uint32_t img_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)img;
                    // (one variant: a second, escape-free copy of the loop made the allocator spill)
                    {
                        constexpr bool E = true;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            __builtin_amdgcn_sched_barrier(0);  // the group's constants live one group at a time
                            const uint32_t p = pq4[q];
                            const uint32_t i0 = l * 64u + 16u * q;
                            part_header(p, i0 != 0 && (i0 & (psz - 1u)) == 0);
                            const bool esc = (p & 0x80u) != 0;
                            const uint32_t wb = p & 0x7Fu, pr = esc ? 0u : p;
                            const uint32_t cl = esc ? wb : pr + 1u;
                            const uint32_t cmask = esc ? ((1u << wb) - 1u) : ((1u << pr) - 1u);
                            const uint32_t cbit = esc ? 0u : (1u << pr);
                            const uint32_t ncl = 64u - cl;
                            uint32_t pa = 8u * img_lds + pos;
#pragma unroll
                            for (int jj = 0; jj < 16; jj++) {
                                const int j = 16 * q + jj;
                                const bool warm = j < KW && l == 0 && (uint32_t)j < k;
                                const int32_t r = (int32_t)s[j];
                                const uint32_t zz = zigzag32(r);
                                const uint32_t src = E ? (esc ? (uint32_t)r : zz) : zz;
                                uint32_t v = (src & cmask) | cbit;
                                uint32_t qz = E ? (esc ? 0u : (zz >> pr)) : (zz >> pr);
                                uint32_t sh = ncl, adv = cl;
                                if (j < KW) {
                                    v = warm ? 0u : v;
                                    qz = warm ? 0u : qz;
                                    sh = warm ? 64u : sh;
                                    adv = warm ? 0u : adv;
                                }
                                pa += qz;
                                const uint64_t t = (uint64_t)v << ((sh - (pa & 31u)) & 63u);
                                lds_or2((pa >> 3) & ~3u, (uint32_t)(t >> 32), (uint32_t)t);
                                pa += adv;
                            }
                            pos = pa - 8u * img_lds;
                        }
                    }
                } else {
                    const uint32_t psz = n >> o;
#pragma unroll
                    for (int j = 0; j < 64; j++) {
                        const uint32_t i = l * 64u + j;
                        const bool ok = i < n;
                        const uint32_t p = ok ? pp[i / psz] : 0u;
                        part_header(p, ok && i != 0 && (i % psz) == 0);
                        code((int32_t)s[j], p, !ok || (l == 0 && (uint32_t)j < k));
                    }
                }
            }
        }
        bar_lds();

        STAMP(4);
        // ---- 4. CRC-16 of the frame: the word stream is front-padded with zero words (a no-op
        // for an init-0 CRC) to NT*2H words; thread t folds its 2H words as two interleaved
        // halves in table-free chains mod Q (crc_lane_q), joins them (x z^(32H) mod Q), scales by
        // z^(16 + 64H(NT-1-t)) mod Q and the workgroup XOR-reduces residue and parity.  H is odd so
        // the per-thread word stride 2H costs at most 2-way conflicts.
        {
            const int32_t Z = (int32_t)(NT * 2u * H) - (int32_t)W4;
            const int32_t va = (int32_t)(tid * 2u * H) - Z, vb = va + (int32_t)H;
            uint32_t sa = 0, sb = 0, px = 0;
            for (uint32_t i = 0; i < H; i++) {
                const int32_t ra = va + (int32_t)i, rb = vb + (int32_t)i;
                const uint32_t wa = ra >= 0 ? img[ra] : 0u, wb = rb >= 0 ? img[rb] : 0u;
                sa = q_word(sa, wa);
                sb = q_word(sb, wb);
                px ^= wa ^ wb;
            }
            const uint32_t ct = q_fold(q_mul(q_fold(sa), crc_jw) ^ sb);
            uint32_t contrib = q_mul(ct, crc_pw) | ((__builtin_popcount(px) & 1u) << 16);
            contrib = wave_xor32(contrib);
            if (l == 0) misc[wave] = contrib;
        }
        bar_lds();
        if (tid == 0) {
            uint32_t qp = 0;
            for (uint32_t i = 0; i < NW; i++) qp ^= misc[i];
            uint32_t crc = crc_from_q(qp);
            for (uint32_t b = W4 * 4u; b < Lb; b++)
                crc = crc_byte_v(crc, (img[b >> 2] >> (24 - 8 * (b & 3))) & 255u);
            put_bits(img, Lb * 8u, crc, 16);
        }
        bar_lds();

        STAMP(5);
        // ---- 5. image -> out[D, D + fbytes)
        store_frame16(img, a.out, D, fbytes, tid, NT);
        // the image / staging area is reused by the next frame: with double buffering it is next
        // written by the DMA issued after the next frame's top barrier, which orders these reads
        // before it; synchronous staging refills it before that barrier
        if (!dbuf) __syncthreads();
        STAMP(6);
        jidx = nxt; job = jn; nxt = nn; jn = jnn; buf ^= dbuf ? 1u : 0u;
    }  // persistent frame loop
#ifdef FG_STAMPS
    if (l0 == 0 && a.stamps)
        for (int i = 0; i < 11; i++) atomicAdd(&a.stamps[16 + i], (unsigned long long)ph_[i]);
#endif
}

#include "fg_pack4.hpp"
#include "fg_packw.hpp"
#if FG_DIAG
#include "fg_ana1.hpp"
#endif

// persistent launch: grid = min(work items, resident workgroups on this device).  The occupancy
// is cached per (kernel, threads, LDS, device); the lock covers only the cache lookup/insert, so
// contexts driven from several host threads (fg_multi.cpp) launch concurrently.  A miss computes
// outside the lock (two racing threads compute the same value).
template <typename KernelT>
static hipError_t launch_persistent(KernelT k, const EncodeArgs &a, uint32_t threads, uint32_t lds, hipStream_t st) {
    struct Occ {
        const void *fn;
        uint32_t threads, lds;
        int device, resident, cus;
    };
    static Occ cache[64];
    static int n_cache = 0;
    static std::mutex mu;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int resident = 0, cus = 0;
    {
        std::lock_guard<std::mutex> lock(mu);
        for (int i = 0; i < n_cache; i++)
            if (cache[i].fn == (const void *)k && cache[i].threads == threads && cache[i].lds == lds &&
                cache[i].device == dev) {
                resident = cache[i].resident;
                cus = cache[i].cus;
                break;
            }
    }
    if (!resident) {
        e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        int nb = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)k, (int)threads, (size_t)lds);
        if (e != hipSuccess) return e;
        resident = nb > 0 ? nb : 1;
        std::lock_guard<std::mutex> lock(mu);
        if (n_cache < 64) cache[n_cache++] = {(const void *)k, threads, lds, dev, resident, cus};
    }
    uint64_t grid = (uint64_t)a.n_jobs << (a.ch_split ? 1 : 0);  // work items (channel halves: two per frame)
    const int per_cu = (a.grid_per_cu && (int)a.grid_per_cu < resident) ? (int)a.grid_per_cu : resident;
    uint64_t cap = (uint64_t)per_cu * (uint64_t)(cus > 0 ? cus : 256);
    // leave room for workgroups of a kernel running beside this one (the stream MD5): without it
    // the persistent grid takes every slot and the other kernel waits for this one to finish
    if (a.grid_reserve && cap > 4u * (uint64_t)a.grid_reserve) cap -= a.grid_reserve;
    if (grid > cap) grid = cap;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k, dim3((uint32_t)grid), dim3(threads), lds, st, a);
    return hipGetLastError();
}

// NC = 2 for two channels, 1 for mono, 0 (runtime) otherwise; MAXT by wave count.
// stage: 0 = analysis, 1 = pack.
template <int B, int CLS, int LPW>
static hipError_t launch_stage_b(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds,
                                 hipStream_t st) {
#define FG_L(NCV, MT)                                                                                     \
    do {                                                                                                  \
        if (stage == 0)                                                                                   \
            return full ? launch_persistent(k_analyze<B, CLS, true, MT, NCV, LPW>, a, threads, lds, st)  \
                        : launch_persistent(k_analyze<B, CLS, false, MT, NCV, LPW>, a, threads, lds, st); \
        return full ? launch_persistent(k_pack<B, CLS, true, MT, NCV, LPW>, a, threads, lds, st)         \
                    : launch_persistent(k_pack<B, CLS, false, MT, NCV, LPW>, a, threads, lds, st);       \
    } while (0)
    if constexpr (B == 2 && CLS == 16 && LPW == 0) {
        // full 16-bit two-channel frames: four waves per written subframe (fg_pack4.hpp)
        if (stage == 1 && full && a.channels == 2 && threads == 512u)
            return launch_persistent(k_pack4<512>, a, threads, lds, st);
#if FG_DIAG
        // fused single-pass encode of full 16-bit stereo frames (fg_fused.hpp)
        if (stage == 2 && full && a.channels == 2 && a.stereo && threads == 256u)
            return launch_persistent(k_analyze<2, 16, true, 256, 2, 0, true>, a, threads, lds, st);
        // one wave per full 16-bit stereo frame (fg_ana1.hpp)
        if (stage == 3 && full && a.channels == 2 && a.stereo && threads == 64u)
            return a.ana1_variant == 2 ? launch_persistent(k_ana1<2>, a, threads, lds, st)
                                       : launch_persistent(k_ana1<1>, a, threads, lds, st);
#endif
    }
    if (stage >= 2) return hipErrorInvalidValue;
    // other full frames: WPS waves per written subframe (fg_packw.hpp); the host marks it by
    // the thread count 64 * n_out * WPS (k_pack runs 64 * n_out)
    if (stage == 1 && full && a.ch_split) {
        // channel halves (k_packw split mode): 2 waves per written subframe of the half
        return launch_persistent(k_packw<B, CLS, 0, LPW, 32, true>, a, threads, lds, st);
    }
    if (stage == 1 && full) {
        const uint32_t n_out = a.stereo ? 2u : a.channels;
        if (threads == 64u * n_out * 4u) {
            if (a.channels == 2) return launch_persistent(k_packw<B, CLS, 2, LPW, 16>, a, threads, lds, st);
            return launch_persistent(k_packw<B, CLS, 0, LPW, 16>, a, threads, lds, st);
        }
        if (threads == 64u * n_out * 2u) return launch_persistent(k_packw<B, CLS, 0, LPW, 32>, a, threads, lds, st);
    }
    if (a.channels == 2) FG_L(2, 256);
    if (a.channels == 1) FG_L(1, 256);
    // four channels (the channel halves of 8-channel frames, c4): compile-time C halves the
    // analysis's spills (VGPR 43 -> 22, SGPR 368 -> 128, scratch 112 -> 64 B per lane); the
    // pack keeps the runtime form (its NC = 4 build spills where NC = 0 does not)
    if constexpr (LPW == 0) {
        static const bool nc4 = !std::getenv("FLACGPU_NC4") || std::getenv("FLACGPU_NC4")[0] != '0';  // A/B knob
        if (nc4 && stage == 0 && full && a.channels == 4 && threads == 256u)
            return launch_persistent(k_analyze<B, CLS, true, 256, 4, 0>, a, threads, lds, st);
    }
    if (threads <= 256) FG_L(0, 256);
    FG_L(0, 512);
#undef FG_L
}

}  // namespace fg
