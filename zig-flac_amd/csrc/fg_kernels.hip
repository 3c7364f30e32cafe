// fg_kernels.hip -- CDNA4 (gfx950) kernels for the FLAC block-encode path.
//
// One workgroup encodes one frame; one 64-lane wave owns one candidate
// subframe (stereo: L, R, M, S; otherwise one wave per channel) and each lane
// owns 64 consecutive samples held in VGPRs.  The whole per-block pipeline of
// toastori/zig-flac's Encoder.writeFrame (src/lib/encoder.zig:234-284) runs
// here: mid/side (encoder.zig:329-350), wasted bits (:556-570), subframe
// choice (:482-554), fixed-order analysis and residuals (fixed.zig:30-201),
// Rice partition/parameter search (rice.zig:87-107,248-405), bit packing
// (frame_writer.zig:40-372), CRC-8/CRC-16 (frame_writer.zig:128-148,
// crc16.zig) -- plus MD5 (md5.zig) in its own kernel.  No MFMA: there is no
// dense contraction on this path.  See DESIGN.md for the layout and roofline.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fg_common.hpp"
#include "fg_layout.hpp"

namespace fg {

// ------------------------------------------------------------------------
// wave helpers (wave64)
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// v_sad_u32: |a - b| (unsigned) + acc
__device__ __forceinline__ uint32_t sad_u32(uint32_t a, uint32_t b, uint32_t acc) {
    uint32_t d;
    asm("v_sad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(acc));
    return d;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_or(T v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v |= __shfl_xor(v, m);
    return v;
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m);
    return v;
}
// exclusive prefix sum over the wave; *total = sum of all lanes
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    uint32_t x = v;
    const uint32_t l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x += y;
    }
    *total = __shfl(x, 63);
    return x - v;
}

__device__ __forceinline__ uint32_t bitlen32(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }
__device__ __forceinline__ uint32_t bitlen64(uint64_t x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }
__device__ __forceinline__ uint32_t zigzag32(int32_t r) { return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31); }
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

// ------------------------------------------------------------------------
// Rice partition decision (rice.zig:343-405) in closed form.
// f(0) = len + 2S; f(p) = (1+p)*len + (S >> (p-1)) - floor(len/2), p >= 1.
// f is convex in p, so the lowest argmin over 0..maxp-1 -- the
// parameter the reference's strict "<" scan keeps -- is the first p whose
// forward difference is >= 0:  p = 0 if S <= ceil(len/2), else p = m + 1 for
// the smallest m with (S >> m) <= 2*len, clamped to maxp - 1.  The escape
// code (5 + width*len, invalid above 31 bits) is the initial candidate and
// wins ties (strict "<" on the rice side).
// ------------------------------------------------------------------------
__device__ __forceinline__ void rice_choose(uint64_t S, uint32_t len, uint32_t width, uint32_t maxp, uint32_t *cost,
                                            uint32_t *param) {
    uint32_t p;
    if (S <= (uint64_t)((len + 1u) >> 1)) {
        p = 0;
    } else {
        uint64_t two = 2ull * len;
        uint32_t m = 0;
        if (S > two) {
            m = bitlen64(S) - bitlen64(two);
            if ((S >> m) > two) m++;
        }
        p = m + 1u;
    }
    if (p > maxp - 1u) p = maxp - 1u;
    uint64_t f = (p == 0) ? (uint64_t)len + (S << 1)
                          : (uint64_t)(1u + p) * len + ((S >> (p - 1u)) - (uint64_t)(len >> 1));
    uint64_t esc = (width <= 31u) ? 5ull + (uint64_t)width * len : ~0ull;
    if (f < esc) {
        *cost = (uint32_t)f;
        *param = p;
    } else {
        *cost = (uint32_t)esc;
        *param = 0x80u | width;
    }
}

// CRC-16/UMTS helpers (crc16.zig; poly 0x8005, init 0).  tab = 4 x 256 u16:
// [0] x*z^40, [1] x*z^32, [2] x*z^24, [3] x*z^16 (mod P).  W is a stream word
// whose first byte sits in bits 31..24.
__device__ __forceinline__ uint32_t crc_word(uint32_t crc, uint32_t W, const uint16_t *tab) {
    uint32_t X = W ^ (crc << 16);
    return (uint32_t)tab[X >> 24] ^ (uint32_t)tab[256 + ((X >> 16) & 255u)] ^
           (uint32_t)tab[512 + ((X >> 8) & 255u)] ^ (uint32_t)tab[768 + (X & 255u)];
}
__device__ __forceinline__ uint32_t crc_byte(uint32_t crc, uint32_t b, const uint16_t *tab) {
    return ((crc << 8) & 0xFFFFu) ^ (uint32_t)tab[768 + (((crc >> 8) ^ b) & 255u)];
}
// a(z) * b(z) mod (z^16 + z^15 + z^2 + 1)
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        r <<= 1;
        if (r & 0x10000u) r ^= 0x18005u;
        if ((a >> i) & 1u) r ^= b;
    }
    return r & 0xFFFFu;
}

// OR `len` (<= 33) bits of v at bit position pos of the big-endian word image.
__device__ __forceinline__ void put_bits(uint32_t *img, uint32_t pos, uint64_t v, uint32_t len) {
    if (len == 0) return;
    uint32_t wi = pos >> 5, o = pos & 31u;
    uint64_t t = v << (64u - o - len);
    atomicOr(&img[wi], (uint32_t)(t >> 32));
    if (o + len > 32u) atomicOr(&img[wi + 1], (uint32_t)t);
}

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
            uint32_t sh = n - remain;
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

// Writes the header into img (zeroed) and returns its length in bytes.
__device__ uint32_t write_frame_header(uint32_t *img, uint64_t frame_number, uint32_t bits, uint32_t channel_code,
                                       uint32_t block_size, uint32_t sample_rate) {
    HdrWriter h;
    h.bits(16, 0xFFF8);
    uint32_t unc_bs = 0;
    uint32_t ctz = (uint32_t)__builtin_ctz(block_size);
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
    } else {
        uint64_t buf = 0, num = frame_number, fbm = 0x3F;
        uint32_t i = 0;
        while (num > fbm) {
            buf |= (0x80ull + (num & 0x3F)) << (8 * i);
            i++;
            num >>= 6;
            fbm >>= 1;
        }
        buf |= ((0xFEull << (6 - i)) | num) << (8 * i);
        uint32_t nb = 8 * (i + 1);
        h.bits(nb, buf & (~0ull >> (64 - nb)));
    }
    if (unc_bs) h.bits(unc_bs, block_size - 1u);
    if (unc_sr == 4) h.bits(8, block_size);  // reference writes the block size here (unmasked)
    else if (unc_sr) h.bits(16, block_size / unc_sr);
    // header bytes so far: words w0 (if stored) then the accumulator's top byte_end bytes
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
// The frame-encode kernel.
//   B    : bytes per PCM sample (1..4, == bits/8)
//   CLS  : 16 (bits <= 16), 24 (bits == 24) or 32 (bits == 32)
//   FULL : every frame of the launch has n == 4096 (lane-owned partitions);
//          otherwise any 1 <= n <= 4096 (tail frames; LDS partition tables)
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
    uint64_t est;
    int64_t cval;
};

// residual of order K from sample x and history q1..q4 (fixed.zig:12-18 COEFF_SCALAR stencil):
// wrapping i32 (narrow, fixed.zig:63-68) or i64 truncated to i32 (wide, fixed.zig:69-74).
template <int K, typename ST>
__device__ __forceinline__ ST fixed_residual(ST x, ST q1, ST q2, ST q3, ST q4) {
    if constexpr (sizeof(ST) == 4) {
        uint32_t ux = (uint32_t)x, u1 = (uint32_t)q1, u2 = (uint32_t)q2, u3 = (uint32_t)q3, u4 = (uint32_t)q4;
        uint32_t r;
        if constexpr (K == 0) r = ux;
        else if constexpr (K == 1) r = ux - u1;
        else if constexpr (K == 2) r = ux - 2u * u1 + u2;
        else if constexpr (K == 3) r = ux - 3u * u1 + 3u * u2 - u3;
        else r = ux - 4u * u1 + 6u * u2 - 4u * u3 + u4;
        return (ST)(int32_t)r;
    } else {
        int64_t r;
        if constexpr (K == 0) r = x;
        else if constexpr (K == 1) r = x - q1;
        else if constexpr (K == 2) r = x - 2 * q1 + q2;
        else if constexpr (K == 3) r = x - 3 * q1 + 3 * q2 - q3;
        else r = x - 4 * q1 + 6 * q2 - 4 * q3 + q4;
        return (ST)(int32_t)(uint32_t)(uint64_t)r;
    }
}

// inverse: sample from residual and history (wrapping i32 / exact i64)
__device__ __forceinline__ int32_t fixed_restore(uint32_t k, int32_t r, int32_t q1, int32_t q2, int32_t q3,
                                                 int32_t q4) {
    uint32_t ur = (uint32_t)r, u1 = (uint32_t)q1, u2 = (uint32_t)q2, u3 = (uint32_t)q3, u4 = (uint32_t)q4, x;
    if (k == 0) x = ur;
    else if (k == 1) x = ur + u1;
    else if (k == 2) x = ur + 2u * u1 - u2;
    else if (k == 3) x = ur + 3u * u1 - 3u * u2 + u3;
    else x = ur + 4u * u1 - 6u * u2 + 4u * u3 - u4;
    return (int32_t)x;
}
__device__ __forceinline__ int64_t fixed_restore(uint32_t k, int64_t r, int64_t q1, int64_t q2, int64_t q3,
                                                 int64_t q4) {
    if (k == 0) return r;
    if (k == 1) return r + q1;
    if (k == 2) return r + 2 * q1 - q2;
    if (k == 3) return r + 3 * q1 - 3 * q2 + q3;
    return r + 4 * q1 - 6 * q2 + 4 * q3 - q4;
}

template <int B, int CLS, bool FULL>
__global__ void __launch_bounds__(512) k_encode(EncodeArgs a) {
    using ST = typename Cls<CLS>::S;
    using SumT = typename Cls<CLS>::Sum;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const uint32_t tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
    const uint32_t wave = tid >> 6, l = lane_id();
    const FrameJob job = a.jobs[blockIdx.x];
    const uint32_t C = a.channels;
    const uint32_t n = FULL ? (uint32_t)kBlock : job.n;
    const LdsLayout LY = lds_layout(C, B, NW, a.image_bytes, FULL);
    uint32_t *img = (uint32_t *)(smem + LY.img);
    uint8_t *par = smem + LY.par + wave * 512u;
    uint32_t *recs = (uint32_t *)(smem + LY.rec);
    uint16_t *crct = (uint16_t *)(smem + LY.crc);
    uint32_t *misc = (uint32_t *)(smem + LY.misc);

    // ---- 1. stage the frame's interleaved PCM into LDS: 64 chunks of 64
    // samples, one pad dword per chunk (conflict-free per-lane reads below)
    const uint32_t cw = 16u * C * B;  // dwords per chunk
    const uint32_t in_bytes = n * C * B;
    {
        const uint32_t *src = (const uint32_t *)(a.pcm + job.pcm_off);
        const uint32_t nchunks = FULL ? 64u : (n + 63u) >> 6;
        for (uint32_t ch = wave; ch < nchunks; ch += NW) {
#pragma unroll 4
            for (uint32_t x = l; x < cw; x += 64) {
                const uint32_t wd = ch * cw + x;
                uint32_t v = 0;
                if (FULL || 4u * wd + 4u <= in_bytes) {
                    v = src[wd];
                } else if (4u * wd < in_bytes) {
                    const uint8_t *sb = (const uint8_t *)src + 4u * wd;
                    for (uint32_t q = 0; 4u * wd + q < in_bytes; q++) v |= (uint32_t)sb[q] << (8 * q);
                }
                img[ch * (cw + 1u) + x] = v;
            }
        }
        for (uint32_t i = tid; i < 1024u; i += NT) crct[i] = a.crc_tab[i];
    }
    __syncthreads();

    // ---- 2. each wave loads its candidate: lane l owns samples [64l, 64l+64)
    const bool stereo = a.stereo != 0;
    const uint32_t cand = wave;
    const uint32_t bd = a.bits + ((stereo && cand == 3) ? 1u : 0u);
    ST s[64];
    {
        const uint8_t *base = (const uint8_t *)img + l * (cw + 1u) * 4u;
        const uint32_t CB = C * B;
        if (stereo) {
#pragma unroll
            for (int j = 0; j < 64; j++) {
                const int64_t L = ld_sample<B>(base + j * CB);
                const int64_t Rr = ld_sample<B>(base + j * CB + B);
                int64_t v;
                if (cand == 0) v = L;
                else if (cand == 1) v = Rr;
                else if (cand == 2) v = (L + Rr) >> 1;  // mid from un-shifted L/R (encoder.zig:337,347)
                else v = L - Rr;                         // side; 33-bit at 32 bps (samples64, encoder.zig:338)
                if (!FULL && l * 64u + j >= n) v = 0;
                s[j] = (ST)v;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 64; j++) {
                int32_t v = ld_sample<B>(base + j * CB + cand * B);
                if (!FULL && l * 64u + j >= n) v = 0;
                s[j] = (ST)v;
            }
        }
    }
    __syncthreads();  // staging is dead from here on (region 0 reused)

    // ---- 3. wasted bits (encoder.zig:556-570)
    CandRes R;
    R.bd = bd;
    R.order = R.porder = R.method = 0;
    R.cval = 0;
    {
        uint64_t o = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) o |= (uint64_t)(int64_t)s[j];
        if (CLS != 32) o &= 0xFFFFFFFFull;
        o = wave_or(o);
        const uint32_t w = (o == 0) ? bd : (uint32_t)__builtin_ctzll(o);
        if (w != 0 && w != bd) {
#pragma unroll
            for (int j = 0; j < 64; j++) s[j] >>= w;
        }
        R.waste = w;
    }
    const uint32_t bps = bd - R.waste;

    // history: the 4 samples before this lane's chunk (lane 0: zeros; its i<k terms are masked)
    ST h1 = __shfl_up(s[63], 1), h2 = __shfl_up(s[62], 1), h3 = __shfl_up(s[61], 1), h4 = __shfl_up(s[60], 1);
    if (l == 0) h1 = h2 = h3 = h4 = 0;

    // ---- 4. CONSTANT / VERBATIM defaults (encoder.zig:493-514)
    bool try_fixed = false;
    if (bps == 0) {
        R.type = 0;
        R.est = 0;
    } else {
        const ST x0 = (ST)__shfl(s[0], 0);
        bool eq = true;
#pragma unroll
        for (int j = 0; j < 64; j++) eq &= (s[j] == x0) || (!FULL && l * 64u + j >= n);
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

    uint32_t k = 0;
    if (try_fixed) {
        // ---- 5. bestOrder (fixed.zig:85-167)
        uint64_t T[5];
        if constexpr (CLS != 32) {
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
            T0 += t0; T1 += t1; T2 += t2; T3 += t3; T4 += t4;
            T[0] = wave_sum(T0); T[1] = wave_sum(T1); T[2] = wave_sum(T2); T[3] = wave_sum(T3); T[4] = wave_sum(T4);
        } else {
            // wide path (i64): an order is invalid if any |e| exceeds i32 (fixed.zig:160-162);
            // applying the check for bps' < 28 too is a no-op there, so one path serves both
            int64_t p0 = h1, p1 = h1 - h2, p2 = h1 - 2 * h2 + h3, p3 = h1 - 3 * h2 + 3 * h3 - h4;
            uint64_t A0 = 0, A1 = 0, A2 = 0, A3 = 0, A4 = 0, O0 = 0, O1 = 0, O2 = 0, O3 = 0, O4 = 0;
#pragma unroll
            for (int j = 0; j < 64; j++) {
                const bool valid = FULL || (l * 64u + j < n);
                const bool z = (l == 0);
                const int64_t e0 = s[j], e1 = e0 - p0, e2 = e1 - p1, e3 = e2 - p2, e4 = e3 - p3;
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
            }
            T[0] = wave_or(O0) > 0x7FFFFFFFull ? ~0ull : wave_sum(A0);
            T[1] = wave_or(O1) > 0x7FFFFFFFull ? ~0ull : wave_sum(A1);
            T[2] = wave_or(O2) > 0x7FFFFFFFull ? ~0ull : wave_sum(A2);
            T[3] = wave_or(O3) > 0x7FFFFFFFull ? ~0ull : wave_sum(A3);
            T[4] = wave_or(O4) > 0x7FFFFFFFull ? ~0ull : wave_sum(A4);
        }
        k = 0;
#pragma unroll
        for (int q = 1; q < 5; q++)
            if (T[q] < T[k]) k = q;  // first minimum (fixed.zig:164)
        if (CLS == 32 && T[k] == ~0ull) try_fixed = false;  // null -> VERBATIM (encoder.zig:520)
    }

    if (try_fixed) {
        // ---- 6. residuals in place, s[j] := e_k (lane 0 keeps its k warm-up samples),
        // and the finest-level partition sums (rice.zig:288-340)
        SumT S8[4] = {0, 0, 0, 0};
        uint32_t O8[4] = {0, 0, 0, 0};
        uint64_t *psum = nullptr;
        uint32_t *pmax = nullptr;
        uint32_t P = a.max_part_order, ps = 0;
        if constexpr (!FULL) {
            // caps of rice.calcParams (rice.zig:97-103).  The while-clamp only changes the
            // reference's result where it would slice res[k..ps] with ps < k (UB there).
            const uint32_t lim = k ? (31u - __builtin_clz(n)) - (31u - __builtin_clz(k)) : 15u;
            const uint32_t ctzn = (uint32_t)__builtin_ctz(n);
            if (ctzn < P) P = ctzn;
            if (lim < P) P = lim;
            while (P > 0 && (n >> P) < k) P--;
            ps = n >> P;
            psum = (uint64_t *)(smem + LY.psum) + wave * 512u;
            pmax = (uint32_t *)(smem + LY.pmax) + wave * 512u;
            for (uint32_t i = l; i < 512u; i += 64) {
                psum[i] = 0;
                pmax[i] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        {
            ST q1 = h1, q2 = h2, q3 = h3, q4 = h4;
            auto body = [&](auto KK) {
                constexpr int K = decltype(KK)::value;
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const ST x = s[j];
                    const ST r = fixed_residual<K, ST>(x, q1, q2, q3, q4);
                    q4 = q3; q3 = q2; q2 = q1; q1 = x;
                    const bool warm = (l == 0 && j < K);
                    if (!warm) s[j] = r;
                    const uint32_t zz = zigzag32((int32_t)r);
                    const uint32_t av = (zz >> 1) + (zz & 1u);  // |r|
                    if constexpr (FULL) {
                        S8[j >> 4] += warm ? 0u : av;
                        O8[j >> 4] |= warm ? 0u : zz;
                    } else {
                        const uint32_t i = l * 64u + j;
                        if (!warm && i < n) {
                            const uint32_t pid = i / ps;
                            atomicAdd((unsigned long long *)&psum[pid], (unsigned long long)av);
                            atomicOr(&pmax[pid], zz);
                        }
                    }
                }
            };
            switch (k) {
                case 0: body(std::integral_constant<int, 0>()); break;
                case 1: body(std::integral_constant<int, 1>()); break;
                case 2: body(std::integral_constant<int, 2>()); break;
                case 3: body(std::integral_constant<int, 3>()); break;
                default: body(std::integral_constant<int, 4>()); break;
            }
        }

        // ---- 7. parameter search for every partition order (rice.zig:248-279,343-395)
        const uint32_t capp = bps > 16 ? 30u : 14u;
        const uint32_t maxp = capp < a.max_param ? capp : a.max_param;
        uint64_t tots[9];
        uint32_t fives[9];
        if constexpr (FULL) {
            uint32_t W8[4];
#pragma unroll
            for (int q = 0; q < 4; q++) W8[q] = bitlen32(O8[q]);
            const uint64_t S7a = (uint64_t)S8[0] + S8[1], S7b = (uint64_t)S8[2] + S8[3];
            const uint32_t W7a = max(W8[0], W8[1]), W7b = max(W8[2], W8[3]);
            const uint64_t S6 = S7a + S7b;
            const uint32_t W6 = max(W7a, W7b);
            uint64_t Sl[6];
            uint32_t Wl[6];
            {
                uint64_t Sg = S6;
                uint32_t Wg = W6;
#pragma unroll
                for (int m = 0; m < 6; m++) {  // Sl[m]: level 5-m, partition spans 2^(m+1) lanes
                    Sg += __shfl_xor(Sg, 1 << m);
                    Wg = max(Wg, (uint32_t)__shfl_xor((int)Wg, 1 << m));
                    Sl[m] = Sg;
                    Wl[m] = Wg;
                }
            }
#pragma unroll
            for (int o = 0; o < 9; o++) {
              if ((uint32_t)o <= P) {
                uint32_t cost = 0;
                bool five = false;
                if (o >= 6) {
                    const int per = 1 << (o - 6);
#pragma unroll
                    for (int q = 0; q < per; q++) {
                        uint64_t S;
                        uint32_t W;
                        if (o == 8) { S = S8[q]; W = W8[q]; }
                        else if (o == 7) { S = q ? S7b : S7a; W = q ? W7b : W7a; }
                        else { S = S6; W = W6; }
                        const uint32_t j = l * per + q;
                        const uint32_t len = (4096u >> o) - (j == 0 ? k : 0u);
                        uint32_t c, p;
                        rice_choose(S, len, W, maxp, &c, &p);
                        cost += c;
                        five |= (p < 0x80u && p > 14u);
                        par[(1u << o) - 1u + j] = (uint8_t)p;
                    }
                } else {
                    const int g = 6 - o;  // a partition spans 2^g lanes
                    const uint32_t j = l >> g;
                    const bool lead = (l & ((1u << g) - 1u)) == 0;
                    const uint32_t len = (4096u >> o) - (j == 0 ? k : 0u);
                    uint32_t c, p;
                    rice_choose(Sl[g - 1], len, Wl[g - 1], maxp, &c, &p);
                    if (lead) {
                        cost = c;
                        five = (p < 0x80u && p > 14u);
                        par[(1u << o) - 1u + j] = (uint8_t)p;
                    }
                }
                tots[o] = wave_sum((uint64_t)cost);
                fives[o] = (maxp > 14u && __any(five)) ? 1u : 0u;
              }
            }
        } else {
            uint64_t *cs = psum, *ns = psum + 256;
            uint32_t *cm = pmax, *nm = pmax + 256;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (int o = 8; o >= 0; o--) {
              if ((uint32_t)o <= P) {
                const uint32_t np = 1u << o, len_full = n >> o;
                uint32_t cost = 0;
                bool five = false;
                for (uint32_t j = l; j < np; j += 64) {
                    const uint32_t len = len_full - (j == 0 ? k : 0u);
                    uint32_t c, p;
                    rice_choose(cs[j], len, bitlen32(cm[j]), maxp, &c, &p);
                    cost += c;
                    five |= (p < 0x80u && p > 14u);
                    par[np - 1u + j] = (uint8_t)p;
                }
                tots[o] = wave_sum((uint64_t)cost);
                fives[o] = (maxp > 14u && __any(five)) ? 1u : 0u;
                if (o > 0) {
                    for (uint32_t j = l; j < (np >> 1); j += 64) {
                        ns[j] = cs[2 * j] + cs[2 * j + 1];
                        nm[j] = cm[2 * j] | cm[2 * j + 1];
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    uint64_t *ts = cs; cs = ns; ns = ts;
                    uint32_t *tm = cm; cm = nm; nm = tm;
                }
              }
            }
        }
        uint64_t best = ~0ull;
        uint32_t best_o = 0, best_m = 0;
#pragma unroll
        for (int o = 0; o < 9; o++) {
            const uint64_t tot = tots[o] + ((uint64_t)(4u + fives[o]) << o);
            if ((uint32_t)o <= P && tot <= best) {  // ascending orders, "<=": the higher order wins ties (rice.zig:271)
                best = tot;
                best_o = (uint32_t)o;
                best_m = fives[o];
            }
        }

        // ---- 8. FIXED iff its estimate < the verbatim estimate (encoder.zig:538)
        if (best < R.est) {
            R.type = 2;
            R.est = best;
            R.order = k;
            R.porder = best_o;
            R.method = best_m;
        } else {
            // verbatim needs the samples back: invert the residual recurrence
            ST q1 = h1, q2 = h2, q3 = h3, q4 = h4;
#pragma unroll
            for (int j = 0; j < 64; j++) {
                const bool warm = (l == 0 && (uint32_t)j < k);
                const ST x = warm ? s[j] : fixed_restore(k, s[j], q1, q2, q3, q4);
                s[j] = x;
                q4 = q3; q3 = q2; q2 = q1; q1 = x;
            }
        }
    }

    // ---- 9. publish the candidate record
    if (l == 0) {
        uint32_t *rc = recs + cand * 16u;
        rc[0] = R.type; rc[1] = R.waste; rc[2] = R.bd; rc[3] = R.order; rc[4] = R.porder; rc[5] = R.method;
        rc[6] = (uint32_t)R.est; rc[7] = (uint32_t)(R.est >> 32);
    }
    __syncthreads();
    // zero the frame image (region 0)
    for (uint32_t i = tid; i < (a.image_bytes >> 4); i += NT) ((uint4 *)img)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();

    // ---- 10. stereo decision (encoder.zig:441-452) or independent channels (:456-475)
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
        channel_code = C - 1u;
        n_out = C;
        my_slot = (int)cand;
    }
    if (tid == 0) misc[16] = 8u * write_frame_header(img, job.number, a.bits, channel_code, n, a.sample_rate);

    // ---- 11. exact subframe lengths (pass A), frame_writer.zig:269-372
    uint32_t lane_off = 0;
    uint32_t pq[4] = {0, 0, 0, 0};
    const uint32_t param_len = 4u + R.method;
    const uint32_t w = R.waste;
    k = R.order;
    const uint8_t *pp = par + ((1u << R.porder) - 1u);
    if (my_slot >= 0) {
        uint32_t seg = 0;
        if (R.type == 0) {
            seg = (l == 0) ? 8u + bd : 0u;
        } else if (R.type == 1) {
            const uint32_t cnt = FULL ? 64u : (n > l * 64u ? min(64u, n - l * 64u) : 0u);
            seg = cnt * bps + ((l == 0) ? 8u + w : 0u);
        } else {
            const uint32_t o = R.porder;
            if (l == 0) {
                const uint32_t p0 = pp[0];
                seg = 8u + w + k * bps + 6u + param_len + ((p0 & 0x80u) ? 5u : 0u);
            }
            if constexpr (FULL) {
                const uint32_t sh = 12u - o, psz = 4096u >> o;
#pragma unroll
                for (int q = 0; q < 4; q++) pq[q] = pp[(l * 64u + 16u * q) >> sh];
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const uint32_t p = pq[j >> 4];
                    const bool esc = (p & 0x80u) != 0;
                    const uint32_t i = l * 64u + j;
                    if ((j & 15) == 0 && i != 0 && (i & (psz - 1u)) == 0) seg += param_len + (esc ? 5u : 0u);
                    const bool warm = (l == 0 && (uint32_t)j < k);
                    const uint32_t zz = zigzag32((int32_t)s[j]);
                    const uint32_t cl = esc ? (p & 0x7Fu) : (zz >> p) + 1u + p;
                    seg += warm ? 0u : cl;
                }
            } else {
                const uint32_t psz = n >> o;
                for (int j = 0; j < 64; j++) {
                    const uint32_t i = l * 64u + j;
                    if (i >= n) break;
                    if (l == 0 && (uint32_t)j < k) continue;
                    const uint32_t p = pp[i / psz];
                    const bool esc = (p & 0x80u) != 0;
                    if (i != 0 && (i % psz) == 0) seg += param_len + (esc ? 5u : 0u);
                    const uint32_t zz = zigzag32((int32_t)s[j]);
                    seg += esc ? (p & 0x7Fu) : (zz >> p) + 1u + p;
                }
            }
        }
        uint32_t total;
        lane_off = wave_excl_scan(seg, &total);
        if (l == 0) misc[my_slot] = total;
    }
    __syncthreads();

    uint32_t total_bits = misc[16];
    uint32_t sub_start = total_bits;
    for (uint32_t i = 0; i < n_out; i++) {
        if ((int)i < my_slot) sub_start += misc[i];
        total_bits += misc[i];
    }

    // ---- 12. pack (pass B)
    if (my_slot >= 0) {
        uint32_t pos = sub_start + lane_off;
        if (R.type == 0) {
            if (l == 0) {  // writeConstantSubframe: header 0x00, value << waste in bd bits (no wasted flag)
                const uint64_t v = ((uint64_t)R.cval << w) & (~0ull >> (64 - bd));
                put_bits(img, pos + 8u, v, bd);
            }
        } else {
            const uint64_t mask = ~0ull >> (64 - bps);
            if (l == 0) {
                const uint32_t hdr = (R.type == 1) ? (w ? 0x03u : 0x02u) : (((8u | k) << 1) | (w ? 1u : 0u));
                put_bits(img, pos, hdr, 8);
                pos += 8;
                if (w) {
                    put_bits(img, pos, 1, w);
                    pos += w;
                }
            }
            if (R.type == 1) {
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    if (FULL || l * 64u + j < n) {
                        put_bits(img, pos, (uint64_t)(int64_t)s[j] & mask, bps);
                        pos += bps;
                    }
                }
            } else {
                const uint32_t o = R.porder;
                auto part_header = [&](uint32_t p) {
                    if (p & 0x80u) {
                        put_bits(img, pos, 0x0Fu | (R.method << 4), param_len);
                        put_bits(img, pos + param_len, p & 0x7Fu, 5);
                        pos += param_len + 5u;
                    } else {
                        put_bits(img, pos, p, param_len);
                        pos += param_len;
                    }
                };
                if (l == 0) {
#pragma unroll
                    for (int j = 0; j < 4; j++) {  // warm-up samples
                        if ((uint32_t)j < k) {
                            put_bits(img, pos, (uint64_t)(int64_t)s[j] & mask, bps);
                            pos += bps;
                        }
                    }
                    put_bits(img, pos, (R.method << 4) | o, 6);
                    pos += 6;
                    part_header(pp[0]);
                }
                auto code = [&](int32_t r, uint32_t p) {
                    const uint32_t zz = zigzag32(r);
                    if (p & 0x80u) {
                        const uint32_t len = p & 0x7Fu;
                        if (len) put_bits(img, pos, (uint64_t)(uint32_t)r & (~0ull >> (64 - len)), len);
                        pos += len;
                    } else {
                        const uint32_t skip = zz >> p;
                        put_bits(img, pos + skip, (1ull << p) | (zz & ((1u << p) - 1u)), p + 1u);
                        pos += skip + p + 1u;
                    }
                };
                if constexpr (FULL) {
                    const uint32_t psz = 4096u >> o;
#pragma unroll
                    for (int j = 0; j < 64; j++) {
                        const uint32_t i = l * 64u + j;
                        if ((j & 15) == 0 && i != 0 && (i & (psz - 1u)) == 0) part_header(pq[j >> 4]);
                        if (!(l == 0 && (uint32_t)j < k)) code((int32_t)s[j], pq[j >> 4]);
                    }
                } else {
                    const uint32_t psz = n >> o;
                    for (int j = 0; j < 64; j++) {
                        const uint32_t i = l * 64u + j;
                        if (i >= n) break;
                        if (l == 0 && (uint32_t)j < k) continue;
                        const uint32_t p = pp[i / psz];
                        if (i != 0 && (i % psz) == 0) part_header(p);
                        code((int32_t)s[j], p);
                    }
                }
            }
        }
    }
    __syncthreads();

    // ---- 13. CRC-16 of the frame (frame_writer.zig:111-125,144-148): the word stream
    // is front-padded with zero words (a no-op for init-0 CRC) to NT*SW words; thread t
    // folds its SW words, then its CRC is shifted by z^(32*SW*(NT-1-t)) and XOR-reduced.
    const uint32_t Lb = (total_bits + 7u) >> 3;
    const uint32_t W4 = Lb >> 2;
    {
        const uint32_t SW = a.crc_seg_words;
        const int32_t Z = (int32_t)(NT * SW) - (int32_t)W4;
        uint32_t crc = 0;
        const int32_t v0 = (int32_t)(tid * SW) - Z;
        for (uint32_t i = 0; i < SW; i++) {
            const int32_t rw = v0 + (int32_t)i;
            if (rw >= 0) crc = crc_word(crc, img[rw], crct);
        }
        uint32_t contrib = crc ? crc_mulmod(crc, a.crc_pow[tid]) : 0u;
        contrib = wave_xor(contrib);
        if (l == 0) misc[24 + wave] = contrib;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t crc = 0;
        for (uint32_t i = 0; i < NW; i++) crc ^= misc[24 + i];
        for (uint32_t b = W4 * 4u; b < Lb; b++) crc = crc_byte(crc, (img[b >> 2] >> (24 - 8 * (b & 3))) & 255u, crct);
        put_bits(img, Lb * 8u, crc, 16);
        const uint32_t fbytes = Lb + 2u;
        if (fbytes + 16u > a.slot_bytes || fbytes > a.image_bytes) atomicOr(a.err, 1u);
        a.frame_bytes[job.slot] = fbytes;
        misc[17] = fbytes;
    }
    __syncthreads();

    // ---- 14. frame image -> its slot (big-endian words to bytes)
    {
        const uint32_t fbytes = misc[17];
        const uint32_t units = min((fbytes + 15u) >> 4, a.slot_bytes >> 4);
        uint4 *dst = (uint4 *)(a.slots + (uint64_t)job.slot * a.slot_bytes);
        for (uint32_t u = tid; u < units; u += NT) {
            uint4 v = ((const uint4 *)img)[u];
            v.x = __builtin_bswap32(v.x);
            v.y = __builtin_bswap32(v.y);
            v.z = __builtin_bswap32(v.z);
            v.w = __builtin_bswap32(v.w);
            dst[u] = v;
        }
    }

    // ---- 15. optional decision records (parity tests)
    if (a.records) {
        FrameRec *fr = a.records + job.slot;
        SubRec *sr = &fr->cand[cand];
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
        }
        const uint32_t np = 1u << R.porder;
        for (uint32_t j = l; j < 256u; j += 64) sr->params[j] = (R.type == 2 && j < np) ? pp[j] : 0;
        if (tid == 0) {
            fr->channel_code = channel_code;
            fr->n_cand = NW;
            fr->frame_bytes = misc[17];
            fr->pad = 0;
        }
    }
}

// ------------------------------------------------------------------------
// frame table for one contiguous stream (wav2flac.zig:66-97)
// ------------------------------------------------------------------------
__global__ void k_make_jobs(FrameJob *jobs, uint64_t n_samples, uint32_t block, uint32_t frame_stride_bytes,
                            uint64_t first_number, uint32_t n_frames) {
    uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    uint64_t start = (uint64_t)f * block;
    uint64_t rem = n_samples - start;
    FrameJob j;
    j.pcm_off = (uint64_t)f * frame_stride_bytes;
    j.number = first_number + f;
    j.n = (uint32_t)(rem < block ? rem : block);
    j.slot = f;
    jobs[f] = j;
}

// ------------------------------------------------------------------------
// exclusive scan of frame sizes -> byte offsets (single workgroup, 1024 thr)
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_scan(const uint32_t *sizes, uint64_t *offsets, uint64_t *total, uint32_t n) {
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x, per = (n + 1023u) / 1024u;
    const uint32_t b = t * per, e = min(n, b + per);
    uint64_t acc = 0;
    for (uint32_t i = b; i < e; i++) acc += sizes[i];
    // block exclusive scan of acc
    uint64_t x = acc;
    const uint32_t l = lane_id(), w = t >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x += y;
    }
    if (l == 63) wsum[w] = x;
    __syncthreads();
    uint64_t pre = 0;
    for (uint32_t i = 0; i < w; i++) pre += wsum[i];
    uint64_t run = pre + x - acc;
    for (uint32_t i = b; i < e; i++) {
        offsets[i] = run;
        run += sizes[i];
    }
    if (t == 1023) {
        uint64_t tot = 0;
        for (int i = 0; i < 16; i++) tot += wsum[i];
        *total = tot;
    }
}

// ------------------------------------------------------------------------
// compaction: frame slots -> contiguous byte stream
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_compact(const uint8_t *slots, uint32_t slot_bytes, const uint32_t *sizes,
                                                 const uint64_t *offsets, uint8_t *out, uint64_t out_cap, uint32_t *err) {
    const uint32_t f = blockIdx.x;
    const uint64_t D = offsets[f];
    const uint32_t len = sizes[f];
    if (D + len > out_cap) {
        if (threadIdx.x == 0) atomicOr(err, 2u);
        return;
    }
    const uint8_t *src = slots + (uint64_t)f * slot_bytes;
    const uint64_t E = D + len;
    const uint64_t w0 = (D + 3) >> 2, w1 = E >> 2;  // fully covered dwords [w0, w1)
    uint32_t *o32 = (uint32_t *)out;
    const uint32_t *s32 = (const uint32_t *)src;
    if (w1 > w0) {
        const uint32_t sh = (uint32_t)((4 * w0 - D) & 3);  // source byte offset of dword w0 is 4*w0 - D
        const uint64_t sbase = 4 * w0 - D;
        for (uint64_t w = w0 + threadIdx.x; w < w1; w += blockDim.x) {
            const uint64_t sb = sbase + 4 * (w - w0);
            const uint32_t lo = s32[sb >> 2];
            uint32_t v = lo;
            if (sh) {
                const uint32_t hi = s32[(sb >> 2) + 1];
                v = __builtin_amdgcn_alignbyte(hi, lo, sh);
            }
            o32[w] = v;
        }
        if (threadIdx.x < 8) {
            // head bytes [D, 4*w0) and tail bytes [4*w1, E)
            uint64_t b = threadIdx.x < 4 ? D + threadIdx.x : 4 * w1 + (threadIdx.x - 4);
            bool ok = threadIdx.x < 4 ? (b < 4 * w0) : (b < E);
            if (ok) out[b] = src[b - D];
        }
    } else {
        for (uint64_t b = D + threadIdx.x; b < E; b += blockDim.x) out[b] = src[b - D];
    }
}

// ------------------------------------------------------------------------
// MD5 (md5.zig / RFC 1321): one lane per independent stream
// ------------------------------------------------------------------------
constexpr uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

#define MD5_STEP(F, a, b, c, d, m, k, s) a = b + rotl(a + F(b, c, d) + (m) + (k), s)
#define MD5_F(b, c, d) (((b) & (c)) | (~(b) & (d)))
#define MD5_G(b, c, d) (((b) & (d)) | ((c) & ~(d)))
#define MD5_H(b, c, d) ((b) ^ (c) ^ (d))
#define MD5_I(b, c, d) ((c) ^ ((b) | ~(d)))

__device__ __forceinline__ void md5_compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        MD5_STEP(MD5_F, a, b, c, d, m[i + 0], kMd5K[i + 0], 7);
        MD5_STEP(MD5_F, d, a, b, c, m[i + 1], kMd5K[i + 1], 12);
        MD5_STEP(MD5_F, c, d, a, b, m[i + 2], kMd5K[i + 2], 17);
        MD5_STEP(MD5_F, b, c, d, a, m[i + 3], kMd5K[i + 3], 22);
    }
#pragma unroll
    for (int i = 16; i < 32; i += 4) {
        MD5_STEP(MD5_G, a, b, c, d, m[(5 * i + 1) & 15], kMd5K[i + 0], 5);
        MD5_STEP(MD5_G, d, a, b, c, m[(5 * i + 6) & 15], kMd5K[i + 1], 9);
        MD5_STEP(MD5_G, c, d, a, b, m[(5 * i + 11) & 15], kMd5K[i + 2], 14);
        MD5_STEP(MD5_G, b, c, d, a, m[(5 * i + 16) & 15], kMd5K[i + 3], 20);
    }
#pragma unroll
    for (int i = 32; i < 48; i += 4) {
        MD5_STEP(MD5_H, a, b, c, d, m[(3 * i + 5) & 15], kMd5K[i + 0], 4);
        MD5_STEP(MD5_H, d, a, b, c, m[(3 * i + 8) & 15], kMd5K[i + 1], 11);
        MD5_STEP(MD5_H, c, d, a, b, m[(3 * i + 11) & 15], kMd5K[i + 2], 16);
        MD5_STEP(MD5_H, b, c, d, a, m[(3 * i + 14) & 15], kMd5K[i + 3], 23);
    }
#pragma unroll
    for (int i = 48; i < 64; i += 4) {
        MD5_STEP(MD5_I, a, b, c, d, m[(7 * i) & 15], kMd5K[i + 0], 6);
        MD5_STEP(MD5_I, d, a, b, c, m[(7 * i + 7) & 15], kMd5K[i + 1], 10);
        MD5_STEP(MD5_I, c, d, a, b, m[(7 * i + 14) & 15], kMd5K[i + 2], 15);
        MD5_STEP(MD5_I, b, c, d, a, m[(7 * i + 21) & 15], kMd5K[i + 3], 21);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// Full digest of n_streams independent byte ranges (offsets 4-byte aligned).
__global__ void __launch_bounds__(64) k_md5_streams(const uint8_t *base, const uint64_t *offs, const uint64_t *lens,
                                                    uint32_t n_streams, uint8_t *digests) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_streams) return;
    const uint8_t *p = base + offs[s];
    const uint64_t len = lens[s];
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const uint64_t full = len >> 6;
    const uint32_t *p32 = (const uint32_t *)p;
    for (uint64_t b = 0; b < full; b++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = p32[b * 16 + i];
        md5_compress(st, m);
    }
    // tail + padding (one or two blocks), assembled straight into message words
    const uint32_t rem = (uint32_t)(len & 63);
    const uint8_t *tp = p + full * 64;
    const uint32_t nb = rem < 56 ? 1u : 2u;
    const uint64_t bits = len * 8;
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t idx = b * 64u + 4u * i + q;
                uint32_t by = idx < rem ? tp[idx] : (idx == rem ? 0x80u : 0u);
                if (b == nb - 1 && 4 * i + q >= 56) by = (uint32_t)(bits >> (8 * (4 * i + q - 56))) & 255u;
                v |= by << (8 * q);
            }
            m[i] = v;
        }
        md5_compress(st, m);
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) digests[16 * s + 4 * i + j] = (uint8_t)(st[i] >> (8 * j));
}

// Streaming update of one MD5 state in device memory by whole 64-byte blocks.
__global__ void k_md5_blocks(uint32_t *state, const uint32_t *blocks, uint64_t n_blocks) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t st[4] = {state[0], state[1], state[2], state[3]};
    for (uint64_t b = 0; b < n_blocks; b++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = blocks[b * 16 + i];
        md5_compress(st, m);
    }
    for (int i = 0; i < 4; i++) state[i] = st[i];
}

// ------------------------------------------------------------------------
// host-side launch wrappers (called from fg_api.cpp)
// ------------------------------------------------------------------------
template <int B, int CLS, bool FULL>
static hipError_t launch_encode_t(const EncodeArgs &a, uint32_t threads, uint32_t lds, hipStream_t st) {
    auto k = k_encode<B, CLS, FULL>;
    hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(a.n_jobs), dim3(threads), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_encode(const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    const uint32_t B = a.bytes_per_sample;
    const int cls = a.bits <= 16 ? 16 : (a.bits <= 24 ? 24 : 32);
#define FG_CASE(BB, CC)                                                            \
    if (B == BB && cls == CC)                                                      \
        return full ? launch_encode_t<BB, CC, true>(a, threads, lds, st)           \
                    : launch_encode_t<BB, CC, false>(a, threads, lds, st);
    FG_CASE(1, 16)
    FG_CASE(2, 16)
    FG_CASE(3, 24)
    FG_CASE(4, 32)
#undef FG_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_make_jobs(FrameJob *jobs, uint64_t n_samples, uint32_t block, uint32_t stride, uint64_t first,
                            uint32_t n_frames, hipStream_t st) {
    if (n_frames == 0) return hipSuccess;
    hipLaunchKernelGGL(k_make_jobs, dim3((n_frames + 255) / 256), dim3(256), 0, st, jobs, n_samples, block, stride,
                       first, n_frames);
    return hipGetLastError();
}

hipError_t launch_scan(const uint32_t *sizes, uint64_t *offsets, uint64_t *total, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, sizes, offsets, total, n);
    return hipGetLastError();
}

hipError_t launch_compact(const uint8_t *slots, uint32_t slot_bytes, const uint32_t *sizes, const uint64_t *offsets,
                          uint8_t *out, uint64_t out_cap, uint32_t *err, uint32_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3(n), dim3(256), 0, st, slots, slot_bytes, sizes, offsets, out, out_cap, err);
    return hipGetLastError();
}

hipError_t launch_md5_streams(const uint8_t *base, const uint64_t *offs, const uint64_t *lens, uint32_t n,
                              uint8_t *digests, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_md5_streams, dim3((n + 63) / 64), dim3(64), 0, st, base, offs, lens, n, digests);
    return hipGetLastError();
}

hipError_t launch_md5_blocks(uint32_t *state, const uint32_t *blocks, uint64_t n_blocks, hipStream_t st) {
    hipLaunchKernelGGL(k_md5_blocks, dim3(1), dim3(64), 0, st, state, blocks, n_blocks);
    return hipGetLastError();
}

}  // namespace fg
