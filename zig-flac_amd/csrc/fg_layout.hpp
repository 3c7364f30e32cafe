// fg_layout.hpp -- LDS layout and size bounds shared by host and device.
#pragma once
#include <stdint.h>

#include "fg_common.hpp"

namespace fg {

// Analysis kernel (one wave per candidate, nw waves).
struct AnaLayout {
    uint32_t stage0; // PCM staging: 64 padded chunks
    uint32_t stage1; // second staging buffer (double-buffered LDS-DMA prefetch), or == stage0
    uint32_t psum;   // tail kernel only: 256 u64 per wave (levels combined in place)
    uint32_t pmax;   // tail kernel only: 256 u32 per wave
    uint32_t par;    // rice params, 512 B per candidate wave (orders 0..8 at offset (1<<o)-1);
                     // with LPC two such buffers per wave (current best / candidate)
    uint32_t par_stride;
    uint32_t lpc;    // LPC: quantised coefficient table, kLpcTab i32 per wave
    uint32_t rec;    // 16 x u32 per candidate wave
    uint32_t misc;   // 64 x u32 scratch (header words)
    uint32_t lbits;  // fused encode: 2 x 64 u32 segment bits of the written subframes (== total without)
    uint32_t total;
};

// Pack kernel (one wave per written subframe): staging, then the frame image.
struct PackLayout {
    uint32_t buf0;   // PCM staging of a frame, then (aliasing it) the frame image (big-endian words)
    uint32_t buf1;   // second buffer: the next frame's PCM arrives by LDS-DMA (== buf0 without)
    uint32_t misc;   // 64 x u32 scratch (crc partials)
    uint32_t dsc;    // k_packw: two LDS copies of a frame descriptor's fields (packw_dsc_dw each)
    uint32_t total;
};

__host__ __device__ inline uint32_t fg_round16(uint32_t x) { return (x + 15u) & ~15u; }

// Staging: 64 chunks (one per lane) of 16*C*B dwords.  16-bit stereo: blocks of 4
// chunks, 1088 B apart, each block the 1 KiB destination of one 16-B LDS-DMA
// instruction with the chunks' 16-B groups interleaved (group g of chunk 4b + c at
// byte 64g + 16c of block b); lane l then reads group g at a per-lane base plus the
// immediate 64g, and a quarter-wave's 16 ds_read_b128 cover all 64 banks (the 64-B
// block pad staggers the four blocks).  Otherwise a pad makes the per-lane reads
// conflict free: 32-bit stereo reads ds_read_b64 (pad 2 dwords), the rest one sample
// at a time (pad 1).  Either way 64 * (16*C*B + pad) dwords.
__host__ __device__ inline bool stage_ilv(uint32_t C, uint32_t B) { return C == 2 && B == 2; }
__host__ __device__ inline uint32_t stage_pad(uint32_t C, uint32_t B) {
    return stage_ilv(C, B) ? 4u : ((C == 2 && B == 4) ? 2u : 1u);
}
__host__ __device__ inline uint32_t stage_bytes(uint32_t C, uint32_t B) {
    return 64u * (16u * C * B + stage_pad(C, B)) * 4u;
}

// The staged PCM of a frame stays valid for the whole analysis (the chosen
// candidate's residuals are recomputed from it for the exact-length pass).
// The full-frame kernel double-buffers it when both buffers fit and DMAs the
// next frame's PCM into the idle one; the tail kernel (and configs whose two
// buffers do not fit) stage synchronously into one buffer.
// fused_img != 0 (the fused encode, fg_fused.hpp): the single staging buffer also holds the frame
// image of that many bytes, and lbits follows misc
__host__ __device__ inline AnaLayout ana_layout(uint32_t C, uint32_t B, uint32_t nw, bool full, bool dbuf,
                                                bool lpc = false, uint32_t fused_img = 0) {
    AnaLayout L;
    uint32_t sb = fg_round16(stage_bytes(C, B));
    if (fused_img > sb) sb = fg_round16(fused_img);
    uint32_t end = sb;
    L.stage0 = L.stage1 = 0;
    if (full && dbuf) {
        L.stage1 = sb;
        end = 2u * sb;
    }
    L.psum = L.pmax = end;
    if (!full) {
        L.pmax = end + nw * 2048u;
        end += nw * 3072u;
    }
    L.par = end;
    L.par_stride = lpc ? 1024u : 512u;
    L.lpc = L.par + nw * L.par_stride;
    L.rec = L.lpc + (lpc ? nw * 4u * (uint32_t)kLpcTab : 0u);
    L.misc = L.rec + nw * 64u;
    L.lbits = L.misc + 256u;
    L.total = fg_round16(L.lbits + (fused_img ? 512u : 0u));
    return L;
}

__host__ __device__ inline PackLayout pack_layout(uint32_t C, uint32_t B, uint32_t image_bytes, bool dbuf) {
    PackLayout L;
    uint32_t r0 = stage_bytes(C, B);
    if (image_bytes > r0) r0 = image_bytes;
    r0 = fg_round16(r0);
    L.buf0 = 0;
    L.buf1 = dbuf ? r0 : 0u;
    // (until round 5 a 4-KiB CRC table area sat here; the table-free CRC of round 3 left it unused)
    L.misc = dbuf ? 2u * r0 : r0;
    L.dsc = L.misc + 256u;
    L.total = fg_round16(L.dsc);
    return L;
}

// k_ana1 (fg_ana1.hpp, one wave per frame): per-wave LDS of the four candidates' Rice parameters
// (512 B each, orders 0..8 at (1 << o) - 1), their decisions (8 u32 each), the frame header words
// (4) and its byte count.
struct Ana1Layout {
    static constexpr uint32_t par = 0, rec = 2048, hdr = 2048 + 128, total = 2048 + 128 + 32;
};

// k_pack4 (fg_pack4.hpp): two staging / image buffers, scratch, and two LDS copies of a frame
// descriptor (320 dwords each, DMA'd a frame ahead)
struct P4Layout {
    uint32_t buf0, buf1, misc, dsc0, dsc1, total;
};
__host__ __device__ inline P4Layout pack4_layout(uint32_t image_bytes) {
    P4Layout L;
    uint32_t r0 = stage_bytes(2, 2);
    if (image_bytes > r0) r0 = image_bytes;
    r0 = fg_round16(r0);
    L.buf0 = 0;
    L.buf1 = r0;
    L.misc = 2u * r0;
    L.dsc0 = L.misc + 256u;
    L.dsc1 = L.dsc0 + 1280u;
    L.total = fg_round16(L.dsc1 + 1280u);
    return L;
}

// k_packw staging (fg_packw.hpp): 64 chunks of 64 samples, each split into WPS sub-chunks of
// 64 / WPS samples (one lane's samples) followed by one pad word each, so the WPS lanes that read
// one chunk start in different banks (with the plain pad they would all hit one: a sub-chunk of
// 16 or 32 samples is a multiple of 32 words for 8-byte and 24-byte sample rows).
__host__ __device__ inline uint32_t packw_cst(uint32_t C, uint32_t B, uint32_t wps) { return 16u * C * B + wps; }
// k_packw's LDS copy of a frame descriptor (fg_packw.hpp, dsc_dma) for nh written subframes per
// workgroup: hc header chunks of 64 dwords (frame fields, the subframes' bit counts, the frame's
// offset, 11 fields per local subframe), then nh chunks of lane bit counts and nh of Rice
// parameters
__host__ __device__ inline uint32_t packw_dsc_hc(uint32_t nh) { return (18u + 11u * nh + 63u) / 64u; }
__host__ __device__ inline uint32_t packw_dsc_dw(uint32_t nh) { return 64u * (packw_dsc_hc(nh) + 2u * nh); }
__host__ __device__ inline PackLayout packw_layout(uint32_t C, uint32_t B, uint32_t wps, uint32_t image_bytes, bool dbuf,
                                                   uint32_t nh) {
    PackLayout L;
    uint32_t r0 = 64u * packw_cst(C, B, wps) * 4u;
    if (image_bytes > r0) r0 = image_bytes;
    r0 = fg_round16(r0);
    L.buf0 = 0;
    L.buf1 = dbuf ? r0 : 0u;
    // (until round 5 a 4-KiB CRC table area sat here; the table-free CRC of round 3 left it unused)
    L.misc = dbuf ? 2u * r0 : r0;
    L.dsc = L.misc + 256u;
    L.total = fg_round16(L.dsc + 2u * 4u * packw_dsc_dw(nh));
    return L;
}

// Upper bound (bytes) of one encoded frame, block n <= 4096:
// header <= 16 B; per subframe <= 14 + 4*bd + n*bd + n/2 bits (a FIXED subframe
// is chosen only when its estimate < n*bps', and the exact Rice length exceeds
// the estimate by at most floor(len/2) per partition); pad + CRC-16.
__host__ __device__ inline uint32_t frame_bound_bytes(uint32_t n, uint32_t C, uint32_t bits, bool stereo) {
    uint64_t b = 16u * 8u;
    for (uint32_t c = 0; c < C; c++) {
        uint32_t bd = bits + ((stereo && c == 1) ? 1u : 0u);
        b += 14u + 4u * bd + (uint64_t)n * bd + n / 2u;
    }
    return (uint32_t)((b + 7u) / 8u + 1u + 2u + 16u);
}

}  // namespace fg
