// fg_common.hpp -- POD types shared by the HIP kernels (fg_device.hpp,
// fg_misc.hip) and the host orchestration behind the C ABI (fg_api.cpp).
// gfx950 only.
#pragma once
#include <stdint.h>

// FG_DIAG=1 (`make diag`, build_diag/): the measured-slower alternatives (the one-wave analysis
// k_ana1, the fused single-pass kernel, the overlapped schedule) and the diagnostic environment
// knobs that can change what a call does (FLACGPU_FILES_MD5, issue priorities, grid reserves).
// The release library (FG_DIAG=0, the default) compiles none of them.
#ifndef FG_DIAG
#define FG_DIAG 0
#endif
#ifndef FG_C3_W
#define FG_C3_W 3  // waves per SIMD of the 24-bit LPC full-frame analysis (k_analyze; fg_api.cpp sizes its staging to match)
#endif

namespace fg {

constexpr int kBlock = 4096;       // Config.default block size (encoder.zig:644)
constexpr int kLaneSamples = 64;   // samples per lane: one wave == one 4096-sample subframe
constexpr int kMaxPartOrder = 8;   // rice.MAX_ORDER (rice.zig:13)
constexpr int kParamBytes = 512;   // params of all orders 0..8: offset (1<<o)-1 (511 used)
constexpr int kCrcThreadsMax = 512;
constexpr uint32_t kCtrSet = 32;    // u32 tickets per work_ctr set (reset_analysis_tickets)
constexpr uint32_t kMd5StreamsPerWg = 256;  // k_md5_streams workgroup size (one stream per lane)
// LPC (build-defined extension; the reference has none, readme.md:27): orders
// 1..12 on the GPU path (the FLAC subset limit), 15-bit coefficients.
constexpr int kLpcMax = 12;
constexpr int kLpcPrec = 15;
constexpr int kLpcTab = 160;       // i32 per wave: [12 orders][13] (12 coefs + shift)

// One frame of work.  pcm_off must be 4-byte aligned.
struct FrameJob {
    uint64_t pcm_off;   // byte offset of the frame's first interleaved sample
    uint64_t number;    // frame number written into the header (u36)
    uint32_t n;         // samples per channel in this frame (1..4096)
    uint32_t slot;      // output slot / frame index within the call
};

// Per-stream MD5 chaining state carried across calls (mirrors flacgpu_md5_state).
struct Md5State {
    uint32_t h[4];
    uint64_t bytes;     // message bytes absorbed so far
    uint32_t flags;     // 1 once the stream's final segment has been padded
    uint32_t pad;
};
static_assert(sizeof(Md5State) == 32, "Md5State layout");

// Per-candidate decision record (SubframeType.Encoding + estimate,
// encoder.zig:678-702).  Mirrors flacgpu_subframe_record.
struct SubRec {
    uint8_t type;       // 0 CONSTANT, 1 VERBATIM, 2 FIXED, 3 LPC
    uint8_t waste;
    uint8_t bits;
    uint8_t order;
    uint8_t part_order;
    uint8_t method;
    uint8_t written;
    uint8_t pad;
    uint32_t pad2;
    uint64_t estimate;
    int64_t constant;
    uint8_t params[256];
    uint8_t lpc_precision;
    int8_t lpc_shift;
    uint8_t pad3[6];
    int32_t lpc_coefs[32];
};

struct FrameRec {
    uint32_t channel_code;
    uint32_t n_cand;
    uint32_t frame_bytes;
    uint32_t pad;
    SubRec cand[8];
};

// Frame descriptor written by the analysis kernel and consumed by the pack
// kernel: everything needed to emit the frame's bits at its final byte offset
// without redoing the search.  Stride: desc_stride(n_out).
struct SubDesc {
    uint8_t type;        // 0 CONSTANT, 1 VERBATIM, 2 FIXED, 3 LPC
    uint8_t waste;
    uint8_t bd;          // bits of the (side: +1) channel before the waste shift
    uint8_t order;       // fixed / LPC predictor order (= warm-up samples)
    uint8_t porder;      // rice partition order
    uint8_t method;      // 0 RICE, 1 RICE2
    uint8_t cand;        // stereo: 0 L, 1 R, 2 M, 3 S; else the channel
    int8_t lpc_shift;    // LPC: quantisation shift
    uint32_t bits;       // exact subframe bits
    uint32_t lpc_prec;   // LPC: coefficient precision
    int64_t cval;        // CONSTANT value (after the waste shift)
    uint32_t lane_bits[64];  // bits of lane l's 64-sample segment (pass A)
    uint8_t params[256];     // rice params of the chosen order (0x80|w = escape)
    int16_t coef[kLpcMax];   // LPC: quantised coefficients
    uint8_t pad3[8];
};
static_assert(sizeof(SubDesc) == 568, "SubDesc layout");

struct FrameDesc {
    uint32_t hdr_bytes;     // frame header bytes incl. CRC-8
    uint32_t total_bits;    // header + subframes (before the byte pad)
    uint32_t channel_code;
    uint32_t n_out;         // subframes written
    uint32_t hdr[4];        // header bytes as big-endian words, zero past hdr_bytes
};
static_assert(sizeof(FrameDesc) == 32, "FrameDesc layout");

// descriptor of a frame: FrameDesc, n_out SubDesc, then 32 B of channel-half pack hand-off
// (k_packw split mode: the halves' CRC partials and shared byte, and the arrival ticket)
__host__ __device__ constexpr uint32_t desc_side_off(uint32_t n_out) { return 32u + n_out * (uint32_t)sizeof(SubDesc); }
__host__ __device__ constexpr uint32_t desc_stride(uint32_t n_out) { return desc_side_off(n_out) + 32u; }

struct EncodeArgs {
    const uint8_t *pcm;         // device PCM base
    const FrameJob *jobs;       // frame table
    uint32_t n_jobs;
    uint32_t channels;
    uint32_t bits;              // bits per sample (8/16/24/32)
    uint32_t bytes_per_sample;  // container bytes (== bits/8)
    uint32_t sample_rate;
    uint32_t stereo;            // 1: stereo decorrelation (channels == 2 && cfg flag)
    uint32_t max_part_order;    // 0..8
    uint32_t max_param;         // 1..30
    uint32_t block_size;        // stream block size (header field for short frames is n)
    uint32_t lpc_order;         // 0: fixed prediction only (the reference); 1..12: LPC search
    uint8_t *desc;              // frame descriptors [slot], desc_stride bytes each
    uint32_t desc_stride;
    uint32_t image_bytes;       // pack kernel LDS frame-image bytes (multiple of 16, >= bound + 16)
    uint32_t stage_dbuf;        // full-frame analysis kernel: double-buffered staging (LDS-DMA prefetch)
    uint32_t pack_dbuf;         // full-frame pack kernel: the same
    uint32_t *frame_bytes;      // [slot] exact frame bytes (analysis kernel)
    const uint64_t *offsets;    // [slot] byte offset of the frame in out (scan)
    uint8_t *out;               // contiguous output bitstream
    uint64_t out_cap;
    uint32_t *work_ctr;         // kCtrSet frame-queue tickets: analysis full/tail, pack full/tail,
                                // per-XCD split-analysis queues (each stage zeroes the other's)
    uint32_t *err;              // device error word (0 = ok; bit 0 invariant, bit 1 output too small)
    const uint16_t *crc_pow;    // [(H-1)*pack_threads + t] = z^(16+64*H*(T-1-t)) mod Q (Q = z^15+z+1), H = 1..crc_hmax
    const uint16_t *crc_join;   // [H-1] = z^(32*H) mod Q
    uint32_t crc_hmax;          // largest half-segment (words) of the CRC fold
    const uint16_t *crc_pow4;   // the same for the four-waves-per-subframe pack kernel (k_pack4, 512 threads)
    uint32_t crc_hmax4;
    FrameRec *records;          // optional decision records [slot]
    unsigned long long *stamps; // diagnostic builds (-DFG_STAMPS): per-phase clock sums
    uint32_t ch_split;          // full-frame analysis: 1 = one workgroup per channel half (channels
                                // = the half's count), frame totals by k_frame_totals
    uint32_t grid_reserve;      // host side: persistent workgroups left unlaunched (room for the
                                // stream-MD5 workgroups queued beside this kernel)
    const uint16_t *crc_x8;     // [i] = z^(8 * 2^i) mod P, i < 24 (channel-half pack: CRC shift)
    uint32_t xcd_queue;         // split analysis: items from per-XCD queues (xcd_ticket, fg_device.hpp)
    uint64_t *status;           // fused encode: per-slot size / inclusive-prefix words (fg_fused.hpp);
                                // the tail analysis before it publishes its frames' sizes there
    uint32_t grid_per_cu;       // host side: at most this many persistent workgroups per CU (0 = as
                                // many as fit) -- the overlapped encode shares each CU between an
                                // analysis grid and a pack grid running on two streams
    uint32_t enc_prio;          // A/B knob: the C2 encode waves at issue priority 1, above the MD5's 0
    uint32_t ana1_variant;      // k_ana1 register budget (fg_ana1.hpp): 1 = 3 waves/SIMD, 2 = 4
};

}  // namespace fg
