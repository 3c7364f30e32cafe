// fg_common.hpp -- POD types shared by the HIP kernels (fg_kernels.hip) and the
// host orchestration behind the C ABI (fg_api.cpp).  gfx950 only.
#pragma once
#include <stdint.h>

namespace fg {

constexpr int kBlock = 4096;       // Config.default block size (encoder.zig:644)
constexpr int kLaneSamples = 64;   // samples per lane: one wave == one 4096-sample subframe
constexpr int kMaxPartOrder = 8;   // rice.MAX_ORDER (rice.zig:13)
constexpr int kParamBytes = 512;   // params of all orders 0..8: offset (1<<o)-1 (511 used)
constexpr int kCrcThreadsMax = 512;

// One frame of work.  pcm_off must be 4-byte aligned.
struct FrameJob {
    uint64_t pcm_off;   // byte offset of the frame's first interleaved sample
    uint64_t number;    // frame number written into the header (u36)
    uint32_t n;         // samples per channel in this frame (1..4096)
    uint32_t slot;      // output slot / frame index within the call
};

// Per-candidate decision record (SubframeType.Encoding + estimate,
// encoder.zig:678-702).  Mirrors flacgpu_subframe_record.
struct SubRec {
    uint8_t type;       // 0 CONSTANT, 1 VERBATIM, 2 FIXED
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
};

struct FrameRec {
    uint32_t channel_code;
    uint32_t n_cand;
    uint32_t frame_bytes;
    uint32_t pad;
    SubRec cand[8];
};

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
    uint8_t *slots;             // frame slots, slot_bytes each
    uint32_t slot_bytes;
    uint32_t image_bytes;       // LDS frame-image bytes (multiple of 16, >= bound)
    uint32_t stage_separate;    // full-frame kernel: staging region separate from the image (DMA prefetch)
    uint32_t *frame_bytes;      // [slot]
    uint32_t *err;              // device error word (0 = ok)
    const uint16_t *crc_tab;    // 4 x 256: z^40, z^32, z^24, z^16 byte tables (CRC-16/UMTS)
    const uint16_t *crc_pow;    // [threads+1]: z^(32*seg_words*(T-1-t)) mod P; [threads] = z^(16*seg_words)
    uint32_t crc_seg_words;     // words per thread in the CRC fold (even)
    FrameRec *records;          // optional decision records [slot]
    unsigned long long *stamps; // diagnostic builds (-DFG_STAMPS): per-phase clock sums
};

}  // namespace fg
