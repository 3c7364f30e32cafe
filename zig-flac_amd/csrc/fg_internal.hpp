// fg_internal.hpp -- library-internal entry points shared by the translation
// units behind the C ABI (not exported in include/flacgpu.h).
#pragma once
#include <stdint.h>

#include "../../include/flacgpu.h"

namespace fg {
// Upload ns interleaved samples (at most max_frames frames) from host memory, encode
// them with frame numbers from first_number, wait; *total = bytes of the encoded
// frames, now in the context's device output; frame_bytes (if non-NULL) receives the
// per-frame sizes.  Device-side errors are reported here.
int ctx_encode_chunk(flacgpu_ctx *c, const uint8_t *src, uint64_t ns, uint64_t first_number, uint64_t *total,
                     uint32_t *frame_bytes);
// Copy the last chunk's `total` encoded bytes to host memory at out.
int ctx_download_chunk(flacgpu_ctx *c, uint8_t *out, uint64_t total);
// n independent streams from host memory, frames numbered from 0 each, through one pipelined
// H2D / encode / D2H schedule that runs on from one stream into the next; out_len[i] = bytes of
// stream i's frames at out[i], frame_bytes[i] (array and entries may be NULL) their sizes.
int ctx_encode_segments(flacgpu_ctx *c, uint32_t n, const uint8_t *const *src, const uint64_t *n_samples,
                        uint8_t *const *out, const size_t *out_cap, size_t *out_len, uint32_t *const *frame_bytes);
uint32_t ctx_max_frames(const flacgpu_ctx *c);
// The device side of a context: where ctx_encode_chunk leaves its frames (d_out), their sizes
// (d_fbytes) and their byte total (d_total), on `stream` of HIP device `device`.
struct CtxDevice {
    int device;
    void *stream;  // hipStream_t
    uint8_t *d_out;
    uint32_t *d_fbytes;
    uint64_t *d_total;
    uint64_t out_cap;
    uint32_t channels, bytes_per_sample, block_size;
};
CtxDevice ctx_device(const flacgpu_ctx *c);
// The context runs the default schedule with no per-context instrumentation (no decision
// records, no kernel timing, no diagnostic schedule): its host-buffer file work may then run on
// the device's shared file pipeline (fg_file.cpp) instead of on its own streams.
bool ctx_plain(const flacgpu_ctx *c);
void ctx_finish(flacgpu_ctx *c);  // fold pending timing events
}  // namespace fg
