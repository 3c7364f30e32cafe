// Multi-GPU host-buffer encode: the frames of one input sharded over several
// contexts (one per GPU), encoded concurrently and concatenated in frame order.
// Frame f depends only on its samples and its number (encoder.zig:234-284), so
// contiguous frame ranges encode independently; the only exchange is the
// concatenation of the variable-length bitstreams.
#include <algorithm>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/flacgpu.h"

struct flacgpu_multi {
    std::vector<flacgpu_ctx *> ctx;
    flacgpu_config cfg{};
};

int flacgpu_open_multi(int n_devices, const int *devices, const flacgpu_config *cfg, uint32_t max_frames_per_call,
                       flacgpu_multi **out) {
    if (!out || !cfg || !devices || n_devices <= 0 || n_devices > 64) return FLACGPU_ERR_INVALID_INPUT;
    *out = nullptr;
    flacgpu_multi *m = new (std::nothrow) flacgpu_multi;
    if (!m) return FLACGPU_ERR_OUT_OF_MEMORY;
    m->cfg = *cfg;
    for (int i = 0; i < n_devices; i++) {
        flacgpu_ctx *c = nullptr;
        const int rc = flacgpu_open(devices[i], cfg, max_frames_per_call, &c);
        if (rc) {
            flacgpu_close_multi(m);
            return rc;
        }
        m->ctx.push_back(c);
    }
    flacgpu_get_config(m->ctx[0], &m->cfg);  // as normalised by flacgpu_open
    *out = m;
    return FLACGPU_OK;
}

void flacgpu_close_multi(flacgpu_multi *m) {
    if (!m) return;
    for (flacgpu_ctx *c : m->ctx) flacgpu_close(c);
    delete m;
}

int flacgpu_multi_encode_frames(flacgpu_multi *m, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                                uint64_t first_frame_number, uint8_t *out, size_t out_cap, size_t *out_len,
                                uint32_t *frame_bytes) {
    if (!m || (!pcm && n_samples) || !out_len) return FLACGPU_ERR_INVALID_INPUT;
    *out_len = 0;
    const uint32_t bs = m->cfg.block_size ? m->cfg.block_size : 4096u;
    const uint64_t frames = (n_samples + bs - 1) / bs;
    const uint64_t n = m->ctx.size();
    const uint64_t per = (frames + n - 1) / (n ? n : 1);
    const uint64_t isz = (uint64_t)m->cfg.channels * bytes_per_sample;  // bytes per interchannel sample
    const size_t fb = flacgpu_frame_bound_bytes(&m->cfg);
    struct Part {
        uint64_t f0 = 0, nf = 0;
        std::vector<uint8_t> buf;
        size_t len = 0;
        int rc = FLACGPU_OK;
    };
    std::vector<Part> parts(n);
    for (uint64_t i = 0; i < n; i++) {  // all staging first: no thread is running on an early return
        Part &p = parts[i];
        p.f0 = std::min(frames, i * per);
        p.nf = std::min(frames, p.f0 + per) - p.f0;
        if (p.nf == 0) continue;
        try {
            p.buf.resize(p.nf * fb + 64);
        } catch (...) {
            return FLACGPU_ERR_OUT_OF_MEMORY;
        }
    }
    std::vector<std::thread> th;
    for (uint64_t i = 0; i < n; i++) {
        if (parts[i].nf == 0) continue;
        const uint64_t s0 = parts[i].f0 * bs, ns = std::min<uint64_t>(parts[i].nf * bs, n_samples - s0);
        th.emplace_back([&, i, s0, ns]() {
            Part &q = parts[i];
            q.rc = flacgpu_encode_frames(m->ctx[i], (const uint8_t *)pcm + s0 * isz, bytes_per_sample, ns,
                                         first_frame_number + q.f0, q.buf.data(), q.buf.size(), &q.len,
                                         frame_bytes ? frame_bytes + q.f0 : nullptr);
        });
    }
    for (std::thread &t : th) t.join();
    size_t written = 0;
    for (const Part &p : parts) {
        if (p.rc) return p.rc;
        if (written + p.len > out_cap) return FLACGPU_ERR_OUTPUT_TOO_SMALL;
        if (p.len) std::memcpy(out + written, p.buf.data(), p.len);
        written += p.len;
    }
    *out_len = written;
    return FLACGPU_OK;
}
