// Multi-GPU host-buffer encode: the frames of one input sharded over several
// contexts (one per GPU), encoded concurrently and concatenated in frame order.
// Frame f depends only on its samples and its number (encoder.zig:234-284), so
// contiguous frame ranges encode independently; the only exchange is the
// concatenation of the variable-length bitstreams (SURVEY.md §8(e),
// wav2flac.zig:66-97 with the frame-order replay of metadata.zig:35-40).
//
// The input is cut into rounds of n_ctx x max_frames frames; in a round, context
// i encodes the i-th contiguous slice.  One host thread per context; after a
// round's encodes every thread knows all the round's byte counts (a barrier), so
// each copies its frames from its GPU straight into the caller's buffer at the
// scanned offset -- no host staging, no second copy.  A thread's download of round
// r overlaps the other contexts' encodes of round r + 1.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <cstring>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "fg_internal.hpp"

struct flacgpu_multi {
    std::vector<flacgpu_ctx *> ctx;
    flacgpu_config cfg{};
};

namespace {

// Reusable barrier for the worker threads of one call.
class Barrier {
  public:
    explicit Barrier(size_t n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(m_);
        const size_t gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            gen_++;
            cv_.notify_all();
            return;
        }
        cv_.wait(lk, [&] { return gen_ != gen; });
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    size_t n_, count_ = 0, gen_ = 0;
};

}  // namespace

extern "C" {

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
    if (bytes_per_sample != m->cfg.bits_per_sample / 8u) return FLACGPU_ERR_INVALID_INPUT;
    const uint64_t bs = m->cfg.block_size;
    const uint64_t frames = (n_samples + bs - 1) / bs;
    if (frames && (first_frame_number >= (1ull << 36) || frames - 1 > (1ull << 36) - 1 - first_frame_number))
        return FLACGPU_ERR_INVALID_INPUT;  // u36 frame numbers
    const uint64_t n = m->ctx.size();
    const uint64_t isz = (uint64_t)m->cfg.channels * bytes_per_sample;  // bytes per interchannel sample
    // frames per context and round: even slices of a round, capped by the context capacity
    const uint64_t cap = fg::ctx_max_frames(m->ctx[0]);
    const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(cap, (frames + n - 1) / n));
    const uint64_t rounds = frames ? (frames + per * n - 1) / (per * n) : 0;
    std::vector<uint64_t> totals;
    try {
        totals.assign(rounds * n, 0);
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    // per-context result: set by its own thread, read by all after a barrier
    std::unique_ptr<std::atomic<int>[]> rcs(new (std::nothrow) std::atomic<int>[n]);
    if (!rcs) return FLACGPU_ERR_OUT_OF_MEMORY;
    for (uint64_t i = 0; i < n; i++) rcs[i] = FLACGPU_OK;
    Barrier bar(n);
    auto slice = [&](uint64_t r, uint64_t i, uint64_t *f0, uint64_t *nf) {
        const uint64_t a = std::min(frames, (r * n + i) * per);
        *f0 = a;
        *nf = std::min(frames, a + per) - a;
    };
    auto work = [&](uint64_t i) {
        flacgpu_ctx *c = m->ctx[i];
        for (uint64_t r = 0; r < rounds; r++) {
            uint64_t f0, nf;
            slice(r, i, &f0, &nf);
            int rc = FLACGPU_OK;
            if (nf && !rcs[i]) {
                const uint64_t s0 = f0 * bs, ns = std::min<uint64_t>(nf * bs, n_samples - s0);
                rc = fg::ctx_encode_chunk(c, (const uint8_t *)pcm + s0 * isz, ns, first_frame_number + f0,
                                          &totals[r * n + i], frame_bytes ? frame_bytes + f0 : nullptr);
                if (rc) rcs[i] = rc;
            }
            bar.wait();  // every total of round r (and every failure so far) is visible
            bool any_fail = false;
            for (uint64_t j = 0; j < n; j++) any_fail |= rcs[j] != FLACGPU_OK;
            if (any_fail) return;  // all threads see the same flags after the barrier: all stop here
            uint64_t off = 0;
            for (uint64_t k = 0; k < r * n + i; k++) off += totals[k];
            const uint64_t t = totals[r * n + i];
            if (off + t > out_cap) {
                rcs[i] = FLACGPU_ERR_OUTPUT_TOO_SMALL;
            } else if (t) {
                rc = fg::ctx_download_chunk(c, out + off, t);
                if (rc) rcs[i] = rc;
            }
        }
    };
    // threads wait at a gate until all exist: if one cannot be created, the others are
    // released with "abort" before any of them reaches the barrier (which counts n)
    std::mutex gm;
    std::condition_variable gcv;
    int gate = 0;  // 0 closed, 1 go, -1 abort
    auto run = [&](uint64_t i) {
        {
            std::unique_lock<std::mutex> lk(gm);
            gcv.wait(lk, [&] { return gate != 0; });
            if (gate < 0) return;
        }
        work(i);
    };
    std::vector<std::thread> th;
    int rc = FLACGPU_OK;
    try {
        th.reserve(n);
        for (uint64_t i = 1; i < n; i++) th.emplace_back(run, i);
    } catch (...) {
        rc = FLACGPU_ERR_OUT_OF_MEMORY;
    }
    {
        std::lock_guard<std::mutex> lk(gm);
        gate = rc ? -1 : 1;
    }
    gcv.notify_all();
    if (!rc) work(0);
    for (std::thread &t : th) t.join();
    if (rc) return rc;
    for (uint64_t i = 0; i < n; i++)
        if (rcs[i]) return rcs[i];
    uint64_t written = 0;
    for (uint64_t t : totals) written += t;
    for (flacgpu_ctx *c : m->ctx) fg::ctx_finish(c);
    *out_len = written;
    return FLACGPU_OK;
}

}  // extern "C"
