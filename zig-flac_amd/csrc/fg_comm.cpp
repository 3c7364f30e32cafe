// Multi-rank encode behind the C ABI: one process per GPU, the bitstream gather over RCCL
// (xGMI point-to-point between the GPUs of one node).  SURVEY.md §8(e): frame f depends
// only on its samples and its number (encoder.zig:234-284, frame_writer.zig:235-251), so
// the ranks encode disjoint frames with no exchange; the one exchange is the gather of the
// variable-length bitstreams and per-frame sizes to the rank that writes the file
// (wav2flac.zig:66-97's output stream; updateFrameSize replayed in frame order,
// metadata.zig:35-40).
//
// The gather is two collectives: an all-gather of every rank's (frames, bytes, error,
// rank-0 capacities) so that every rank takes the same decision, then one RCCL group of
// point-to-point transfers straight into slices of rank 0's receive buffer (the stream
// arrives contiguous and in frame order; no concatenation pass).
//
// librccl.so.1 is opened at the first communicator: an RCCL already loaded in the process
// (a framework's: torch ships one with the same soname) is reused, else /opt/rocm/lib's.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "fg_internal.hpp"

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // already in the process
        if (!h) {
            if (const char *p = std::getenv("FLACGPU_RCCL")) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        auto sym = [&](const char *n) { return dlsym(h, n); };
        r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))sym("ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))sym("ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))sym("ncclAllGather");
        r.send = (decltype(r.send))sym("ncclSend");
        r.recv = (decltype(r.recv))sym("ncclRecv");
        r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
        r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.send && r.recv &&
               r.group_start && r.group_end;
    });
    return r;
}

int hip_rc(hipError_t e) { return e == hipSuccess ? FLACGPU_OK : (e == hipErrorOutOfMemory ? FLACGPU_ERR_OUT_OF_MEMORY : FLACGPU_ERR_DEVICE); }
#define CHK_HIP(x)                                  \
    do {                                            \
        const hipError_t e_ = (x);                  \
        if (e_ != hipSuccess) return hip_rc(e_);    \
    } while (0)
#define CHK_NCCL(x)                                  \
    do {                                             \
        if ((x) != ncclSuccess) return FLACGPU_ERR_DEVICE; \
    } while (0)

// one rank's entry of the count all-gather
enum { kFrames = 0, kBytes, kErr, kRecvCap, kRecvSizesCap, kWords = 8 };

}  // namespace

struct flacgpu_comm {
    ncclComm_t nc = nullptr;
    int world = 0, rank = 0, device = 0;
    uint64_t *d_cnt = nullptr;  // kWords u64: this rank's entry
    uint64_t *d_all = nullptr;  // world x kWords u64
    uint64_t *h_all = nullptr;  // pinned host copy of d_all
    uint64_t *h_cnt = nullptr;  // pinned staging of this rank's entry
    // encode_frames_sharded: rank 0's receive buffers (grow-only)
    uint8_t *d_recv = nullptr;
    uint32_t *d_recv_sizes = nullptr;
    uint64_t recv_cap = 0, recv_sizes_cap = 0;
    // FLACGPU_COMM_SELF_P2P=1 (read at init; output-invariant): rank 0 moves its own slice into the
    // receive buffer by RCCL send/recv to itself instead of a device copy, so that a one-GPU box runs
    // the grouped point-to-point code the other ranks' slices take
    bool self_p2p = false;
};

namespace {

// The all-gather of every rank's entry; returns with comm->h_all filled (stream synchronised).
int exchange_counts(flacgpu_comm *m, const uint64_t entry[kWords], const uint64_t *d_nbytes, hipStream_t st) {
    const Rccl &r = rccl();
    std::memcpy(m->h_cnt, entry, kWords * sizeof(uint64_t));
    CHK_HIP(hipMemcpyAsync(m->d_cnt, m->h_cnt, kWords * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if (d_nbytes) CHK_HIP(hipMemcpyAsync(m->d_cnt + kBytes, d_nbytes, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    CHK_NCCL(r.all_gather(m->d_cnt, m->d_all, kWords, ncclUint64, m->nc, st));
    CHK_HIP(hipMemcpyAsync(m->h_all, m->d_all, (size_t)m->world * kWords * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    CHK_HIP(hipStreamSynchronize(st));
    return FLACGPU_OK;
}

// The transfers once every rank knows every count (comm->h_all): rank 0 receives rank r's bytes
// and sizes at the running offsets, the others send theirs.  Returns the agreed result.
int transfer(flacgpu_comm *m, const uint8_t *d_frames, const uint32_t *d_sizes, uint8_t *d_recv, uint32_t *d_recv_sizes,
             uint64_t *total_bytes, uint64_t *total_frames, hipStream_t st) {
    const Rccl &r = rccl();
    const uint64_t *all = m->h_all;
    uint64_t tb = 0, tf = 0;
    int err = FLACGPU_OK;
    for (int k = 0; k < m->world; k++) {
        tb += all[k * kWords + kBytes];
        tf += all[k * kWords + kFrames];
        if (all[k * kWords + kErr] && !err) err = -(int)all[k * kWords + kErr];
    }
    if (total_bytes) *total_bytes = err ? 0 : tb;
    if (total_frames) *total_frames = err ? 0 : tf;
    if (err) return err;  // a rank failed before the gather: every rank reports it, nothing moves
    if (tb > all[kRecvCap] || tf > all[kRecvSizesCap]) {
        if (total_bytes) *total_bytes = 0;
        if (total_frames) *total_frames = 0;
        return FLACGPU_ERR_OUTPUT_TOO_SMALL;  // rank 0's capacities: the same decision everywhere
    }
    const uint64_t my_b = all[m->rank * kWords + kBytes], my_f = all[m->rank * kWords + kFrames];
    if (m->rank == 0) {
        // its own slice: in place, a device copy, or (self_p2p) send/recv to itself
        const bool pb = my_b && d_frames != d_recv, pf = my_f && d_sizes != d_recv_sizes;
        if (pb && !m->self_p2p) CHK_HIP(hipMemcpyAsync(d_recv, d_frames, my_b, hipMemcpyDeviceToDevice, st));
        if (pf && !m->self_p2p)
            CHK_HIP(hipMemcpyAsync(d_recv_sizes, d_sizes, my_f * 4, hipMemcpyDeviceToDevice, st));
        const bool self = m->self_p2p && (pb || pf);
        if (m->world == 1 && !self) return FLACGPU_OK;
        CHK_NCCL(r.group_start());
        uint64_t ob = my_b, of = my_f;
        bool bad = false;
        if (self && pf) {
            bad |= r.recv(d_recv_sizes, my_f, ncclUint32, 0, m->nc, st) != ncclSuccess;
            bad |= r.send(d_sizes, my_f, ncclUint32, 0, m->nc, st) != ncclSuccess;
        }
        if (self && pb) {
            bad |= r.recv(d_recv, my_b, ncclUint8, 0, m->nc, st) != ncclSuccess;
            bad |= r.send(d_frames, my_b, ncclUint8, 0, m->nc, st) != ncclSuccess;
        }
        for (int k = 1; k < m->world; k++) {
            const uint64_t nb = all[k * kWords + kBytes], nf = all[k * kWords + kFrames];
            if (nf) bad |= r.recv(d_recv_sizes + of, nf, ncclUint32, k, m->nc, st) != ncclSuccess;
            if (nb) bad |= r.recv(d_recv + ob, nb, ncclUint8, k, m->nc, st) != ncclSuccess;
            ob += nb;
            of += nf;
        }
        bad |= r.group_end() != ncclSuccess;
        return bad ? FLACGPU_ERR_DEVICE : FLACGPU_OK;
    }
    if (!my_b && !my_f) return FLACGPU_OK;
    CHK_NCCL(r.group_start());
    bool bad = false;
    if (my_f) bad |= r.send(d_sizes, my_f, ncclUint32, 0, m->nc, st) != ncclSuccess;
    if (my_b) bad |= r.send(d_frames, my_b, ncclUint8, 0, m->nc, st) != ncclSuccess;
    bad |= r.group_end() != ncclSuccess;
    return bad ? FLACGPU_ERR_DEVICE : FLACGPU_OK;
}

hipStream_t as_stream(void *s) { return s == FLACGPU_STREAM_LEGACY ? (hipStream_t)0 : (hipStream_t)s; }

}  // namespace

extern "C" {

int flacgpu_comm_unique_id(uint8_t id[FLACGPU_COMM_ID_BYTES]) {
    if (!id) return FLACGPU_ERR_INVALID_INPUT;
    const Rccl &r = rccl();
    if (!r.ok) return FLACGPU_ERR_DEVICE;
    ncclUniqueId u;
    CHK_NCCL(r.get_unique_id(&u));
    static_assert(sizeof(u) == FLACGPU_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof u);
    return FLACGPU_OK;
}

int flacgpu_comm_init(const uint8_t id[FLACGPU_COMM_ID_BYTES], int world, int rank, int device, flacgpu_comm **out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world || device < 0) return FLACGPU_ERR_INVALID_INPUT;
    *out = nullptr;
    const Rccl &r = rccl();
    if (!r.ok) return FLACGPU_ERR_DEVICE;
    CHK_HIP(hipSetDevice(device));
    flacgpu_comm *m = new (std::nothrow) flacgpu_comm;
    if (!m) return FLACGPU_ERR_OUT_OF_MEMORY;
    m->world = world;
    m->rank = rank;
    m->device = device;
    if (const char *e = std::getenv("FLACGPU_COMM_SELF_P2P")) m->self_p2p = std::atoi(e) != 0;
    auto fail = [&](int rc) {
        flacgpu_comm_destroy(m);
        return rc;
    };
    if (hipMalloc(&m->d_cnt, kWords * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&m->d_all, (size_t)world * kWords * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&m->h_all, (size_t)world * kWords * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&m->h_cnt, kWords * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
        return fail(FLACGPU_ERR_OUT_OF_MEMORY);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (r.comm_init_rank(&m->nc, world, u, rank) != ncclSuccess) {
        m->nc = nullptr;
        return fail(FLACGPU_ERR_DEVICE);
    }
    *out = m;
    return FLACGPU_OK;
}

void flacgpu_comm_destroy(flacgpu_comm *m) {
    if (!m) return;
    hipSetDevice(m->device);
    if (m->nc) rccl().comm_destroy(m->nc);
    hipFree(m->d_cnt);
    hipFree(m->d_all);
    hipHostFree(m->h_all);
    hipHostFree(m->h_cnt);
    hipFree(m->d_recv);
    hipFree(m->d_recv_sizes);
    delete m;
}

int flacgpu_comm_rank(const flacgpu_comm *m) { return m ? m->rank : FLACGPU_ERR_INVALID_INPUT; }
int flacgpu_comm_size(const flacgpu_comm *m) { return m ? m->world : FLACGPU_ERR_INVALID_INPUT; }

int flacgpu_gather_frames_device(flacgpu_comm *m, const uint8_t *d_frames, uint64_t nbytes, const uint64_t *d_nbytes,
                                 const uint32_t *d_sizes, uint64_t n_frames, uint8_t *d_recv, uint64_t recv_cap,
                                 uint32_t *d_recv_sizes, uint64_t recv_sizes_cap, uint64_t *total_bytes,
                                 uint64_t *total_frames, void *hip_stream) {
    if (!m) return FLACGPU_ERR_INVALID_INPUT;
    // a bad argument on one rank must not leave the others waiting in the collective: it is
    // reported through the all-gather and every rank returns it
    int local = FLACGPU_OK;
    if ((n_frames && !d_sizes) || ((nbytes || d_nbytes) && !d_frames) ||
        (m->rank == 0 && ((recv_cap && !d_recv) || (recv_sizes_cap && !d_recv_sizes))))
        local = FLACGPU_ERR_INVALID_INPUT;
    CHK_HIP(hipSetDevice(m->device));
    const hipStream_t st = as_stream(hip_stream);
    uint64_t e[kWords] = {};
    e[kFrames] = local ? 0 : n_frames;
    e[kBytes] = local ? 0 : nbytes;
    e[kErr] = (uint64_t)(-local);
    e[kRecvCap] = recv_cap;
    e[kRecvSizesCap] = recv_sizes_cap;
    int rc = exchange_counts(m, e, local ? nullptr : d_nbytes, st);
    if (rc) return rc;
    return transfer(m, d_frames, d_sizes, d_recv, d_recv_sizes, total_bytes, total_frames, st);
}

int flacgpu_encode_frames_sharded(flacgpu_ctx *ctx, flacgpu_comm *m, const void *pcm, uint32_t bytes_per_sample,
                                  uint64_t n_samples, uint64_t first_frame_number, uint8_t *out, size_t out_cap,
                                  size_t *out_len, uint32_t *frame_bytes) {
    if (!m) return FLACGPU_ERR_INVALID_INPUT;
    if (out_len) *out_len = 0;
    int local = FLACGPU_OK;
    if (!ctx || (!pcm && n_samples) || (m->rank == 0 && !out_len)) local = FLACGPU_ERR_INVALID_INPUT;
    fg::CtxDevice d{};
    if (!local) {
        d = fg::ctx_device(ctx);
        if (d.device != m->device || bytes_per_sample != d.bytes_per_sample) local = FLACGPU_ERR_INVALID_INPUT;
    }
    const uint64_t bs = local ? 4096 : d.block_size;
    const uint64_t frames = (n_samples + bs - 1) / bs;
    if (!local && frames && (first_frame_number >= (1ull << 36) || frames - 1 > (1ull << 36) - 1 - first_frame_number))
        local = FLACGPU_ERR_INVALID_INPUT;  // u36 frame numbers
    const uint64_t per = local ? 1 : fg::ctx_max_frames(ctx);  // frames per rank per window
    const uint64_t isz = local ? 0 : (uint64_t)d.channels * bytes_per_sample;
    // every rank must run the same number of windows: agree on it (and on any argument error)
    // through one count exchange before the first window
    CHK_HIP(hipSetDevice(m->device));
    hipStream_t st = local ? (hipStream_t)0 : (hipStream_t)d.stream;
    uint64_t e[kWords] = {};
    e[kFrames] = frames;
    e[kBytes] = per;
    e[kErr] = (uint64_t)(-local);
    int rc = exchange_counts(m, e, nullptr, st);
    if (rc) return rc;
    uint64_t windows = 0;
    for (int k = 0; k < m->world; k++) {
        const uint64_t *a = m->h_all + k * kWords;
        if (a[kErr]) return -(int)a[kErr];
        if (a[kFrames] != frames || a[kBytes] != per) return FLACGPU_ERR_INVALID_INPUT;  // not the same call
    }
    const uint64_t wf = per * (uint64_t)m->world;  // frames per window
    windows = (frames + wf - 1) / wf;
    // rank 0's receive buffers: one window of every rank's frames
    if (m->rank == 0) {
        const uint64_t need = (uint64_t)m->world * d.out_cap, need_f = wf;
        if (need > m->recv_cap) {
            hipFree(m->d_recv);
            m->d_recv = nullptr;
            m->recv_cap = 0;
            if (hipMalloc(&m->d_recv, need) == hipSuccess) m->recv_cap = need;
        }
        if (need_f > m->recv_sizes_cap) {
            hipFree(m->d_recv_sizes);
            m->d_recv_sizes = nullptr;
            m->recv_sizes_cap = 0;
            if (hipMalloc(&m->d_recv_sizes, need_f * 4) == hipSuccess) m->recv_sizes_cap = need_f;
        }
    }
    uint64_t written = 0, frames_out = 0;
    int err = FLACGPU_OK;
    for (uint64_t w = 0; w < windows; w++) {
        // this rank's slice of window w
        const uint64_t f0 = std::min(frames, w * wf + (uint64_t)m->rank * per);
        const uint64_t nf = std::min(frames, f0 + per) - f0;
        uint64_t total = 0;
        int lrc = err;
        if (!lrc && m->rank == 0 && (!m->d_recv || !m->d_recv_sizes)) lrc = FLACGPU_ERR_OUT_OF_MEMORY;
        if (!lrc && nf) {
            const uint64_t s0 = f0 * bs, ns = std::min<uint64_t>(nf * bs, n_samples - s0);
            lrc = fg::ctx_encode_chunk(ctx, (const uint8_t *)pcm + s0 * isz, ns, first_frame_number + f0, &total, nullptr);
        }
        uint64_t ge[kWords] = {};
        ge[kFrames] = lrc ? 0 : nf;
        ge[kBytes] = lrc ? 0 : total;
        ge[kErr] = (uint64_t)(-lrc);
        ge[kRecvCap] = m->recv_cap;
        ge[kRecvSizesCap] = m->recv_sizes_cap;
        if ((rc = exchange_counts(m, ge, nullptr, st))) return rc;  // the collective itself failed
        uint64_t tb = 0, tf = 0;
        rc = transfer(m, d.d_out, d.d_fbytes, m->d_recv, m->d_recv_sizes, &tb, &tf, st);
        if (rc) {
            err = rc;
            break;  // every rank took the same decision (the counts are shared): all leave here
        }
        if (m->rank == 0) {
            if (written + tb > out_cap) {
                err = FLACGPU_ERR_OUTPUT_TOO_SMALL;  // rank 0 only: reported to the others next window
            } else {
                if (tb) CHK_HIP(hipMemcpyAsync(out + written, m->d_recv, tb, hipMemcpyDeviceToHost, st));
                if (tf && frame_bytes)
                    CHK_HIP(hipMemcpyAsync(frame_bytes + frames_out, m->d_recv_sizes, tf * 4, hipMemcpyDeviceToHost, st));
                CHK_HIP(hipStreamSynchronize(st));
                written += tb;
                frames_out += tf;
            }
        }
    }
    if (!err && m->rank == 0 && frames_out != frames) err = FLACGPU_ERR_INTERNAL;
    // rank 0's last-window output error reaches every rank through one more exchange
    uint64_t fe[kWords] = {};
    fe[kErr] = (uint64_t)(-err);
    if ((rc = exchange_counts(m, fe, nullptr, st))) return rc;
    for (int k = 0; k < m->world; k++)
        if (m->h_all[k * kWords + kErr]) return -(int)m->h_all[k * kWords + kErr];
    fg::ctx_finish(ctx);
    if (m->rank == 0 && out_len) *out_len = written;
    return FLACGPU_OK;
}

}  // extern "C"
