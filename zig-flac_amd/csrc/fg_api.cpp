// fg_api.cpp -- the C ABI of libflacgpu.so (include/flacgpu.h): device
// memory planning, frame tables, launches and host <-> device movement for
// the gfx950 kernels (fg_device.hpp, fg_misc.hip).  No CPU encoding path exists: every
// encode goes through the HIP kernels, and a missing/unsupported device is an
// error (FLACGPU_ERR_DEVICE), never a fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/flacgpu.h"
#include "fg_common.hpp"
#include "fg_internal.hpp"
#include "fg_layout.hpp"
#include "fg_md5_host.hpp"

namespace fg {
hipError_t launch_stage(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st);
hipError_t launch_make_jobs(FrameJob *jobs, uint64_t n_samples, uint32_t block, uint32_t stride, uint64_t first,
                            uint32_t n_frames, hipStream_t st);
hipError_t launch_frame_totals(const EncodeArgs &a, hipStream_t st);
hipError_t launch_scan(const uint32_t *sizes, uint64_t *offsets, uint64_t *total, uint32_t n, uint64_t *part,
                       hipStream_t st, const uint64_t *base = nullptr);
hipError_t launch_md5_streams(const uint8_t *base, const uint64_t *offs, const uint64_t *lens, const uint8_t *fin,
                              uint32_t n, Md5State *states, uint8_t *digests, hipStream_t st, int kernel, int prio);
hipError_t launch_advance_jobs(FrameJob *jobs, uint64_t n, uint64_t delta, hipStream_t st);
hipError_t launch_md5_blocks(uint32_t *state, const uint32_t *blocks, uint64_t n_blocks, hipStream_t st);
uint32_t md5_workgroups(uint32_t n, int kernel);
hipError_t launch_streaminfo_replay(const uint32_t *sizes, uint64_t n, uint32_t *minmax, hipStream_t st);
}  // namespace fg

using namespace fg;

static_assert(sizeof(SubRec) == sizeof(flacgpu_subframe_record), "record layout");
static_assert(sizeof(FrameRec) == sizeof(flacgpu_frame_record), "record layout");
static_assert(sizeof(Md5State) == sizeof(flacgpu_md5_state), "md5 state layout");

namespace {

constexpr uint32_t kCrcPoly = 0x8005u;

uint32_t crc_mulmod_host(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 15; i >= 0; i--) {
        r <<= 1;
        if (r & 0x10000u) r ^= 0x10000u | kCrcPoly;
        if ((a >> i) & 1u) r ^= b;
    }
    return r & 0xFFFFu;
}
// z^e mod P
uint32_t crc_zpow(uint64_t e) {
    uint32_t result = 1, base = 2;  // z
    while (e) {
        if (e & 1) result = crc_mulmod_host(result, base);
        base = crc_mulmod_host(base, base);
        e >>= 1;
    }
    return result;
}

// z^e mod Q, Q = z^15 + z + 1 (a factor of P): the shift constants of the table-free CRC fold
// (fg_device.hpp crc_lane_q)
uint32_t q_zpow(uint64_t e) {
    const uint32_t r = crc_zpow(e);
    return (r & 0x8000u) ? r ^ 0x8003u : r;
}

struct TimedLaunch {
    int kernel;
    hipEvent_t start, stop;
};

}  // namespace

// chunk sets of the pipelined host-buffer path (encode_pipelined): chunk i uploads into set i % 3
// while chunk i-1 encodes and chunks i-2, i-3 download -- with two sets the upload of chunk i had
// to wait for the encode of chunk i-2 and the encode for the download of chunk i-2, so a slow
// download or a late host thread stalled both directions of PCIe (round-4 batches reached 33-44 GB/s
// of H2D against 57 GB/s measured alone)
constexpr uint32_t kPipeSets = 4;  // the most; flacgpu_ctx::pipe_sets is the number in use (2..4)
constexpr uint32_t kPipeSetsDefault = 3;

struct flacgpu_ctx {
    int device = 0;
    flacgpu_config cfg{};
    uint32_t max_frames = 0;
    uint32_t C = 0, B = 0, bits = 0, stereo = 0, nt = 0, nt_pack = 0;
    uint32_t image_bytes = 0, desc_stride = 0, lds = 0, lds_tail = 0, lds_pack = 0, crc_hmax = 0;
    bool stage_dbuf = false;
    bool pack_dbuf = false;
    hipStream_t stream = nullptr, aux = nullptr;
    hipStream_t dl = nullptr;  // download stream of the pipelined host-buffer path
    hipStream_t up = nullptr;  // its upload stream (chunk i+1's upload beside chunk i's encode)
    hipEvent_t up_done[kPipeSets] = {};  // a chunk set's upload landed (GPU-side waits)
    hipEvent_t set_done[kPipeSets] = {};  // a chunk set's encode finished (GPU-side waits)
    hipEvent_t dl_done[kPipeSets] = {};   // a chunk set's frames downloaded (GPU-side waits)
    uint32_t pipe_sets = kPipeSetsDefault;  // chunk sets in use (FLACGPU_PIPE_SETS = 2: the round-4 schedule; 4)
    hipEvent_t fork = nullptr, join = nullptr;
    // host waits of the pipelined host-buffer path (the download stream, the end; the chunk sets'
    // own events are set_done below):
    // blocking-sync events, so a waiting thread sleeps instead of spinning on a core the MD5 pool
    // and the other files' threads need (FLACGPU_SPIN_SYNC=1: spinning events, A/B)
    hipEvent_t hw[4] = {nullptr, nullptr, nullptr, nullptr};
    uint16_t *d_crc_pow = nullptr, *d_crc_join = nullptr, *d_crc_pow4 = nullptr;
    // full 16-bit two-channel frames are packed by k_pack4 (four waves per subframe): 512 threads
    uint32_t nt_pack4 = 0, lds_pack4 = 0, crc_hmax4 = 0;
    uint32_t *d_err = nullptr, *d_ctr = nullptr;
    FrameJob *d_jobs = nullptr;
    uint8_t *d_desc = nullptr;
    uint32_t *d_fbytes = nullptr;
    uint64_t *d_offsets = nullptr, *d_total = nullptr;
    uint8_t *d_pcm = nullptr;
    uint64_t pcm_cap = 0;
    uint8_t *d_out = nullptr;
    uint64_t out_cap = 0;
    FrameRec *d_records = nullptr;
    unsigned long long *d_stamps = nullptr;
    bool records_on = false;
    bool records_keep = false;  // encode_files with records: every file's records, concatenated
    bool ana_split = false;  // full-frame analysis in channel halves (fg_device.hpp k_analyze)
    bool pack_split = false;  // full-frame pack in channel halves (fg_packw.hpp k_packw<..., true>)
    uint32_t nt_psplit = 0, lds_psplit = 0, image_split = 0, crc_hmaxs = 0;
    uint16_t *d_crc_pows = nullptr;  // CRC fold shifts for the split pack's thread count
    uint16_t *d_crc_x8 = nullptr;    // z^(8 * 2^i) mod P, i < 24
    uint32_t nt_split = 0, lds_split = 0;
    uint64_t *d_scan_part = nullptr;  // per-4096-frame block sums of the multi-workgroup scan
    uint32_t scan_part_cap = 0;
    std::vector<FrameRec> h_records;
    bool timing = false;
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
    uint64_t launches[FLACGPU_K_COUNT] = {};
    double ms[FLACGPU_K_COUNT] = {};
    // streaming MD5 (one stream): a host core by default (FLACGPU_MD5_HOST), or one GPU
    // lane fed by bounded chunks (FLACGPU_MD5_DEVICE, opt-in)
    int md5_engine = FLACGPU_MD5_HOST;
    int md5_kernel = 1;  // batched stream MD5: 1 = coalesced LDS-DMA ring, 0 = per-lane loads (A/B knob)
    int md5_prio = 0;    // issue priority of the MD5 waves beside the encode (A/B knob)
    uint32_t enc_prio = 0;  // issue priority 1 for the C2 encode waves (A/B knob FLACGPU_ENC_PRIO)
    int md5_reserve = -1;  // 1: the analysis grid leaves one workgroup slot per stream-MD5 workgroup
                           //    queued beside it, 2: the pack grid too, 0: none, -1: auto (A/B knob)
    uint32_t grid_reserve = 0;  // per call: slots the next analysis / pack launches leave free
    // overlapped encode (encode_core): the full frames in `ovl_chunks` ranges, the analysis of
    // range i+1 on `stream` beside the scan + pack of range i on `ovl`, each grid capped to
    // ovl_ana / ovl_pack workgroups per CU so both are resident on every CU
    uint32_t ovl_chunks = 0, ovl_ana = 2, ovl_pack = 2, ovl_min_frames = 4096;
    bool xcd_queue = true;  // split analysis: per-XCD item queues (fg_device.hpp xcd_ticket)
    bool pack_xcdq = true;  // split pack: the same (fg_packw.hpp)
    // split analysis (bit 0) / pack (bit 1): each item's ticket taken right before its DMA, so a
    // frame's two halves are staged close together (c4 A/B r4l: analysis 5.03 -> 4.95 ms, analysis
    // traffic 1.82x -> 1.44x of the PCM (r4n); the pack's bit measured no gain, r4o)
    uint32_t split_jit = 1;
    // fused single-pass encode of full 16-bit stereo frames (fg_fused.hpp): analysis and pack in
    // one kernel, frame offsets by an in-kernel look-back over per-slot status words
    bool fused = false;
    // one wave per full 16-bit stereo frame (fg_ana1.hpp k_ana1) instead of one per candidate
    bool ana1 = false;
    uint32_t ana1_variant = 1;
    uint32_t lds_fused = 0, crc_hmaxf = 0;
    uint16_t *d_crc_powf = nullptr;  // CRC fold shifts for its 256 threads
    uint64_t *d_status = nullptr;    // per-slot status words, grow-only
    uint64_t status_cap = 0;
    hipStream_t ovl = nullptr;
    uint64_t *d_cum = nullptr;  // [chunk] bytes of the frames before the chunk's slot range
    HostMd5 host_md5;
    uint32_t *d_md5_state = nullptr;
    uint32_t *d_md5_blocks = nullptr;
    uint8_t md5_buf[64] = {};
    uint32_t md5_fill = 0;
    uint64_t md5_len = 0;
};

// device MD5 engine: whole blocks move through one bounded device buffer
constexpr uint64_t kMd5ChunkBlocks = (64ull << 20) / 64;
// overlapped encode: at most this many frame ranges per call (one ticket set of 4 u32 each)
constexpr uint32_t kOvlMaxChunks = 64;

struct flacgpu_plan {
    flacgpu_ctx *ctx = nullptr;
    uint32_t n_streams = 0;
    uint32_t B = 0;
    uint64_t n_frames = 0, n_full = 0, n_tail = 0;
    FrameJob *d_jobs = nullptr;  // full jobs first, then tail jobs
    uint64_t *d_md5_offs = nullptr, *d_md5_lens = nullptr;
    uint8_t *d_md5_fin = nullptr;  // per-stream final-segment flags (NULL: all final)
    uint64_t md5_max_len = 0;      // longest stream segment (bytes): the MD5 chain of one call
    uint64_t max_number = 0;       // largest frame number in the table (u36 check on advance)
    std::vector<uint64_t> first_frame;
    std::vector<uint32_t> full_slots;  // slot of each full job (host copy: ranges of the overlapped encode)
    // host copies of the MD5 segments (the host engine, flacgpu_md5_plan_host)
    std::vector<uint64_t> h_md5_offs, h_md5_lens;
    std::vector<uint8_t> h_md5_fin;  // empty: all final
    uint64_t md5_total = 0;          // bytes of all segments
    uint64_t out_bound = 0;
    uint8_t *d_desc = nullptr;  // per-plan descriptor area when larger than the context's
};

namespace {

hipEvent_t get_event(flacgpu_ctx *c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void resolve_timing(flacgpu_ctx *c) {
    for (auto &t : c->pending) {
        hipEventSynchronize(t.stop);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.start, t.stop) == hipSuccess) {
            c->launches[t.kernel]++;
            c->ms[t.kernel] += ms;
        }
        c->event_pool.push_back(t.start);
        c->event_pool.push_back(t.stop);
    }
    c->pending.clear();
}

struct Timed {
    flacgpu_ctx *c;
    int k;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    Timed(flacgpu_ctx *c_, int k_, hipStream_t st_) : c(c_), k(k_), st(st_) {
        if (c->timing) {
            a = get_event(c);
            b = get_event(c);
            if (a) hipEventRecord(a, st);
        }
    }
    ~Timed() {
        if (c->timing && a && b) {
            hipEventRecord(b, st);
            c->pending.push_back({k, a, b});
        }
    }
};

int hip_err(hipError_t e) { return e == hipSuccess ? FLACGPU_OK : (e == hipErrorOutOfMemory ? FLACGPU_ERR_OUT_OF_MEMORY : FLACGPU_ERR_DEVICE); }

#define HIPCHK(x)                               \
    do {                                        \
        hipError_t e_ = (x);                    \
        if (e_ != hipSuccess) return hip_err(e_); \
    } while (0)

// The C ABI's hip_stream: NULL = the context's own stream, FLACGPU_STREAM_LEGACY = the HIP null
// stream (legacy default-stream semantics: the handle-0 stream of a framework), else a hipStream_t.
static hipStream_t pick_stream(const flacgpu_ctx *c, void *hip_stream) {
    if (!hip_stream) return c->stream;
    if (hip_stream == FLACGPU_STREAM_LEGACY) return (hipStream_t)0;
    return (hipStream_t)hip_stream;
}

int validate(const flacgpu_config *cfg) {
    if (!cfg) return FLACGPU_ERR_INVALID_INPUT;
    if (cfg->channels < 1 || cfg->channels > 8) return FLACGPU_ERR_INVALID_CONFIG;
    const uint32_t b = cfg->bits_per_sample;
    if (b != 8 && b != 16 && b != 24 && b != 32) return FLACGPU_ERR_INVALID_CONFIG;  // frame_writer.zig:221-233
    if (cfg->block_size < 1 || cfg->block_size > kBlock) return FLACGPU_ERR_INVALID_CONFIG;
    if (cfg->max_rice_part_order > kMaxPartOrder) return FLACGPU_ERR_INVALID_CONFIG;  // rice.zig:13 buffers
    if (cfg->max_rice_param < 1 || cfg->max_rice_param > 30) return FLACGPU_ERR_INVALID_CONFIG;
    if (cfg->sample_rate >= (1u << 20)) return FLACGPU_ERR_INVALID_CONFIG;  // u20 (wav_reader.zig:98)
    // prediction: 0 = fixed only (the reference); 1..12 = LPC search up to that order
    // (build-defined extension; the FLAC subset limit)
    if (cfg->prediction > kLpcMax) return FLACGPU_ERR_INVALID_CONFIG;
    return FLACGPU_OK;
}

uint64_t frames_for(uint64_t n_samples, uint32_t bs) { return (n_samples + bs - 1) / bs; }

// Queue the encode of n_full full frames (jobs[0..n_full)) and n_tail short ones
// (jobs[n_full..)): analysis (descriptors + exact sizes), scan (byte offsets),
// pack (frames written at their offsets in d_out).  full_slots: the slot of each full job
// (NULL: slot == job index); full jobs are in increasing slot order.
//
// Overlapped schedule (c->ovl_chunks > 1 and enough full frames): the tail frames are analysed
// first, then the full frames in K ranges: the analysis of range i+1 runs on `st` while the scan
// of range i's slot span (carried base: the bytes before it) and its pack run on c->ovl, each
// persistent grid capped per CU so that an analysis grid and a pack grid share every CU (the
// analysis is VALU/issue bound, the pack LDS/latency bound).  Each range has its own set of
// frame-queue tickets.  Output bytes are identical to the serial schedule.
int encode_core(flacgpu_ctx *c, const uint8_t *d_pcm, const FrameJob *d_jobs, uint64_t n_full, uint64_t n_tail,
                uint8_t *d_desc, uint32_t *d_fbytes, uint8_t *d_out, uint64_t out_cap, uint64_t *d_offsets,
                uint64_t *d_total, hipStream_t st, const uint32_t *full_slots = nullptr) {
    const uint64_t n_frames = n_full + n_tail;
    if (n_frames == 0) {
        HIPCHK(hipMemsetAsync(d_total, 0, sizeof(uint64_t), st));
        return FLACGPU_OK;
    }
    if (n_frames > 0xFFFFFFFFull) return FLACGPU_ERR_INVALID_INPUT;
    EncodeArgs a{};
    a.pcm = d_pcm;
    a.channels = c->C;
    a.bits = c->bits;
    a.bytes_per_sample = c->B;
    a.sample_rate = c->cfg.sample_rate;
    a.stereo = c->stereo;
    a.max_part_order = c->cfg.max_rice_part_order;
    a.max_param = c->cfg.max_rice_param;
    a.lpc_order = c->cfg.prediction;
    a.block_size = c->cfg.block_size;
    a.desc = d_desc;
    a.desc_stride = c->desc_stride;
    a.image_bytes = c->image_bytes;
    a.stage_dbuf = c->stage_dbuf ? 1u : 0u;
    a.pack_dbuf = c->pack_dbuf ? 1u : 0u;
    a.enc_prio = c->enc_prio;
    a.ana1_variant = c->ana1_variant;
    a.frame_bytes = d_fbytes;
    a.offsets = d_offsets;
    a.out = d_out;
    a.out_cap = out_cap;
    a.err = c->d_err;
    a.work_ctr = c->d_ctr;
    a.crc_pow = c->d_crc_pow;
    a.crc_pow4 = c->d_crc_pow4;
    a.crc_hmax4 = c->crc_hmax4;
    a.crc_join = c->d_crc_join;
    a.crc_hmax = c->crc_hmax;
    a.records = c->records_on ? c->d_records : nullptr;
    a.stamps = c->d_stamps;
    a.crc_x8 = c->d_crc_x8;

    // full-frame analysis of jobs[j0, j0 + n) with ticket set `set`
    auto analyze_full = [&](uint64_t j0, uint64_t n, uint32_t set, uint32_t per_cu, hipStream_t s) -> int {
        Timed t(c, FLACGPU_K_ANALYZE, s);
        EncodeArgs h = a;
        h.jobs = d_jobs + j0;
        h.n_jobs = (uint32_t)n;
        h.work_ctr = c->d_ctr + kCtrSet * set;
        h.grid_reserve = c->grid_reserve;
        h.grid_per_cu = per_cu;
        if (c->ana_split) {
            h.channels = c->C / 2u;
            h.ch_split = 1;
            h.xcd_queue = c->xcd_queue ? ((c->split_jit & 1u) ? 3u : 1u) : 0u;
            HIPCHK(launch_stage(0, h, true, c->nt_split, c->lds_split, s));
            HIPCHK(launch_frame_totals(h, s));
        } else if (c->ana1) {
            HIPCHK(launch_stage(3, h, true, 64u, (uint32_t)Ana1Layout::total, s));
        } else {
            HIPCHK(launch_stage(0, h, true, c->nt, c->lds, s));
        }
        return FLACGPU_OK;
    };
    auto pack_full = [&](uint64_t j0, uint64_t n, uint32_t set, uint32_t per_cu, hipStream_t s) -> int {
        Timed t(c, FLACGPU_K_PACK, s);
        EncodeArgs h = a;
        h.jobs = d_jobs + j0;
        h.n_jobs = (uint32_t)n;
        h.work_ctr = c->d_ctr + kCtrSet * set;
        h.grid_reserve = c->md5_reserve == 2 ? c->grid_reserve : 0u;
        h.grid_per_cu = per_cu;
        if (c->pack_split) {
            h.channels = c->C / 2u;
            h.ch_split = 1;
            h.image_bytes = c->image_split;
            h.crc_pow4 = c->d_crc_pows;
            h.crc_hmax4 = c->crc_hmaxs;
            h.xcd_queue = c->pack_xcdq ? ((c->split_jit & 2u) ? 3u : 1u) : 0u;
            HIPCHK(launch_stage(1, h, true, c->nt_psplit, c->lds_psplit, s));
        } else if (c->nt_pack4) {
            HIPCHK(launch_stage(1, h, true, c->nt_pack4, c->lds_pack4, s));
        } else {
            HIPCHK(launch_stage(1, h, true, c->nt_pack, c->lds_pack, s));
        }
        return FLACGPU_OK;
    };
    auto analyze_tail = [&](hipStream_t s) -> int {
        Timed t(c, FLACGPU_K_ANALYZE_TAIL, s);
        EncodeArgs h = a;
        h.jobs = d_jobs + n_full;
        h.n_jobs = (uint32_t)n_tail;
        HIPCHK(launch_stage(0, h, false, c->nt, c->lds_tail, s));
        return FLACGPU_OK;
    };
    auto pack_tail = [&](hipStream_t s) -> int {
        Timed t(c, FLACGPU_K_PACK, s);
        EncodeArgs h = a;
        h.jobs = d_jobs + n_full;
        h.n_jobs = (uint32_t)n_tail;
        HIPCHK(launch_stage(1, h, false, c->nt_pack, c->lds_pack, s));
        return FLACGPU_OK;
    };
    // the multi-workgroup scan's per-block sums: a grow-only context buffer
    const uint32_t nb = (uint32_t)((n_frames + 4095u) / 4096u);
    if (nb > c->scan_part_cap) {
        hipFree(c->d_scan_part);
        c->d_scan_part = nullptr;
        c->scan_part_cap = 0;
        HIPCHK(hipMalloc(&c->d_scan_part, (size_t)nb * 8u));
        c->scan_part_cap = nb;
    }

    if (c->fused && n_full) {
        // fused: the tail frames' analysis first (it publishes their sizes), then analysis + pack of
        // the full frames in one kernel whose frames find their offsets by look-back, then the scan
        // (offsets of every frame, the total) and the tail frames' pack
        if (n_frames > c->status_cap) {
            hipFree(c->d_status);
            c->d_status = nullptr;
            c->status_cap = 0;
            HIPCHK(hipMalloc(&c->d_status, (size_t)n_frames * 8u));
            c->status_cap = n_frames;
        }
        HIPCHK(hipMemsetAsync(c->d_status, 0, (size_t)n_frames * 8u, st));
        HIPCHK(hipMemsetAsync(c->d_ctr, 0, 4, st));  // the fused kernel's frame queue (ticket 0)
        a.status = c->d_status;
        int rc;
        if (n_tail && (rc = analyze_tail(st))) return rc;
        {
            Timed t(c, FLACGPU_K_ANALYZE, st);
            EncodeArgs h = a;
            h.jobs = d_jobs;
            h.n_jobs = (uint32_t)n_full;
            h.stage_dbuf = 0;
            h.crc_pow4 = c->d_crc_powf;
            h.crc_hmax4 = c->crc_hmaxf;
            h.grid_reserve = c->grid_reserve;
            HIPCHK(launch_stage(2, h, true, 256u, c->lds_fused, st));
        }
        a.status = nullptr;
        {
            Timed t(c, FLACGPU_K_SCAN, st);
            HIPCHK(launch_scan(d_fbytes, d_offsets, d_total, (uint32_t)n_frames, c->d_scan_part, st));
        }
        if (n_tail && (rc = pack_tail(st))) return rc;
        return FLACGPU_OK;
    }

    uint32_t K = c->ovl_chunks;
    if (K > kOvlMaxChunks) K = kOvlMaxChunks;
    while (K > 1 && n_full / K < c->ovl_min_frames) K--;
    if (K > 1) {
        int rc;
        if (n_tail && (rc = analyze_tail(st))) return rc;
        auto slot_of = [&](uint64_t j) -> uint64_t { return full_slots ? full_slots[j] : j; };
        auto j_begin = [&](uint32_t i) -> uint64_t { return n_full * i / K; };
        std::vector<hipEvent_t> evs;
        auto release = [&]() {
            for (auto e : evs) c->event_pool.push_back(e);
        };
        for (uint32_t i = 0; i < K; i++) {
            const uint64_t j0 = j_begin(i), j1 = j_begin(i + 1);
            if ((rc = analyze_full(j0, j1 - j0, i, c->ovl_ana, st))) return release(), rc;
            hipEvent_t ev = get_event(c);
            if (!ev) return release(), FLACGPU_ERR_DEVICE;
            evs.push_back(ev);
            if (hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(c->ovl, ev, 0) != hipSuccess)
                return release(), FLACGPU_ERR_DEVICE;
            // the slot span of range i: from its first full job (0 for the first range) to the next
            // range's first full job (n_frames for the last); tail slots inside it were analysed first
            const uint64_t s0 = i == 0 ? 0 : slot_of(j0), s1 = i + 1 == K ? n_frames : slot_of(j1);
            {
                Timed t(c, FLACGPU_K_SCAN, c->ovl);
                if (i == 0 && hipMemsetAsync(c->d_cum, 0, sizeof(uint64_t), c->ovl) != hipSuccess)
                    return release(), FLACGPU_ERR_DEVICE;
                const hipError_t e = launch_scan(d_fbytes + s0, d_offsets + s0, i + 1 == K ? d_total : c->d_cum + i + 1,
                                                 (uint32_t)(s1 - s0), c->d_scan_part, c->ovl, c->d_cum + i);
                if (e != hipSuccess) return release(), hip_err(e);
            }
            if ((rc = pack_full(j0, j1 - j0, i, c->ovl_pack, c->ovl))) return release(), rc;
        }
        if (n_tail && (rc = pack_tail(c->ovl))) return release(), rc;
        // st continues after the last pack
        hipEvent_t done = get_event(c);
        if (!done) return release(), FLACGPU_ERR_DEVICE;
        evs.push_back(done);
        if (hipEventRecord(done, c->ovl) != hipSuccess || hipStreamWaitEvent(st, done, 0) != hipSuccess)
            return release(), FLACGPU_ERR_DEVICE;
        release();  // the waits are enqueued: the events can be recorded again
        return FLACGPU_OK;
    }

    int rc;
    if (n_full && (rc = analyze_full(0, n_full, 0, 0, st))) return rc;
    if (n_tail && (rc = analyze_tail(st))) return rc;
    {
        Timed t(c, FLACGPU_K_SCAN, st);
        HIPCHK(launch_scan(d_fbytes, d_offsets, d_total, (uint32_t)n_frames, c->d_scan_part, st));
    }
    if (n_full && (rc = pack_full(0, n_full, 0, 0, st))) return rc;
    if (n_tail && (rc = pack_tail(st))) return rc;
    return FLACGPU_OK;
}

int check_device_error(flacgpu_ctx *c) {
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, c->d_err, 4, hipMemcpyDeviceToHost));
    if (err) {
        hipMemset(c->d_err, 0, 4);
        return (err & 2u) && !(err & 1u) ? FLACGPU_ERR_OUTPUT_TOO_SMALL : FLACGPU_ERR_INTERNAL;
    }
    return FLACGPU_OK;
}

// Wait on the host for everything queued on st so far, through the context's event i (blocking
// sync: the thread sleeps).
hipError_t wait_host(flacgpu_ctx *c, hipStream_t st, int i) {
    hipError_t e = hipEventRecord(c->hw[i], st);
    return e != hipSuccess ? e : hipEventSynchronize(c->hw[i]);
}

// check_device_error after a blocking wait on st (the pipelined path's end)
int check_device_error_on(flacgpu_ctx *c, hipStream_t st) {
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, c->d_err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(wait_host(c, st, 3));
    if (err) {
        hipMemset(c->d_err, 0, 4);
        return (err & 2u) && !(err & 1u) ? FLACGPU_ERR_OUTPUT_TOO_SMALL : FLACGPU_ERR_INTERNAL;
    }
    return FLACGPU_OK;
}

int fetch_records(flacgpu_ctx *c, uint64_t n_frames, hipStream_t st) {
    if (!c->records_on) return FLACGPU_OK;
    const size_t base = c->h_records.size();
    c->h_records.resize(base + n_frames);
    HIPCHK(hipMemcpyAsync(c->h_records.data() + base, c->d_records, n_frames * sizeof(FrameRec),
                          hipMemcpyDeviceToHost, st));
    return FLACGPU_OK;
}

}  // namespace

// One chunk of at most max_frames frames (fg_internal.hpp): upload, encode, wait; the
// frames stay in the context's device output until ctx_download_chunk.
int fg::ctx_encode_chunk(flacgpu_ctx *c, const uint8_t *src, uint64_t ns, uint64_t first_number, uint64_t *total,
                         uint32_t *frame_bytes) {
    const uint32_t bs = c->cfg.block_size;
    const uint64_t nf = frames_for(ns, bs);
    if (nf > c->max_frames || !total) return FLACGPU_ERR_INVALID_INPUT;
    *total = 0;
    if (nf == 0) return FLACGPU_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->d_pcm, src, ns * c->C * c->B, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_make_jobs(c->d_jobs, ns, bs, (uint32_t)((uint64_t)bs * c->C * c->B), first_number, (uint32_t)nf,
                            c->stream));
    // frames with n == 4096 take the lane-owned-partition kernel, the rest the general one
    const uint64_t n_full = (bs == (uint32_t)kBlock) ? ns / kBlock : 0;
    int rc = encode_core(c, c->d_pcm, c->d_jobs, n_full, nf - n_full, c->d_desc, c->d_fbytes, c->d_out, c->out_cap,
                         c->d_offsets, c->d_total, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(total, c->d_total, 8, hipMemcpyDeviceToHost, c->stream));
    if (frame_bytes) HIPCHK(hipMemcpyAsync(frame_bytes, c->d_fbytes, nf * 4, hipMemcpyDeviceToHost, c->stream));
    if ((rc = fetch_records(c, nf, c->stream))) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return check_device_error(c);
}

int fg::ctx_download_chunk(flacgpu_ctx *c, uint8_t *out, uint64_t total) {
    if (!total) return FLACGPU_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(out, c->d_out, total, hipMemcpyDeviceToHost));
    return FLACGPU_OK;
}

uint32_t fg::ctx_max_frames(const flacgpu_ctx *c) { return c->max_frames; }
bool fg::ctx_plain(const flacgpu_ctx *c) { return !c->records_on && !c->timing && c->ovl_chunks <= 1 && !c->fused; }
fg::CtxDevice fg::ctx_device(const flacgpu_ctx *c) {
    return {c->device, (void *)c->stream, c->d_out, c->d_fbytes, c->d_total, c->out_cap, c->C, c->B,
            c->cfg.block_size};
}
void fg::ctx_finish(flacgpu_ctx *c) { resolve_timing(c); }

extern "C" {

flacgpu_config flacgpu_config_default(uint32_t channels, uint32_t bits_per_sample, uint32_t sample_rate) {
    flacgpu_config c{};
    c.sample_rate = sample_rate;
    c.block_size = 4096;
    c.channels = (uint8_t)channels;
    c.bits_per_sample = (uint8_t)bits_per_sample;
    c.stereo_decorrelation = 1;
    c.max_rice_part_order = 8;
    c.max_rice_param = 30;
    c.prediction = 0;
    return c;
}

const char *flacgpu_strerror(int code) {
    switch (code) {
        case FLACGPU_OK: return "ok";
        case FLACGPU_ERR_INVALID_CONFIG: return "invalid config";
        case FLACGPU_ERR_INVALID_INPUT: return "invalid input";
        case FLACGPU_ERR_OUT_OF_MEMORY: return "out of memory";
        case FLACGPU_ERR_OUTPUT_TOO_SMALL: return "output buffer too small";
        case FLACGPU_ERR_DEVICE: return "HIP device error (no usable gfx950 device?)";
        case FLACGPU_ERR_INTERNAL: return "device-side invariant violated";
        default: return "unknown error";
    }
}

int flacgpu_abi_version(void) { return FLACGPU_ABI_VERSION; }

uint32_t flacgpu_build_flags(void) {
    uint32_t f = 0;
#if FG_DIAG
    f |= FLACGPU_BUILD_DIAG;
#endif
#ifdef FG_STAMPS
    f |= FLACGPU_BUILD_STAMPS;
#endif
    return f;
}

int flacgpu_get_config(const flacgpu_ctx *c, flacgpu_config *out) {
    if (!c || !out) return FLACGPU_ERR_INVALID_INPUT;
    *out = c->cfg;
    return FLACGPU_OK;
}

size_t flacgpu_reference_max_frame_bytes(const flacgpu_config *cfg) {
    if (!cfg) return 0;
    // maxFrameBytes(block_size, bit_depth, channels, compute_waste_bits=true) (encoder.zig:55-60,583-595)
    const size_t bps = cfg->channels == 2 ? cfg->bits_per_sample + 1u : cfg->bits_per_sample;
    return 14u + 8u * cfg->channels + (size_t)cfg->block_size * ((bps + 7) / 8) * (cfg->channels + 1u) + 2u;
}

size_t flacgpu_frame_bound_bytes(const flacgpu_config *cfg) {
    if (!cfg) return 0;
    const bool stereo = cfg->channels == 2 && cfg->stereo_decorrelation;
    return frame_bound_bytes(kBlock, cfg->channels, cfg->bits_per_sample, stereo);
}

int flacgpu_open(int device, const flacgpu_config *cfg, uint32_t max_frames_per_call, flacgpu_ctx **out) {
    if (!out) return FLACGPU_ERR_INVALID_INPUT;
    *out = nullptr;
    int rc = validate(cfg);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return FLACGPU_ERR_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return FLACGPU_ERR_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FLACGPU_ERR_DEVICE;  // code objects are gfx950-only
    HIPCHK(hipSetDevice(device));

    auto *c = new (std::nothrow) flacgpu_ctx();
    if (!c) return FLACGPU_ERR_OUT_OF_MEMORY;
    c->device = device;
    c->cfg = *cfg;
    c->max_frames = max_frames_per_call ? max_frames_per_call : 32768u;
    c->C = cfg->channels;
    c->bits = cfg->bits_per_sample;
    c->B = c->bits / 8;
    c->stereo = (c->C == 2 && cfg->stereo_decorrelation) ? 1u : 0u;
    const uint32_t nw = c->stereo ? 4u : c->C;
    const uint32_t n_out = c->stereo ? 2u : c->C;
    c->nt = 64u * nw;
    c->nt_pack = 64u * n_out;
    c->image_bytes = fg_round16(frame_bound_bytes(kBlock, c->C, c->bits, c->stereo != 0) + 16u);
    c->desc_stride = desc_stride(n_out);
    const bool lpc = c->cfg.prediction != 0;
    // 24-bit LPC analysis runs three waves per SIMD (fg_device.hpp): double-buffer only where
    // three workgroups still fit the LDS
    const uint32_t ana_wgs = (lpc && c->B == 3) ? (FG_C3_W == 3 ? 3u : 2u) : 1u;
    c->stage_dbuf = ana_layout(c->C, c->B, nw, true, true, lpc).total * ana_wgs <= 160u * 1024u;
    c->lds = ana_layout(c->C, c->B, nw, true, c->stage_dbuf, lpc).total;
    c->lds_tail = ana_layout(c->C, c->B, nw, false, false, lpc).total;
    // Frames of 4+ independent channels too large to double-buffer: analyse them in channel
    // halves (one workgroup per half, staged single-buffered) when a half is whole dwords of
    // every interchannel row and two halves fit a CU -- c4: three 51-KiB workgroups per CU
    // instead of one 96-KiB frame (analysis 5.35 -> 4.77 ms per 65536 frames, same-box A/B).
    if (!c->stereo && c->C >= 4u && (c->C & 1u) == 0 && ((c->C / 2u) * c->B) % 4u == 0 && !c->stage_dbuf) {
        const uint32_t ch = c->C / 2u, lh = ana_layout(ch, c->B, ch, true, false, lpc).total;
        if (2u * lh <= 160u * 1024u) {
            c->ana_split = true;
            c->nt_split = 64u * ch;
            c->lds_split = lh;
        }
    }
    // pack: double-buffer the staging when that keeps the register-limited occupancy
    // (4 workgroups per CU; 2 for 32-bit samples)
    const uint32_t pack_wgs = c->B == 4 ? 2u : 4u;
    c->pack_dbuf = pack_layout(c->C, c->B, c->image_bytes, true).total * pack_wgs <= 160u * 1024u;
    // output-invariant tuning knobs (schedule / kernel-variant choices; every setting is
    // parity-tested: tests/test_gpu_parity.py, test_gpu_plan.py; INTEGRATION.md lists them)
    if (const char *e = std::getenv("FLACGPU_PACK_DBUF")) c->pack_dbuf = c->pack_dbuf && e[0] == '1';
    // 32-bit samples (c5): the 48-KiB three-chunk ring (kernel 2) -- same-box A/B r4m, 2 reps:
    // c5 24.19-24.25k -> 24.67-24.68k MS/s (MD5 10.1 -> 9.5 ms, analysis 8.84 -> 8.58 ms beside
    // it); c3 neutral, C2 -4 %, so the others keep kernel 1
    if (c->B == 4u) c->md5_kernel = 2;
    if (const char *e = std::getenv("FLACGPU_MD5_KERNEL")) c->md5_kernel = std::atoi(e);
    if (const char *e = std::getenv("FLACGPU_XCD_QUEUE")) c->xcd_queue = e[0] != '0';
    if (const char *e = std::getenv("FLACGPU_PACK_XCDQ")) c->pack_xcdq = e[0] != '0';
    if (const char *e = std::getenv("FLACGPU_SPLIT_JIT")) c->split_jit = (uint32_t)std::atoi(e) & 3u;
    if (const char *e = std::getenv("FLACGPU_PIPE_SETS")) {
        const int v = std::atoi(e);
        c->pipe_sets = v >= 2 && v <= (int)kPipeSets ? (uint32_t)v : kPipeSetsDefault;
    }
    // issue priority of the stream-MD5 waves (output-invariant): 1 trades 2-5 % of the encode for a
    // 35-58 % shorter MD5 chain -- for a workload whose MD5 would bind the step
    if (const char *e = std::getenv("FLACGPU_MD5_PRIO")) c->md5_prio = std::atoi(e) ? 1 : 0;
#if FG_DIAG
    // diagnostic build only: grid reserves, the overlapped schedule's shape
    if (const char *e = std::getenv("FLACGPU_ENC_PRIO")) c->enc_prio = e[0] == '1' ? 1u : 0u;
    if (const char *e = std::getenv("FLACGPU_MD5_RESERVE")) c->md5_reserve = std::atoi(e);
    if (const char *e = std::getenv("FLACGPU_MD5_DIAG")) c->md5_prio |= std::atoi(e) << 8;
    if (const char *e = std::getenv("FLACGPU_OVERLAP")) c->ovl_chunks = (uint32_t)std::atoi(e);
    if (const char *e = std::getenv("FLACGPU_OVL_ANA")) c->ovl_ana = (uint32_t)std::atoi(e);
    if (const char *e = std::getenv("FLACGPU_OVL_PACK")) c->ovl_pack = (uint32_t)std::atoi(e);
    if (const char *e = std::getenv("FLACGPU_OVL_MIN")) c->ovl_min_frames = (uint32_t)std::max(1, std::atoi(e));
#endif
    c->lds_pack = pack_layout(c->C, c->B, c->image_bytes, c->pack_dbuf).total;
    // CRC fold: half-segments of H words (odd), H <= ceil(image words / (2 * pack threads))
    c->crc_hmax = ((c->image_bytes / 4u + 2u * c->nt_pack - 1u) / (2u * c->nt_pack)) | 1u;
    if (c->C == 2 && c->B == 2 && !lpc) {
        c->nt_pack4 = 512u;
        if (const char *e = std::getenv("FLACGPU_PACK4")) c->nt_pack4 = e[0] == '0' ? 0u : 512u;  // A/B knob
    }
    bool packw_dbuf = true;
    // k_packw (fg_packw.hpp) where k_pack's occupancy is poor: 32-bit samples (i64 lanes, 2 waves
    // per SIMD) or more than two written subframes (one workgroup per CU).  Mono/stereo 8-24-bit
    // frames stay on k_pack: its small single-buffered workgroups keep 4-5 frames in flight per
    // CU, which measured faster (c3 pack alone: 1.26 ms vs 1.40-1.66 ms for the packw variants).
    bool use_packw = c->B == 4u || n_out > 2u;
    if (const char *e = std::getenv("FLACGPU_PACKW")) use_packw = e[0] == '1' ? true : (e[0] == '0' ? false : use_packw);  // A/B knob
    if (!c->nt_pack4 && use_packw) {
        // WPS waves per written subframe, 16 (<= 4 subframes) or 32 samples per lane;
        // double-buffered staging where two workgroups per CU still fit
        uint32_t wps = n_out <= 4u ? 4u : 2u;
        if (const char *e = std::getenv("FLACGPU_PACKW_WPS")) wps = (e[0] == '2' && n_out <= 8u) ? 2u : wps;  // tuning knob
        c->nt_pack4 = 64u * n_out * wps;
        packw_dbuf = packw_layout(c->C, c->B, wps, c->image_bytes, true, n_out).total * 2u <= 160u * 1024u;
        if (const char *e = std::getenv("FLACGPU_PACKW_DBUF")) packw_dbuf = packw_dbuf && e[0] == '1';  // tuning knob
        c->pack_dbuf = packw_dbuf;  // k_pack then runs tail frames only (never double-buffered)
    }
    if (c->nt_pack4) {
        c->lds_pack4 = (c->C == 2 && c->B == 2 && !lpc) ? pack4_layout(c->image_bytes).total
                                                         : packw_layout(c->C, c->B, c->nt_pack4 / (64u * n_out), c->image_bytes, packw_dbuf, n_out).total;
        c->crc_hmax4 = ((c->image_bytes / 4u + 2u * c->nt_pack4 - 1u) / (2u * c->nt_pack4)) | 1u;
    }
    // Frames whose single-buffered k_packw staging admits one workgroup per CU and whose analysis
    // runs in channel halves are packed in channel halves too (two workgroups per CU, see k_packw)
    if (c->ana_split && use_packw && !packw_dbuf) {
        const uint32_t ch = c->C / 2u;
        const uint32_t img = fg_round16(frame_bound_bytes(kBlock, ch, c->bits, false) + 16u);
        const uint32_t lh = packw_layout(ch, c->B, 2u, img, false, ch).total;
        bool on = 2u * lh <= 160u * 1024u;
        if (const char *e = std::getenv("FLACGPU_PACK_SPLIT")) on = on && e[0] != '0';  // A/B knob
        if (on) {
            c->pack_split = true;
            c->nt_psplit = 64u * ch * 2u;
            c->lds_psplit = lh;
            c->image_split = img;
            c->crc_hmaxs = ((img / 4u + 2u * c->nt_psplit - 1u) / (2u * c->nt_psplit)) | 1u;
        }
    }
#if FG_DIAG
    if (c->C == 2 && c->B == 2 && !lpc && c->stereo) {
        c->ana1 = false;  // measured slower than k_analyze so far: opt-in
        if (const char *e = std::getenv("FLACGPU_ANA1")) {  // A/B knob: 0 = k_analyze, 1 / 2 = k_ana1 variant
            c->ana1 = e[0] != '0';
            c->ana1_variant = e[0] == '2' ? 2u : 1u;
        }
        c->fused = false;
        if (const char *e = std::getenv("FLACGPU_FUSED")) c->fused = e[0] == '1';  // A/B knob
        c->lds_fused = ana_layout(2, 2, 4, true, false, false, c->image_bytes).total;
        c->crc_hmaxf = ((c->image_bytes / 4u + 2u * 256u - 1u) / (2u * 256u)) | 1u;
    }
#endif
    if (c->lds > 160u * 1024u || c->lds_tail > 160u * 1024u || c->lds_pack > 160u * 1024u ||
        c->lds_pack4 > 160u * 1024u) {
        delete c;
        return FLACGPU_ERR_INVALID_CONFIG;
    }

    auto fail = [&](int code) {
        flacgpu_close(c);
        return code;
    };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipStreamCreateWithFlags(&c->dl, hipStreamNonBlocking) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    for (hipEvent_t &ev : c->up_done)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipStreamCreateWithFlags(&c->ovl, hipStreamNonBlocking) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    if (hipEventCreateWithFlags(&c->join, hipEventDisableTiming) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    {
        unsigned fl = hipEventDisableTiming | hipEventBlockingSync;
#if FG_DIAG
        if (const char *e = std::getenv("FLACGPU_SPIN_SYNC")) fl = e[0] == '1' ? hipEventDisableTiming : fl;
#endif
        for (hipEvent_t &ev : c->hw)
            if (hipEventCreateWithFlags(&ev, fl) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
        for (hipEvent_t &ev : c->set_done)
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
        for (hipEvent_t &ev : c->dl_done)
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(FLACGPU_ERR_DEVICE);
    }

    // CRC-16 shift constants of the table-free fold (mod Q, fg_device.hpp crc_lane_q): thread t
    // of T folds 2H words, followed by 2H (T - 1 - t) words and the CRC's z^16
    const uint32_t T = c->nt_pack, HM = c->crc_hmax;
    std::vector<uint16_t> pw((size_t)HM * T), pj(HM);
    for (uint32_t h = 1; h <= HM; h++) {
        pj[h - 1] = (uint16_t)q_zpow(32ull * h);
        for (uint32_t t = 0; t < T; t++) pw[(size_t)(h - 1) * T + t] = (uint16_t)q_zpow(16ull + 64ull * h * (T - 1u - t));
    }
    const uint32_t T4 = c->nt_pack4, HM4 = c->crc_hmax4;
    std::vector<uint16_t> pw4((size_t)HM4 * T4 + 1);
    for (uint32_t h = 1; h <= HM4; h++)
        for (uint32_t t = 0; t < T4; t++) pw4[(size_t)(h - 1) * T4 + t] = (uint16_t)q_zpow(16ull + 64ull * h * (T4 - 1u - t));

    if (c->crc_hmaxf) {
        std::vector<uint16_t> pwf((size_t)c->crc_hmaxf * 256u);
        for (uint32_t h = 1; h <= c->crc_hmaxf; h++)
            for (uint32_t t = 0; t < 256u; t++) pwf[(size_t)(h - 1) * 256u + t] = (uint16_t)q_zpow(16ull + 64ull * h * (255u - t));
        if (hipMalloc(&c->d_crc_powf, pwf.size() * 2) ||
            hipMemcpy(c->d_crc_powf, pwf.data(), pwf.size() * 2, hipMemcpyHostToDevice))
            return fail(FLACGPU_ERR_DEVICE);
    }
    std::vector<uint16_t> pws((size_t)c->crc_hmaxs * c->nt_psplit + 1), x8(24);
    for (uint32_t h = 1; h <= c->crc_hmaxs; h++)
        for (uint32_t t = 0; t < c->nt_psplit; t++)
            pws[(size_t)(h - 1) * c->nt_psplit + t] = (uint16_t)q_zpow(16ull + 64ull * h * (c->nt_psplit - 1u - t));
    for (uint32_t i = 0; i < 24; i++) x8[i] = (uint16_t)crc_zpow(8ull << i);
    if (hipMalloc(&c->d_crc_pows, pws.size() * 2) || hipMalloc(&c->d_crc_x8, 48) ||
        hipMemcpy(c->d_crc_pows, pws.data(), pws.size() * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(c->d_crc_x8, x8.data(), 48, hipMemcpyHostToDevice))
        return fail(FLACGPU_ERR_DEVICE);

    const uint64_t F = c->max_frames;
    c->pcm_cap = F * (uint64_t)kBlock * c->C * c->B + 64;
    c->out_cap = F * (uint64_t)c->image_bytes;
    if (hipMalloc(&c->d_crc_pow, pw.size() * 2) ||
        hipMalloc(&c->d_crc_pow4, pw4.size() * 2) ||
        hipMalloc(&c->d_crc_join, pj.size() * 2) || hipMalloc(&c->d_err, 16) || hipMalloc(&c->d_ctr, 4u * kCtrSet * kOvlMaxChunks) ||
        hipMalloc(&c->d_cum, 8u * (kOvlMaxChunks + 1u)) ||
        hipMalloc(&c->d_jobs, F * sizeof(FrameJob)) || hipMalloc(&c->d_desc, F * (uint64_t)c->desc_stride) ||
        hipMalloc(&c->d_fbytes, F * 4) || hipMalloc(&c->d_offsets, F * 8) || hipMalloc(&c->d_total, 8u * (kPipeSets + 1u)) ||
        hipMalloc(&c->d_pcm, c->pcm_cap) || hipMalloc(&c->d_out, c->out_cap) || hipMalloc(&c->d_md5_state, 16) || hipMalloc(&c->d_stamps, 32 * 8))
        return fail(FLACGPU_ERR_OUT_OF_MEMORY);
    if (hipMemcpy(c->d_crc_pow, pw.data(), pw.size() * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(c->d_crc_pow4, pw4.data(), pw4.size() * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(c->d_crc_join, pj.data(), pj.size() * 2, hipMemcpyHostToDevice) || hipMemset(c->d_err, 0, 16) || hipMemset(c->d_ctr, 0, 4u * kCtrSet * kOvlMaxChunks) ||
        hipMemset(c->d_stamps, 0, 32 * 8))
        return fail(FLACGPU_ERR_DEVICE);
    flacgpu_md5_init(c);
    *out = c;
    return FLACGPU_OK;
}

void flacgpu_close(flacgpu_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    resolve_timing(c);
    for (auto e : c->event_pool) hipEventDestroy(e);
    hipFree(c->d_crc_pow);
    hipFree(c->d_crc_pow4);
    hipFree(c->d_crc_powf);
    hipFree(c->d_status);
    hipFree(c->d_crc_join);
    hipFree(c->d_scan_part);
    hipFree(c->d_err);
    hipFree(c->d_ctr);
    hipFree(c->d_cum);
    hipFree(c->d_jobs);
    hipFree(c->d_desc);
    hipFree(c->d_fbytes);
    hipFree(c->d_offsets);
    hipFree(c->d_total);
    hipFree(c->d_pcm);
    hipFree(c->d_out);
    hipFree(c->d_records);
    hipFree(c->d_stamps);
    hipFree(c->d_crc_pows);
    hipFree(c->d_crc_x8);
    hipFree(c->d_md5_state);
    hipFree(c->d_md5_blocks);
    if (c->fork) hipEventDestroy(c->fork);
    if (c->join) hipEventDestroy(c->join);
    for (hipEvent_t e : c->hw)
        if (e) hipEventDestroy(e);
    if (c->aux) hipStreamDestroy(c->aux);
    if (c->dl) hipStreamDestroy(c->dl);
    if (c->up) hipStreamDestroy(c->up);
    for (hipEvent_t e : c->up_done)
        if (e) hipEventDestroy(e);
    for (hipEvent_t e : c->set_done)
        if (e) hipEventDestroy(e);
    for (hipEvent_t e : c->dl_done)
        if (e) hipEventDestroy(e);
    if (c->ovl) hipStreamDestroy(c->ovl);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

// Host buffers in, host buffers out, with both PCIe directions and the encode overlapped: the
// context's device buffers split into kPipeSets (3) chunk sets; chunk i+1 uploads on c->up while
// chunk i encodes on c->stream and the frames of chunks i-1, i-2 download on c->dl, issued by one
// worker thread (pageable copies block the issuing thread, so the download needs a thread of its own).
// Output bytes and frame sizes are identical to the sequential loop; only the schedule differs.
// The input is a list of segments (files, flacgpu_encode_files): chunks never span two, and the
// pipeline runs on from one segment into the next instead of draining at each file's end.
struct PipeSeg {
    const uint8_t *src;
    uint64_t n_samples, first_frame_number;
    uint8_t *out;
    size_t out_cap, written;
    uint32_t *frame_bytes;  // may be NULL
};

// encode_pipelined could not start its download thread: nothing was queued, encode sequentially
constexpr int kNoWorker = -1000;

static int encode_pipelined(flacgpu_ctx *c, PipeSeg *segs, size_t nseg) {
    const uint32_t bs = c->cfg.block_size;
    const uint64_t stride = (uint64_t)bs * c->C * c->B;
    // chunks of at most 2048 frames (32 MiB of 16-bit stereo) so that long inputs keep both
    // PCIe directions busy; the thirds of the context's buffers hold one chunk each
    const uint32_t NS = c->pipe_sets;
    const uint64_t part = c->max_frames / NS;  // frames of one chunk set
    const uint64_t F = std::min<uint64_t>(part, 2048u);
    const uint64_t pcm_half = part * kBlock * c->C * c->B;  // 16-B multiple
    const uint64_t out_half = part * c->image_bytes;
    const uint64_t fb_half = part;
    hipEvent_t *done = c->set_done;  // a chunk set's encode finished
    struct Dl {
        int set;
        PipeSeg *sg;
        uint64_t frame0, nf;
    };
    // the download worker: one thread for the whole call, fed chunk by chunk
    std::mutex m;
    std::condition_variable cv;
    std::deque<Dl> q;
    uint64_t n_done = 0;  // downloads issued (in chunk order; dl_done[set] marks their completion)
    bool closing = false;
    int wrc = FLACGPU_OK;  // the first download error
    // One host wait per chunk: the download stream waits for the chunk's encode on the GPU, the
    // worker reads the chunk's byte count (it places the next chunk of the segment), then issues
    // the copies and records dl_done[set], on which the next encode into that set waits GPU-side.
    // (Round 4 slept on three blocking-sync events per chunk -- encode done, count, copies done --
    // and the 64-file batch moved 33 GB/s of PCM against 56 GB/s of chunked H2D beside D2H.)
    auto download = [&](const Dl &d) -> int {
        PipeSeg *sg = d.sg;
        uint64_t total = 0;
        if (hipSetDevice(c->device) != hipSuccess || hipStreamWaitEvent(c->dl, done[d.set], 0) != hipSuccess ||
            hipMemcpyAsync(&total, c->d_total + d.set, 8, hipMemcpyDeviceToHost, c->dl) != hipSuccess ||
            wait_host(c, c->dl, 2) != hipSuccess)
            return FLACGPU_ERR_DEVICE;
        if (sg->written + total > sg->out_cap) return FLACGPU_ERR_OUTPUT_TOO_SMALL;
        if ((sg->frame_bytes && hipMemcpyAsync(sg->frame_bytes + d.frame0, c->d_fbytes + d.set * fb_half, d.nf * 4,
                                               hipMemcpyDeviceToHost, c->dl) != hipSuccess) ||
            hipMemcpyAsync(sg->out + sg->written, c->d_out + d.set * out_half, total, hipMemcpyDeviceToHost, c->dl) !=
                hipSuccess ||
            hipEventRecord(c->dl_done[d.set], c->dl) != hipSuccess)
            return FLACGPU_ERR_DEVICE;
        sg->written += total;
        return FLACGPU_OK;
    };
    auto work = [&]() {
        for (;;) {
            Dl d;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return closing || !q.empty(); });
                if (q.empty()) return;
                d = q.front();
                q.pop_front();
            }
            const int r = wrc == FLACGPU_OK ? download(d) : FLACGPU_OK;  // after an error: drain only
            {
                std::lock_guard<std::mutex> lk(m);
                if (r != FLACGPU_OK && wrc == FLACGPU_OK) wrc = r;
                n_done++;
            }
            cv.notify_all();
        }
    };
    std::thread worker;
    try {
        worker = std::thread(work);
    } catch (const std::system_error &) {
        return kNoWorker;  // the caller encodes chunk by chunk on this thread instead
    }
    // wait (host) until at least `k` downloads have been issued; the first download error
    auto wait_done = [&](uint64_t k) -> int {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return n_done >= k || wrc != FLACGPU_OK; });
        return wrc;
    };
    int rc = FLACGPU_OK;
    uint64_t chunk = 0;  // chunks issued so far
    for (size_t si = 0; si < nseg && rc == FLACGPU_OK; si++) {
        PipeSeg *sg = &segs[si];
        sg->written = 0;
        const uint64_t total_frames = frames_for(sg->n_samples, bs);
        for (uint64_t frame0 = 0; frame0 < total_frames && rc == FLACGPU_OK; chunk++) {
            const int set = (int)(chunk % NS);
            const uint64_t nf = std::min<uint64_t>(F, total_frames - frame0);
            const uint64_t s0 = frame0 * bs;
            const uint64_t ns = std::min<uint64_t>(nf * bs, sg->n_samples - s0);
            uint8_t *dp = c->d_pcm + set * pcm_half;
            // upload: the PCM part was last read by chunk i-3's encode (its `done` event, a GPU-side
            // wait); it runs beside chunk i-1's encode and the downloads of chunks i-2, i-3
            if ((chunk >= NS && hipStreamWaitEvent(c->up, done[set], 0) != hipSuccess) ||
                hipMemcpyAsync(dp, sg->src + s0 * c->C * c->B, ns * c->C * c->B, hipMemcpyHostToDevice, c->up) !=
                    hipSuccess ||
                hipEventRecord(c->up_done[set], c->up) != hipSuccess) {
                rc = FLACGPU_ERR_DEVICE;
                break;
            }
            // the encode writes the output part chunk i-3's download reads: that download first
            // (issued by the worker: then the encode stream waits for its copies on the GPU)
            if (chunk >= NS && (rc = wait_done(chunk - NS + 1))) break;
            if ((chunk >= NS && hipStreamWaitEvent(c->stream, c->dl_done[set], 0) != hipSuccess) ||
                hipStreamWaitEvent(c->stream, c->up_done[set], 0) != hipSuccess ||
                launch_make_jobs(c->d_jobs, ns, bs, (uint32_t)stride, sg->first_frame_number + frame0, (uint32_t)nf,
                                 c->stream) != hipSuccess) {
                rc = FLACGPU_ERR_DEVICE;
                break;
            }
            const uint64_t n_full = (bs == (uint32_t)kBlock) ? ns / kBlock : 0;
            if ((rc = encode_core(c, dp, c->d_jobs, n_full, nf - n_full, c->d_desc, c->d_fbytes + set * fb_half,
                                  c->d_out + set * out_half, out_half, c->d_offsets, c->d_total + set, c->stream)))
                break;
            if (hipEventRecord(done[set], c->stream) != hipSuccess) {
                rc = FLACGPU_ERR_DEVICE;
                break;
            }
            {
                std::lock_guard<std::mutex> lk(m);
                q.push_back(Dl{set, sg, frame0, nf});
            }
            cv.notify_all();
            frame0 += nf;
        }
    }
    {
        std::lock_guard<std::mutex> lk(m);
        closing = true;
    }
    cv.notify_all();
    worker.join();
    if (rc == FLACGPU_OK) rc = wrc;
    const hipError_t se = hipStreamSynchronize(c->dl);  // the last chunks' copies
    if (rc == FLACGPU_OK && se != hipSuccess) rc = FLACGPU_ERR_DEVICE;
    if (rc) {
        hipStreamSynchronize(c->up);
        hipStreamSynchronize(c->stream);
        return rc;
    }
    return check_device_error_on(c, c->stream);
}

}  // extern "C"

int fg::ctx_encode_segments(flacgpu_ctx *c, uint32_t n, const uint8_t *const *src, const uint64_t *n_samples,
                            uint8_t *const *out, const size_t *out_cap, size_t *out_len, uint32_t *const *frame_bytes) {
    HIPCHK(hipSetDevice(c->device));
    // contexts the pipeline cannot serve (one frame per call, decision records on), or no thread
    // for its downloads: each file through flacgpu_encode_frames, which is what
    // flacgpu_encode_file does for them
    auto one_by_one = [&]() -> int {
        for (uint32_t i = 0; i < n; i++) out_len[i] = 0;
        // with decision records on, the records of EVERY file are kept, file after file in frame
        // order (flacgpu_get_records), not only the last file's
        if (c->records_on) c->h_records.clear();
        c->records_keep = true;
        for (uint32_t i = 0; i < n; i++) {
            const int r = flacgpu_encode_frames(c, src[i], c->B, n_samples[i], 0, out[i], out_cap[i], &out_len[i],
                                                frame_bytes ? frame_bytes[i] : nullptr);
            if (r) {
                c->records_keep = false;
                for (uint32_t j = 0; j < n; j++) out_len[j] = 0;
                return r;
            }
        }
        c->records_keep = false;
        return FLACGPU_OK;
    };
    if (c->max_frames < c->pipe_sets || c->records_on) return one_by_one();
    std::vector<PipeSeg> segs;
    try {
        segs.resize(n);
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t nf = frames_for(n_samples[i], c->cfg.block_size);
        if (nf && nf - 1 > (1ull << 36) - 1) return FLACGPU_ERR_INVALID_INPUT;  // u36 frame numbers
        segs[i] = PipeSeg{src[i], n_samples[i], 0, out[i], out_cap[i], 0, frame_bytes ? frame_bytes[i] : nullptr};
    }
    const int rc = encode_pipelined(c, segs.data(), n);
    if (rc == kNoWorker) return one_by_one();
    resolve_timing(c);
    for (uint32_t i = 0; i < n; i++) out_len[i] = rc ? 0 : segs[i].written;
    return rc;
}

extern "C" {

int flacgpu_encode_frames(flacgpu_ctx *c, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                          uint64_t first_frame_number, uint8_t *out, size_t out_cap, size_t *out_len,
                          uint32_t *frame_bytes) {
    if (!c || (!pcm && n_samples) || !out_len) return FLACGPU_ERR_INVALID_INPUT;
    if (bytes_per_sample != c->B) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    *out_len = 0;
    const uint32_t bs = c->cfg.block_size;
    const uint64_t stride = (uint64_t)bs * c->C * c->B;
    const uint64_t total_frames = frames_for(n_samples, bs);
    // frame numbers are u36 (frame_writer.zig:153, wav2flac.zig:75)
    if (total_frames && (first_frame_number >= (1ull << 36) || total_frames - 1 > (1ull << 36) - 1 - first_frame_number))
        return FLACGPU_ERR_INVALID_INPUT;
    const uint8_t *src = (const uint8_t *)pcm;
    uint64_t frame0 = 0;
    size_t written = 0;
    if (c->records_on && !c->records_keep) c->h_records.clear();
    if (!c->records_on && c->max_frames >= c->pipe_sets &&
        total_frames > std::min<uint64_t>(c->max_frames / c->pipe_sets, 2048u)) {
        PipeSeg seg{src, n_samples, first_frame_number, out, out_cap, 0, frame_bytes};
        const int rc = encode_pipelined(c, &seg, 1);
        if (rc != kNoWorker) {
            resolve_timing(c);
            if (rc == FLACGPU_OK) *out_len = seg.written;
            return rc;
        }
    }
    (void)stride;
    while (frame0 < total_frames) {
        const uint64_t nf = std::min<uint64_t>(c->max_frames, total_frames - frame0);
        const uint64_t s0 = frame0 * bs;
        const uint64_t ns = std::min<uint64_t>(nf * bs, n_samples - s0);
        uint64_t total = 0;
        int rc = fg::ctx_encode_chunk(c, src + s0 * c->C * c->B, ns, first_frame_number + frame0, &total,
                                      frame_bytes ? frame_bytes + frame0 : nullptr);
        if (rc) return rc;
        if (written + total > out_cap) return FLACGPU_ERR_OUTPUT_TOO_SMALL;
        if ((rc = fg::ctx_download_chunk(c, out + written, total))) return rc;
        written += total;
        frame0 += nf;
    }
    resolve_timing(c);
    *out_len = written;
    return FLACGPU_OK;
}

int flacgpu_encode_frame_planar(flacgpu_ctx *c, const int32_t *const planes[8], uint32_t n, uint64_t frame_number,
                                uint8_t *out, size_t out_cap, uint32_t *frame_bytes) {
    if (!c || !planes || !out || n == 0 || n > c->cfg.block_size) return FLACGPU_ERR_INVALID_INPUT;
    for (uint32_t ch = 0; ch < c->C; ch++)
        if (!planes[ch]) return FLACGPU_ERR_INVALID_INPUT;
    // Encoder.samples[ch][0..n] -> the little-endian interleaved layout the kernels stage
    std::vector<uint8_t> pcm((size_t)n * c->C * c->B + 4);
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t ch = 0; ch < c->C; ch++) {
            const uint32_t v = (uint32_t)planes[ch][i];
            uint8_t *d = &pcm[((size_t)i * c->C + ch) * c->B];
            for (uint32_t k = 0; k < c->B; k++) d[k] = (uint8_t)(v >> (8 * k));
        }
    size_t len = 0;
    uint32_t fb = 0;
    int rc = flacgpu_encode_frames(c, pcm.data(), c->B, n, frame_number, out, out_cap, &len, &fb);
    if (rc) return rc;
    if (frame_bytes) *frame_bytes = fb;
    return FLACGPU_OK;
}

// ---- streaming MD5 --------------------------------------------------------
int flacgpu_md5_set_engine(flacgpu_ctx *c, int engine) {
    if (!c || (engine != FLACGPU_MD5_HOST && engine != FLACGPU_MD5_DEVICE)) return FLACGPU_ERR_INVALID_INPUT;
    c->md5_engine = engine;
    return flacgpu_md5_init(c);
}

int flacgpu_md5_get_engine(const flacgpu_ctx *c) { return c ? c->md5_engine : FLACGPU_ERR_INVALID_INPUT; }

int flacgpu_md5_init(flacgpu_ctx *c) {
    if (!c) return FLACGPU_ERR_INVALID_INPUT;
    c->host_md5.reset();
    c->md5_fill = 0;
    c->md5_len = 0;
    if (c->md5_engine != FLACGPU_MD5_DEVICE) return FLACGPU_OK;
    const uint32_t iv[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(c->d_md5_state, iv, 16, hipMemcpyHostToDevice));
    return FLACGPU_OK;
}

// device engine: whole blocks through one bounded buffer (kMd5ChunkBlocks per launch)
static int md5_push_blocks(flacgpu_ctx *c, const uint8_t *p, uint64_t nblocks) {
    if (!nblocks) return FLACGPU_OK;
    if (!c->d_md5_blocks) HIPCHK(hipMalloc(&c->d_md5_blocks, kMd5ChunkBlocks * 64));
    for (uint64_t b = 0; b < nblocks; b += kMd5ChunkBlocks) {
        const uint64_t nb = std::min<uint64_t>(kMd5ChunkBlocks, nblocks - b);
        HIPCHK(hipMemcpyAsync(c->d_md5_blocks, p + b * 64, nb * 64, hipMemcpyHostToDevice, c->stream));
        {
            Timed t(c, FLACGPU_K_MD5, c->stream);
            HIPCHK(launch_md5_blocks(c->d_md5_state, c->d_md5_blocks, nb, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return FLACGPU_OK;
}

int flacgpu_md5_update(flacgpu_ctx *c, const void *data, size_t len) {
    if (!c || (!data && len)) return FLACGPU_ERR_INVALID_INPUT;
    if (c->md5_engine != FLACGPU_MD5_DEVICE) {
        c->host_md5.update(data, len);
        return FLACGPU_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    const uint8_t *p = (const uint8_t *)data;
    c->md5_len += len;
    if (c->md5_fill) {
        const size_t take = std::min<size_t>(64 - c->md5_fill, len);
        std::memcpy(c->md5_buf + c->md5_fill, p, take);
        c->md5_fill += (uint32_t)take;
        p += take;
        len -= take;
        if (c->md5_fill == 64) {
            int rc = md5_push_blocks(c, c->md5_buf, 1);
            if (rc) return rc;
            c->md5_fill = 0;
        }
    }
    const uint64_t nb = len / 64;
    int rc = md5_push_blocks(c, p, nb);
    if (rc) return rc;
    p += nb * 64;
    len -= nb * 64;
    std::memcpy(c->md5_buf, p, len);
    c->md5_fill = (uint32_t)len;
    return FLACGPU_OK;
}

int flacgpu_md5_final(flacgpu_ctx *c, uint8_t digest[16]) {
    if (!c || !digest) return FLACGPU_ERR_INVALID_INPUT;
    if (c->md5_engine != FLACGPU_MD5_DEVICE) {
        c->host_md5.final(digest);
        return FLACGPU_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    uint8_t tail[128] = {};
    std::memcpy(tail, c->md5_buf, c->md5_fill);
    tail[c->md5_fill] = 0x80;
    const uint32_t nb = c->md5_fill < 56 ? 1 : 2;
    const uint64_t bits = c->md5_len * 8;
    for (int i = 0; i < 8; i++) tail[nb * 64 - 8 + i] = (uint8_t)(bits >> (8 * i));
    int rc = md5_push_blocks(c, tail, nb);
    if (rc) return rc;
    uint32_t st[4];
    HIPCHK(hipMemcpy(st, c->d_md5_state, 16, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) digest[4 * i + j] = (uint8_t)(st[i] >> (8 * j));
    resolve_timing(c);
    return flacgpu_md5_init(c);
}

void flacgpu_md5_state_init(flacgpu_md5_state *s, size_t n) {
    for (size_t i = 0; s && i < n; i++) {
        s[i].h[0] = 0x67452301u;
        s[i].h[1] = 0xefcdab89u;
        s[i].h[2] = 0x98badcfeu;
        s[i].h[3] = 0x10325476u;
        s[i].bytes = 0;
        s[i].finished = 0;
        s[i].reserved = 0;
    }
}

int flacgpu_md5_many(uint32_t n, const void *const *data, const uint64_t *lens, const uint8_t *final,
                     flacgpu_md5_state *states, uint8_t *digests) {
    if (n && (!data || !lens)) return FLACGPU_ERR_INVALID_INPUT;
    for (uint32_t i = 0; i < n; i++) {
        const bool fin = !final || final[i];
        // the state carries no partial block: a chain continues only after whole 64-byte blocks
        if (!fin && (!states || lens[i] % 64u)) return FLACGPU_ERR_INVALID_INPUT;
        if (lens[i] && !data[i]) return FLACGPU_ERR_INVALID_INPUT;
    }
    std::vector<fg::HostMd5> hs;
    std::vector<fg::HostMd5 *> hp;
    std::vector<const uint8_t *> ps;
    std::vector<size_t> ls;
    std::vector<uint32_t> idx;
    try {
        hs.resize(n);
        hp.reserve(n);
        ps.reserve(n);
        ls.reserve(n);
        idx.reserve(n);
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    for (uint32_t i = 0; i < n; i++) {
        const bool fin = !final || final[i];
        if (states && (states[i].finished & 1u)) {
            // a finished chain stays as it is; a final segment reports its digest again
            if (fin && digests)
                for (int w = 0; w < 4; w++)
                    for (int b = 0; b < 4; b++) digests[16 * i + 4 * w + b] = (uint8_t)(states[i].h[w] >> (8 * b));
            continue;
        }
        if (states) {
            std::memcpy(hs[i].h, states[i].h, 16);
            hs[i].bytes = states[i].bytes;
        }
        hp.push_back(&hs[i]);
        ps.push_back((const uint8_t *)data[i]);
        ls.push_back((size_t)lens[i]);
        idx.push_back(i);
    }
    fg::md5_pool_update_many(hp.data(), ps.data(), ls.data(), hp.size());
    for (uint32_t i : idx) {
        const bool fin = !final || final[i];
        const uint64_t bytes = hs[i].bytes;
        uint8_t dg[16];
        if (fin) {
            hs[i].final(dg);
            if (digests) std::memcpy(digests + 16 * (size_t)i, dg, 16);
        }
        if (states) {
            if (fin)
                for (int w = 0; w < 4; w++)
                    states[i].h[w] = (uint32_t)dg[4 * w] | (uint32_t)dg[4 * w + 1] << 8 | (uint32_t)dg[4 * w + 2] << 16 |
                                     (uint32_t)dg[4 * w + 3] << 24;
            else
                std::memcpy(states[i].h, hs[i].h, 16);
            states[i].bytes = bytes;
            states[i].finished = fin ? 1u : 0u;
            states[i].reserved = 0;
        }
    }
    return FLACGPU_OK;
}

int flacgpu_md5_plan_host(const flacgpu_plan *p, const void *h_pcm, flacgpu_md5_state *states, uint8_t *digests) {
    if (!p || (p->n_streams && !h_pcm)) return FLACGPU_ERR_INVALID_INPUT;
    std::vector<const void *> ptrs;
    try {
        ptrs.resize(p->n_streams);
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    for (uint32_t s = 0; s < p->n_streams; s++) ptrs[s] = (const uint8_t *)h_pcm + p->h_md5_offs[s];
    return flacgpu_md5_many(p->n_streams, ptrs.data(), p->h_md5_lens.data(),
                            p->h_md5_fin.empty() ? nullptr : p->h_md5_fin.data(), states, digests);
}

// The engine rates: device figures from bench.py's stream_curve on MI355X (DESIGN.md section 5.2:
// one lane per stream at ~72 MB/s beside the encode, at most ~600 GB/s over the chip -- 16384
// streams: 4.3 GB of MD5 in 7.1 ms); host figures measured on this machine the first time the
// choice is made (fg::md5_measure_rates: the fixed 0.95 GB/s-per-chain constants of round 4 were
// 1.6-3x off on the driver's box, where the picker then chose the slower engine).
static std::mutex g_rates_mu;
static flacgpu_md5_rates g_rates{};
static bool g_rates_set = false;

static flacgpu_md5_rates md5_rates() {
    std::lock_guard<std::mutex> lk(g_rates_mu);
    if (!g_rates_set) {
        flacgpu_md5_rates r{};
        const bool contended = fg::md5_measure_rates(r.host_chain, r.host_chains);
        r.device_lane = 72e6;
        r.device_chip = 600e9;
        r.host_workers = fg::md5_pool_workers();
        r.measured = contended ? 3 : 1;
        g_rates = r;
        g_rates_set = true;
    }
    return g_rates;
}

int flacgpu_md5_get_rates(flacgpu_md5_rates *out) {
    if (!out) return FLACGPU_ERR_INVALID_INPUT;
    *out = md5_rates();
    return FLACGPU_OK;
}

int flacgpu_md5_set_rates(const flacgpu_md5_rates *r) {
    // the whole struct is validated on a local copy first: a rejected call leaves the rates in use
    // (measured or set earlier) as they were
    flacgpu_md5_rates v{};
    if (r) {
        v = *r;
        for (double x : v.host_chain)
            if (!(x > 0)) return FLACGPU_ERR_INVALID_INPUT;
        if (!(v.device_lane > 0) || !(v.device_chip > 0) || v.host_workers < 0) return FLACGPU_ERR_INVALID_INPUT;
        if (!v.host_chains[0])
            for (uint32_t i = 0; i < 4; i++) v.host_chains[i] = i + 1u;
        for (uint32_t i = 1; i < 4; i++)
            if (v.host_chains[i] <= v.host_chains[i - 1]) return FLACGPU_ERR_INVALID_INPUT;
        v.measured = 2;
    }
    std::lock_guard<std::mutex> lk(g_rates_mu);
    if (r) g_rates = v;
    g_rates_set = r != nullptr;
    return FLACGPU_OK;
}

int flacgpu_md5_engine_for(uint32_t n_streams, uint64_t max_len, uint64_t total_len) {
    if (!n_streams || !total_len) return FLACGPU_MD5_DEVICE;
    const flacgpu_md5_rates r = md5_rates();
    const double n = n_streams;
    const double t_dev = std::max((double)max_len / r.device_lane, (double)total_len / r.device_chip);
    double t_host;
    if (r.host_workers <= 0) {
        t_host = (double)total_len / r.host_chain[0];  // no pool: the caller hashes chain after chain
    } else {
        // k chains per worker: the per-worker rate interpolated between the measured points, flat
        // past the last (more chains are time-sliced); with fewer chains than workers, one chain
        // each on n workers
        const double w = r.host_workers;
        const double k = std::ceil(n / w);
        double rw = r.host_chain[3];
        for (int i = 0; i < 4; i++) {
            const double pk = r.host_chains[i] ? r.host_chains[i] : i + 1.0;
            if (k <= pk) {
                if (i == 0) {
                    rw = r.host_chain[0];
                } else {
                    const double p0 = r.host_chains[i - 1] ? r.host_chains[i - 1] : i;
                    rw = r.host_chain[i - 1] + (r.host_chain[i] - r.host_chain[i - 1]) * (k - p0) / (pk - p0);
                }
                break;
            }
        }
        t_host = std::max((double)total_len / (rw * std::min(n, w)), (double)max_len / r.host_chain[0]);
    }
    return t_host < t_dev ? FLACGPU_MD5_HOST : FLACGPU_MD5_DEVICE;
}

int flacgpu_plan_md5_engine(const flacgpu_plan *p) {
    if (!p || !p->n_streams) return FLACGPU_MD5_DEVICE;
    return flacgpu_md5_engine_for(p->n_streams, p->md5_max_len, p->md5_total);
}

// ---- plans (device-resident batches of independent streams) --------------
int flacgpu_plan_create_segments(flacgpu_ctx *c, uint32_t n_streams, const uint64_t *offs, const uint64_t *samples,
                                 uint32_t bytes_per_sample, const uint64_t *first_frame_numbers,
                                 const uint8_t *final_segment, flacgpu_plan **out) {
    if (!c || !out || (n_streams && (!offs || !samples)) || bytes_per_sample != c->B) return FLACGPU_ERR_INVALID_INPUT;
    *out = nullptr;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t bs = c->cfg.block_size;
    const uint64_t fbytes_in = (uint64_t)c->C * c->B;
    std::vector<FrameJob> full, tail;
    std::vector<uint64_t> lens(n_streams);
    uint64_t max_number = 0;
    // validate everything before any allocation
    for (uint32_t s = 0; s < n_streams; s++) {
        // stream starts: 4-byte aligned (the kernels' dword / 16-byte vector loads)
        if (offs[s] & 3u) return FLACGPU_ERR_INVALID_INPUT;
        const uint64_t nf = frames_for(samples[s], bs);
        const uint64_t f0 = first_frame_numbers ? first_frame_numbers[s] : 0;
        if (nf && (f0 >= (1ull << 36) || nf - 1 > (1ull << 36) - 1 - f0)) return FLACGPU_ERR_INVALID_INPUT;  // u36
        if (nf) max_number = std::max(max_number, f0 + nf - 1);
        // a segment that the stream continues after: whole frames and whole MD5 blocks
        if (final_segment && !final_segment[s] && (samples[s] % bs || (samples[s] * fbytes_in) % 64))
            return FLACGPU_ERR_INVALID_INPUT;
    }
    auto *p = new (std::nothrow) flacgpu_plan();
    if (!p) return FLACGPU_ERR_OUT_OF_MEMORY;
    p->ctx = c;
    p->n_streams = n_streams;
    p->B = bytes_per_sample;
    p->max_number = max_number;
    uint64_t slot = 0;
    try {
        p->first_frame.resize(n_streams);
        for (uint32_t s = 0; s < n_streams; s++) {
            p->first_frame[s] = slot;
            lens[s] = samples[s] * fbytes_in;
            p->md5_max_len = std::max(p->md5_max_len, lens[s]);
            p->md5_total += lens[s];
            const uint64_t nf = frames_for(samples[s], bs);
            const uint64_t f0 = first_frame_numbers ? first_frame_numbers[s] : 0;
            for (uint64_t f = 0; f < nf; f++, slot++) {
                FrameJob j;
                j.pcm_off = offs[s] + f * bs * fbytes_in;
                j.number = f0 + f;
                j.n = (uint32_t)std::min<uint64_t>(bs, samples[s] - f * bs);
                j.slot = (uint32_t)slot;
                (j.n == (uint32_t)kBlock ? full : tail).push_back(j);
                if (j.n == (uint32_t)kBlock) p->full_slots.push_back(j.slot);
            }
        }
        full.insert(full.end(), tail.begin(), tail.end());
        p->h_md5_offs.assign(offs, offs + n_streams);
        p->h_md5_lens = lens;
        if (final_segment) p->h_md5_fin.assign(final_segment, final_segment + n_streams);
    } catch (...) {
        delete p;
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    p->n_frames = slot;
    p->n_full = full.size() - tail.size();
    p->n_tail = tail.size();
    p->out_bound = slot * (uint64_t)c->image_bytes;
    auto fail = [&](int code) {
        flacgpu_plan_destroy(p);
        return code;
    };
    if (slot > 0xFFFFFFFFull) return fail(FLACGPU_ERR_INVALID_INPUT);
    if (slot) {
        if (hipMalloc(&p->d_jobs, slot * sizeof(FrameJob))) return fail(FLACGPU_ERR_OUT_OF_MEMORY);
        if (hipMemcpy(p->d_jobs, full.data(), slot * sizeof(FrameJob), hipMemcpyHostToDevice))
            return fail(FLACGPU_ERR_DEVICE);
    }
    if (n_streams) {
        if (hipMalloc(&p->d_md5_offs, n_streams * 8) || hipMalloc(&p->d_md5_lens, n_streams * 8))
            return fail(FLACGPU_ERR_OUT_OF_MEMORY);
        if (hipMemcpy(p->d_md5_offs, offs, n_streams * 8, hipMemcpyHostToDevice) ||
            hipMemcpy(p->d_md5_lens, lens.data(), n_streams * 8, hipMemcpyHostToDevice))
            return fail(FLACGPU_ERR_DEVICE);
        if (final_segment) {
            if (hipMalloc(&p->d_md5_fin, n_streams)) return fail(FLACGPU_ERR_OUT_OF_MEMORY);
            if (hipMemcpy(p->d_md5_fin, final_segment, n_streams, hipMemcpyHostToDevice)) return fail(FLACGPU_ERR_DEVICE);
        }
    }
    if (slot > c->max_frames && hipMalloc(&p->d_desc, slot * (uint64_t)c->desc_stride))
        return fail(FLACGPU_ERR_OUT_OF_MEMORY);
    *out = p;
    return FLACGPU_OK;
}

int flacgpu_plan_create(flacgpu_ctx *c, uint32_t n_streams, const uint64_t *offs, const uint64_t *samples,
                        uint32_t bytes_per_sample, flacgpu_plan **out) {
    return flacgpu_plan_create_segments(c, n_streams, offs, samples, bytes_per_sample, nullptr, nullptr, out);
}

void flacgpu_plan_destroy(flacgpu_plan *p) {
    if (!p) return;
    hipFree(p->d_jobs);
    hipFree(p->d_md5_offs);
    hipFree(p->d_md5_lens);
    hipFree(p->d_md5_fin);
    hipFree(p->d_desc);
    delete p;
}

uint64_t flacgpu_plan_frames(const flacgpu_plan *p) { return p ? p->n_frames : 0; }
uint64_t flacgpu_plan_out_bound(const flacgpu_plan *p) { return p ? p->out_bound : 0; }
uint64_t flacgpu_plan_stream_first_frame(const flacgpu_plan *p, uint32_t s) {
    return (p && s < p->n_streams) ? p->first_frame[s] : 0;
}

int flacgpu_plan_advance(flacgpu_plan *p, uint64_t frames, void *hip_stream) {
    if (!p) return FLACGPU_ERR_INVALID_INPUT;
    if (!frames || !p->n_frames) return FLACGPU_OK;
    if (frames > (1ull << 36) - 1 - p->max_number) return FLACGPU_ERR_INVALID_INPUT;  // u36 frame numbers
    flacgpu_ctx *c = p->ctx;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = pick_stream(c, hip_stream);
    HIPCHK(launch_advance_jobs(p->d_jobs, p->n_frames, frames, st));
    p->max_number += frames;
    return FLACGPU_OK;
}

int flacgpu_encode_plan_device_ex(flacgpu_ctx *c, const flacgpu_plan *p, const void *d_pcm, uint8_t *d_out,
                                  uint64_t out_cap, uint32_t *d_frame_bytes, uint64_t *d_frame_offsets,
                                  uint64_t *d_total, flacgpu_md5_state *d_md5_state, uint8_t *d_md5, void *hip_stream,
                                  void *md5_stream) {
    if (!c || !p || p->ctx != c || !d_pcm || !d_out || !d_frame_bytes || !d_frame_offsets || !d_total)
        return FLACGPU_ERR_INVALID_INPUT;
    // a stream that continues past this segment has no digest yet: its state must be carried
    if (p->d_md5_fin && d_md5 && !d_md5_state) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = pick_stream(c, hip_stream);
    if (c->records_on && p->n_frames > c->max_frames) return FLACGPU_ERR_INVALID_INPUT;
    uint8_t *desc = p->d_desc ? p->d_desc : c->d_desc;
    // MD5 of every stream on a second stream, overlapping the encode kernels (joined back into
    // st unless the caller owns the MD5 stream)
    const bool join = md5_stream == nullptr;
    hipStream_t ms = join ? c->aux : pick_stream(c, md5_stream);
    const bool md5 = (d_md5 || d_md5_state) && p->n_streams;
    if (md5) {
        hipEvent_t fork = join ? c->fork : get_event(c);
        if (!fork) return FLACGPU_ERR_DEVICE;
        HIPCHK(hipEventRecord(fork, st));
        HIPCHK(hipStreamWaitEvent(ms, fork, 0));
        if (!join) c->event_pool.push_back(fork);  // recycled: the wait is already enqueued
        {
            Timed t(c, FLACGPU_K_MD5, ms);
            HIPCHK(launch_md5_streams((const uint8_t *)d_pcm, p->d_md5_offs, p->d_md5_lens, p->d_md5_fin, p->n_streams,
                                      (Md5State *)d_md5_state, d_md5, ms, c->md5_kernel, c->md5_prio));
        }
        if (join) HIPCHK(hipEventRecord(c->join, ms));
    }
    // the MD5 workgroups were queued first: the encode kernels' persistent grids leave their slots
    // auto: only for long chains (>= 4096 blocks per stream per call, e.g. c4's 4 x 96-KiB frames).  A
    // persistent grid cannot grow back, so the reserved slots idle once the MD5 is done; a shorter
    // chain started late (after the analysis) still ends before the pack
    const bool reserve = c->md5_reserve > 0 || (c->md5_reserve < 0 && p->md5_max_len >= (256u << 10));
    c->grid_reserve = (md5 && reserve) ? md5_workgroups(p->n_streams, c->md5_kernel) : 0u;
    int rc = encode_core(c, (const uint8_t *)d_pcm, p->d_jobs, p->n_full, p->n_tail, desc, d_frame_bytes, d_out,
                         out_cap, d_frame_offsets, d_total, st, p->full_slots.data());
    c->grid_reserve = 0;
    if (rc) return rc;
    if (join && md5) HIPCHK(hipStreamWaitEvent(st, c->join, 0));
    return FLACGPU_OK;
}

int flacgpu_encode_plan_device_md5_async(flacgpu_ctx *c, const flacgpu_plan *p, const void *d_pcm, uint8_t *d_out,
                                         uint64_t out_cap, uint32_t *d_frame_bytes, uint64_t *d_frame_offsets,
                                         uint64_t *d_total, uint8_t *d_md5, void *hip_stream, void *md5_stream) {
    return flacgpu_encode_plan_device_ex(c, p, d_pcm, d_out, out_cap, d_frame_bytes, d_frame_offsets, d_total, nullptr,
                                         d_md5, hip_stream, md5_stream);
}

int flacgpu_encode_plan_device(flacgpu_ctx *c, const flacgpu_plan *p, const void *d_pcm, uint8_t *d_out,
                               uint64_t out_cap, uint32_t *d_frame_bytes, uint64_t *d_frame_offsets, uint64_t *d_total,
                               uint8_t *d_md5, void *hip_stream) {
    return flacgpu_encode_plan_device_ex(c, p, d_pcm, d_out, out_cap, d_frame_bytes, d_frame_offsets, d_total, nullptr,
                                         d_md5, hip_stream, nullptr);
}

int flacgpu_streaminfo_replay_device(flacgpu_ctx *c, const uint32_t *d_frame_bytes, uint64_t n_frames,
                                     uint32_t *d_minmax, void *hip_stream) {
    if (!c || !d_minmax || (n_frames && !d_frame_bytes)) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = pick_stream(c, hip_stream);
    HIPCHK(launch_streaminfo_replay(d_frame_bytes, n_frames, d_minmax, st));
    return FLACGPU_OK;
}

int flacgpu_sync_check(flacgpu_ctx *c, void *hip_stream) {
    if (!c) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(pick_stream(c, hip_stream)));
    return check_device_error(c);
}

// ---- instrumentation ---------------------------------------------------------
int flacgpu_set_timing(flacgpu_ctx *c, int enable) {
    if (!c) return FLACGPU_ERR_INVALID_INPUT;
    c->timing = enable != 0;
    return FLACGPU_OK;
}

int flacgpu_kernel_time(flacgpu_ctx *c, int kernel, uint64_t *launches, double *total_ms) {
    if (!c || kernel < 0 || kernel >= FLACGPU_K_COUNT) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    resolve_timing(c);
    if (launches) *launches = c->launches[kernel];
    if (total_ms) *total_ms = c->ms[kernel];
    return FLACGPU_OK;
}

int flacgpu_reset_timing(flacgpu_ctx *c) {
    if (!c) return FLACGPU_ERR_INVALID_INPUT;
    resolve_timing(c);
    for (int k = 0; k < FLACGPU_K_COUNT; k++) {
        c->launches[k] = 0;
        c->ms[k] = 0;
    }
    return FLACGPU_OK;
}

int flacgpu_set_overlap(flacgpu_ctx *c, uint32_t ranges, uint32_t ana_per_cu, uint32_t pack_per_cu,
                        uint32_t min_frames) {
    if (!c || ranges > kOvlMaxChunks || min_frames == 0) return FLACGPU_ERR_INVALID_INPUT;
    // the overlapped schedule measured slower: diagnostic builds only
    if (!FG_DIAG && ranges > 1) return FLACGPU_ERR_INVALID_CONFIG;
    c->ovl_chunks = ranges;
    c->ovl_ana = ana_per_cu;
    c->ovl_pack = pack_per_cu;
    c->ovl_min_frames = min_frames;
    return FLACGPU_OK;
}

int flacgpu_set_records(flacgpu_ctx *c, int enable) {
    if (!c) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    if (enable && !c->d_records) HIPCHK(hipMalloc(&c->d_records, (uint64_t)c->max_frames * sizeof(FrameRec)));
    if (enable) HIPCHK(hipMemset(c->d_records, 0, (uint64_t)c->max_frames * sizeof(FrameRec)));
    c->records_on = enable != 0;
    return FLACGPU_OK;
}

int flacgpu_get_records(flacgpu_ctx *c, flacgpu_frame_record *out, uint64_t max_frames, uint64_t *n_frames) {
    if (!c || !n_frames) return FLACGPU_ERR_INVALID_INPUT;
    const uint64_t n = std::min<uint64_t>(max_frames, c->h_records.size());
    if (out && n) std::memcpy(out, c->h_records.data(), n * sizeof(FrameRec));
    *n_frames = c->h_records.size();
    return FLACGPU_OK;
}

// Diagnostic build only (-DFG_STAMPS): per-phase shader-clock sums of the encode kernel.
int flacgpu_debug_stamps(flacgpu_ctx *c, uint64_t *out32, int reset) {
    if (!c || !out32) return FLACGPU_ERR_INVALID_INPUT;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(out32, c->d_stamps, 32 * 8, hipMemcpyDeviceToHost));
    if (reset) HIPCHK(hipMemset(c->d_stamps, 0, 32 * 8));
    return FLACGPU_OK;
}

}  // extern "C"
