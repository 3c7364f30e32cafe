// fg_file.cpp -- host-side file assembly around the GPU frame encoder: WAV
// header parsing (WavReader.init/getFmt, src/lib/wav_reader.zig:92-170),
// StreamInfo (src/lib/metadata.zig:18-68), the metadata writers of the
// reference Encoder (skipHeader/writeHeader/writeVorbisComment,
// src/lib/encoder.zig:177-226) and the wav2flac driver
// (src/cli/wav2flac.zig:10-97).  Pure host code: every sample goes through the
// GPU kernels via flacgpu_encode_frames; only the 73 metadata bytes are built
// here.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <system_error>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/flacgpu.h"
#include "fg_common.hpp"
#include "fg_internal.hpp"
#include "fg_md5_host.hpp"

namespace {

constexpr char kVendor[] = "toastori FLAC 0.0.0";  // encoder.zig:212
constexpr uint32_t kVendorLen = sizeof(kVendor) - 1;

uint32_t rd_le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint16_t rd_le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }
void wr_be(uint8_t *p, uint64_t v, int n) {
    for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * (n - 1 - i)));
}

// ---- The device's shared file pipeline --------------------------------------------------
// The reference converts one file per encoder (wav2flac.zig:10-63).  Many such encoders on one GPU,
// each with its own streams and chunk pipeline, contend for the device's few hardware queues
// (GPU_MAX_HW_QUEUES = 4) and each launch their persistent grids over a small chunk: 64 concurrent
// flacgpu_encode_file calls ran at 0.25 of the host-MD5 bound.  So a
// flacgpu_encode_file call on a plain context (fg::ctx_plain) with the host MD5 engine queues its
// file on the shared pipeline of (device, config): one caller at a time is the leader and runs
// every file queued by then as ONE flacgpu_encode_files batch on the pipeline's own context (one
// H2D / encode / D2H schedule running on from file to file, all MD5s on the host pool); the other
// callers wait for their file and take over as leader when the batch ends.  Output bytes are those
// of flacgpu_encode_file (flacgpu_encode_files' contract).  FLACGPU_FILE_SHARED=0 turns it off.
struct FileReq {
    const void *pcm;
    uint64_t n;
    uint8_t *out;
    size_t cap, len = 0;
    int rc = FLACGPU_OK;
    bool done = false;
};

struct FilePipe {
    std::mutex m;
    std::condition_variable cv;
    std::deque<FileReq *> q;
    bool leading = false;
    flacgpu_ctx *ctx = nullptr;  // opened by the first leader, kept for the process lifetime
    int open_rc = FLACGPU_OK;
};

constexpr uint32_t kPipeFrames = 6144;  // three 2048-frame chunk sets (the pipelined schedule)

FilePipe &file_pipe(int device, const flacgpu_config &c) {
    static std::mutex mm;
    static std::map<std::tuple<int, uint32_t, uint32_t, uint32_t, uint32_t>, FilePipe *> pipes;
    const auto key = std::make_tuple(device, c.sample_rate, (uint32_t)c.block_size | ((uint32_t)c.channels << 16) |
                                                                ((uint32_t)c.bits_per_sample << 24),
                                     (uint32_t)c.stereo_decorrelation | ((uint32_t)c.max_rice_part_order << 8) |
                                         ((uint32_t)c.max_rice_param << 16),
                                     (uint32_t)c.prediction);
    std::lock_guard<std::mutex> lk(mm);
    FilePipe *&p = pipes[key];
    if (!p) p = new FilePipe;  // never freed: callers may still hold it at exit
    return *p;
}

bool file_pipe_on() {
    const char *e = std::getenv("FLACGPU_FILE_SHARED");
    return !(e && e[0] == '0');
}

// Queue one file on the shared pipeline and return when it is encoded (maybe by another caller).
int file_pipe_encode(int device, const flacgpu_config &cfg, const void *pcm, uint32_t bytes_per_sample, uint64_t n,
                     uint8_t *out, size_t cap, size_t *out_len) {
    FilePipe &P = file_pipe(device, cfg);
    FileReq me{pcm, n, out, cap};
    std::unique_lock<std::mutex> lk(P.m);
    P.q.push_back(&me);
    P.cv.notify_all();
    for (;;) {
        P.cv.wait(lk, [&] { return me.done || !P.leading; });
        if (me.done) break;
        // no batch running and this file still queued: lead.  Give callers that start at about the
        // same moment a window to queue theirs: the batch closes once no file has arrived for 1 ms
        // (at most 20 ms; a batch of ten-minute files runs for ~100 ms, and every file left out of
        // it waits for the whole next batch)
        P.leading = true;
        const auto t_lead = std::chrono::steady_clock::now();
        for (;;) {
            const size_t before = P.q.size();
            P.cv.wait_for(lk, std::chrono::milliseconds(1), [&] { return P.q.size() != before; });
            if (P.q.size() == before || std::chrono::steady_clock::now() - t_lead > std::chrono::milliseconds(20)) break;
        }
        std::vector<FileReq *> batch(P.q.begin(), P.q.end());
        P.q.clear();
        lk.unlock();
        int rc = FLACGPU_OK;
        if (!P.ctx && P.open_rc == FLACGPU_OK) P.open_rc = flacgpu_open(device, &cfg, kPipeFrames, &P.ctx);
        rc = P.ctx ? FLACGPU_OK : (P.open_rc ? P.open_rc : FLACGPU_ERR_DEVICE);
        const uint32_t nb = (uint32_t)batch.size();
        std::vector<const void *> src(nb);
        std::vector<uint64_t> ns(nb);
        std::vector<uint8_t *> outs(nb);
        std::vector<size_t> caps(nb), lens(nb, 0);
        for (uint32_t i = 0; i < nb; i++) {
            src[i] = batch[i]->pcm;
            ns[i] = batch[i]->n;
            outs[i] = batch[i]->out;
            caps[i] = batch[i]->cap;
        }
        if (!rc) rc = flacgpu_encode_files(P.ctx, nb, src.data(), bytes_per_sample, ns.data(), outs.data(), caps.data(),
                                           lens.data());
        if (rc == FLACGPU_ERR_OUTPUT_TOO_SMALL || rc == FLACGPU_ERR_INVALID_INPUT) {
            // one file's buffer is too small (or its pointer bad): every file of the batch alone,
            // so that each caller gets its own file's result
            for (uint32_t i = 0; i < nb; i++) {
                size_t l = 0;
                batch[i]->rc = flacgpu_encode_files(P.ctx, 1, &src[i], bytes_per_sample, &ns[i], &outs[i], &caps[i], &l);
                batch[i]->len = l;
            }
        } else {
            for (uint32_t i = 0; i < nb; i++) {
                batch[i]->rc = rc;
                batch[i]->len = rc ? 0 : lens[i];
            }
        }
        lk.lock();
        for (FileReq *r : batch) r->done = true;
        P.leading = false;
        P.cv.notify_all();
    }
    *out_len = me.len;
    return me.rc;
}

}  // namespace

extern "C" {

// WavReader.init + getFmt (wav_reader.zig:116-170) + flacStreaminfo checks (:92-108).
int flacgpu_wav_parse(const void *wav, size_t len, flacgpu_wav_info *info) {
    if (!wav || !info) return FLACGPU_ERR_INVALID_INPUT;
    const uint8_t *p = (const uint8_t *)wav;
    size_t pos = 0;
    auto need = [&](size_t n) { return pos + n <= len; };
    if (!need(12) || std::memcmp(p, "RIFF", 4) || std::memcmp(p + 8, "WAVE", 4)) return FLACGPU_ERR_INVALID_INPUT;
    pos = 12;
    // skip chunks until "fmt " (wav_reader.zig:125-128)
    for (;;) {
        if (!need(8)) return FLACGPU_ERR_INVALID_INPUT;
        if (!std::memcmp(p + pos, "fmt ", 4)) break;
        pos += 8 + rd_le32(p + pos + 4);
    }
    pos += 8;  // tag + fmt size (the size field is not used, as in the reference)
    if (!need(16)) return FLACGPU_ERR_INVALID_INPUT;
    const uint16_t codec = rd_le16(p + pos);
    if (codec != 1 && codec != 0xFFFE) return FLACGPU_ERR_INVALID_CONFIG;  // UnsupportCodec
    const uint32_t channels = rd_le16(p + pos + 2);
    const uint32_t rate = rd_le32(p + pos + 4);
    const uint32_t byte_rate = rd_le32(p + pos + 8);
    const uint32_t block_align = rd_le16(p + pos + 12);
    uint32_t bit_depth = rd_le16(p + pos + 14);
    pos += 16;
    if (bit_depth < 4 || bit_depth > 32 || channels == 0) return FLACGPU_ERR_INVALID_CONFIG;
    const uint32_t bytes_per_sample = block_align / channels;
    if (byte_rate != rate * channels * bytes_per_sample) return FLACGPU_ERR_INVALID_INPUT;  // BitRateUnmatch
    if (codec == 0xFFFE) {  // extension size, valid bits, channel mask, subformat
        if (!need(24)) return FLACGPU_ERR_INVALID_INPUT;
        bit_depth = rd_le16(p + pos + 2);
        pos += 24;
    }
    for (;;) {  // skip unknown subchunks until "data"
        if (!need(8)) return FLACGPU_ERR_INVALID_INPUT;  // DataNotFound
        if (!std::memcmp(p + pos, "data", 4)) break;
        pos += 8 + rd_le32(p + pos + 4);
    }
    const uint32_t data_len = rd_le32(p + pos + 4);
    pos += 8;
    if (block_align == 0 || data_len % block_align != 0) return FLACGPU_ERR_INVALID_INPUT;  // InvalidDataLen
    if (bit_depth / 8 == 0) return FLACGPU_ERR_INVALID_CONFIG;
    const uint64_t samples = data_len / (channels * (bit_depth / 8));  // wav_reader.zig:169
    // flacStreaminfo (wav_reader.zig:92-108)
    if (bit_depth < 4 || bit_depth > 32 || channels > 8 || rate >= (1u << 20) || samples >= (1ull << 36))
        return FLACGPU_ERR_INVALID_CONFIG;
    info->sample_rate = rate;
    info->channels = (uint16_t)channels;
    info->bits_per_sample = (uint16_t)bit_depth;
    info->bytes_per_sample = (uint16_t)bytes_per_sample;
    info->samples = samples;
    info->data_offset = pos;
    info->data_bytes = std::min<uint64_t>(data_len, len - pos);
    return FLACGPU_OK;
}

// StreamInfo defaults (metadata.zig:18-33; wav_reader.zig:98-107 sets block sizes = 4096).
void flacgpu_streaminfo_init(flacgpu_streaminfo *si, uint32_t sample_rate, uint32_t channels, uint32_t bit_depth,
                             uint64_t interchannel_samples, uint32_t block_size) {
    if (!si) return;
    std::memset(si, 0, sizeof(*si));
    si->min_frame_size = 0xFFFFFFu;
    si->max_frame_size = 0;
    si->sample_rate = sample_rate;
    si->channels = (uint8_t)channels;
    si->bit_depth = (uint8_t)bit_depth;
    si->interchannel_samples = interchannel_samples;
    si->min_block_size = (uint16_t)block_size;
    si->max_block_size = (uint16_t)block_size;
}

// updateFrameSize (metadata.zig:35-40), including its else-if: a frame that raises
// max never lowers min.
void flacgpu_streaminfo_update_frame_size(flacgpu_streaminfo *si, uint32_t frame_size) {
    if (!si) return;
    frame_size &= 0xFFFFFFu;
    if (frame_size > si->max_frame_size) si->max_frame_size = frame_size;
    else if (frame_size < si->min_frame_size) si->min_frame_size = frame_size;
}

// StreamInfo.bytes (metadata.zig:42-68): 34 big-endian bytes.
void flacgpu_streaminfo_bytes(const flacgpu_streaminfo *si, uint8_t out[34]) {
    wr_be(out + 0, si->min_block_size, 2);
    wr_be(out + 2, si->max_block_size, 2);
    wr_be(out + 4, si->min_frame_size & 0xFFFFFFu, 3);
    wr_be(out + 7, si->max_frame_size & 0xFFFFFFu, 3);
    // 20-bit rate, 3-bit channels-1, 5-bit bits-1, 36-bit samples
    const uint64_t packed = ((uint64_t)(si->sample_rate & 0xFFFFFu) << 44) |
                            ((uint64_t)((si->channels - 1u) & 7u) << 41) |
                            ((uint64_t)((si->bit_depth - 1u) & 31u) << 36) |
                            (si->interchannel_samples & 0xFFFFFFFFFull);
    wr_be(out + 10, packed, 8);
    std::memcpy(out + 18, si->md5, 16);
}

// writeHeader (encoder.zig:192-206): "fLaC", STREAMINFO block header, 34 bytes.
size_t flacgpu_header_bytes(const flacgpu_streaminfo *si, int last_metadata, uint8_t out[42]) {
    std::memcpy(out, "fLaC", 4);
    out[4] = (uint8_t)((last_metadata ? 0x80u : 0u) | 0u);  // BlockHeader{type StreamInfo}
    wr_be(out + 5, 34, 3);
    flacgpu_streaminfo_bytes(si, out + 8);
    return 42;
}

// writeVorbisComment (encoder.zig:211-226): vendor string, no tags.
size_t flacgpu_vorbis_comment_bytes(int last_metadata, uint8_t out[31]) {
    out[0] = (uint8_t)((last_metadata ? 0x80u : 0u) | 4u);  // BlockHeader{type VorbisComment}
    wr_be(out + 1, kVendorLen + 8, 3);
    out[4] = (uint8_t)kVendorLen;
    out[5] = out[6] = out[7] = 0;
    std::memcpy(out + 8, kVendor, kVendorLen);
    std::memset(out + 8 + kVendorLen, 0, 4);
    return 12 + kVendorLen;
}

// wav2flac.main + encode (wav2flac.zig:10-97) for PCM already in memory (on a plain context with
// the host MD5 engine: through the device's shared file pipeline above): skipHeader,
// writeVorbisComment(true), every frame through the GPU (sizes replayed into
// updateFrameSize in frame order), the MD5 of the PCM bytes, then the header written
// last.  With the host MD5 engine (the default) the hash runs on its own thread while
// the GPU encodes (the reference interleaves the two per block on one thread,
// wav_reader.zig:66 beside encoder.zig:234); the device engine hashes after the encode.
int flacgpu_encode_file(flacgpu_ctx *ctx, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                        uint8_t *out, size_t out_cap, size_t *out_len) {
    if (!ctx || !out || !out_len || (!pcm && n_samples)) return FLACGPU_ERR_INVALID_INPUT;
    *out_len = 0;
    flacgpu_config cfg;
    int rc = flacgpu_get_config(ctx, &cfg);
    if (rc) return rc;
    if (out_cap < 73) return FLACGPU_ERR_OUTPUT_TOO_SMALL;
    if (bytes_per_sample != cfg.bits_per_sample / 8u) return FLACGPU_ERR_INVALID_INPUT;
    if (flacgpu_md5_get_engine(ctx) == FLACGPU_MD5_HOST && fg::ctx_plain(ctx) && file_pipe_on())
        return file_pipe_encode(fg::ctx_device(ctx).device, cfg, pcm, bytes_per_sample, n_samples, out, out_cap,
                                out_len);
    const uint64_t block = cfg.block_size;
    const uint64_t n_frames = (n_samples + block - 1) / block;
    const size_t pcm_bytes = (size_t)(n_samples * cfg.channels * bytes_per_sample);
    std::vector<uint32_t> sizes;
    try {
        sizes.resize(n_frames ? n_frames : 1);
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
    flacgpu_streaminfo si;
    flacgpu_streaminfo_init(&si, cfg.sample_rate, cfg.channels, cfg.bits_per_sample, n_samples, cfg.block_size);
    fg::HostMd5 md5;
    std::thread hasher;
    const bool host_md5 = flacgpu_md5_get_engine(ctx) == FLACGPU_MD5_HOST;
    if (host_md5) {
        try {
            // the process-wide pool interleaves this file's chain with other files hashed at once
            hasher = std::thread([&]() { fg::md5_pool_update(&md5, pcm, pcm_bytes); });
        } catch (const std::system_error &) {
            md5.update(pcm, pcm_bytes);  // no thread to be had: hash here, before the encode
        }
    }
    size_t frames_len = 0;
    rc = flacgpu_encode_frames(ctx, pcm, bytes_per_sample, n_samples, 0, out + 73, out_cap - 73, &frames_len,
                               sizes.data());
    if (hasher.joinable()) hasher.join();
    if (rc) return rc;
    for (uint64_t f = 0; f < n_frames; f++) flacgpu_streaminfo_update_frame_size(&si, sizes[f]);
    if (host_md5) {
        md5.final(si.md5);
    } else {
        if ((rc = flacgpu_md5_init(ctx))) return rc;
        if ((rc = flacgpu_md5_update(ctx, pcm, pcm_bytes))) return rc;
        if ((rc = flacgpu_md5_final(ctx, si.md5))) return rc;
    }
    flacgpu_header_bytes(&si, 0, out);
    flacgpu_vorbis_comment_bytes(1, out + 42);
    *out_len = 73 + frames_len;
    return FLACGPU_OK;
}

// wav2flac for n files at once on one context: every file's frames through ONE pipelined
// H2D / encode / D2H schedule (fg::ctx_encode_segments: the pipeline runs on from file to file;
// one context's streams, not one context per file contending for the GPU's hardware queues),
// and every file's MD5 on the host hashing pool in one batch beside it (md5_pool_update_many:
// up to eight chains per core).  Each out[i] receives exactly what flacgpu_encode_file writes.
// Diagnostic builds only (FG_DIAG, `make diag`): FLACGPU_FILES_MD5=0 times the GPU / PCIe schedule
// alone, skipping the hashing and leaving the STREAMINFO MD5 zero ("not computed").  The release
// library always finalises the MD5 into STREAMINFO (encoder.zig:168-170).
int flacgpu_encode_files(flacgpu_ctx *ctx, uint32_t n_files, const void *const *pcm, uint32_t bytes_per_sample,
                         const uint64_t *n_samples, uint8_t *const *out, const size_t *out_cap, size_t *out_len) {
    if (!ctx || (n_files && (!pcm || !n_samples || !out || !out_cap || !out_len))) return FLACGPU_ERR_INVALID_INPUT;
    flacgpu_config cfg;
    int rc = flacgpu_get_config(ctx, &cfg);
    if (rc) return rc;
    if (bytes_per_sample != cfg.bits_per_sample / 8u) return FLACGPU_ERR_INVALID_INPUT;
    for (uint32_t i = 0; i < n_files; i++) {
        out_len[i] = 0;
        if (!out[i] || (!pcm[i] && n_samples[i])) return FLACGPU_ERR_INVALID_INPUT;
    }
    for (uint32_t i = 0; i < n_files; i++)
        if (out_cap[i] < 73) return FLACGPU_ERR_OUTPUT_TOO_SMALL;
    std::vector<fg::HostMd5> md5;
    std::vector<fg::HostMd5 *> hp;
    std::vector<const uint8_t *> src;
    std::vector<size_t> bytes, caps, lens;
    std::vector<uint8_t *> frames_out;
    std::vector<std::vector<uint32_t>> sizes;
    std::vector<uint32_t *> sizes_p;
    try {
        md5.resize(n_files);
        hp.resize(n_files);
        src.resize(n_files);
        bytes.resize(n_files);
        caps.resize(n_files);
        lens.resize(n_files);
        frames_out.resize(n_files);
        sizes.resize(n_files);
        sizes_p.resize(n_files);
        for (uint32_t i = 0; i < n_files; i++) {
            hp[i] = &md5[i];
            src[i] = (const uint8_t *)pcm[i];
            bytes[i] = (size_t)(n_samples[i] * cfg.channels * bytes_per_sample);
            caps[i] = out_cap[i] - 73;
            frames_out[i] = out[i] + 73;
            sizes[i].resize((n_samples[i] + cfg.block_size - 1) / cfg.block_size + 1);
            sizes_p[i] = sizes[i].data();
        }
    } catch (...) {
        return FLACGPU_ERR_OUT_OF_MEMORY;
    }
#if FG_DIAG
    const char *mk = std::getenv("FLACGPU_FILES_MD5");
    const bool no_md5 = mk && mk[0] == '0';
#else
    const bool no_md5 = false;
#endif
    const bool host_md5 = no_md5 || flacgpu_md5_get_engine(ctx) == FLACGPU_MD5_HOST;
    std::thread hasher;
    if (host_md5 && !no_md5) {
        try {
            hasher = std::thread([&]() { fg::md5_pool_update_many(hp.data(), src.data(), bytes.data(), n_files); });
        } catch (const std::system_error &) {
            fg::md5_pool_update_many(hp.data(), src.data(), bytes.data(), n_files);  // before the encode
        }
    }
    rc = fg::ctx_encode_segments(ctx, n_files, src.data(), n_samples, frames_out.data(), caps.data(), lens.data(),
                                 sizes_p.data());
    if (hasher.joinable()) hasher.join();
    if (rc) return rc;
    for (uint32_t i = 0; i < n_files; i++) {
        flacgpu_streaminfo si;
        flacgpu_streaminfo_init(&si, cfg.sample_rate, cfg.channels, cfg.bits_per_sample, n_samples[i], cfg.block_size);
        const uint64_t nf = (n_samples[i] + cfg.block_size - 1) / cfg.block_size;
        for (uint64_t f = 0; f < nf; f++) flacgpu_streaminfo_update_frame_size(&si, sizes[i][f]);
        if (no_md5) {
            memset(si.md5, 0, 16);
        } else if (host_md5) {
            md5[i].final(si.md5);
        } else {
            if ((rc = flacgpu_md5_init(ctx)) || (rc = flacgpu_md5_update(ctx, pcm[i], bytes[i])) ||
                (rc = flacgpu_md5_final(ctx, si.md5))) {
                for (uint32_t j = 0; j < n_files; j++) out_len[j] = 0;
                return rc;
            }
        }
        flacgpu_header_bytes(&si, 0, out[i]);
        flacgpu_vorbis_comment_bytes(1, out[i] + 42);
        out_len[i] = 73 + lens[i];
    }
    return FLACGPU_OK;
}

// The whole wav2flac conversion of an in-memory WAV file on GPU `device`.
int flacgpu_wav_to_flac(int device, const void *wav, size_t wav_len, uint8_t *out, size_t out_cap, size_t *out_len) {
    if (!out_len) return FLACGPU_ERR_INVALID_INPUT;
    *out_len = 0;
    flacgpu_wav_info wi;
    int rc = flacgpu_wav_parse(wav, wav_len, &wi);
    if (rc) return rc;
    if (wi.bytes_per_sample * 8u != wi.bits_per_sample) return FLACGPU_ERR_INVALID_CONFIG;  // container == depth only
    // 8-bit WAV data is unsigned; the reference's 8-bit conversion is broken
    // (wav_reader.zig:71-78), so there is no behaviour to match.
    if (wi.bits_per_sample == 8) return FLACGPU_ERR_INVALID_CONFIG;
    if (wi.data_bytes < wi.samples * wi.channels * wi.bytes_per_sample) return FLACGPU_ERR_INVALID_INPUT;
    const flacgpu_config cfg = flacgpu_config_default(wi.channels, wi.bits_per_sample, wi.sample_rate);
    flacgpu_ctx *ctx = nullptr;
    if ((rc = flacgpu_open(device, &cfg, 0, &ctx))) return rc;
    rc = flacgpu_encode_file(ctx, (const uint8_t *)wav + wi.data_offset, wi.bytes_per_sample, wi.samples, out, out_cap,
                             out_len);
    flacgpu_close(ctx);
    return rc;
}

}  // extern "C"
