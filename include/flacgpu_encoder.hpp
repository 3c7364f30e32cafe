// flacgpu_encoder.hpp -- C++ host mirror of toastori/zig-flac's Encoder API
// (src/lib.zig re-exports; src/lib/encoder.zig, src/lib/metadata.zig) over the
// C ABI of libflacgpu.so.  Same method names, argument meaning and call order
// as the Zig API, so a C++ host reads like wav2flac.zig:10-97:
//
//   flacgpu::Encoder enc = flacgpu::Encoder::init(writer, flacgpu::Config::make(2, 16, 44100));
//   enc.skipHeader();  enc.writeVorbisComment(true);
//   for (frame ...) { fill enc.samples[ch][0..n]; enc.md5.update(bytes);
//                     si.updateFrameSize(enc.writeFrame(idx, {16, 2, n, 44100})); }
//   enc.finalizeStreamInfoMd5(si);  writer.seekTo(0);  enc.writeHeader(si, false);
//
// Errors are thrown as flacgpu::Error carrying the C ABI code (the Zig error
// union members: OutOfMemory, WriteFailed, DeviceError, InvalidConfig, ...).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "flacgpu.h"

namespace flacgpu {

struct Error : std::runtime_error {
    int code;
    Error(int c, const char *where)
        : std::runtime_error(std::string(where) + ": " + flacgpu_strerror(c)), code(c) {}
};
inline void check(int rc, const char *where) {
    if (rc != FLACGPU_OK) throw Error(rc, where);
}

// std.Io.Writer as the encoder uses it: sequential writes + seekTo(0) at the end.
struct Writer {
    virtual ~Writer() = default;
    virtual void writeAll(const uint8_t *p, size_t n) = 0;
    virtual void seekTo(uint64_t pos) = 0;
};

// Writer over a growable byte buffer (the tests' and in-memory users' writer).
struct BufferWriter : Writer {
    std::vector<uint8_t> buf;
    size_t pos = 0;
    void writeAll(const uint8_t *p, size_t n) override {
        if (pos + n > buf.size()) buf.resize(pos + n);
        std::memcpy(buf.data() + pos, p, n);
        pos += n;
    }
    void seekTo(uint64_t p) override { pos = (size_t)p; }
};

// Encoder.Config (encoder.zig:609-656).
struct Config {
    flacgpu_config c;
    static Config make(uint32_t channels, uint32_t bit_depth, uint32_t sample_rate) {
        return Config{flacgpu_config_default(channels, bit_depth, sample_rate)};
    }
};

// FrameInfo (encoder.zig:658-663).
struct FrameInfo {
    uint32_t bit_depth;
    uint32_t channels;
    uint32_t samples_count;
    uint32_t sample_rate;
};

// metadata.StreamInfo (metadata.zig:18-68).
struct StreamInfo {
    flacgpu_streaminfo s;
    static StreamInfo make(uint32_t sample_rate, uint32_t channels, uint32_t bit_depth, uint64_t samples,
                           uint32_t block_size = 4096) {
        StreamInfo si;
        flacgpu_streaminfo_init(&si.s, sample_rate, channels, bit_depth, samples, block_size);
        return si;
    }
    void updateFrameSize(uint32_t frame_size) { flacgpu_streaminfo_update_frame_size(&s, frame_size); }
    void bytes(uint8_t out[34]) const { flacgpu_streaminfo_bytes(&s, out); }
};

// Md5 (md5.zig), computed on the encoder's GPU.
class Md5 {
   public:
    explicit Md5(flacgpu_ctx *c = nullptr) : ctx_(c) {}
    void update(const void *p, size_t n) { check(flacgpu_md5_update(ctx_, p, n), "Md5.update"); }
    void final(uint8_t out[16]) { check(flacgpu_md5_final(ctx_, out), "Md5.final"); }

   private:
    flacgpu_ctx *ctx_;
};

class Encoder {
   public:
    // Encoder.samples (encoder.zig:23): planar i32, block_size per channel.
    std::vector<std::vector<int32_t>> samples;
    Md5 md5;

    // Encoder.init (encoder.zig:44-118).
    static Encoder init(Writer &writer, const Config &config, int device = 0, uint32_t max_frames = 64) {
        Encoder e(writer);
        check(flacgpu_open(device, &config.c, max_frames, &e.ctx_), "Encoder.init");
        e.cfg_ = config.c;
        e.samples.assign(config.c.channels, std::vector<int32_t>(config.c.block_size, 0));
        e.md5 = Md5(e.ctx_);
        e.frame_.resize(flacgpu_frame_bound_bytes(&config.c));
        return e;
    }
    Encoder(Encoder &&o) noexcept
        : samples(std::move(o.samples)), md5(o.md5), w_(o.w_), ctx_(o.ctx_), cfg_(o.cfg_), frame_(std::move(o.frame_)) {
        o.ctx_ = nullptr;
    }
    Encoder(const Encoder &) = delete;
    Encoder &operator=(const Encoder &) = delete;
    ~Encoder() { deinit(); }

    // Encoder.deinit (encoder.zig:121-164).
    void deinit() {
        if (ctx_) flacgpu_close(ctx_);
        ctx_ = nullptr;
    }

    // skipHeader (encoder.zig:177-186): 4 + 1 + 3 + 34 zero bytes.
    void skipHeader() {
        const uint8_t z[42] = {};
        w_->writeAll(z, sizeof z);
    }
    // writeHeader (encoder.zig:192-206).
    void writeHeader(const StreamInfo &si, bool last_metadata) {
        uint8_t h[42];
        w_->writeAll(h, flacgpu_header_bytes(&si.s, last_metadata ? 1 : 0, h));
    }
    // writeVorbisComment (encoder.zig:211-226).
    void writeVorbisComment(bool last_metadata) {
        uint8_t v[31];
        w_->writeAll(v, flacgpu_vorbis_comment_bytes(last_metadata ? 1 : 0, v));
    }
    // writeFrame (encoder.zig:234-284): the frame from samples[ch][0..n] through the GPU;
    // returns its byte count (u24).
    uint32_t writeFrame(uint64_t frame_number, const FrameInfo &info) {
        if (info.channels != cfg_.channels || info.bit_depth != cfg_.bits_per_sample ||
            info.sample_rate != cfg_.sample_rate)
            throw Error(FLACGPU_ERR_INVALID_INPUT, "Encoder.writeFrame");
        const int32_t *planes[8] = {};
        for (uint32_t ch = 0; ch < info.channels; ch++) planes[ch] = samples[ch].data();
        uint32_t n = 0;
        check(flacgpu_encode_frame_planar(ctx_, planes, info.samples_count, frame_number, frame_.data(),
                                          frame_.size(), &n),
              "Encoder.writeFrame");
        w_->writeAll(frame_.data(), n);
        return n;
    }
    // finalizeStreamInfoMd5 (encoder.zig:168-170).
    void finalizeStreamInfoMd5(StreamInfo &si) { md5.final(si.s.md5); }

    flacgpu_ctx *ctx() const { return ctx_; }

   private:
    explicit Encoder(Writer &w) : w_(&w) {}
    Writer *w_;
    flacgpu_ctx *ctx_ = nullptr;
    flacgpu_config cfg_{};
    std::vector<uint8_t> frame_;
};

}  // namespace flacgpu
