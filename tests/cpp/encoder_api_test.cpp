// encoder_api_test.cpp -- drives libflacgpu.so through the C++ mirror of the
// reference Encoder API (include/flacgpu_encoder.hpp) exactly the way
// wav2flac.zig:10-97 drives the Zig encoder: skipHeader, writeVorbisComment,
// one writeFrame per block with updateFrameSize, MD5, seek back, writeHeader.
// Usage: encoder_api_test <pcm.raw> <channels> <bits> <rate> <out.flac>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "flacgpu_encoder.hpp"

int main(int argc, char **argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s pcm channels bits rate out\n", argv[0]);
        return 2;
    }
    const uint32_t ch = std::atoi(argv[2]), bits = std::atoi(argv[3]), rate = std::atoi(argv[4]);
    const uint32_t B = bits / 8;
    std::FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> pcm;
    uint8_t tmp[1 << 16];
    size_t r;
    while ((r = std::fread(tmp, 1, sizeof tmp, f)) > 0) pcm.insert(pcm.end(), tmp, tmp + r);
    std::fclose(f);
    const uint64_t samples = pcm.size() / (ch * B);
    try {
        flacgpu::BufferWriter w;
        auto enc = flacgpu::Encoder::init(w, flacgpu::Config::make(ch, bits, rate));
        auto si = flacgpu::StreamInfo::make(rate, ch, bits, samples);
        enc.skipHeader();
        enc.writeVorbisComment(true);
        uint64_t done = 0;
        for (uint64_t frame = 0; done < samples; frame++) {
            const uint32_t n = (uint32_t)std::min<uint64_t>(4096, samples - done);
            // WavReader.fillSamples (wav_reader.zig:44-91): LE bytes -> planar i32, MD5 of the bytes
            const uint8_t *src = pcm.data() + done * ch * B;
            for (uint32_t i = 0; i < n; i++)
                for (uint32_t c = 0; c < ch; c++) {
                    const uint8_t *p = src + ((size_t)i * ch + c) * B;
                    uint32_t v = 0;
                    for (uint32_t k = 0; k < B; k++) v |= (uint32_t)p[k] << (8 * k);
                    enc.samples[c][i] = (int32_t)(v << (32 - bits)) >> (32 - bits);
                }
            enc.md5.update(src, (size_t)n * ch * B);
            si.updateFrameSize(enc.writeFrame(frame, {bits, ch, n, rate}));
            done += n;
        }
        enc.finalizeStreamInfoMd5(si);
        w.seekTo(0);
        enc.writeHeader(si, false);
        std::FILE *o = std::fopen(argv[5], "wb");
        std::fwrite(w.buf.data(), 1, w.buf.size(), o);
        std::fclose(o);
    } catch (const flacgpu::Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
