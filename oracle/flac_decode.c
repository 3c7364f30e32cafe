/*
 * flac_decode.c -- minimal FLAC decoder used as a round-trip VERIFIER.
 * TEST INFRASTRUCTURE ONLY (loaded by tests/ and bench.py's checks).
 *
 * Written from the FLAC format specification (RFC 9639: frame header,
 * CONSTANT / VERBATIM / FIXED / LPC subframes, partitioned Rice coding with
 * escapes, stereo decorrelation, CRC-8 / CRC-16), sharing no code with the
 * encoder restatement in flac_oracle.c or with the GPU encoder.  Every frame
 * header CRC-8 and frame CRC-16 is checked; any mismatch is an error.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    const uint8_t *p;
    size_t nbytes;
    uint64_t pos; /* bit position */
    int err;
} br_t;

static inline uint32_t br_bit(br_t *b) {
    if ((b->pos >> 3) >= b->nbytes) { b->err = 1; return 0; }
    uint32_t v = (b->p[b->pos >> 3] >> (7 - (b->pos & 7))) & 1u;
    b->pos++;
    return v;
}

static uint64_t br_u(br_t *b, unsigned n) {
    uint64_t v = 0;
    /* fast path: byte-wise when aligned */
    while (n >= 8 && (b->pos & 7) == 0) {
        if ((b->pos >> 3) >= b->nbytes) { b->err = 1; return 0; }
        v = (v << 8) | b->p[b->pos >> 3];
        b->pos += 8;
        n -= 8;
    }
    while (n--) v = (v << 1) | br_bit(b);
    return v;
}

static int64_t br_s(br_t *b, unsigned n) {
    if (n == 0) return 0;
    uint64_t v = br_u(b, n);
    if (n < 64 && (v >> (n - 1)) & 1) v |= ~0ULL << n;
    return (int64_t)v;
}

static uint64_t br_unary(br_t *b) {
    uint64_t z = 0;
    for (;;) {
        if ((b->pos >> 3) >= b->nbytes) { b->err = 1; return 0; }
        uint8_t byte = (uint8_t)(b->p[b->pos >> 3] << (b->pos & 7));
        unsigned avail = 8 - (unsigned)(b->pos & 7);
        if (byte == 0) { z += avail; b->pos += avail; continue; }
        unsigned lead = (unsigned)__builtin_clz((unsigned)byte) - 24;
        z += lead;
        b->pos += lead + 1;
        return z;
    }
}

static uint8_t crc8_spec(const uint8_t *p, size_t n) {
    uint8_t c = 0;
    while (n--) {
        c ^= *p++;
        for (int i = 0; i < 8; i++) c = (uint8_t)(c & 0x80 ? (c << 1) ^ 0x07 : c << 1);
    }
    return c;
}

static uint16_t crc16_tab[256];
static int crc16_init_done;
static uint16_t crc16_spec(const uint8_t *p, size_t n) {
    if (!crc16_init_done) {
        for (int i = 0; i < 256; i++) {
            uint16_t c = (uint16_t)(i << 8);
            for (int k = 0; k < 8; k++) c = (uint16_t)(c & 0x8000 ? (c << 1) ^ 0x8005 : c << 1);
            crc16_tab[i] = c;
        }
        crc16_init_done = 1;
    }
    uint16_t c = 0;
    while (n--) c = (uint16_t)((c << 8) ^ crc16_tab[((c >> 8) ^ *p++) & 0xFF]);
    return c;
}

typedef struct {
    uint32_t block_size;
    uint32_t sample_rate;
    uint32_t channel_assign;
    uint32_t bits;
    uint64_t number;
    uint32_t frame_bytes;
    uint32_t sub_type[8];   /* 0 const 1 verbatim 2 fixed 3 lpc */
    uint32_t sub_order[8];
    uint32_t sub_waste[8];
} fdec_frame_info;

enum { FD_OK = 0, FD_ESYNC = -1, FD_EHDR = -2, FD_ECRC8 = -3, FD_ESUB = -4, FD_ECRC16 = -5, FD_EEOF = -6, FD_ERANGE = -7 };

static int decode_residual(br_t *b, uint32_t bs, uint32_t order, int64_t *res) {
    uint32_t method = (uint32_t)br_u(b, 2);
    if (method > 1) return FD_ESUB;
    uint32_t pbits = method ? 5 : 4, esc = method ? 31 : 15;
    uint32_t porder = (uint32_t)br_u(b, 4);
    uint32_t nparts = 1u << porder;
    if ((bs >> porder) < order || (bs % nparts) != 0) return FD_ESUB;
    uint32_t i = order;
    for (uint32_t pt = 0; pt < nparts; pt++) {
        uint32_t cnt = (bs >> porder) - (pt == 0 ? order : 0);
        uint32_t k = (uint32_t)br_u(b, pbits);
        if (k == esc) {
            uint32_t w = (uint32_t)br_u(b, 5);
            for (uint32_t j = 0; j < cnt; j++) res[i++] = w ? br_s(b, w) : 0;
        } else {
            for (uint32_t j = 0; j < cnt; j++) {
                uint64_t q = br_unary(b);
                uint64_t u = (q << k) | (k ? br_u(b, k) : 0);
                res[i++] = (u & 1) ? -(int64_t)(u >> 1) - 1 : (int64_t)(u >> 1);
            }
        }
        if (b->err) return FD_EEOF;
    }
    return FD_OK;
}

static int decode_subframe(br_t *b, uint32_t bs, uint32_t bps, int64_t *out, fdec_frame_info *fi, int ch) {
    if (br_u(b, 1) != 0) return FD_ESUB;
    uint32_t t = (uint32_t)br_u(b, 6);
    uint32_t waste = 0;
    if (br_u(b, 1)) waste = (uint32_t)br_unary(b) + 1;
    if (waste >= bps && !(t == 0)) { /* constant with waste is legal in theory */
        if (waste > bps) return FD_ESUB;
    }
    uint32_t sbps = bps - waste;
    fi->sub_waste[ch] = waste;
    if (t == 0) {
        fi->sub_type[ch] = 0;
        int64_t v = br_s(b, sbps);
        for (uint32_t i = 0; i < bs; i++) out[i] = v;
    } else if (t == 1) {
        fi->sub_type[ch] = 1;
        for (uint32_t i = 0; i < bs; i++) out[i] = br_s(b, sbps);
    } else if (t >= 8 && t <= 12) {
        uint32_t order = t - 8;
        fi->sub_type[ch] = 2;
        fi->sub_order[ch] = order;
        if (order > bs) return FD_ESUB;
        for (uint32_t i = 0; i < order; i++) out[i] = br_s(b, sbps);
        int rc = decode_residual(b, bs, order, out);
        if (rc) return rc;
        for (uint32_t i = order; i < bs; i++) {
            int64_t p = 0;
            switch (order) {
            case 1: p = out[i - 1]; break;
            case 2: p = 2 * out[i - 1] - out[i - 2]; break;
            case 3: p = 3 * out[i - 1] - 3 * out[i - 2] + out[i - 3]; break;
            case 4: p = 4 * out[i - 1] - 6 * out[i - 2] + 4 * out[i - 3] - out[i - 4]; break;
            default: p = 0;
            }
            out[i] += p;
        }
    } else if (t >= 32) {
        uint32_t order = (t & 31) + 1;
        fi->sub_type[ch] = 3;
        fi->sub_order[ch] = order;
        if (order > bs) return FD_ESUB;
        for (uint32_t i = 0; i < order; i++) out[i] = br_s(b, sbps);
        uint32_t prec = (uint32_t)br_u(b, 4) + 1;
        if (prec == 16) return FD_ESUB;
        int32_t shift = (int32_t)br_s(b, 5);
        if (shift < 0) return FD_ESUB;
        int64_t coef[32];
        for (uint32_t j = 0; j < order; j++) coef[j] = br_s(b, prec);
        int rc = decode_residual(b, bs, order, out);
        if (rc) return rc;
        for (uint32_t i = order; i < bs; i++) {
            int64_t acc = 0;
            for (uint32_t j = 0; j < order; j++) acc += coef[j] * out[i - 1 - j];
            out[i] += acc >> shift;
        }
    } else {
        return FD_ESUB;
    }
    if (waste)
        for (uint32_t i = 0; i < bs; i++) out[i] = (int64_t)((uint64_t)out[i] << waste);
    return b->err ? FD_EEOF : FD_OK;
}

static const uint32_t RATE_TAB[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
static const uint32_t BITS_TAB[8] = {0, 8, 12, 0, 16, 20, 24, 32};

/* Decode one frame starting at buf.  stream_bits/stream_rate substitute for
 * "from STREAMINFO" codes.  planes: 8 x >= block_size int64.  Returns bytes
 * consumed or a negative FD_* code. */
long fdec_frame(const uint8_t *buf, size_t len, uint32_t stream_bits, uint32_t stream_rate, int64_t *const *planes,
                uint32_t max_block, fdec_frame_info *fi) {
    br_t b = {buf, len, 0, 0};
    memset(fi, 0, sizeof(*fi));
    if (br_u(&b, 15) != 0x7FFC) return FD_ESYNC;
    uint32_t blocking = (uint32_t)br_u(&b, 1);
    (void)blocking;
    uint32_t bsc = (uint32_t)br_u(&b, 4), src = (uint32_t)br_u(&b, 4);
    uint32_t chc = (uint32_t)br_u(&b, 4), bitc = (uint32_t)br_u(&b, 3);
    if (br_u(&b, 1) != 0) return FD_EHDR;
    /* coded number: UTF-8-like, up to 7 bytes */
    uint32_t first = (uint32_t)br_u(&b, 8);
    uint64_t num;
    int extra;
    if (!(first & 0x80)) { num = first; extra = 0; }
    else if ((first & 0xE0) == 0xC0) { num = first & 0x1F; extra = 1; }
    else if ((first & 0xF0) == 0xE0) { num = first & 0x0F; extra = 2; }
    else if ((first & 0xF8) == 0xF0) { num = first & 0x07; extra = 3; }
    else if ((first & 0xFC) == 0xF8) { num = first & 0x03; extra = 4; }
    else if ((first & 0xFE) == 0xFC) { num = first & 0x01; extra = 5; }
    else if (first == 0xFE) { num = 0; extra = 6; }
    else return FD_EHDR;
    for (int i = 0; i < extra; i++) {
        uint32_t c = (uint32_t)br_u(&b, 8);
        if ((c & 0xC0) != 0x80) return FD_EHDR;
        num = (num << 6) | (c & 0x3F);
    }
    uint32_t bs;
    if (bsc == 0) return FD_EHDR;
    else if (bsc == 1) bs = 192;
    else if (bsc <= 5) bs = 576u << (bsc - 2);
    else if (bsc == 6) bs = (uint32_t)br_u(&b, 8) + 1;
    else if (bsc == 7) bs = (uint32_t)br_u(&b, 16) + 1;
    else bs = 256u << (bsc - 8);
    uint32_t rate;
    if (src == 0) rate = stream_rate;
    else if (src <= 11) rate = RATE_TAB[src];
    else if (src == 12) rate = (uint32_t)br_u(&b, 8) * 1000;
    else if (src == 13) rate = (uint32_t)br_u(&b, 16);
    else if (src == 14) rate = (uint32_t)br_u(&b, 16) * 10;
    else return FD_EHDR;
    uint32_t bits = bitc == 0 ? stream_bits : BITS_TAB[bitc];
    if (bits == 0) return FD_EHDR;
    size_t hdr_bytes = (size_t)(b.pos >> 3);
    uint32_t crc8 = (uint32_t)br_u(&b, 8);
    if (b.err) return FD_EEOF;
    if (crc8 != crc8_spec(buf, hdr_bytes)) return FD_ECRC8;
    if (bs > max_block) return FD_ERANGE;
    uint32_t nch = chc <= 7 ? chc + 1 : (chc <= 10 ? 2 : 0);
    if (nch == 0) return FD_EHDR;
    fi->block_size = bs; fi->sample_rate = rate; fi->channel_assign = chc; fi->bits = bits; fi->number = num;
    for (uint32_t c = 0; c < nch; c++) {
        uint32_t sb = bits;
        if ((chc == 8 && c == 1) || (chc == 9 && c == 0) || (chc == 10 && c == 1)) sb = bits + 1;
        int rc = decode_subframe(&b, bs, sb, planes[c], fi, (int)c);
        if (rc) return rc;
    }
    /* undo decorrelation */
    for (uint32_t i = 0; i < bs; i++) {
        int64_t a = planes[0][i], s = nch > 1 ? planes[1][i] : 0;
        if (chc == 8) { planes[1][i] = a - s; }
        else if (chc == 9) { planes[0][i] = a + s; }
        else if (chc == 10) {
            int64_t mid = a * 2 + (s & 1);
            planes[0][i] = (mid + s) >> 1;
            planes[1][i] = (mid - s) >> 1;
        }
    }
    /* byte align (padding must be zero), then CRC-16 */
    while (b.pos & 7) if (br_bit(&b) != 0) return FD_ESUB;
    size_t body = (size_t)(b.pos >> 3);
    uint32_t crc16 = (uint32_t)br_u(&b, 16);
    if (b.err) return FD_EEOF;
    if (crc16 != crc16_spec(buf, body)) return FD_ECRC16;
    fi->frame_bytes = (uint32_t)(body + 2);
    return (long)(body + 2);
}

/* Decode a run of frames back to little-endian interleaved PCM with
 * `bytes_per_sample` bytes per sample.  Returns samples decoded (per
 * channel) or a negative FD_* code; *consumed gets the bytes used. */
long fdec_frames_to_pcm(const uint8_t *buf, size_t len, uint32_t channels, uint32_t bits, uint32_t rate,
                        uint32_t bytes_per_sample, uint8_t *pcm_out, uint64_t max_samples, uint64_t first_number,
                        uint32_t *frame_sizes, uint64_t max_frames) {
    int64_t *planes[8];
    for (int c = 0; c < 8; c++) planes[c] = (int64_t *)malloc(65536 * sizeof(int64_t));
    size_t pos = 0;
    uint64_t total = 0, f = 0;
    long rc = 0;
    fdec_frame_info fi;
    while (pos < len) {
        long n = fdec_frame(buf + pos, len - pos, bits, rate, planes, 65535, &fi);
        if (n < 0) { rc = n; break; }
        uint32_t nch = fi.channel_assign <= 7 ? fi.channel_assign + 1 : 2;
        if (nch != channels || fi.bits != bits || fi.number != first_number + f) { rc = FD_EHDR; break; }
        if (total + fi.block_size > max_samples) { rc = FD_ERANGE; break; }
        for (uint32_t i = 0; i < fi.block_size; i++)
            for (uint32_t c = 0; c < channels; c++) {
                int64_t v = planes[c][i];
                if (bits < 64 && (v < -(1LL << (bits - 1)) || v >= (1LL << (bits - 1)))) { rc = FD_ERANGE; goto done; }
                uint8_t *d = pcm_out + ((total + i) * channels + c) * bytes_per_sample;
                for (uint32_t k = 0; k < bytes_per_sample; k++) d[k] = (uint8_t)((uint64_t)v >> (8 * k));
            }
        if (frame_sizes && f < max_frames) frame_sizes[f] = (uint32_t)n;
        total += fi.block_size;
        pos += (size_t)n;
        f++;
    }
done:
    for (int c = 0; c < 8; c++) free(planes[c]);
    return rc < 0 ? rc : (long)total;
}
