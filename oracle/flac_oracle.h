/*
 * flac_oracle.h -- CPU restatement of toastori/zig-flac's block-encode path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product path (zig-flac_amd/, libflacgpu.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline -- never as the thing shipped.
 *
 * Parity status: the reference (Zig 0.16) cannot be built here or on the GPU
 * box (no zig toolchain), and it ships no tests, fixtures or golden vectors
 * (SURVEY.md section 4, 8c).  Whole-frame parity against reference OUTPUT is
 * therefore UNPINNED.  What pins this restatement instead:
 *   - published known-answer tests for the third-party primitives it relies on
 *     (CRC-8/SMBUS, CRC-16/UMTS, MD5 / RFC 1321, UTF-8 coded numbers);
 *   - lossless round trips through an independent FLAC decoder
 *     (oracle/flac_decode.c, written from the FLAC format spec, no code shared
 *     with this file), including CRC-8/CRC-16/MD5 verification;
 *   - hand-derived known-answer frames for every decision quirk listed in
 *     SURVEY.md Appendix A (tests/test_oracle_quirks.py).
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef FLAC_ORACLE_H
#define FLAC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Encoder.Config / Feature (src/lib/encoder.zig:609-656). */
typedef struct {
    uint32_t sample_rate;
    uint16_t block_size;          /* 4096 in Config.default (encoder.zig:644) */
    uint8_t channels;             /* 1..8 */
    uint8_t bits_per_sample;      /* 8, 16, 24, 32 (frame_writer.zig:221-233) */
    uint8_t stereo_decorrelation; /* default true */
    uint8_t max_rice_part_order;  /* default 8 */
    uint8_t max_rice_param;       /* default 30 (rice.MAX_PARAM) */
    uint8_t prediction;           /* unused by the reference (encoder.zig:629-640).  Build-defined
                                     extension: 0 = fixed prediction only (the reference's output,
                                     bit for bit); 1..32 = also search LPC orders 1..prediction
                                     (see the LPC contract in flac_oracle.c / DESIGN.md) */
} oracle_config;

enum { OR_CONSTANT = 0, OR_VERBATIM = 1, OR_FIXED = 2, OR_LPC = 3 };
#define ORACLE_LPC_MAX_ORDER 32
#define ORACLE_LPC_PRECISION 15   /* quantised coefficient bits (FLAC field max) */

/* Decision record of one evaluated subframe (SubframeType.Encoding,
 * encoder.zig:678-702, plus the estimate returned by chooseSubframeEncoding). */
typedef struct {
    uint8_t type;        /* OR_CONSTANT / OR_VERBATIM / OR_FIXED */
    uint8_t waste;       /* wasted bits */
    uint8_t bits;        /* channel bit depth before waste removal (bd, +1 for side) */
    uint8_t order;       /* fixed order (FIXED only) */
    uint8_t part_order;  /* rice partition order (FIXED only) */
    uint8_t method;      /* 0 = FOUR, 1 = FIVE (FIXED only) */
    uint8_t wide;        /* 1 if the wide (i64 / >=28 bit) path was used */
    uint8_t ub_clamped;  /* 1 if the partition order had to be clamped (reference UB) */
    uint64_t estimate;   /* bit estimate used for decisions */
    int64_t constant;    /* CONSTANT value (shifted), 0 when undefined (bps'==0) */
    uint8_t params[256]; /* rice Param.p for the chosen order: p, or 0x80|bits */
    /* LPC only (build-defined extension) */
    uint8_t lpc_precision;
    int8_t lpc_shift;
    uint8_t pad2[6];
    int32_t lpc_coefs[ORACLE_LPC_MAX_ORDER];
} oracle_subframe;

typedef struct {
    uint8_t channel_code;      /* header channel assignment: ch-1, 8, 9, 10 */
    uint8_t n_sub;             /* subframes written */
    uint8_t n_cand;            /* candidates evaluated (4 for stereo) */
    uint8_t pad;
    uint32_t frame_bytes;
    oracle_subframe written[8];  /* in bitstream order */
    oracle_subframe cand[8];     /* stereo: L, R, M, S; indep: per channel */
} oracle_frame_record;

/* ---- primitives ---- */
uint8_t oracle_crc8(const uint8_t *p, size_t n);               /* CRC-8/SMBUS */
uint16_t oracle_crc16(uint16_t crc, const uint8_t *p, size_t n); /* CRC-16/UMTS */
uint16_t oracle_crc16_bitwise(uint16_t crc, const uint8_t *p, size_t n); /* the same, one bit per step */

typedef struct {
    uint32_t a, b, c, d;
    uint64_t len;
    uint8_t buf[64];
    uint32_t fill;
} oracle_md5_ctx;
void oracle_md5_init(oracle_md5_ctx *c);
void oracle_md5_update(oracle_md5_ctx *c, const void *p, size_t n);
void oracle_md5_final(oracle_md5_ctx *c, uint8_t out[16]);
void oracle_md5(const void *p, size_t n, uint8_t out[16]);

/* UTF-8-style frame number coder of frame_writer.zig:235-251; returns bytes. */
int oracle_utf8_number(uint64_t v, uint8_t out[8]);

/* WavReader.fillSamples de-interleave + sign extension
 * (wav_reader.zig:44-91,172-249) for 2/3/4-byte containers. */
void oracle_unpack_pcm(const uint8_t *bytes, uint32_t bytes_per_sample, uint32_t channels,
                       uint32_t bit_depth, uint32_t n, int32_t *const *planes);

/* Encoder.writeFrame (encoder.zig:234-284).  planes[ch][0..n) are the raw
 * (unshifted) samples; they are copied, not modified.  Returns the frame byte
 * count (> 0) or a negative error code. */
long oracle_encode_frame(const oracle_config *cfg, const int32_t *const *planes, uint32_t n,
                         uint64_t frame_number, uint8_t *out, size_t cap,
                         oracle_frame_record *rec);

/* wav2flac.encode loop (wav2flac.zig:66-97) over interleaved little-endian
 * PCM: frames of cfg->block_size, last one short.  Writes the concatenated
 * frames, per-frame sizes, and (optionally) the MD5 of the raw bytes.
 * Returns total bytes or negative error. */
long oracle_encode_stream(const oracle_config *cfg, const uint8_t *pcm, uint32_t bytes_per_sample,
                          uint64_t n_samples, uint64_t first_frame, uint8_t *out, size_t cap,
                          uint32_t *frame_bytes, uint8_t md5_out[16]);

/* Whole file as wav2flac.main produces it (wav2flac.zig:10-63):
 * fLaC + STREAMINFO + VORBIS_COMMENT(last) + frames. */
long oracle_encode_file(const oracle_config *cfg, const uint8_t *pcm, uint32_t bytes_per_sample,
                        uint64_t n_samples, uint8_t *out, size_t cap);

/* StreamInfo.bytes (metadata.zig:42-68) and updateFrameSize (metadata.zig:35-40). */
typedef struct {
    uint8_t md5[16];
    uint64_t interchannel_samples;
    uint32_t min_frame_size, max_frame_size;
    uint32_t sample_rate;
    uint16_t min_block_size, max_block_size;
    uint8_t channels, bit_depth;
} oracle_streaminfo;
void oracle_streaminfo_init(oracle_streaminfo *si);
void oracle_streaminfo_update(oracle_streaminfo *si, uint32_t frame_size);
void oracle_streaminfo_bytes(const oracle_streaminfo *si, uint8_t out[34]);

/* maxFrameBytes (encoder.zig:583-595). */
size_t oracle_max_frame_bytes(uint32_t block_size, uint32_t bit_depth, uint32_t channels);

/* LPC pieces (build-defined; exposed for unit tests).  x: n shifted samples.
 * autocorr: R[0..max_lag] exact (returns the scaling shift sh).
 * levinson: coefs[(q-1)*32 + t] for orders q = 1..max_order; returns the
 * number of orders with valid coefficients.
 * quantize: returns 0 and the shift, or -1 if the order is not representable. */
int oracle_lpc_autocorr(const int64_t *x, uint32_t n, unsigned max_lag, int64_t *R);
int oracle_lpc_levinson(const int64_t *R, unsigned max_order, double *coefs);
int oracle_lpc_levinson_err(const int64_t *R, unsigned max_order, double *coefs, double *errs);
double oracle_lpc_order_key(double err, unsigned q, uint32_t n, unsigned bps);
int oracle_lpc_quantize(const double *a, unsigned order, unsigned precision, int32_t *q, int *shift);
/* analysis mode (not the contract): exhaustive LPC order search, for compression comparisons */
void oracle_set_lpc_exhaustive(int on);

/* Exposed pieces for unit tests. */
uint64_t oracle_rice_part_size(uint64_t len, uint32_t param, uint64_t abs_sum);
int oracle_best_order(const int64_t *s, uint32_t n, int wide, uint64_t totals[5]);

#ifdef __cplusplus
}
#endif
#endif
