/*
 * flacgpu.h -- C ABI of libflacgpu.so, the MI355X (gfx950) FLAC block encoder.
 *
 * Drop-in boundary for toastori/zig-flac's per-block encode path
 * (reference: src/lib.zig re-exports; the hot call is Encoder.writeFrame,
 * src/lib/encoder.zig:234-284).  Plain pointers and sizes only; no torch or
 * HIP types in any signature except the opaque `void *hip_stream` of the
 * device-resident entry points.  Each entry point cites the reference
 * interface it replaces.  The Zig `extern` declarations a maintainer adds to
 * the reference are in INTEGRATION.md.
 *
 * Output bytes are identical to the reference encoder's for the same input
 * (see DESIGN.md for the parity evidence and the one documented divergence,
 * a reference undefined-behaviour case).
 *
 * Threading: one context per GPU per host thread; a context is not
 * thread-safe.  All functions return FLACGPU_OK (0) or a negative error code.
 *
 * Streams: `void *hip_stream` is a hipStream_t, except two values: NULL selects
 * the context's own (non-blocking) stream, and FLACGPU_STREAM_LEGACY selects the
 * HIP null stream (legacy default-stream semantics), which orders the work
 * against default-stream producers and consumers (e.g. a framework whose
 * current stream handle is 0).
 */
#ifndef FLACGPU_H
#define FLACGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLACGPU_ABI_VERSION 5

/* the HIP null (legacy default) stream as a hip_stream argument */
#define FLACGPU_STREAM_LEGACY ((void *)1)

/* Error codes (map to the Zig error set
 * {OutOfMemory, WriteFailed, DeviceError, InvalidConfig, InvalidInput}). */
enum {
    FLACGPU_OK = 0,
    FLACGPU_ERR_INVALID_CONFIG = -1, /* Config outside what the reference accepts */
    FLACGPU_ERR_INVALID_INPUT = -2,  /* bad pointer / size / alignment */
    FLACGPU_ERR_OUT_OF_MEMORY = -3,  /* Allocator.Error.OutOfMemory (encoder.zig:48) */
    FLACGPU_ERR_OUTPUT_TOO_SMALL = -4, /* Writer.Error.WriteFailed analogue */
    FLACGPU_ERR_DEVICE = -5,         /* HIP runtime failure or no gfx950 device */
    FLACGPU_ERR_INTERNAL = -6        /* device-side invariant violated */
};

/* Encoder.Config + Config.Feature (encoder.zig:609-656) and the per-frame
 * FrameInfo fields that are constant over a stream (encoder.zig:658-663). */
typedef struct {
    uint32_t sample_rate;          /* FrameInfo.sample_rate (u20) */
    uint16_t block_size;           /* Config.block_size: 1..4096 (default 4096, encoder.zig:644) */
    uint8_t channels;              /* 1..8 */
    uint8_t bits_per_sample;       /* 8, 16, 24 or 32 (frame_writer.zig:221-233) */
    uint8_t stereo_decorrelation;  /* Feature.stereo_decorrelation (default 1) */
    uint8_t max_rice_part_order;   /* Feature.max_rice_order, 0..8 (default 8) */
    uint8_t max_rice_param;        /* Feature.max_rice_param, 1..30 (default 30) */
    uint8_t prediction;            /* Feature.prediction: 0 = fixed (the only value the
                                      reference implements; it never reads the field).
                                      Build-defined extension: 1..12 = also search LPC
                                      orders 1..prediction (DESIGN.md "LPC") */
} flacgpu_config;

/* Config.default(channels, bit_depth) (encoder.zig:642-655). */
flacgpu_config flacgpu_config_default(uint32_t channels, uint32_t bits_per_sample, uint32_t sample_rate);

typedef struct flacgpu_ctx flacgpu_ctx;

/* Encoder.init (encoder.zig:44-118): allocates all device scratch up front
 * for up to `max_frames_per_call` frames per call (0 = 32768).  device is the
 * HIP ordinal. */
int flacgpu_open(int device, const flacgpu_config *cfg, uint32_t max_frames_per_call, flacgpu_ctx **out);
/* Encoder.deinit (encoder.zig:121-164). */
void flacgpu_close(flacgpu_ctx *ctx);

const char *flacgpu_strerror(int code);
int flacgpu_abi_version(void);

/* How this libflacgpu.so was built (no reference counterpart: library introspection).
 * FLACGPU_BUILD_DIAG: a diagnostic build (`make diag`) with the measured-slower alternative
 * kernels / schedules and the diagnostic environment knobs compiled in; the release build has
 * none of them.  FLACGPU_BUILD_STAMPS: per-phase clock stamps (-DFG_STAMPS). */
#define FLACGPU_BUILD_DIAG 1u
#define FLACGPU_BUILD_STAMPS 2u
uint32_t flacgpu_build_flags(void);

/* maxFrameBytes (encoder.zig:583-595) of the reference, and the tight bound
 * the GPU path uses for its per-frame LDS image. */
size_t flacgpu_reference_max_frame_bytes(const flacgpu_config *cfg);
size_t flacgpu_frame_bound_bytes(const flacgpu_config *cfg);

/* ---- Host-buffer entry points (synchronous) ---------------------------- */

/* Batched Encoder.writeFrame (encoder.zig:234) driven the way wav2flac.encode
 * drives it (wav2flac.zig:66-97): `pcm` holds n_samples interleaved
 * little-endian samples of bytes_per_sample (= bits/8) bytes, exactly as a WAV
 * data chunk stores them (WavReader.fillSamples, wav_reader.zig:44-91).  Frames
 * of cfg.block_size samples are numbered from first_frame_number; the last
 * one may be short.  Writes the concatenated frames to out[0..*out_len) and
 * the per-frame byte counts (the u24 writeFrame returns) to frame_bytes[],
 * in frame order.  As in the reference, the caller drives the MD5
 * separately (flacgpu_md5_update with the same bytes). */
int flacgpu_encode_frames(flacgpu_ctx *ctx, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                          uint64_t first_frame_number, uint8_t *out, size_t out_cap, size_t *out_len,
                          uint32_t *frame_bytes);

/* ---- Multi-GPU host-buffer encode (SURVEY.md §8(b) "flacgpu_open_multi") --
 * One process, n_devices contexts (device ordinals may repeat).  A call shards
 * the input's frames into contiguous ranges, one per context, encodes them
 * concurrently (one host thread per context, each with its own PCIe link) and
 * concatenates the frames in frame order into out -- the bitstream
 * concatenation step of the multi-rank path, done in host memory because the
 * caller's output already lives there.  Same arguments, errors and output as
 * flacgpu_encode_frames (byte-identical to one context encoding it all). */
typedef struct flacgpu_multi flacgpu_multi;
int flacgpu_open_multi(int n_devices, const int *devices, const flacgpu_config *cfg, uint32_t max_frames_per_call,
                       flacgpu_multi **out);
void flacgpu_close_multi(flacgpu_multi *m);
int flacgpu_multi_encode_frames(flacgpu_multi *m, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                                uint64_t first_frame_number, uint8_t *out, size_t out_cap, size_t *out_len,
                                uint32_t *frame_bytes);

/* ---- Multi-rank encode: one process per GPU, RCCL over xGMI (SURVEY.md §8(b)
 *      "flacgpu_open_multi ... shards frames and gathers via RCCL", §8(e); BASELINE
 *      config 4) -----------------------------------------------------------------
 * The sharded form of wav2flac's block loop (wav2flac.zig:66-97): frame f of a
 * stream depends only on its samples and its number (encoder.zig:234-284), so the
 * ranks encode disjoint frames, and the only exchange is the gather of the
 * variable-length bitstreams and the per-frame sizes (the u24 writeFrame returns,
 * replayed by updateFrameSize in frame order, metadata.zig:35-40) to rank 0.
 * librccl.so.1 is loaded on first use (an RCCL already in the process, e.g. a
 * framework's, is reused; else /opt/rocm/lib); without it these return
 * FLACGPU_ERR_DEVICE.  Every call below is collective: every rank of the
 * communicator makes it, in the same order.  A communicator is used by one host
 * thread at a time (as a flacgpu_ctx is): its count buffers are per communicator. */
typedef struct flacgpu_comm flacgpu_comm;
#define FLACGPU_COMM_ID_BYTES 128
/* Rank 0 creates the communicator id; the host hands it to every rank (a file,
 * a socket, torch.distributed's store: any channel).  No GPU work. */
int flacgpu_comm_unique_id(uint8_t id[FLACGPU_COMM_ID_BYTES]);
/* Join the communicator as `rank` of `world` on HIP device `device` (one rank
 * per GPU: RCCL rejects two ranks on one device). */
int flacgpu_comm_init(const uint8_t id[FLACGPU_COMM_ID_BYTES], int world, int rank, int device,
                      flacgpu_comm **out);
void flacgpu_comm_destroy(flacgpu_comm *comm);
int flacgpu_comm_rank(const flacgpu_comm *comm);
int flacgpu_comm_size(const flacgpu_comm *comm);

/* Gather every rank's device-resident frames to rank 0, in rank order, into ONE
 * device buffer (xGMI point-to-point; nothing crosses PCIe).  Each rank gives its
 * n_frames frames: d_frames (device) holding nbytes valid bytes -- or, if
 * d_nbytes is non-NULL, the count in device memory (a u64, e.g. the d_total of
 * flacgpu_encode_plan_device_ex, read without a separate host sync) -- and
 * d_sizes (device u32 per frame).  Rank 0 passes d_recv (capacity recv_cap
 * bytes) and d_recv_sizes (capacity recv_sizes_cap entries); rank 0's own frames
 * are copied to their head unless d_frames == d_recv (encoded in place).  Every
 * rank gets *total_bytes / *total_frames (NULL: not wanted) = the gathered
 * totals.  Queued on hip_stream (NULL: the HIP null stream) and synchronised
 * with it once (the counts are read on the host to size the transfers).  If
 * rank 0's capacities are too small, EVERY rank returns
 * FLACGPU_ERR_OUTPUT_TOO_SMALL and nothing is transferred. */
int flacgpu_gather_frames_device(flacgpu_comm *comm, const uint8_t *d_frames, uint64_t nbytes, const uint64_t *d_nbytes,
                                 const uint32_t *d_sizes, uint64_t n_frames, uint8_t *d_recv, uint64_t recv_cap,
                                 uint32_t *d_recv_sizes, uint64_t recv_sizes_cap, uint64_t *total_bytes,
                                 uint64_t *total_frames, void *hip_stream);

/* flacgpu_encode_frames across the ranks of comm: every rank passes the SAME
 * arguments (pcm = the whole stream in host memory, e.g. each rank's mmap of the
 * WAV data chunk; n_samples; first_frame_number).  The frames are cut into
 * windows of world x max_frames_per_call frames; rank r encodes the r-th slice of
 * every window on its GPU, and each window's frames are gathered to rank 0's GPU
 * over RCCL and appended to rank 0's out (frame order).  Rank 0 gets exactly the
 * bytes and frame sizes flacgpu_encode_frames would write for the whole input;
 * other ranks get *out_len = 0 (out / frame_bytes unused, may be NULL).  A failure
 * on any rank is returned by every rank.  ctx must be open on comm's device with
 * the same config on every rank. */
int flacgpu_encode_frames_sharded(flacgpu_ctx *ctx, flacgpu_comm *comm, const void *pcm, uint32_t bytes_per_sample,
                                  uint64_t n_samples, uint64_t first_frame_number, uint8_t *out, size_t out_cap,
                                  size_t *out_len, uint32_t *frame_bytes);

/* Encoder.writeFrame for one frame, exactly the reference call: the caller
 * provides planar i32 samples (the reference's Encoder.samples[ch][0..n],
 * encoder.zig:23, each within bits_per_sample signed range), the frame number
 * (u36) and n = FrameInfo.samples_count (1..block_size).  Writes the frame to
 * out and its size to *frame_bytes. */
int flacgpu_encode_frame_planar(flacgpu_ctx *ctx, const int32_t *const planes[8], uint32_t n,
                                uint64_t frame_number, uint8_t *out, size_t out_cap, uint32_t *frame_bytes);

/* ---- Streaming MD5 (md5.zig, fed by wav_reader.zig:66; finalised by
 *      Encoder.finalizeStreamInfoMd5, encoder.zig:168-170) -------------------
 * One stream's MD5 is a strictly sequential chain.  The default engine hashes
 * on a host core (about 10x one GPU lane's rate, and the bytes are already in
 * host memory on this path); FLACGPU_MD5_DEVICE runs the chain on one GPU
 * lane (opt-in; the device-resident plans below hash many streams at once, one
 * lane per stream).  set_engine resets the running hash. */
enum { FLACGPU_MD5_HOST = 0, FLACGPU_MD5_DEVICE = 1 };
int flacgpu_md5_set_engine(flacgpu_ctx *ctx, int engine);
int flacgpu_md5_get_engine(const flacgpu_ctx *ctx);
int flacgpu_md5_init(flacgpu_ctx *ctx);
int flacgpu_md5_update(flacgpu_ctx *ctx, const void *data, size_t len);
int flacgpu_md5_final(flacgpu_ctx *ctx, uint8_t digest[16]);

/* ---- Device-resident entry points (asynchronous on hip_stream) --------- */

/* A plan describes a batch of independent streams (files) laid out in one
 * device PCM buffer: stream s holds stream_samples[s] interleaved samples
 * starting at byte offset stream_offsets[s] (4-byte aligned).  Frames of
 * every stream are numbered from 0.  The plan precomputes the frame table
 * (device memory) so repeated calls launch no host work. */
typedef struct flacgpu_plan flacgpu_plan;
int flacgpu_plan_create(flacgpu_ctx *ctx, uint32_t n_streams, const uint64_t *stream_offsets,
                        const uint64_t *stream_samples, uint32_t bytes_per_sample, flacgpu_plan **out);
void flacgpu_plan_destroy(flacgpu_plan *plan);
uint64_t flacgpu_plan_frames(const flacgpu_plan *plan);
/* Bytes of device output capacity the plan may need (sum of frame bounds). */
uint64_t flacgpu_plan_out_bound(const flacgpu_plan *plan);
/* First frame index of stream s inside the plan's frame table. */
uint64_t flacgpu_plan_stream_first_frame(const flacgpu_plan *plan, uint32_t s);

/* A plan whose streams are SEGMENTS of longer streams (a stream spans several
 * batches, as the reference's block loop spans a whole file, wav2flac.zig:66-97):
 * stream s's frames are numbered from first_frame_numbers[s] (NULL: 0) and
 * final_segment[s] == 0 marks a segment the stream continues after (NULL: every
 * segment final).  A non-final segment must hold whole frames of block_size
 * samples and a whole number of 64-byte MD5 blocks (always true at 4096). */
int flacgpu_plan_create_segments(flacgpu_ctx *ctx, uint32_t n_streams, const uint64_t *stream_offsets,
                                 const uint64_t *stream_samples, uint32_t bytes_per_sample,
                                 const uint64_t *first_frame_numbers, const uint8_t *final_segment,
                                 flacgpu_plan **out);
/* Move every frame number of the plan on by `frames`, queued on hip_stream: the
 * next window of the same streams at the same device offsets (a ring buffer the
 * caller refills).  Frame numbers stay u36. */
int flacgpu_plan_advance(flacgpu_plan *plan, uint64_t frames, void *hip_stream);

/* Per-stream MD5 chaining state carried from one call to the next (device
 * memory, 32 bytes per stream; initialise with flacgpu_md5_state_init and copy
 * to the device). */
typedef struct {
    uint32_t h[4];      /* MD5 chaining value */
    uint64_t bytes;     /* message bytes absorbed */
    uint32_t finished;  /* 1 once the final segment has been padded: h is then the digest, and
                           later calls leave the state unchanged (a final segment passed again
                           reports the same digest); re-initialise it to start a new stream */
    uint32_t reserved;
} flacgpu_md5_state;
void flacgpu_md5_state_init(flacgpu_md5_state *states, size_t n);

/* Encode every frame of the plan from device PCM d_pcm into the contiguous
 * device buffer d_out (capacity out_cap).  Per frame: d_frame_bytes[f] (u32)
 * and d_frame_offsets[f] (u64 byte offset of frame f in d_out; stream s's
 * bitstream is the contiguous range starting at its first frame's offset).
 * d_total (u64) receives the total byte count.  If d_md5 is non-NULL, the MD5
 * of every stream's raw PCM bytes is computed on the GPU into d_md5[16*s].
 * Nothing is synchronised; all work is queued on hip_stream (NULL = the
 * context's own stream). */
int flacgpu_encode_plan_device(flacgpu_ctx *ctx, const flacgpu_plan *plan, const void *d_pcm, uint8_t *d_out,
                               uint64_t out_cap, uint32_t *d_frame_bytes, uint64_t *d_frame_offsets,
                               uint64_t *d_total, uint8_t *d_md5, void *hip_stream);

/* As flacgpu_encode_plan_device, but the MD5 of the streams is queued on
 * md5_stream (after the PCM is ready on hip_stream) and NOT joined back into
 * hip_stream: the encode of the next batch can start while this batch's MD5
 * chains finish (the MD5 is per-stream sequential and latency-bound, the
 * encode is throughput-bound, so consecutive batches overlap).  The caller
 * synchronises md5_stream before reading d_md5 or reusing d_pcm.
 * md5_stream == NULL behaves exactly like flacgpu_encode_plan_device. */
int flacgpu_encode_plan_device_md5_async(flacgpu_ctx *ctx, const flacgpu_plan *plan, const void *d_pcm,
                                         uint8_t *d_out, uint64_t out_cap, uint32_t *d_frame_bytes,
                                         uint64_t *d_frame_offsets, uint64_t *d_total, uint8_t *d_md5,
                                         void *hip_stream, void *md5_stream);

/* flacgpu_encode_plan_device with carried MD5 state: if d_md5_state is non-NULL,
 * each stream's state is read, advanced by its segment and written back (the
 * MD5 of a stream spanning many calls); segments marked final are padded and
 * their digest written to d_md5[16 s] (if non-NULL).  With d_md5_state NULL every
 * segment must be final (fresh state, digest to d_md5).  md5_stream as in
 * flacgpu_encode_plan_device_md5_async (NULL: joined into hip_stream). */
int flacgpu_encode_plan_device_ex(flacgpu_ctx *ctx, const flacgpu_plan *plan, const void *d_pcm, uint8_t *d_out,
                                  uint64_t out_cap, uint32_t *d_frame_bytes, uint64_t *d_frame_offsets,
                                  uint64_t *d_total, flacgpu_md5_state *d_md5_state, uint8_t *d_md5,
                                  void *hip_stream, void *md5_stream);

/* The host engine of the same MD5 (md5.zig:3-31 over the bytes wav_reader.zig:66
 * feeds it; finalised as Encoder.finalizeStreamInfoMd5, encoder.zig:168-170).
 * flacgpu_md5_many advances n independent chains on the library's host hashing
 * pool: chain i absorbs lens[i] bytes at data[i] from states[i] (host memory,
 * the layout and `finished` rules of the device path above, so a stream's state
 * may pass between the engines from one call to the next); final[i] != 0 (final
 * NULL: every chain) pads the chain and writes its digest to digests[16 i] (if
 * non-NULL).  states NULL: fresh chains, all final.  A chain that continues
 * after the call must absorb whole 64-byte blocks.  Needs no GPU; blocks. */
int flacgpu_md5_many(uint32_t n, const void *const *data, const uint64_t *lens, const uint8_t *final,
                     flacgpu_md5_state *states, uint8_t *digests);
/* flacgpu_md5_many over every segment of `plan`, read from h_pcm, a host copy
 * of the device PCM buffer (same offsets), with the plan's final flags.  Run it
 * on a host thread beside flacgpu_encode_plan_device_ex called with
 * d_md5_state = d_md5 = NULL: few long streams then hash at host-core speed
 * instead of one GPU lane each. */
int flacgpu_md5_plan_host(const flacgpu_plan *plan, const void *h_pcm, flacgpu_md5_state *states, uint8_t *digests);
/* The faster MD5 engine for this plan's segments: FLACGPU_MD5_HOST below the
 * stream-count crossover (a few long chains), FLACGPU_MD5_DEVICE above it:
 * flacgpu_md5_engine_for(plan's stream count, longest segment, total bytes). */
int flacgpu_plan_md5_engine(const flacgpu_plan *plan);

/* The rates the engine choice is priced with (no reference
 * counterpart: the reference hashes on its one thread).  host_chain[i]: bytes/s
 * per pool worker when every worker holds host_chains[i] chains (1, 2, 3, 4 for the
 * scalar interleave; 1, 4, 8, 16 where the host has AVX-512), MEASURED on this
 * machine by running the pool the first time they are needed
 * (flacgpu_md5_get_rates); host_workers: the pool's size (0: no pool, host_chain
 * is one chain on the caller); device_lane / device_chip: bytes/s of one stream's
 * GPU lane beside the encode and of all lanes together (MI355X measurements). */
typedef struct {
    double host_chain[4];
    uint32_t host_chains[4]; /* chains per worker of each host_chain entry (0s: 1, 2, 3, 4) */
    double device_lane;
    double device_chip;
    int32_t host_workers;
    int32_t measured; /* 1: host_chain measured in this process; 2: set by the caller; 3: measured while
                         other chains were hashing on the pool (possibly low: set_rates(NULL) re-measures) */
} flacgpu_md5_rates;
/* The current rates (measures the host ones on first use, ~2 ms).  Needs no GPU. */
int flacgpu_md5_get_rates(flacgpu_md5_rates *out);
/* Replace the rates (NULL: measure again); e.g. a caller's own measurement. */
int flacgpu_md5_set_rates(const flacgpu_md5_rates *rates);
/* The engine the rates predict faster for n_streams chains of at most max_len
 * bytes, total_len bytes in all: host time = total / (pool throughput at
 * ceil(n / workers) chains per worker, interpolated between the measured points
 * and flat past the last: time-sliced), device time =
 * max(max_len / device_lane, total / device_chip).  Needs no GPU. */
int flacgpu_md5_engine_for(uint32_t n_streams, uint64_t max_len, uint64_t total_len);

/* Synchronise hip_stream (NULL: the context's stream) and report the device-side
 * error word of the kernels queued so far (FLACGPU_ERR_OUTPUT_TOO_SMALL when a
 * frame would not fit out_cap, FLACGPU_ERR_INTERNAL on a violated invariant);
 * clears it.  The device-resident entry points are asynchronous: this is how
 * their caller learns of a failure. */
int flacgpu_sync_check(flacgpu_ctx *ctx, void *hip_stream);

/* ---- File level (host code around the GPU frame path) --------------------- */

/* The context's configuration (what flacgpu_open was given). */
int flacgpu_get_config(const flacgpu_ctx *ctx, flacgpu_config *out);

/* WavReader.init / getFmt (wav_reader.zig:116-170) and the flacStreaminfo checks
 * (wav_reader.zig:92-108) on an in-memory WAV file: the PCM data chunk starts at
 * data_offset; samples = data_len / (channels * (bits/8)) as in wav_reader.zig:169. */
typedef struct {
    uint32_t sample_rate;
    uint16_t channels;
    uint16_t bits_per_sample;   /* valid bits (EXTENSIBLE) or the fmt bit depth */
    uint16_t bytes_per_sample;  /* block_align / channels */
    uint16_t pad;
    uint64_t samples;           /* interchannel samples */
    uint64_t data_offset;
    uint64_t data_bytes;
} flacgpu_wav_info;
int flacgpu_wav_parse(const void *wav, size_t len, flacgpu_wav_info *info);

/* StreamInfo (metadata.zig:18-68). */
typedef struct {
    uint8_t md5[16];
    uint64_t interchannel_samples;
    uint32_t min_frame_size;    /* u24; starts at 0xFFFFFF */
    uint32_t max_frame_size;    /* u24; starts at 0 */
    uint32_t sample_rate;
    uint16_t min_block_size;
    uint16_t max_block_size;
    uint8_t channels;
    uint8_t bit_depth;
    uint8_t pad[6];
} flacgpu_streaminfo;
void flacgpu_streaminfo_init(flacgpu_streaminfo *si, uint32_t sample_rate, uint32_t channels, uint32_t bit_depth,
                             uint64_t interchannel_samples, uint32_t block_size);
/* StreamInfo.updateFrameSize (metadata.zig:35-40), with its else-if. */
void flacgpu_streaminfo_update_frame_size(flacgpu_streaminfo *si, uint32_t frame_size);
/* StreamInfo.updateFrameSize replayed over n_frames device-resident frame sizes in frame
 * order (metadata.zig:35-40, the caller's loop at wav2flac.zig:94): d_minmax (device, u32[2])
 * holds {min_frame_size, max_frame_size} on entry (0xFFFFFF, 0 for a new stream, or the
 * state after earlier windows) and on exit, with the reference's else-if quirk: a frame that
 * raises the running max never lowers the min.  One workgroup, queued on hip_stream; the
 * bitstream of a sharded encode never leaves HBM for its STREAMINFO. */
int flacgpu_streaminfo_replay_device(flacgpu_ctx *ctx, const uint32_t *d_frame_bytes, uint64_t n_frames,
                                     uint32_t *d_minmax, void *hip_stream);
/* StreamInfo.bytes (metadata.zig:42-68). */
void flacgpu_streaminfo_bytes(const flacgpu_streaminfo *si, uint8_t out[34]);
/* Encoder.writeHeader (encoder.zig:192-206): "fLaC" + STREAMINFO block; returns 42. */
size_t flacgpu_header_bytes(const flacgpu_streaminfo *si, int last_metadata, uint8_t out[42]);
/* Encoder.writeVorbisComment (encoder.zig:211-226): vendor "toastori FLAC 0.0.0", no tags; returns 31. */
size_t flacgpu_vorbis_comment_bytes(int last_metadata, uint8_t out[31]);

/* wav2flac (wav2flac.zig:10-97) for PCM in memory: the 73-byte header (STREAMINFO not
 * last, VORBIS_COMMENT last) + every frame, STREAMINFO carrying the frame-size
 * min/max (from the GPU's per-frame sizes, replayed in frame order) and the MD5 of
 * the PCM bytes (the context's MD5 engine; the host engine hashes on a thread
 * that runs beside the GPU encode). */
int flacgpu_encode_file(flacgpu_ctx *ctx, const void *pcm, uint32_t bytes_per_sample, uint64_t n_samples,
                        uint8_t *out, size_t out_cap, size_t *out_len);
/* flacgpu_encode_file for n_files PCM buffers at once on one context: out[i]
 * (capacity out_cap[i]) receives exactly the bytes flacgpu_encode_file writes for
 * file i, out_len[i] their count (all 0 on an error).  Every file's frames go
 * through one pipelined upload / encode / download schedule that runs on from
 * file to file, and every file's MD5 is hashed on the host pool in one batch
 * beside it: the many-files-per-GPU form of wav2flac.zig:10-97. */
int flacgpu_encode_files(flacgpu_ctx *ctx, uint32_t n_files, const void *const *pcm, uint32_t bytes_per_sample,
                         const uint64_t *n_samples, uint8_t *const *out, const size_t *out_cap, size_t *out_len);
/* The whole conversion of an in-memory WAV file on HIP device `device`
 * (Config.default for the WAV's channels and bit depth). */
int flacgpu_wav_to_flac(int device, const void *wav, size_t wav_len, uint8_t *out, size_t out_cap, size_t *out_len);

/* ---- Instrumentation ---------------------------------------------------- */
/* Kernel ids for flacgpu_kernel_time: frame analysis (4096-sample frames /
 * short frames), frame-size scan, frame packing (all frames), stream MD5. */
enum { FLACGPU_K_ANALYZE = 0, FLACGPU_K_ANALYZE_TAIL = 1, FLACGPU_K_SCAN = 2, FLACGPU_K_PACK = 3, FLACGPU_K_MD5 = 4,
       FLACGPU_K_COUNT = 5 };
/* When enabled, every launch of kernel k is bracketed by HIP events on the
 * stream it runs on; flacgpu_kernel_time returns the number of timed launches
 * and their summed device milliseconds since the last reset. */
int flacgpu_set_timing(flacgpu_ctx *ctx, int enable);
int flacgpu_kernel_time(flacgpu_ctx *ctx, int kernel, uint64_t *launches, double *total_ms);
int flacgpu_reset_timing(flacgpu_ctx *ctx);

/* Decision records (for parity tests): when enabled, each encode call also
 * stores one flacgpu_frame_record per frame, readable with
 * flacgpu_get_records after a synchronous call (flacgpu_encode_files: the
 * records of every file, file after file, in frame order). */
typedef struct {
    uint8_t type;       /* 0 CONSTANT, 1 VERBATIM, 2 FIXED, 3 LPC */
    uint8_t waste;
    uint8_t bits;       /* channel bit depth before waste removal */
    uint8_t order;
    uint8_t part_order;
    uint8_t method;     /* 0 FOUR, 1 FIVE */
    uint8_t written;    /* 1 if this candidate is in the bitstream */
    uint8_t pad;
    uint32_t pad2;
    uint64_t estimate;
    int64_t constant;
    uint8_t params[256];
    uint8_t lpc_precision;  /* LPC only */
    int8_t lpc_shift;
    uint8_t pad3[6];
    int32_t lpc_coefs[32];
} flacgpu_subframe_record;

typedef struct {
    uint32_t channel_code;
    uint32_t n_cand;
    uint32_t frame_bytes;
    uint32_t pad;
    flacgpu_subframe_record cand[8];
} flacgpu_frame_record;

int flacgpu_set_records(flacgpu_ctx *ctx, int enable);

/* Encode schedule (no reference counterpart: how the device runs the writeFrame loop).
 * ranges > 1: each call's full frames are encoded in that many frame ranges, the analysis of
 * range i+1 beside the scan + pack of range i on a second HIP stream, the two persistent grids
 * capped at ana_per_cu / pack_per_cu workgroups per CU (0 = no cap); calls with fewer than
 * ranges * min_frames full frames use fewer ranges.  ranges <= 1: one analysis, scan and pack
 * launch per call.  Output bytes are the same either way.  The overlapped schedule measured
 * slower than the serial one: ranges > 1 is FLACGPU_ERR_INVALID_CONFIG unless the library is a
 * diagnostic build (flacgpu_build_flags() & FLACGPU_BUILD_DIAG). */
int flacgpu_set_overlap(flacgpu_ctx *ctx, uint32_t ranges, uint32_t ana_per_cu, uint32_t pack_per_cu,
                        uint32_t min_frames);
int flacgpu_get_records(flacgpu_ctx *ctx, flacgpu_frame_record *out, uint64_t max_frames, uint64_t *n_frames);

#ifdef __cplusplus
}
#endif
#endif
