// fg_misc.hip -- the small kernels around the frame encoder (gfx950): frame
// table, frame-size scan, MD5 (md5.zig / RFC 1321) with one lane per
// independent stream, and the per-width dispatcher of the analysis / pack
// kernels.
#include <hip/hip_runtime.h>

#include "fg_common.hpp"

namespace fg {

__device__ __forceinline__ uint32_t lane_id_m() { return __lane_id(); }

#define FG_DECL(B, W) \
    hipError_t launch_stage_b##B##_l##W(int, const EncodeArgs &, bool, uint32_t, uint32_t, hipStream_t);
#define FG_DECL3(B) FG_DECL(B, 0) FG_DECL(B, 8) FG_DECL(B, 12)
FG_DECL3(1)
FG_DECL3(2)
FG_DECL3(3)
FG_DECL3(4)

// LPC taps held in registers for a configured maximum LPC order (0 = fixed only)
uint32_t lpc_taps(uint32_t lpc_order) { return lpc_order == 0 ? 0u : (lpc_order <= 8 ? 8u : 12u); }

// stage 0: analysis kernel, 1: pack kernel
hipError_t launch_stage(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    const uint32_t w = lpc_taps(a.lpc_order);
#define FG_CASE(B)                                                                              \
    case B:                                                                                     \
        if (w == 0) return launch_stage_b##B##_l0(stage, a, full, threads, lds, st);            \
        if (w == 8) return launch_stage_b##B##_l8(stage, a, full, threads, lds, st);            \
        return launch_stage_b##B##_l12(stage, a, full, threads, lds, st);
    switch (a.bytes_per_sample) {
        FG_CASE(1)
        FG_CASE(2)
        FG_CASE(3)
        FG_CASE(4)
        default: return hipErrorInvalidValue;
    }
#undef FG_CASE
}

// ------------------------------------------------------------------------
// frame table for one contiguous stream (wav2flac.zig:66-97)
// ------------------------------------------------------------------------
__global__ void k_make_jobs(FrameJob *jobs, uint64_t n_samples, uint32_t block, uint32_t frame_stride_bytes,
                            uint64_t first_number, uint32_t n_frames) {
    uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_frames) return;
    uint64_t start = (uint64_t)f * block;
    uint64_t rem = n_samples - start;
    FrameJob j;
    j.pcm_off = (uint64_t)f * frame_stride_bytes;
    j.number = first_number + f;
    j.n = (uint32_t)(rem < block ? rem : block);
    j.slot = f;
    jobs[f] = j;
}

// the same streams' next window (flacgpu_plan_advance): frame numbers move on by delta
__global__ void k_advance_jobs(FrameJob *jobs, uint64_t n, uint64_t delta) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) jobs[i].number += delta;
}

// ------------------------------------------------------------------------
// exclusive scan of frame sizes -> byte offsets (single workgroup, 1024 thr).
// Thread t owns a contiguous run of `per` sizes (a multiple of 4), read as
// 16-byte vectors and written back as 16-byte pairs of u64 offsets; the
// thread totals are scanned across the workgroup with wave shuffles.
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_scan(const uint32_t *sizes, uint64_t *offsets, uint64_t *total, uint32_t n) {
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (((n + 1023u) / 1024u) + 3u) & ~3u;
    const uint32_t b = t * per, e = min(n, b + per);
    // 16-byte vectors only when both buffers are 16-byte aligned (caller-provided pointers)
    const bool vec = ((reinterpret_cast<uintptr_t>(sizes) | reinterpret_cast<uintptr_t>(offsets)) & 15u) == 0;
    uint64_t acc = 0;
    if (vec && b + per <= n) {
        const uint4 *s4 = (const uint4 *)(sizes + b);
        for (uint32_t i = 0; i < per / 4u; i++) {
            const uint4 v = s4[i];
            acc += (uint64_t)v.x + v.y + v.z + v.w;
        }
    } else {
        for (uint32_t i = b; i < e; i++) acc += sizes[i];
    }
    // block exclusive scan of acc
    uint64_t x = acc;
    const uint32_t l = lane_id_m(), w = t >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x += y;
    }
    if (l == 63) wsum[w] = x;
    __syncthreads();
    uint64_t pre = 0;
    for (uint32_t i = 0; i < w; i++) pre += wsum[i];
    uint64_t run = pre + x - acc;
    if (vec && b + per <= n) {
        const uint4 *s4 = (const uint4 *)(sizes + b);
        ulonglong2 *o2 = (ulonglong2 *)(offsets + b);
        for (uint32_t i = 0; i < per / 4u; i++) {
            const uint4 v = s4[i];
            ulonglong2 a, c;
            a.x = run; run += v.x;
            a.y = run; run += v.y;
            c.x = run; run += v.z;
            c.y = run; run += v.w;
            o2[2 * i] = a;
            o2[2 * i + 1] = c;
        }
    } else {
        for (uint32_t i = b; i < e; i++) {
            offsets[i] = run;
            run += sizes[i];
        }
    }
    if (t == 1023) {
        uint64_t tot = 0;
        for (int i = 0; i < 16; i++) tot += wsum[i];
        *total = tot;
    }
}

// ------------------------------------------------------------------------
// The same scan over many workgroups (k_scan, one workgroup, took ~60 us for 65536 frames:
// one CU's memory latency): block b = frames [4096 b, 4096 b + 4096), four per thread.
// k_scan_part writes each block's sum; k_scan_blocks adds the sums of the blocks before
// its own to its workgroup's exclusive scan.
// ------------------------------------------------------------------------
constexpr uint32_t kScanBlock = 4096;

__device__ __forceinline__ void scan_load4(const uint32_t *sizes, uint32_t i0, uint32_t n, bool vec, uint32_t (&v)[4]) {
    if (vec && i0 + 4u <= n) {
        const uint4 q = *(const uint4 *)(sizes + i0);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = (i0 + (uint32_t)k < n) ? sizes[i0 + k] : 0u;
    }
}

// workgroup exclusive scan of one u64 per thread (1024 threads); *blk = the workgroup total
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t acc, uint64_t *wsum, uint64_t *blk) {
    const uint32_t t = threadIdx.x, l = lane_id_m(), w = t >> 6;
    uint64_t x = acc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x += y;
    }
    if (l == 63) wsum[w] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
        const uint64_t v = wsum[i];
        pre += i < w ? v : 0u;
        tot += v;
    }
    *blk = tot;
    return pre + x - acc;
}

__global__ void __launch_bounds__(1024) k_scan_part(const uint32_t *sizes, uint64_t *part, uint32_t n) {
    __shared__ uint64_t wsum[16];
    const bool vec = (reinterpret_cast<uintptr_t>(sizes) & 15u) == 0;
    uint32_t v[4];
    scan_load4(sizes, blockIdx.x * kScanBlock + 4u * threadIdx.x, n, vec, v);
    uint64_t blk;
    (void)block_excl_scan((uint64_t)v[0] + v[1] + v[2] + v[3], wsum, &blk);
    if (threadIdx.x == 0) part[blockIdx.x] = blk;
}

__global__ void __launch_bounds__(1024) k_scan_blocks(const uint32_t *sizes, uint64_t *offsets, uint64_t *total,
                                                      const uint64_t *part, uint32_t n, const uint64_t *base) {
    __shared__ uint64_t wsum[16], bsum[16];
    const uint32_t t = threadIdx.x, b = blockIdx.x;
    // sum of the blocks before this one (plus the carried base of the frames before the range)
    uint64_t p = (base && t == 0) ? *base : 0;
    for (uint32_t j = t; j < b; j += 1024u) p += part[j];
    uint64_t before;
    (void)block_excl_scan(p, bsum, &before);
    const uint32_t i0 = b * kScanBlock + 4u * t;
    const bool vec = ((reinterpret_cast<uintptr_t>(sizes) | reinterpret_cast<uintptr_t>(offsets)) & 15u) == 0;
    uint32_t v[4];
    scan_load4(sizes, i0, n, vec, v);
    uint64_t blk;
    uint64_t run = before + block_excl_scan((uint64_t)v[0] + v[1] + v[2] + v[3], wsum, &blk);
    uint64_t o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        o[k] = run;
        run += v[k];
    }
    if (vec && i0 + 4u <= n) {
        ulonglong2 *o2 = (ulonglong2 *)(offsets + i0);
        o2[0] = make_ulonglong2(o[0], o[1]);
        o2[1] = make_ulonglong2(o[2], o[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i0 + (uint32_t)k < n) offsets[i0 + k] = o[k];
    }
    if (b == gridDim.x - 1u && t == 0) *total = before + blk;
}

// ------------------------------------------------------------------------
// Frame totals after a channel-split analysis (k_analyze, a.ch_split): the two halves wrote
// their subframes' descriptors and half 0 the frame header; total bits = header + every
// subframe, exact frame bytes, the pack kernel's image bound and the records' frame size.
// ------------------------------------------------------------------------
__global__ void k_frame_totals(EncodeArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_jobs) return;
    const uint32_t slot = a.jobs[i].slot;
    FrameDesc *f = (FrameDesc *)(a.desc + (uint64_t)slot * a.desc_stride);
    const SubDesc *sd = (const SubDesc *)((const uint8_t *)f + sizeof(FrameDesc));
    uint32_t total = 8u * f->hdr_bytes;
    for (uint32_t c = 0; c < f->n_out; c++) total += sd[c].bits;
    f->total_bits = total;
    // channel-half pack hand-off word (k_packw split mode) starts empty
    *(unsigned long long *)((uint8_t *)f + desc_side_off(f->n_out)) = 0ull;
    const uint32_t fbytes = ((total + 7u) >> 3) + 2u;
    if (fbytes + 16u > a.image_bytes) atomicOr(a.err, 1u);
    a.frame_bytes[slot] = fbytes;
    if (a.records) a.records[slot].frame_bytes = fbytes;
}

// ------------------------------------------------------------------------
// StreamInfo.updateFrameSize over device-resident sizes (metadata.zig:35-40):
//   if (sz > max) max = sz; else if (sz < min) min = sz;
// in frame order.  max ends as the plain maximum; frame f can lower min only when it does
// not raise the max, i.e. when sz_f <= M_f = max(max_in, sz_0 .. sz_{f-1}).  So
// min = min(min_in, min{ sz_f : sz_f <= M_f }).  Thread t owns a contiguous run of frames:
// run maxima -> exclusive max-scan across the workgroup -> each run replayed from its M.
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_streaminfo_replay(const uint32_t *sizes, uint64_t n, uint32_t *minmax) {
    __shared__ uint32_t wmax[16], wmin[16];
    const uint32_t t = threadIdx.x, l = lane_id_m(), w = t >> 6;
    const uint64_t per = (n + 1023u) / 1024u;
    const uint64_t b = (uint64_t)t * per, e = b + per < n ? b + per : n;
    const uint32_t min_in = minmax[0], max_in = minmax[1];
    uint32_t rmax = 0;
    for (uint64_t i = b; i < e; i++) rmax = max(rmax, sizes[i]);
    // inclusive max-scan within the wave, then across waves
    uint32_t x = rmax;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (l >= (uint32_t)d) x = max(x, y);
    }
    if (l == 63) wmax[w] = x;
    __syncthreads();
    uint32_t before = max_in, all = max_in;
    for (uint32_t i = 0; i < 16; i++) {
        all = max(all, wmax[i]);
        if (i < w) before = max(before, wmax[i]);
    }
    const uint32_t excl = __shfl_up(x, 1);
    uint32_t M = l ? max(before, excl) : before;  // running max entering this thread's run
    uint32_t mn = 0xFFFFFFFFu;
    for (uint64_t i = b; i < e; i++) {
        const uint32_t sz = sizes[i];
        if (sz > M) M = sz;
        else mn = min(mn, sz);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mn = min(mn, __shfl_xor(mn, d));
    if (l == 0) wmin[w] = mn;
    __syncthreads();
    if (t == 0) {
        uint32_t m = min_in;
        for (int i = 0; i < 16; i++) m = min(m, wmin[i]);
        minmax[0] = m;
        minmax[1] = all;
    }
}

// ------------------------------------------------------------------------
// MD5 (md5.zig / RFC 1321): one lane per independent stream
// ------------------------------------------------------------------------
constexpr uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

#define MD5_STEP(F, a, b, c, d, m, k, s) a = b + rotl(a + F(b, c, d) + (m) + (k), s)
// H round: (b ^ (c ^ d)) + (a + m + k) as one v_xad_u32 whose other operands are off the
// critical path -- 3 dependent ops per step instead of 4 (tools/micro/md5_micro.hip variant 4)
__device__ __forceinline__ uint32_t xad_u32(uint32_t x, uint32_t y, uint32_t z) {
    uint32_t r;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}
#define MD5_STEP_H(a, b, c, d, m, k, s) a = b + rotl(xad_u32(b, (c) ^ (d), a + (m) + (k)), s)
#define MD5_F(b, c, d) (((b) & (c)) | (~(b) & (d)))
#define MD5_G(b, c, d) (((b) & (d)) | ((c) & ~(d)))
#define MD5_I(b, c, d) ((c) ^ ((b) | ~(d)))

__device__ __forceinline__ void md5_compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        MD5_STEP(MD5_F, a, b, c, d, m[i + 0], kMd5K[i + 0], 7);
        MD5_STEP(MD5_F, d, a, b, c, m[i + 1], kMd5K[i + 1], 12);
        MD5_STEP(MD5_F, c, d, a, b, m[i + 2], kMd5K[i + 2], 17);
        MD5_STEP(MD5_F, b, c, d, a, m[i + 3], kMd5K[i + 3], 22);
    }
#pragma unroll
    for (int i = 16; i < 32; i += 4) {
        MD5_STEP(MD5_G, a, b, c, d, m[(5 * i + 1) & 15], kMd5K[i + 0], 5);
        MD5_STEP(MD5_G, d, a, b, c, m[(5 * i + 6) & 15], kMd5K[i + 1], 9);
        MD5_STEP(MD5_G, c, d, a, b, m[(5 * i + 11) & 15], kMd5K[i + 2], 14);
        MD5_STEP(MD5_G, b, c, d, a, m[(5 * i + 16) & 15], kMd5K[i + 3], 20);
    }
#pragma unroll
    for (int i = 32; i < 48; i += 4) {
        MD5_STEP_H(a, b, c, d, m[(3 * i + 5) & 15], kMd5K[i + 0], 4);
        MD5_STEP_H(d, a, b, c, m[(3 * i + 8) & 15], kMd5K[i + 1], 11);
        MD5_STEP_H(c, d, a, b, m[(3 * i + 11) & 15], kMd5K[i + 2], 16);
        MD5_STEP_H(b, c, d, a, m[(3 * i + 14) & 15], kMd5K[i + 3], 23);
    }
#pragma unroll
    for (int i = 48; i < 64; i += 4) {
        MD5_STEP(MD5_I, a, b, c, d, m[(7 * i) & 15], kMd5K[i + 0], 6);
        MD5_STEP(MD5_I, d, a, b, c, m[(7 * i + 7) & 15], kMd5K[i + 1], 10);
        MD5_STEP(MD5_I, c, d, a, b, m[(7 * i + 14) & 15], kMd5K[i + 2], 15);
        MD5_STEP(MD5_I, b, c, d, a, m[(7 * i + 21) & 15], kMd5K[i + 3], 21);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// MD5 of n_streams independent byte ranges (segments), one lane per stream.
// A segment may continue a stream begun by an earlier call: `states` (if
// non-NULL) holds each stream's chaining value and byte count in and out
// (Md5.update over successive blocks, wav_reader.zig:66).  A non-final segment
// is a whole number of 64-byte blocks (checked on the host); a final one is
// padded and its digest written to digests[16 s] (Md5.final,
// encoder.zig:168-170).  `final_flags` NULL = every segment final.
// Messages are read as 16-byte vectors (segment starts are 4-byte aligned;
// the unaligned-access mode of the HSA runtime serves them) and prefetched
// kMd5Ahead blocks ahead: 4 vector loads per block instead of 16 dword loads
// keep the texture-address path, which the encode kernels' LDS-DMA staging
// shares on the same CU, 4x less busy.
typedef uint32_t md5_v4 __attribute__((ext_vector_type(4), aligned(4)));
#ifndef FG_MD5_AHEAD
#define FG_MD5_AHEAD 2
#endif
// waves per SIMD the MD5 kernel is compiled for: at 7 it fits 72 VGPRs (one message block in flight ahead), so its waves take
// little of the register file the encode kernels running beside it occupy
#ifndef FG_MD5_WPE
#define FG_MD5_WPE 7
#endif
constexpr int kMd5Ahead = FG_MD5_AHEAD;
#ifndef FG_MD5_PRIO
#define FG_MD5_PRIO 0
#endif
// Streams per MD5 workgroup.  The encode kernels fill their SIMDs' register files (k_analyze
// 4 x 128 VGPRs, k_pack4 8 x 64), so a SIMD that holds an MD5 wave loses one encode wave and its
// CU one encode workgroup.  Four MD5 waves per workgroup (one per SIMD of one CU) confine that
// loss to a quarter of the CUs that one-wave workgroups spread it over: C2 step 2.19 -> 2.12 ms
// (tools/ab_env.sh, FLACGPU_MD5_WG A/B).
constexpr uint32_t kMd5Wg = kMd5StreamsPerWg;

__device__ __forceinline__ void md5_load_block(const uint8_t *p, uint32_t (&m)[16]) {
#if defined(FG_MD5_DIAG) && FG_MD5_DIAG == 1
    p = (const uint8_t *)((uintptr_t)p & ~(uintptr_t)0xFFFF);  // diagnostics: a cache-resident block
#endif
    const md5_v4 *q = (const md5_v4 *)p;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const md5_v4 v = q[i];
        m[4 * i + 0] = v.x;
        m[4 * i + 1] = v.y;
        m[4 * i + 2] = v.z;
        m[4 * i + 3] = v.w;
    }
}

__global__ void __launch_bounds__(kMd5Wg) __attribute__((amdgpu_waves_per_eu(FG_MD5_WPE, 8))) k_md5_streams(const uint8_t *base, const uint64_t *offs, const uint64_t *lens,
                                                    const uint8_t *final_flags, uint32_t n_streams, Md5State *states,
                                                    uint8_t *digests) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_streams) return;
    // The chain is latency-bound and these few waves share SIMDs with the encode kernels.  At
    // issue priority 3 they win every arbitration and the encode waves beside them lose issue
    // slots; at the default 0 the encode runs ~5-10 % faster with 16384 streams while each MD5
    // chain slows only slightly (tools/ab_md5.sh A/B).
    __builtin_amdgcn_s_setprio(FG_MD5_PRIO);
    const uint8_t *p = base + offs[s];
    const uint64_t len = lens[s];
    const bool fin = final_flags ? final_flags[s] != 0 : true;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint64_t done = 0;  // bytes absorbed by earlier segments
    if (states) {
        const Md5State in = states[s];
        st[0] = in.h[0];
        st[1] = in.h[1];
        st[2] = in.h[2];
        st[3] = in.h[3];
        done = in.bytes;
        if (in.flags & 1u) {
            // already finalised (Md5.final ran, encoder.zig:168-170): h IS the digest.  Absorbing
            // more bytes or padding again would corrupt it, so the state is left as it is and a
            // requested digest is the finished one (re-initialise a state before reusing it)
            if (fin && digests)
                for (int i = 0; i < 4; i++)
                    for (int j = 0; j < 4; j++) digests[16 * s + 4 * i + j] = (uint8_t)(st[i] >> (8 * j));
            return;
        }
    }
    const uint64_t full = len >> 6;
    // Ring of R = kMd5Ahead + 1 message blocks in registers: block b is compressed while blocks
    // b + 1 .. b + kMd5Ahead are in flight.  The loads inside the loop are UNCONDITIONAL (the
    // block index is clamped to the lane's last block, a harmless re-read): a load under a
    // per-lane condition makes the compiler merge "loaded" and "old" ring values at the join,
    // i.e. copy the whole ring through v_mov behind an s_waitcnt vmcnt(0) -- which waited for
    // the blocks just issued and exposed one full memory latency per loop trip (beside the
    // encode kernels' traffic, ~1 us per 64-B block; tools/micro/md5_lab.hip).
    constexpr int R = kMd5Ahead + 1;
    uint32_t m[R][16];
    const uint64_t last = full ? full - 1 : 0;
    if (full)
#pragma unroll
        for (int k = 0; k < R; k++) md5_load_block(p + 64u * min((uint64_t)k, last), m[k]);
    uint64_t b = 0;
    for (; b + R <= full; b += R) {
#pragma unroll
        for (int k = 0; k < R; k++) {
            md5_compress(st, m[k]);
            md5_load_block(p + 64u * min(b + k + R, last), m[k]);
            // keep the refill here, R - 1 compressions ahead of its use: without a fence the
            // scheduler sinks every refill to the end of the trip (prefetch distance ~0)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int k = 0; k < R - 1; k++)
        if (b + k < full) md5_compress(st, m[k]);
    if (fin) {
        // tail + padding (one or two blocks): the rem < 64 tail bytes as dwords (the dword holding
        // the end assembled from bytes: nothing past the segment is read), then 0x80 and the
        // bit length
        const uint32_t rem = (uint32_t)(len & 63);
        const uint8_t *tp = p + full * 64;
        const uint32_t *tp32 = (const uint32_t *)tp;
        uint32_t mt[16];
        const uint32_t wr = rem >> 2, br = rem & 3u;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t v = 0;
            if ((uint32_t)i < wr) {
                v = tp32[i];
            } else if ((uint32_t)i == wr) {
                for (uint32_t q = 0; q < br; q++) v |= (uint32_t)tp[4u * i + q] << (8u * q);
                v |= 0x80u << (8u * br);
            }
            mt[i] = v;
        }
        const uint64_t bits = (done + len) * 8;
        if (rem < 56) {
            mt[14] = (uint32_t)bits;
            mt[15] = (uint32_t)(bits >> 32);
            md5_compress(st, mt);
        } else {
            md5_compress(st, mt);
#pragma unroll
            for (int i = 0; i < 14; i++) mt[i] = 0;
            mt[14] = (uint32_t)bits;
            mt[15] = (uint32_t)(bits >> 32);
            md5_compress(st, mt);
        }
        if (digests)
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++) digests[16 * s + 4 * i + j] = (uint8_t)(st[i] >> (8 * j));
    }
    if (states) {
        Md5State o;
        o.h[0] = st[0];
        o.h[1] = st[1];
        o.h[2] = st[2];
        o.h[3] = st[3];
        o.bytes = done + len;
        o.flags = fin ? 1u : 0u;
        o.pad = 0;
        states[s] = o;
    }
}

// ------------------------------------------------------------------------
// The same MD5 with COALESCED message loads through an LDS ring (the default).
//
// k_md5_streams above loads each lane's own 16-B pieces: one dwordx4 touches 64 cache lines
// 64 KiB apart.  Beside the encode kernels' LDS-DMA staging on the same CUs those loads queue
// in the texture path, and a block's load latency, not the 64-step chain, sets the rate
// (tools/micro/md5_lab.hip: 1.86 us per block beside an LDS-DMA streamer, 1.2 alone, against
// 0.5 with no loads at all).  Here the blocks arrive by LDS-DMA in whole cache lines: chunk c of
// a stream is its blocks CB c .. CB c + CB - 1; DMA instruction i of a chunk moves 16 / CB
// streams' chunks (64 CB bytes each, one line for CB = 2) into LDS rows of 64 CB bytes, the
// 16-B pieces of a row rotated by the stream index so that the 16 lanes of a ds_read_b128
// quarter read 16 distinct bank groups.  R chunks are in flight per wave; the wave waits for
// chunk c with vmcnt(4 CB (R - 1)) and re-fills its slot once the chunk is in registers.  All
// lanes take part in every DMA (a lane fetches OTHER streams' pieces), so the chunk loop is
// wave-uniform and a lane whose segment has ended only skips the compression.
// ------------------------------------------------------------------------
// chunk of CB blocks (1 or 2), R chunks in flight per wave, NWV waves (64 streams each) per workgroup
template <uint32_t CB> struct Md5Geo {
    static constexpr uint32_t Chunk = 4096u * CB;  // LDS bytes per chunk per wave (64 streams)
    static constexpr uint32_t Per = 16u / CB;      // streams per DMA instruction
    static constexpr uint32_t Pcs = 4u * CB;       // 16-B pieces per stream chunk = DMAs per chunk
};

// rotation of stream sl's row: the lanes of a 16-lane quarter (consecutive sl) that share a
// 256-B bank window get distinct 16-B slots
template <uint32_t CB>
__device__ __forceinline__ uint32_t md5_rot(uint32_t sl) { return CB == 2 ? (sl >> 1) : (sl >> 2); }

template <uint32_t CB, uint32_t R, uint32_t NWV>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_md5_streams_lds(const uint8_t *base, const uint64_t *offs, const uint64_t *lens, const uint8_t *final_flags,
                  uint32_t n_streams, Md5State *states, uint8_t *digests, const uint8_t *dummy, uint32_t prio,
                  uint32_t diag) {
    constexpr uint32_t kMd5CB = CB, kMd5R = R;
    constexpr uint32_t kMd5Chunk = Md5Geo<CB>::Chunk, kMd5Per = Md5Geo<CB>::Per, kMd5Pcs = Md5Geo<CB>::Pcs;
    __shared__ __attribute__((aligned(16))) uint8_t ring[NWV][R][kMd5Chunk];
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (prio) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(0);
    const bool live = s < n_streams;
    const uint8_t *p = dummy;
    uint64_t len = 0, done = 0;
    bool fin = false;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (live) {
        p = base + offs[s];
        len = lens[s];
        fin = final_flags ? final_flags[s] != 0 : true;
        if (states) {
            const Md5State in = states[s];
            st[0] = in.h[0];
            st[1] = in.h[1];
            st[2] = in.h[2];
            st[3] = in.h[3];
            done = in.bytes;
            if (in.flags & 1u) {
                // already finalised (Md5.final ran, encoder.zig:168-170): h IS the digest; the
                // state stays as it is and a requested digest is the finished one
                if (fin && digests)
                    for (int i = 0; i < 4; i++)
                        for (int j = 0; j < 4; j++) digests[16 * s + 4 * i + j] = (uint8_t)(st[i] >> (8 * j));
                len = 0;
                fin = false;
                states = nullptr;  // nothing to store back for this lane
            }
        }
    }
    const uint64_t full = len >> 6;
    if (!full) p = dummy;  // a lane with no whole block serves its DMA pieces from a valid address
    // the pointer / whole-block count of the stream each of this lane's DMA pieces belongs to
    const uint8_t *src_p[kMd5Pcs];
    uint64_t src_full[kMd5Pcs];
    uint32_t src_rot[kMd5Pcs];
#pragma unroll
    for (uint32_t i = 0; i < kMd5Pcs; i++) {
        const uint32_t sl = kMd5Per * i + l / kMd5Pcs;
        src_p[i] = (const uint8_t *)__shfl((unsigned long long)(uintptr_t)p, (int)sl);
        src_full[i] = __shfl((unsigned long long)full, (int)sl);
        src_rot[i] = ((l % kMd5Pcs) - md5_rot<CB>(sl)) % kMd5Pcs;  // piece index this lane moves
    }
    // wave-uniform chunk count
    uint64_t wmax = full;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) wmax = max(wmax, (uint64_t)__shfl_xor((unsigned long long)wmax, d));
    const uint64_t nch = (wmax + kMd5CB - 1) / kMd5CB;
    uint8_t *wr = &ring[wave][0][0];
    // chunk c into ring slot `slot` (normally c % R)
    auto issue = [&](uint32_t slot, uint64_t c) {
        uint8_t *dst = wr + slot * kMd5Chunk;
#pragma unroll
        for (uint32_t i = 0; i < kMd5Pcs; i++) {
            // piece src_rot[i] of chunk c of stream sl; pieces past the stream's whole blocks
            // re-read its first piece (never compressed)
            const uint64_t off = 64u * kMd5CB * c + 16u * src_rot[i];
            const uint8_t *q = src_p[i] + (off + 16u <= 64u * src_full[i] ? off : 0u);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)q,
                                             (__attribute__((address_space(3))) void *)(dst + 1024u * i), 16, 0, 0);
        }
    };
    // diag (diagnostics only, wrong digests): bit 0 = no LDS reads (message words from registers),
    // bit 1 = no DMA and no waits
    const bool dma = !(diag & 2u), rd = !(diag & 1u);
    if (dma)
        for (uint32_t c = 0; c < kMd5R; c++) issue(c, c < nch ? c : 0);
    const uint32_t row = 64u * kMd5CB * l, rot = md5_rot<CB>(l);
    for (uint64_t c = 0; c < nch; c++) {
        // chunk c has landed once at most the R - 1 younger chunks' DMAs are outstanding
        if (!dma) {
        } else if constexpr (kMd5R * kMd5Pcs == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if constexpr (kMd5R * kMd5Pcs == 12 && kMd5Pcs == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr (kMd5R * kMd5Pcs == 16 && kMd5Pcs == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr (kMd5R * kMd5Pcs == 16 && kMd5Pcs == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if constexpr (kMd5R * kMd5Pcs == 24) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint8_t *buf = wr + (uint32_t)(c % kMd5R) * kMd5Chunk + row;
        uint32_t m[kMd5CB][16];
#pragma unroll
        for (uint32_t k = 0; k < kMd5CB; k++)
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t pc = 4u * k + q;
                const md5_v4 v = rd ? *(const md5_v4 *)(buf + 16u * ((pc + rot) % kMd5Pcs))
                                    : md5_v4{st[0] + pc, st[1], st[2], st[3]};
                m[k][4 * q] = v.x;
                m[k][4 * q + 1] = v.y;
                m[k][4 * q + 2] = v.z;
                m[k][4 * q + 3] = v.w;
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // the slot is free once its words are in registers: re-fill it with chunk c + R (past the
        // end: chunk c again, into the same slot -- a redundant DMA that keeps the vmcnt
        // arithmetic uniform and never lands in a slot that is still to be read)
        if (dma) issue((uint32_t)(c % kMd5R), c + kMd5R < nch ? c + kMd5R : c);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (uint32_t k = 0; k < kMd5CB; k++)
            if (kMd5CB * c + k < full) md5_compress(st, m[k]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!live) return;
    if (fin) {
        // tail + padding, as in k_md5_streams
        const uint32_t rem = (uint32_t)(len & 63);
        const uint8_t *tp = base + offs[s] + full * 64;
        const uint32_t *tp32 = (const uint32_t *)tp;
        uint32_t mt[16];
        const uint32_t wrm = rem >> 2, br = rem & 3u;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t v = 0;
            if ((uint32_t)i < wrm) {
                v = tp32[i];
            } else if ((uint32_t)i == wrm) {
                for (uint32_t q = 0; q < br; q++) v |= (uint32_t)tp[4u * i + q] << (8u * q);
                v |= 0x80u << (8u * br);
            }
            mt[i] = v;
        }
        const uint64_t bits = (done + len) * 8;
        if (rem < 56) {
            mt[14] = (uint32_t)bits;
            mt[15] = (uint32_t)(bits >> 32);
            md5_compress(st, mt);
        } else {
            md5_compress(st, mt);
#pragma unroll
            for (int i = 0; i < 14; i++) mt[i] = 0;
            mt[14] = (uint32_t)bits;
            mt[15] = (uint32_t)(bits >> 32);
            md5_compress(st, mt);
        }
        if (digests)
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++) digests[16 * s + 4 * i + j] = (uint8_t)(st[i] >> (8 * j));
    }
    if (states) {
        Md5State o;
        o.h[0] = st[0];
        o.h[1] = st[1];
        o.h[2] = st[2];
        o.h[3] = st[3];
        o.bytes = done + len;
        o.flags = fin ? 1u : 0u;
        o.pad = 0;
        states[s] = o;
    }
}

// Streaming update of one MD5 state in device memory by whole 64-byte blocks.
__global__ void k_md5_blocks(uint32_t *state, const uint32_t *blocks, uint64_t n_blocks) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t st[4] = {state[0], state[1], state[2], state[3]};
    for (uint64_t b = 0; b < n_blocks; b++) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = blocks[b * 16 + i];
        md5_compress(st, m);
    }
    for (int i = 0; i < 4; i++) state[i] = st[i];
}

// ------------------------------------------------------------------------
// host-side launch wrappers (called from fg_api.cpp)
// ------------------------------------------------------------------------
hipError_t launch_make_jobs(FrameJob *jobs, uint64_t n_samples, uint32_t block, uint32_t stride, uint64_t first,
                            uint32_t n_frames, hipStream_t st) {
    if (n_frames == 0) return hipSuccess;
    hipLaunchKernelGGL(k_make_jobs, dim3((n_frames + 255) / 256), dim3(256), 0, st, jobs, n_samples, block, stride,
                       first, n_frames);
    return hipGetLastError();
}

hipError_t launch_advance_jobs(FrameJob *jobs, uint64_t n, uint64_t delta, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_advance_jobs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, jobs, n, delta);
    return hipGetLastError();
}

hipError_t launch_frame_totals(const EncodeArgs &a, hipStream_t st) {
    if (a.n_jobs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_frame_totals, dim3((a.n_jobs + 255u) / 256u), dim3(256), 0, st, a);
    return hipGetLastError();
}

// part: ceil(n / 4096) u64 of scratch (NULL: the one-workgroup k_scan).  base (multi-workgroup
// form only): a device u64 added to every offset -- the bytes of the frames before the range,
// for a call scanned range by range (overlapped encode, fg_api.cpp)
hipError_t launch_scan(const uint32_t *sizes, uint64_t *offsets, uint64_t *total, uint32_t n, uint64_t *part,
                       hipStream_t st, const uint64_t *base) {
    if (base && !part) return hipErrorInvalidValue;
    if (!part) {
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, sizes, offsets, total, n);
        return hipGetLastError();
    }
    const uint32_t nb = (n + kScanBlock - 1u) / kScanBlock;
    if (nb > 1u) hipLaunchKernelGGL(k_scan_part, dim3(nb), dim3(1024), 0, st, sizes, part, n);
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, st, sizes, offsets, total, part, n, base);
    return hipGetLastError();
}

hipError_t launch_streaminfo_replay(const uint32_t *sizes, uint64_t n, uint32_t *minmax, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_streaminfo_replay, dim3(1), dim3(1024), 0, st, sizes, n, minmax);
    return hipGetLastError();
}

// kernel 0: per-lane loads (k_md5_streams); otherwise the coalesced LDS-DMA ring
// (k_md5_streams_lds) in geometry `kernel` (1 = the default, 2.. = A/B variants); prio: issue
// priority of the MD5 waves (0 or 3)
template <uint32_t CB, uint32_t R, uint32_t NWV>
static void launch_md5_lds(const uint8_t *base, const uint64_t *offs, const uint64_t *lens, const uint8_t *fin,
                           uint32_t n, Md5State *states, uint8_t *digests, uint32_t prio, uint32_t diag,
                           hipStream_t st) {
    const uint8_t *dummy = states ? (const uint8_t *)states : digests;  // >= 16 valid bytes
    const uint32_t wg = 64u * NWV;
    hipLaunchKernelGGL((k_md5_streams_lds<CB, R, NWV>), dim3((n + wg - 1) / wg), dim3(wg), 0, st, base, offs, lens, fin, n,
                       states, digests, dummy, prio, diag);
}

hipError_t launch_md5_streams(const uint8_t *base, const uint64_t *offs, const uint64_t *lens, const uint8_t *fin,
                              uint32_t n, Md5State *states, uint8_t *digests, hipStream_t st, int kernel, int prio) {
    if (n == 0) return hipSuccess;
    const uint32_t pr = prio & 1u, dg = (uint32_t)prio >> 8;  // prio bits 8..9: diagnostics
    switch (kernel) {
        case 0:
            hipLaunchKernelGGL(k_md5_streams, dim3((n + kMd5Wg - 1) / kMd5Wg), dim3(kMd5Wg), 0, st, base, offs, lens, fin,
                               n, states, digests);
            break;
        case 2: launch_md5_lds<1, 3, 4>(base, offs, lens, fin, n, states, digests, pr, dg, st); break;  // 48 KiB
        case 3: launch_md5_lds<2, 3, 2>(base, offs, lens, fin, n, states, digests, pr, dg, st); break;  // 48 KiB
        case 4: launch_md5_lds<2, 2, 4>(base, offs, lens, fin, n, states, digests, pr, dg, st); break;  // 64 KiB
        case 5: launch_md5_lds<2, 2, 2>(base, offs, lens, fin, n, states, digests, pr, dg, st); break;  // 32 KiB
        // default: one-block chunks, two in flight, four waves = 32 KiB of LDS, one workgroup in the
        // footprint of one k_analyze workgroup (37 KiB, 4 x 128 VGPRs)
        default: launch_md5_lds<1, 2, 4>(base, offs, lens, fin, n, states, digests, pr, dg, st); break;
    }
    return hipGetLastError();
}

// workgroups a launch_md5_streams(kernel) of n streams occupies
uint32_t md5_workgroups(uint32_t n, int kernel) {
    const uint32_t wg = (kernel == 3 || kernel == 5) ? 128u : 256u;
    return (n + wg - 1u) / wg;
}

hipError_t launch_md5_blocks(uint32_t *state, const uint32_t *blocks, uint64_t n_blocks, hipStream_t st) {
    hipLaunchKernelGGL(k_md5_blocks, dim3(1), dim3(64), 0, st, state, blocks, n_blocks);
    return hipGetLastError();
}

}  // namespace fg
