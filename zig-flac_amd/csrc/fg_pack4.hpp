// fg_pack4.hpp -- frame packing for full 16-bit two-channel frames with four waves per
// written subframe (included by fg_device.hpp inside namespace fg).
//
// The general pack kernel (k_pack) gives each written subframe one wave of 64-sample
// lanes: 8 waves per CU, each lane emitting 64 codes in one dependent chain, so the
// kernel is latency bound.  Here a lane owns 16 consecutive samples (wave 4s+q of the
// workgroup packs quarter q of written subframe s), which gives 4x the waves and
// 4x shorter chains.  Per frame (frame_writer.zig:269-372 restated):
//   1. PCM arrives by 16-B LDS-DMA in a rotated layout: 16-sample chunk j holds its
//      4-sample group g in 16-B slot (g + (j >> 2)) & 3, so the 16 lanes of a
//      quarter-wave read 16 distinct bank groups (ds_read_b128, conflict free);
//   2. each lane rebuilds its candidate samples (L, R, mid, side; encoder.zig:329-350)
//      plus the 4 samples before them, applies the waste shift and the fixed-order
//      residual (fixed.zig:30-76);
//   3. code lengths (rice: (zz >> p) + 1 + p, escape: width; rice.zig / frame_writer.zig)
//      -> a wave prefix scan on top of the quarter's base, which is the sum of the
//      analysis kernel's exact 64-sample segment lengths before it;
//   4. the codes are ORed into the zeroed LDS frame image, CRC-16 by the same
//      front-padded parallel fold as k_pack, and the frame is stored at its final offset.
#pragma once

#ifndef FG_PACK4_MINW
#define FG_PACK4_MINW 8
#endif


// 16 instructions of 1 KiB: lane i of instruction k fills slot i & 3 of chunk 16k + (i >> 2)
// from that chunk's 4-sample group ((i & 3) - (chunk >> 2)) & 3.
__device__ __forceinline__ void stage_dma_rot(const uint8_t *pcm, uint64_t off, uint32_t *stg, uint32_t wave,
                                              uint32_t NW, uint32_t l) {
    const uint32_t *src = (const uint32_t *)(pcm + off);
    for (uint32_t k = wave; k < 16u; k += NW) {
        const uint32_t j = 16u * k + (l >> 2);
        const uint32_t g = ((l & 3u) - (j >> 2)) & 3u;
        lds_dma<16>(src + 16u * j + 4u * g, stg + 256u * k);
    }
}

// dword offset of 4-sample group g of 16-sample chunk j in the rotated layout
__device__ __forceinline__ uint32_t rot_off(uint32_t j, uint32_t g) { return 16u * j + 4u * ((g + (j >> 2)) & 3u); }

// The frame descriptor in LDS (P4Layout dsc0 / dsc1, 320 dwords), DMA'd during the previous frame
// together with the job record of the frame after it: [0..7] FrameDesc, [8..11] and [12..15] bytes
// 0..15 of SubDesc 0 and 1 (type .. cand, lpc_shift, bits, lpc_prec), [16..17] the frame's byte
// offset, [18..23] the next frame's FrameJob, [64..127] / [128..191] lane_bits of SubDesc 0 / 1,
// [192..255] / [256..319] their Rice parameters.  Five 4-byte LDS-DMA instructions (waves 0..4).
// Loaded at the top of their own frame, the two dependent round trips to the descriptor table
// (written by the analysis kernel: an Infinity-Cache or HBM read) were 21 % of every pack wave's
// time (r3g stamps), and the next job record's load waited behind the frame's PCM DMA.
__device__ __forceinline__ void p4_dsc_dma(const EncodeArgs &a, uint32_t slot, uint32_t nxt_job, uint32_t *dsc,
                                           uint32_t wave, uint32_t l) {
    if (wave >= 5u) return;
    const uint8_t *fd = a.desc + (uint64_t)slot * a.desc_stride;
    const uint8_t *src;
    if (wave == 0) {
        if (l < 8u) src = fd + 4u * l;
        else if (l < 12u) src = fd + 32u + 4u * (l - 8u);
        else if (l < 16u) src = fd + 32u + sizeof(SubDesc) + 4u * (l - 12u);
        else if (l < 18u) src = (const uint8_t *)(a.offsets + slot) + 4u * (l - 16u);
        else if (l < 24u && nxt_job < a.n_jobs) src = (const uint8_t *)(a.jobs + nxt_job) + 4u * (l - 18u);
        else src = fd;
    } else if (wave <= 2u) {
        src = fd + 32u + (wave - 1u) * sizeof(SubDesc) + offsetof(SubDesc, lane_bits) + 4u * l;
    } else {
        src = fd + 32u + (wave - 3u) * sizeof(SubDesc) + offsetof(SubDesc, params) + 4u * l;
    }
    lds_dma<4>(src, dsc + 64u * wave);
}

template <int MAXT>
__global__ void __launch_bounds__(MAXT, FG_PACK4_MINW) k_pack4(EncodeArgs a) {
    if (a.enc_prio) __builtin_amdgcn_s_setprio(1);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const uint32_t tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)), l0 = lane_id();
    const uint32_t sfi = wave >> 2, qw = wave & 3u;  // written subframe, quarter
    const P4Layout LY = pack4_layout(a.image_bytes);
    uint32_t *misc = (uint32_t *)(smem + LY.misc);
    const bool stereo = a.stereo != 0;

    // Tickets run two frames ahead.  The one for frame i+2 is taken at the END of frame i-1, after
    // its output stores: the atomic's round trip then overlaps the wait for those stores that the
    // top of frame i has anyway (taken after the DMAs of frame i, the wait for the atomic's value
    // also waited for them), and it is published at the top of frame i.
    uint32_t *ctr = a.work_ctr + 2u;
    reset_analysis_tickets(a.work_ctr, tid);  // the analysis kernel's queues
    if (tid == 0) misc[21] = gridDim.x + atomicAdd(ctr, 1u);
    __syncthreads();
    uint32_t jidx = blockIdx.x, buf = 0;
    uint32_t nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[21]);
    uint32_t tk = 0;
    if (tid == 0) tk = gridDim.x + atomicAdd(ctr, 1u);
    uint32_t slot = 0;
    if (jidx < a.n_jobs) {
        const FrameJob job = a.jobs[jidx];
        slot = job.slot;
        stage_dma_rot(a.pcm, job.pcm_off, (uint32_t *)(smem + LY.buf0), wave, NW, l0);
        p4_dsc_dma(a, job.slot, nxt, (uint32_t *)(smem + LY.dsc0), wave, l0);
    }
#ifdef FG_STAMPS
    uint64_t ph_[16] = {};
    uint64_t tprev_ = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t i0 = 1024u * qw + 16u * l0;  // first sample of this lane
    while (jidx < a.n_jobs) {
        const uint32_t l = opaque(l0);
        uint32_t *stg = (uint32_t *)(smem + (buf ? LY.buf1 : LY.buf0));
        uint32_t *img = stg;  // the image reuses the staging buffer once the samples are in VGPRs
        const uint32_t *dsc = (const uint32_t *)(smem + (buf ? LY.dsc1 : LY.dsc0));

        // ---- 1. PCM and descriptor (DMA'd during the previous frame) -> this lane's samples
        STAMP(7);
        if (tid == 0) misc[20] = tk;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(8);
        __syncthreads();
        STAMP(0);
        const uint32_t nn = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[20]);  // frame i+2
        const uint32_t total_bits = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[1]);
        const uint32_t fbytes = ((total_bits + 7u) >> 3) + 2u;
        const uint64_t D = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[17]) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[16]);
        const uint32_t Lb = (total_bits + 7u) >> 3;
        const uint32_t W4 = Lb >> 2;
        const uint32_t H = max((W4 + 2u * NT - 1u) / (2u * NT), 1u);  // words per thread / 2
        const uint32_t hq = min(H, a.crc_hmax4) - 1u;
        const bool skip = fbytes + 16u > a.image_bytes || D + fbytes > a.out_cap;  // uniform
        const uint32_t sdw0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[8u + 4u * sfi]),
                       sdw1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[9u + 4u * sfi]);
        const uint32_t type = sdw0 & 255u, w = (sdw0 >> 8) & 255u, bd = (sdw0 >> 16) & 255u, k = sdw0 >> 24,
                       o = sdw1 & 255u, method = (sdw1 >> 8) & 255u, cand = (sdw1 >> 16) & 255u;
        const uint32_t p = ((const uint8_t *)(dsc + 192u + 64u * sfi))[i0 >> (12u - o)];
        const uint32_t lb = dsc[64u + 64u * sfi + l];
        uint32_t sub_start = 8u * (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[0]);
        if (sfi) sub_start += (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[10]);
        const uint32_t hdrw = dsc[4u + (l & 3u)];
        const uint64_t jn_off = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[19]) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[18]);
        const uint32_t jn_slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[23]);
        const uint32_t crc_pw = a.crc_pow4[hq * NT + tid];   // first used in the CRC phase
        if (nxt < a.n_jobs) {
            stage_dma_rot(a.pcm, jn_off, (uint32_t *)(smem + (buf ? LY.buf0 : LY.buf1)), wave, NW, l);
            p4_dsc_dma(a, jn_slot, nn, (uint32_t *)(smem + (buf ? LY.dsc0 : LY.dsc1)), wave, l);
        }
        if (skip) {
            if (tid == 0) {
                atomicOr(a.err, fbytes + 16u > a.image_bytes ? 1u : 2u);
                tk = gridDim.x + atomicAdd(ctr, 1u);
            }
            __syncthreads();
            jidx = nxt; nxt = nn; slot = jn_slot; buf ^= 1u;
            continue;
        }
        const uint32_t j = 64u * qw + l;  // this lane's 16-sample chunk
        uint32_t raw[20];                 // [0..3] the group before the chunk, [4..19] the chunk
        {
            const uint4 hv = j ? *(const uint4 *)(stg + rot_off(j - 1u, 3u)) : make_uint4(0, 0, 0, 0);
            raw[0] = hv.x; raw[1] = hv.y; raw[2] = hv.z; raw[3] = hv.w;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const uint4 v = *(const uint4 *)(stg + rot_off(j, (uint32_t)g));
                raw[4 + 4 * g] = v.x; raw[5 + 4 * g] = v.y; raw[6 + 4 * g] = v.z; raw[7 + 4 * g] = v.w;
            }
        }
        STAMP(9);
        // candidate samples (stereo: 0 L, 1 R, 2 mid, 3 side; otherwise channel `cand`).  The
        // candidate and the predictor order are uniform: one dispatch each around the whole lane
        // loop, not a branch ladder per sample.
        const uint32_t kind = stereo ? cand : (cand ? 1u : 0u);
        int32_t x[20];
        auto unpack = [&](auto KD) {
            constexpr uint32_t KND = decltype(KD)::value;
#pragma unroll
            for (int i = 0; i < 20; i++) {
                const int32_t L = (int32_t)(raw[i] << 16) >> 16, R = (int32_t)raw[i] >> 16;
                x[i] = KND == 0 ? L : KND == 1 ? R : KND == 2 ? (L + R) >> 1 : L - R;
            }
        };
        if (kind == 0) unpack(ic<0>{});
        else if (kind == 1) unpack(ic<1>{});
        else if (kind == 2) unpack(ic<2>{});
        else unpack(ic<3>{});
        // lane offsets: quarter base = the analysis kernel's segment lengths before it
        const uint32_t lbs = wave_incl_scan32(lb);
        const uint32_t qbase = qw ? rdl(lbs, (int)(16u * qw - 1u)) : 0u;
        STAMP(10);
        bar_lds();  // staging dead: zero the image
        STAMP(1);
        const uint32_t Wz = (fbytes + 3u) / 4u + 2u;
        for (uint32_t i = tid; i < Wz; i += NT) img[i] = 0;
        STAMP(2);

        // ---- 2. waste shift and residuals (fixed.zig:30-81), lengths of this lane's codes
        const uint32_t bps = bd - w;
        if (type != 0 && w != 0) {
#pragma unroll
            for (int i = 0; i < 20; i++) x[i] >>= w;
        }
        const bool first = (qw == 0) && (l == 0);
        const uint32_t param_len = 4u + method;
        const bool esc = (p & 0x80u) != 0;
        const uint32_t wb = p & 0x7Fu, pr = esc ? 0u : p;
        uint32_t r[16];
        auto resid = [&](auto KO) {
            constexpr uint32_t K = decltype(KO)::value;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t u0 = (uint32_t)x[4 + i], u1 = (uint32_t)x[3 + i], u2 = (uint32_t)x[2 + i],
                               u3 = (uint32_t)x[1 + i], u4 = (uint32_t)x[i];
                if constexpr (K == 0) r[i] = u0;
                else if constexpr (K == 1) r[i] = u0 - u1;
                else if constexpr (K == 2) r[i] = (u0 + u2) - 2u * u1;
                else if constexpr (K == 3) r[i] = (u0 - u3) + 3u * (u2 - u1);
                else r[i] = (u0 + u4) - 4u * (u1 + u3) + 6u * u2;
            }
        };
        if (type != 2 || k == 0) resid(ic<0>{});
        else if (k == 1) resid(ic<1>{});
        else if (k == 2) resid(ic<2>{});
        else if (k == 3) resid(ic<3>{});
        else resid(ic<4>{});
        // per-lane code shape (a lane's 16 samples share one partition, >= 16 samples):
        // rice = q zeros, then (1 << p) | low p bits in cl = p + 1 bits; escape = the raw
        // wb-bit two's complement value, no unary part.  Warm-up samples (the subframe's first
        // k, lane 0 of quarter 0) are written by the header writer and code as nothing here.
        const uint32_t cl = esc ? wb : pr + 1u;
        const uint32_t cmask = esc ? ((1u << wb) - 1u) : ((1u << pr) - 1u);  // wb <= 31
        const uint32_t cbit = esc ? 0u : (1u << pr);
        const uint32_t qmask = esc ? 0u : ~0u;
        const uint32_t nwarm = (first && type == 2) ? k : 0u;
        auto warm_at = [&](int i) -> bool { return i < 4 && (uint32_t)i < nwarm; };
        // header bits (lane 0 of the subframe) and partition header bits (a lane opening a partition)
        uint32_t len = 0;
        if (first) {
            if (type == 0) len = 8u + bd;
            else if (type == 1) len = 8u + w;
            else len = 8u + w + k * bps + 6u + param_len + (esc ? 5u : 0u);
        } else if (type == 2 && (i0 & ((4096u >> o) - 1u)) == 0) {
            len = param_len + (esc ? 5u : 0u);
        }
        if (type == 1) {
            len += 16u * bps;
        } else if (type == 2) {
            uint32_t qs = 0;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t qz = zigzag32((int32_t)r[i]) >> pr;
                qs = add_chain(qs, warm_at(i) ? 0u : qz);
            }
            len += (qs & qmask) + (16u - nwarm) * cl;
        }
        const uint32_t lane_off = wave_incl_scan32(len) - len;
        bar_lds();  // image zeroed
        STAMP(3);
        if (tid < 4 && hdrw) atomicOr(&img[tid], hdrw);

        // ---- 3. pack: each lane ORs its codes into the image at its bit offset
        {
            uint32_t pos = sub_start + qbase + lane_off;
            const uint64_t mask = ~0ull >> (64 - (bps ? bps : 1u));
            if (first) {
                AtomicWriter bw;
                bw.init(img, pos);
                if (type == 0) {  // writeConstantSubframe: 0x00, value << waste in bd bits
                    bw.put(0, 8);
                    const SubDesc *sd = (const SubDesc *)(a.desc + (uint64_t)slot * a.desc_stride + sizeof(FrameDesc)) + sfi;
                    bw.put(((uint64_t)sd->cval << w) & (~0ull >> (64 - bd)), bd);
                } else {
                    const uint32_t tc = (type == 1) ? 1u : (8u | k);
                    bw.put((tc << 1) | (w ? 1u : 0u), 8);
                    if (w) bw.put(1, w);
                    if (type == 2) {
#pragma unroll
                        for (int i = 0; i < 4; i++)  // warm-up samples
                            if ((uint32_t)i < k) bw.put((uint64_t)(int64_t)x[4 + i] & mask, bps);
                        bw.put((method << 4) | o, 6);
                        if (esc) {
                            bw.put(0x0Fu | (method << 4), 4u + method);
                            bw.put(wb, 5);
                        } else {
                            bw.put(p, 4u + method);
                        }
                    }
                }
                pos = bw.pos;
            } else if (type == 2 && (i0 & ((4096u >> o) - 1u)) == 0) {
                const uint32_t esc_code = (0x0Fu | (method << 4)) << 5;
                const uint32_t hl = param_len + (esc ? 5u : 0u);
                put_or2(img, pos, esc ? (esc_code | wb) : p, hl);
                pos += hl;
            }
            if (type == 1) {
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    put_or2(img, pos, (uint64_t)(int64_t)(int32_t)r[i] & mask, bps);
                    pos += bps;
                }
            } else if (type == 2) {
                // pa: bit address from the LDS base, so a code's word address is (pa >> 5) * 4 and
                // its 64-bit window shift is (64 - cl) - (pa & 31): v < 2^cl, cl <= 32
                const uint32_t img_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)img;
                uint32_t pa = 8u * img_lds + pos;
                const uint32_t ncl = 64u - cl;
                auto emit = [&](auto ESC) {
                    constexpr bool E = decltype(ESC)::value != 0;
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const bool warm = warm_at(i);
                        const uint32_t zz = zigzag32((int32_t)r[i]);
                        // escape: the residual's two's complement bits
                        const uint32_t src = E ? (esc ? r[i] : zz) : zz;
                        uint32_t v = (src & cmask) | cbit;
                        uint32_t q = E ? ((zz >> pr) & qmask) : (zz >> pr);
                        uint32_t sh = ncl, adv = cl;
                        if (i < 4) {
                            v = warm ? 0u : v;
                            q = warm ? 0u : q;
                            sh = warm ? 64u : sh;
                            adv = warm ? 0u : adv;
                        }
                        pa += q;
                        const uint64_t t = (uint64_t)v << ((sh - (pa & 31u)) & 63u);
                        lds_or2((pa >> 3) & ~3u, (uint32_t)(t >> 32), (uint32_t)t);
                        pa += adv;
                    }
                };
                if (__any(esc)) emit(ic<1>{});
                else emit(ic<0>{});
            }
        }
        bar_lds();
        STAMP(4);

        // ---- 4. CRC-16 of the frame: the word stream front-padded with zero words (a no-op for
        // an init-0 CRC) to NT * 2H words; thread t folds its 2H words in one table-free chain mod
        // Q (crc_lane_q) scaled by z^(16 + 64H(NT-1-t)) mod Q, with its words' parity; the
        // workgroup XOR-reduces both and thread 0 recombines them into the CRC (crc_from_q).
        {
            const int32_t Z = (int32_t)(NT * 2u * H) - (int32_t)W4;
            const int32_t va = (int32_t)(tid * 2u * H) - Z;
            uint32_t contrib = crc_lane_q(img, va, 2u * H, crc_pw);
            contrib = wave_xor32(contrib);
            if (l == 0) misc[wave] = contrib;
        }
        bar_lds();
        if (tid == 0) {
            uint32_t qp = 0;
            for (uint32_t i = 0; i < NW; i++) qp ^= misc[i];
            uint32_t crc = crc_from_q(qp);
            for (uint32_t b = W4 * 4u; b < Lb; b++)
                crc = crc_byte_v(crc, (img[b >> 2] >> (24 - 8 * (b & 3))) & 255u);
            put_bits(img, Lb * 8u, crc, 16);
        }
        bar_lds();
        STAMP(5);

        // ---- 5. image -> out[D, D + fbytes)
        store_frame16(img, a.out, D, fbytes, tid, NT);
        // no barrier here: the image / staging area is next written by the DMA issued after the
        // next frame's top barrier, which already orders this frame's last reads before it
        STAMP(6);
        if (tid == 0) tk = gridDim.x + atomicAdd(ctr, 1u);  // frame i+3, behind this frame's stores
        jidx = nxt; nxt = nn; slot = jn_slot; buf ^= 1u;
    }  // persistent frame loop
#ifdef FG_STAMPS
    if (l0 == 0 && a.stamps)
        for (int i = 0; i < 11; i++) atomicAdd(&a.stamps[16 + i], (unsigned long long)ph_[i]);
#endif
}
