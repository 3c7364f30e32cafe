// fg_packw.hpp -- frame packing with several waves per written subframe for every full-frame
// configuration k_pack4 does not cover: 24/32-bit samples, mono and multichannel streams,
// LPC subframes (included by fg_device.hpp inside namespace fg).
//
// k_pack gives each written subframe one wave of 64-sample lanes: one dependent chain of 64
// codes per lane, and for 8 channels only 8 waves per CU (the 96 KiB staging admits one
// workgroup).  Here WPS = 64 / SPL waves share a subframe and a lane owns SPL (16 or 32)
// consecutive samples: wave w packs part hq = w % WPS of written subframe w / WPS.  Per frame
// (frame_writer.zig:269-372 restated):
//   1. the lane loads its SPL samples and the KH before them (fixed: 4, LPC: the taps) of its
//      candidate from the staged PCM (encoder.zig:329-350), applies the waste shift and the
//      predictor of the descriptor (fixed.zig:30-81; LPC: the build-defined contract, §4b);
//   2. code lengths -> a wave prefix scan on top of the part's base, which is the prefix of the
//      analysis kernel's exact 64-sample segment lengths;
//   3. branch-free code emission into the zeroed LDS frame image, CRC-16 (one chain per thread,
//      one shift multiply), 16-byte stores at the frame's final byte offset.
#pragma once

// Sample at byte `byte` of the staged frame, sign-extended.
template <int B>
__device__ __forceinline__ int32_t staged_at(const uint32_t *stg, uint32_t byte) {
    if constexpr (B == 4) {
        return (int32_t)stg[byte >> 2];
    } else if constexpr (B == 3) {
        const uint32_t wd = byte >> 2, o = byte & 3u;
        const uint32_t v = __builtin_amdgcn_alignbyte(stg[wd + 1u], stg[wd], o);
        return (int32_t)(v << 8) >> 8;
    } else if constexpr (B == 2) {
        const uint32_t v = stg[byte >> 2];
        return (int32_t)((byte & 2u) ? v : (v << 16)) >> 16;
    } else {
        const uint32_t v = stg[byte >> 2];
        return (int32_t)(v << (24u - 8u * (byte & 3u))) >> 24;
    }
}

// Byte of sample i, channel c in the k_packw staging (packw_layout): chunk i >> 6, sub-chunk
// (i & 63) / SPL of sw words + 1 pad word each.
template <int B, int SPL>
__device__ __forceinline__ uint32_t packw_byte(uint32_t i, uint32_t c, uint32_t cst, uint32_t sw, uint32_t CB) {
    return (i >> 6) * cst * 4u + ((i & 63u) / (uint32_t)SPL) * (sw + 1u) * 4u + (i & (uint32_t)(SPL - 1)) * CB + c * (uint32_t)B;
}

// LDS-DMA one frame into the k_packw staging: LDS word k = 64 xi + l of a chunk holds source
// word k - sub(k), or (pad slot) a dummy; `code` packs sub (2 bits) and the pad flag of every
// slot xi in 3 bits per lane, computed once per kernel.
// drh != 0 (channel halves): the staged chunk holds the drh dwords [half drh, half drh + drh) of
// every 2 drh-dword interchannel row (cw = the half row's dwords x 64), as k_analyze's split mode.
__device__ __forceinline__ void stage_dma_w(const uint8_t *pcm, uint64_t off, uint32_t *stg, uint32_t cw, uint32_t cst,
                                            uint32_t code, uint32_t wave, uint32_t NW, uint32_t l, uint32_t drh = 0,
                                            uint32_t half = 0) {
    const uint32_t *src = (const uint32_t *)(pcm + off);
    const float inv = drh ? 1.0f / (float)drh : 0.0f;  // x / drh exactly for x < 2^10, drh <= 4
    for (uint32_t ch = wave; ch < 64u; ch += NW) {
#pragma unroll
        for (uint32_t xi = 0; xi < 9u; xi++) {
            const uint32_t cd = (code >> (3u * xi)) & 7u;
            uint32_t so = (cd & 4u) ? 0u : 64u * xi + l - cd;
            uint32_t base = ch * cw;
            if (drh) {
                const uint32_t r = (uint32_t)((float)so * inv);
                so = r * 2u * drh + half * drh + (so - r * drh);
                base = ch * 2u * cw;
            }
            if (64u * xi < cst && 64u * xi + l < cst)
                lds_dma<4>(src + base + so, stg + ch * cst + 64u * xi);
        }
    }
}

// z^(8 m) mod P for m < 2^24, wave-parallel: lane i < 24 contributes z^(8 * 2^i) when bit i of
// m is set, the 32-lane product by a butterfly of table-assisted carry-less multiplies
__device__ __forceinline__ uint32_t crc_zpow8(uint32_t m, const uint16_t *x8, uint32_t l) {
    uint32_t f = (l < 24u && ((m >> l) & 1u)) ? (uint32_t)x8[l] : 1u;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) f = crc_mulmod_v(f, (uint32_t)__shfl_xor((int)f, d));
    return f;
}

// SPLIT: channel halves (frames of 4+ independent channels whose staging admits one workgroup
// per CU, c4): a work item is (frame, half), the workgroup stages only its half's channels and
// packs its half's subframes into its own image -- half 0 the header and subframes
// [0, n/2), half 1 the rest, its image starting at the byte that holds its first bit.  The
// frame's CRC-16 is linear in the message: CRC(frame) = CRC(img0) z^(8 (Lb - e0)) ^ CRC(img1)
// (init 0: leading zero bytes do not change a CRC), so each half folds its own image, stores
// its bytes except the one byte both halves share, and hands its CRC partial and its part of
// that byte to the frame's descriptor; the second to arrive (atomic ticket) writes the shared
// byte and the CRC.  Two 55-KiB halves per CU overlap one half's DMA / store with the other's
// compute, where one 101-KiB whole frame per CU ran those phases back to back.
template <int B, int CLS, int NC, int LPW, int SPL, bool SPLIT = false>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 8))) k_packw(EncodeArgs a) {
    using ST = typename Cls<CLS>::S;
    constexpr int KH = LPW > 4 ? LPW : 4;  // history samples (most warm-ups of any predictor)
    constexpr uint32_t WPS = 64u / SPL;     // waves per written subframe
    constexpr int NG = SPL / 16;            // 16-sample groups per lane (one Rice partition each)
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const uint32_t tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)), l0 = lane_id();
    const uint32_t sfi = wave / WPS, hq = wave % WPS;  // written subframe (of the half), part
    const uint32_t NH = NW / WPS;                      // written subframes of this workgroup
    constexpr uint32_t ssh = SPLIT ? 1u : 0u;
    const uint32_t C = NC ? (uint32_t)NC : a.channels;  // split: the half's channels
    const uint32_t drh = SPLIT ? C * (uint32_t)B / 4u : 0u;  // split: dwords of a half row
    const uint32_t CB = C * (uint32_t)B;
    const uint32_t cw = 16u * C * B, cst = packw_cst(C, B, WPS);
    const uint32_t sw = (uint32_t)SPL * CB / 4u;  // words of one lane's sub-chunk
    const bool dbuf = a.pack_dbuf != 0;
    const PackLayout LY = packw_layout(C, B, WPS, a.image_bytes, dbuf, NW / WPS);
    uint32_t dcode = 0;  // per lane, 3 bits per DMA slot (cst <= 516 words: 9 slots)
#pragma unroll
    for (uint32_t xi = 0; xi < 9u; xi++) {
        const uint32_t k = 64u * xi + l0, sub = k / (sw + 1u), o = k - sub * (sw + 1u);
        dcode |= (((o == sw || k >= cst) ? 4u : 0u) | (sub & 3u)) << (3u * xi);
    }
    uint32_t *misc = (uint32_t *)(smem + LY.misc);
    const bool stereo = a.stereo != 0;

    uint32_t *ctr = a.work_ctr + 2u;
    reset_analysis_tickets(a.work_ctr, tid);  // the analysis kernel's queues
    // split: items from per-XCD queues (work_ctr[16..23], zeroed by the analysis kernel), so the
    // two halves of a frame -- which fetch the same lines of its interleaved rows -- are taken
    // by workgroups of one XCD at about the same time and the second fetch can hit its L2
    // (the analysis's xcd_ticket placement; tools/micro/fetch_micro.hip: 2.0x -> 1.28x)
    const bool xq = SPLIT && a.xcd_queue;
    // jit (xcd_queue bit 1, single-buffered staging): each item's ticket right before its DMA,
    // as k_analyze's split mode, so a frame's halves are staged about one ticket interval apart
    const bool jit = xq && !dbuf && (a.xcd_queue & 2u);
    uint32_t *xqc = a.work_ctr + 16;
    if (tid == 0) {
        if (xq) {
            misc[22] = xcd_ticket(xqc, a.n_jobs);
            misc[21] = jit ? 0xFFFFFFFFu : xcd_ticket(xqc, a.n_jobs);
        } else {
            misc[21] = gridDim.x + atomicAdd(ctr, 1u);
        }
    }
    __syncthreads();
    const uint32_t n_items = a.n_jobs << ssh;
    uint32_t jidx = xq ? (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]) : blockIdx.x, buf = 0;
    uint32_t nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[21]);
    FrameJob job{}, jn{};
    if (jidx < n_items) job = a.jobs[jidx >> ssh];
    if (nxt < n_items) jn = a.jobs[nxt >> ssh];
    if (dbuf && jidx < n_items)
        stage_dma_w(a.pcm, job.pcm_off, (uint32_t *)(smem + LY.buf0), cw, cst, dcode, wave, NW, l0, drh, jidx & ssh);
    // The frame descriptor's fields this workgroup reads, in LDS (two slots, packw_dsc_dw): one
    // frame's copy is DMA'd during the frame before it, so the top of a frame reads them from LDS
    // instead of running dependent global round trips to the table the analysis kernel wrote (the
    // subframes' bit counts -> their prefix -> the image size -> the CRC constants: 28 % of a c4
    // pack wave's time in r5q's stamps).  Dwords: [0..7] FrameDesc, [8..15] SubDesc.bits of the
    // frame's subframes, [16..17] the frame's byte offset, then 11 per local subframe (SubDesc
    // dwords 0, 1, 3, 4, 5, 134..139: fields, lpc_prec, cval, coef); chunk HC + s: lane_bits of
    // local subframe s; chunk HC + NH + s: its Rice parameters.
    const uint32_t HC = packw_dsc_hc(NH), DSC_DW = packw_dsc_dw(NH);
    uint32_t *dscb = (uint32_t *)(smem + LY.dsc);
    auto dsc_dma = [&](uint32_t fslot, uint32_t hf, uint32_t ds) {
        const uint8_t *fdp = a.desc + (uint64_t)fslot * a.desc_stride;
        uint32_t *dst = dscb + ds * DSC_DW;
        const uint32_t nsubx = NH << ssh;
        const uint32_t ll = opaque(l0);
        for (uint32_t kc = wave; kc < HC + 2u * NH; kc += NW) {
            const uint8_t *src = fdp;
            if (kc < HC) {
                const uint32_t q = 64u * kc + ll;
                if (q < 8u) src = fdp + 4u * q;
                else if (q < 16u) src = (q - 8u < nsubx) ? fdp + 32u + (q - 8u) * (uint32_t)sizeof(SubDesc) + 8u : fdp;
                else if (q < 18u) src = (const uint8_t *)(a.offsets + fslot) + 4u * (q - 16u);
                else if (q < 18u + 11u * NH) {
                    const uint32_t sl = (q - 18u) / 11u, f = (q - 18u) - 11u * sl;
                    const uint32_t dw = f < 2u ? f : (f == 2u ? 3u : (f < 5u ? f + 1u : 129u + f));
                    src = fdp + 32u + (hf * NH + sl) * (uint32_t)sizeof(SubDesc) + 4u * dw;
                }
            } else if (kc < HC + NH) {
                src = fdp + 32u + (hf * NH + (kc - HC)) * (uint32_t)sizeof(SubDesc) + 24u + 4u * ll;
            } else {
                src = fdp + 32u + (hf * NH + (kc - HC - NH)) * (uint32_t)sizeof(SubDesc) + 280u + 4u * ll;
            }
            lds_dma<4>(src, dst + 64u * kc);
        }
    };
    uint32_t dslot = 0;      // the LDS slot holding (or receiving) the current frame's descriptor
    bool dsc_ready = false;  // it was DMA'd during the previous frame
#ifdef FG_STAMPS
    uint64_t ph_[16] = {};
    uint64_t tprev_ = __builtin_amdgcn_s_memtime();
#endif
    while (jidx < n_items) {
        const uint32_t l = opaque(l0);
        const uint32_t half = jidx & ssh;
        if (tid == 0 && !jit) misc[20] = xq ? xcd_ticket(xqc, a.n_jobs) : gridDim.x + atomicAdd(ctr, 1u);
        uint32_t *stg = (uint32_t *)(smem + (buf ? LY.buf1 : LY.buf0));
        uint32_t *img = stg;  // the image reuses the staging buffer once the samples are in VGPRs
        // single buffer: the frame's DMA first, so the descriptor's dependent loads below run
        // under it instead of ahead of it (the previous frame's last barrier freed the buffer)
        if (!dbuf) stage_dma_w(a.pcm, job.pcm_off, stg, cw, cst, dcode, wave, NW, l, drh, half);
        if (!dsc_ready) dsc_dma(job.slot, half, dslot);  // (first frame, or jit: no look-ahead)
        const uint32_t *dsc = dscb + dslot * DSC_DW;

        // ---- 1. PCM (double-buffered: DMA'd during the previous frame) -> samples
        STAMP(7);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(8);
        __syncthreads();
        STAMP(0);
        const uint32_t sidx = half * NH + sfi;  // this wave's subframe in the frame
        const uint32_t *sdh = dsc + 18u + 11u * sfi;  // its fields (see dsc_dma)
        const uint32_t hdr_bytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[0]);
        const uint32_t total_bits = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[1]);
        const uint32_t n_out_f = (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[3]);
        const uint32_t Lt = (total_bits + 7u) >> 3;  // the frame's bytes before the CRC
        const uint64_t D = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[17]) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)dsc[16]);
        // split: half 0 ends at bit b0 (header + its subframes); half 1's image starts at byte
        // b0 / 8 and ends with the frame.  Lb = this image's bytes (whole frame: Lt)
        const uint32_t nsub = NH << ssh;
        const uint32_t sbits = l < nsub ? dsc[8u + l] : 0u;
        uint32_t b0 = 0, base = 0, Lb = Lt;
        if (SPLIT) {
            b0 = 8u * hdr_bytes;
            for (uint32_t t = 0; t < NH; t++) b0 += rdl(sbits, (int)t);
            base = half ? (b0 >> 3) : 0u;
            Lb = half ? Lt - base : (b0 + 7u) >> 3;
        }
        const uint32_t fbytes = SPLIT ? Lb : Lt + 2u;  // image bytes this workgroup fills
        const uint32_t W4 = Lb >> 2;
        const uint32_t H = max((W4 + 2u * NT - 1u) / (2u * NT), 1u);  // words per thread / 2
        const uint32_t hcq = min(H, a.crc_hmax4) - 1u;
        const uint32_t crc_pw = a.crc_pow4[hcq * NT + tid];  // first used in the CRC phase
        const bool skip = fbytes + 16u > a.image_bytes || D + Lt + 2u > a.out_cap;  // uniform
        const uint32_t sw0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)sdh[0]),
                       sw1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)sdh[1]);
        const uint32_t type = sw0 & 255u, w = (sw0 >> 8) & 255u, bd = (sw0 >> 16) & 255u, k = sw0 >> 24,
                       o = sw1 & 255u, method = (sw1 >> 8) & 255u, cand = (sw1 >> 16) & 255u;
        const int32_t lpc_shift = (int32_t)(int8_t)(sw1 >> 24);
        const uint32_t lpc_prec = (uint32_t)__builtin_amdgcn_readfirstlane((int)sdh[2]);
        const int64_t cval = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)sdh[4]) << 32) |
                                       (uint32_t)__builtin_amdgcn_readfirstlane((int)sdh[3]));
        const uint16_t *coef = (const uint16_t *)(sdh + 5);
        const uint32_t i0 = hq * 64u * SPL + SPL * l0;  // first sample of this lane
        uint32_t pq[NG];
        const uint8_t *prm = (const uint8_t *)(dsc + 64u * (HC + NH + sfi));
#pragma unroll
        for (int g = 0; g < NG; g++) pq[g] = prm[(i0 + 16u * g) >> (12u - o)];
        const uint32_t lb = dsc[64u * (HC + sfi) + l0];
        uint32_t sub_start = 8u * hdr_bytes;
        for (uint32_t t = 0; t < sidx; t++) sub_start += rdl(sbits, (int)t);
        sub_start -= 8u * base;
        const uint32_t nn = jit ? 0xFFFFFFFFu : (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[20]);
        // the job record of the frame after next before the DMAs: waiting for it then never
        // waits for them (vmcnt completes in order)
        FrameJob jnn{};
        if (nn < n_items) jnn = a.jobs[nn >> ssh];
        // the next frame's descriptor into the other slot (landed by the next frame's top wait;
        // this frame reads its own slot through `dsc`)
        dsc_ready = !jit && nxt < n_items;
        if (dsc_ready) {
            dsc_dma(jn.slot, nxt & ssh, dslot ^ 1u);
            dslot ^= 1u;
        }
        if (dbuf && nxt < n_items)
            stage_dma_w(a.pcm, jn.pcm_off, (uint32_t *)(smem + (buf ? LY.buf0 : LY.buf1)), cw, cst, dcode, wave, NW, l, drh,
                        nxt & ssh);
        if (skip) {
            if (tid == 0) atomicOr(a.err, fbytes + 16u > a.image_bytes ? 1u : 2u);
            __syncthreads();
            if (jit) {
                if (tid == 0) misc[22] = xcd_ticket(xqc, a.n_jobs);
                __syncthreads();
                jidx = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]);
                if (jidx < n_items) job = a.jobs[jidx >> ssh];
                continue;
            }
            jidx = nxt; job = jn; nxt = nn; jn = jnn; buf ^= dbuf ? 1u : 0u;
            continue;
        }
        // x[KH + j] = sample i0 + j of the candidate, x[KH - 1 - t] = sample i0 - 1 - t (0 before
        // the subframe: only lane 0 of part 0, whose first k samples are warm-ups)
        ST x[KH + SPL];
        {
            const uint32_t ia = SPL * l + hq * 64u * SPL;  // == i0, from the opaque lane id
            const uint32_t kind = stereo ? cand : 0u;        // 0 plain channel, 1 R, 2 mid, 3 side
            const uint32_t chan = stereo ? (cand == 1 ? 1u : 0u) : cand - half * C;  // split: of the half
            // the lane's own samples sit in one sub-chunk: a per-lane base plus immediates
            const uint32_t lbase = packw_byte<B, SPL>(ia, 0u, cst, sw, CB);
            auto fill = [&](auto KD) {
                constexpr uint32_t KND = decltype(KD)::value;
                auto get = [&](uint32_t byte) -> int64_t {
                    if constexpr (KND <= 1) {
                        return staged_at<B>(stg, byte + chan * (uint32_t)B);
                    } else {
                        const int64_t L = staged_at<B>(stg, byte), R = staged_at<B>(stg, byte + (uint32_t)B);
                        return KND == 2 ? (L + R) >> 1 : L - R;
                    }
                };
#pragma unroll
                for (int j = 0; j < KH; j++) {  // history: the previous sub-chunk / chunk
                    const bool before = ia + (uint32_t)j < (uint32_t)KH;  // sample index < 0
                    const uint32_t i = before ? 0u : ia + (uint32_t)j - (uint32_t)KH;
                    const int64_t v = get(packw_byte<B, SPL>(i, 0u, cst, sw, CB));
                    x[j] = before ? (ST)0 : (ST)v;
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < SPL; j++) {
                    x[KH + j] = (ST)get(lbase + (uint32_t)j * CB);
                    if ((j & 15) == 15) __builtin_amdgcn_sched_barrier(0);
                }
            };
            if (kind <= 1) fill(ic<0>{});
            else if (kind == 2) fill(ic<2>{});
            else fill(ic<3>{});
        }
        STAMP(9);
        // lane offsets: the part's base = the analysis kernel's segment lengths before it
        const uint32_t lbs = wave_incl_scan32(lb);
        const uint32_t qbase = hq ? rdl(lbs, (int)(SPL * hq - 1u)) : 0u;
        STAMP(10);
        bar_lds();  // staging dead: zero the image
        STAMP(1);
        const uint32_t Wz = (fbytes + 3u) / 4u + 2u;
        for (uint32_t i = tid; i < Wz; i += NT) img[i] = 0;
        STAMP(2);

        // ---- 2. waste shift and residuals, lengths of this lane's codes (k_packw)
        const uint32_t bps = bd - w;
        if (type != 0 && w != 0) {
#pragma unroll
            for (int j = 0; j < KH + SPL; j++) x[j] >>= w;
        }
        const bool first = (hq == 0) && (l == 0);
        const uint32_t param_len = 4u + method;
        uint32_t r[SPL];
        if (type == 2) {
            auto fixed = [&](auto KO) {
                constexpr int K = (int)decltype(KO)::value;
#pragma unroll
                for (int j = 0; j < SPL; j++) {
                    ST q1 = x[KH + j - 1], q2 = x[KH + j - 2], q3 = x[KH + j - 3], q4 = x[KH + j - 4];
                    r[j] = (uint32_t)(int32_t)fixed_residual<K, ST>(x[KH + j], q1, q2, q3, q4);
                }
            };
            if (k == 0) fixed(ic<0>{});
            else if (k == 1) fixed(ic<1>{});
            else if (k == 2) fixed(ic<2>{});
            else if (k == 3) fixed(ic<3>{});
            else fixed(ic<4>{});
        } else if (LPW > 0 && type == 3) {
            if constexpr (LPW > 0) {
                int32_t c[LPW];
#pragma unroll
                for (int t = 0; t < LPW; t++) c[t] = __builtin_amdgcn_readfirstlane((int32_t)(int16_t)coef[t < kLpcMax ? t : 0]);
                const uint32_t shift = (uint32_t)lpc_shift;
                // LPC runs on i32 samples only (contract step 0), so every product is a
                // v_mad_i64_i32 even for 32-bit input; taps bucketed by order (c[t] = 0 past it)
                auto lpc = [&](auto WT) {
                    constexpr int W = decltype(WT)::value;
#pragma unroll
                    for (int j = 0; j < SPL; j++) {
                        int64_t acc = 0;
#pragma unroll
                        for (int t = 0; t < W; t++) acc += (int64_t)c[t] * (int64_t)(int32_t)x[KH + j - 1 - t];
                        r[j] = (uint32_t)((int32_t)x[KH + j] - (int32_t)(acc >> shift));
                    }
                };
                if (k <= 4u) lpc(ic<4>{});
                else if (LPW <= 8 || k <= 8u) lpc(ic<(LPW < 8 ? LPW : 8)>{});
                else lpc(ic<LPW>{});
            }
        } else {
#pragma unroll
            for (int j = 0; j < SPL; j++) r[j] = (uint32_t)(int32_t)x[KH + j];
        }
        // per 16-sample group the code shape is lane-constant (see k_pack4): rice = q zeros then
        // (1 << p) | low p bits in p + 1 bits, escape = the raw wb-bit value; warm-ups (the
        // subframe's first k samples, lane 0 of part 0) are written by the header writer
        const uint32_t nwarm = (first && type >= 2) ? k : 0u;
        auto warm_at = [&](int j) -> bool { return j < KH && (uint32_t)j < nwarm; };
        uint32_t len = 0;
        if (first) {
            const uint32_t p0 = pq[0];
            if (type == 0) len = 8u + bd;
            else if (type == 1) len = 8u + w;
            else len = 8u + w + k * bps + 6u + param_len + ((p0 & 0x80u) ? 5u : 0u) +
                       (type == 3 ? 4u + 5u + k * lpc_prec : 0u);
        }
        if (type == 1) {
            len += SPL * bps;
        } else if (type >= 2) {
            const uint32_t psz = 4096u >> o;
#pragma unroll
            for (int g = 0; g < NG; g++) {
                const uint32_t p = pq[g], ig = i0 + 16u * g;
                const bool esc = (p & 0x80u) != 0;
                const uint32_t pr = esc ? 0u : p, cl = esc ? (p & 0x7Fu) : pr + 1u;
                if (ig != 0 && (ig & (psz - 1u)) == 0) len += param_len + (esc ? 5u : 0u);
                uint32_t qs = 0, nc = 16;
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = 16 * g + jj;
                    const uint32_t qz = zigzag32((int32_t)r[j]) >> pr;
                    const bool wm = warm_at(j);
                    qs = add_chain(qs, wm ? 0u : qz);
                    if (j < KH) nc -= wm ? 1u : 0u;
                }
                len += (esc ? 0u : qs) + nc * cl;
            }
        }
        const uint32_t lane_off = wave_incl_scan32(len) - len;
        bar_lds();  // image zeroed
        STAMP(3);
        if (tid < 4 && half == 0) {
            const uint32_t hv = dsc[4u + tid];
            if (hv) atomicOr(&img[tid], hv);
        }

        // ---- 3. pack: each lane ORs its codes into the image at its bit offset
        {
            uint32_t pos = sub_start + qbase + lane_off;
            const uint64_t mask = ~0ull >> (64 - (bps ? bps : 1u));
            if (first) {
                AtomicWriter bw;
                bw.init(img, pos);
                if (type == 0) {  // writeConstantSubframe: 0x00, value << waste in bd bits
                    bw.put(0, 8);
                    bw.put(((uint64_t)cval << w) & (~0ull >> (64 - bd)), bd);
                } else {
                    // type code: VERBATIM 1, FIXED 8|k, LPC 0x20|(k-1) (build-defined)
                    const uint32_t tc = (type == 1) ? 1u : (type == 2 ? (8u | k) : (0x20u | (k - 1u)));
                    bw.put((tc << 1) | (w ? 1u : 0u), 8);
                    if (w) bw.put(1, w);
                    if (type >= 2) {
#pragma unroll
                        for (int j = 0; j < KH; j++)  // warm-up samples
                            if ((uint32_t)j < k) bw.put((uint64_t)(int64_t)x[KH + j] & mask, bps);
                        if (type == 3) {
                            const uint32_t prec = lpc_prec;
                            bw.put(prec - 1u, 4);
                            bw.put((uint32_t)lpc_shift & 31u, 5);
                            for (uint32_t t = 0; t < k; t++)
                                bw.put((uint64_t)(int64_t)(int16_t)coef[t] & (~0ull >> (64 - prec)), prec);
                        }
                        bw.put((method << 4) | o, 6);
                        const uint32_t p0 = pq[0];
                        if (p0 & 0x80u) {
                            bw.put(0x0Fu | (method << 4), 4u + method);
                            bw.put(p0 & 0x7Fu, 5);
                        } else {
                            bw.put(p0, 4u + method);
                        }
                    }
                }
                pos = bw.pos;
            }
            if (type == 1) {  // verbatim: the (waste-shifted) samples, up to 33 bits (32-bit side)
#pragma unroll
                for (int j = 0; j < SPL; j++) {
                    put_or2(img, pos, (uint64_t)(int64_t)x[KH + j] & mask, bps);
                    pos += bps;
                }
            } else if (type >= 2) {
                const uint32_t psz = 4096u >> o;
                const uint32_t esc_code = (0x0Fu | (method << 4)) << 5;
                const uint32_t img_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)img;
#pragma unroll
                for (int g = 0; g < NG; g++) {
                    __builtin_amdgcn_sched_barrier(0);  // the group's constants live one group at a time
                    const uint32_t p = pq[g], ig = i0 + 16u * g;
                    const bool esc = (p & 0x80u) != 0;
                    const uint32_t wb = p & 0x7Fu, pr = esc ? 0u : p;
                    if (ig != 0 && (ig & (psz - 1u)) == 0) {  // partition header
                        const uint32_t hl = param_len + (esc ? 5u : 0u);
                        put_or2(img, pos, esc ? (esc_code | wb) : p, hl);
                        pos += hl;
                    }
                    const uint32_t cl = esc ? wb : pr + 1u;
                    const uint32_t cmask = esc ? ((1u << wb) - 1u) : ((1u << pr) - 1u);  // wb <= 31
                    const uint32_t cbit = esc ? 0u : (1u << pr);
                    const uint32_t ncl = 64u - cl;
                    uint32_t pa = 8u * img_lds + pos;
#pragma unroll
                    for (int jj = 0; jj < 16; jj++) {
                        const int j = 16 * g + jj;
                        const bool warm = warm_at(j);
                        const uint32_t zz = zigzag32((int32_t)r[j]);
                        uint32_t v = ((esc ? r[j] : zz) & cmask) | cbit;
                        uint32_t qz = esc ? 0u : (zz >> pr);
                        uint32_t sh = ncl, adv = cl;
                        if (j < KH) {
                            v = warm ? 0u : v;
                            qz = warm ? 0u : qz;
                            sh = warm ? 64u : sh;
                            adv = warm ? 0u : adv;
                        }
                        pa += qz;
                        const uint64_t t = (uint64_t)v << ((sh - (pa & 31u)) & 63u);
                        lds_or2((pa >> 3) & ~3u, (uint32_t)(t >> 32), (uint32_t)t);
                        pa += adv;
                    }
                    pos = pa - 8u * img_lds;
                }
            }
        }
        bar_lds();
        STAMP(4);

        // ---- 4. CRC-16 of the frame (one table-free chain of 2H words per thread, see k_pack4)
        {
            const int32_t Z = (int32_t)(NT * 2u * H) - (int32_t)W4;
            const int32_t va = (int32_t)(tid * 2u * H) - Z;
            uint32_t contrib = crc_lane_q(img, va, 2u * H, crc_pw);
            contrib = wave_xor32(contrib);
            if (l == 0) misc[wave] = contrib;
        }
        bar_lds();
        if (!SPLIT) {
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
        } else if (wave == 0) {
            // ---- 4b. this half's CRC partial (half 0: shifted past the bytes after its image)
            uint32_t qp = 0;
            for (uint32_t i = 0; i < NW; i++) qp ^= misc[i];
            uint32_t crc = crc_from_q(qp);
            if (l == 0)
                for (uint32_t b = W4 * 4u; b < Lb; b++)
                    crc = crc_byte_v(crc, (img[b >> 2] >> (24 - 8 * (b & 3))) & 255u);
            crc = (uint32_t)__shfl((int)crc, 0);
            if (half == 0) crc = crc_mulmod_v(crc, crc_zpow8(Lt - Lb, a.crc_x8, l));
            const bool shared = (b0 & 7u) != 0;  // one byte holds bits of both halves
            const uint32_t sb = shared ? (half ? img[0] >> 24 : (img[(Lb - 1u) >> 2] >> (24 - 8 * ((Lb - 1u) & 3))) & 255u)
                                       : 0u;
            // hand-off in ONE 64-bit word per frame, half h in bits [32 h, 32 h + 32): present bit 31,
            // shared-byte bits 16..23, CRC partial 0..15.  A single device-scope atomicOr publishes a
            // half and returns the other's: no fence (a release fence writes back the XCD's L2,
            // which the pack's output stores keep full -- measured 2.2x slower)
            unsigned long long *side =
                (unsigned long long *)(a.desc + (uint64_t)job.slot * a.desc_stride + desc_side_off(n_out_f));
            if (l == 0) {
                const unsigned long long mine = (unsigned long long)(0x80000000u | (sb << 16) | (crc & 0xFFFFu)) << (32u * half);
                const unsigned long long old = atomicOr(side, mine);
                const uint32_t other = (uint32_t)(old >> (32u * (half ^ 1u)));
                if (other & 0x80000000u) {  // the other half is already in: write the shared byte and the CRC
                    const uint32_t c16 = (crc ^ other) & 0xFFFFu;
                    if (shared) a.out[D + (b0 >> 3)] = (uint8_t)(sb | (other >> 16));
                    a.out[D + Lt] = (uint8_t)(c16 >> 8);
                    a.out[D + Lt + 1u] = (uint8_t)c16;
                }
            }
        }
        if (SPLIT) {
            // ---- 5b. this half's bytes of out[D, D + Lt), the shared byte left to the hand-off
            const bool shared = (b0 & 7u) != 0;
            if (half == 0) store_frame16(img, a.out, D, shared ? Lb - 1u : Lb, tid, NT);
            else store_frame16(img, a.out, D + base, Lb, tid, NT, shared ? 1u : 0u);
            STAMP(5);
        }
        // single buffer: the next frame's staging overwrites the image
        if (!dbuf) __syncthreads();
        STAMP(6);
        if (jit) {
            if (tid == 0) misc[22] = xcd_ticket(xqc, a.n_jobs);
            __syncthreads();
            jidx = (uint32_t)__builtin_amdgcn_readfirstlane((int)misc[22]);
            if (jidx < n_items) job = a.jobs[jidx >> ssh];
            continue;
        }
        jidx = nxt; job = jn; nxt = nn; jn = jnn; buf ^= dbuf ? 1u : 0u;
    }  // persistent frame loop (k_packw)
#ifdef FG_STAMPS
    if (l0 == 0 && a.stamps)
        for (int i = 0; i < 11; i++) atomicAdd(&a.stamps[16 + i], (unsigned long long)ph_[i]);
#endif
}
