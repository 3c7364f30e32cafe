// fg_ana1.hpp -- full-frame analysis of 16-bit stereo (BASELINE config 2, the headline) with ONE
// wave per frame.  Included by fg_device.hpp (uses its wave helpers, rice_choose and
// write_frame_header).
//
// k_analyze gives each candidate subframe (L, R, M, S) its own wave of a 256-thread workgroup, so
// a frame costs three workgroup barriers (staged PCM, the estimates for the stereo decision, the
// descriptor), and the two waves whose candidates are not written idle through the exact-length
// pass of the two that are.  Here one wave owns the whole frame and runs the four candidates one
// after the other: no barrier, no idle wave, no LDS staging.
//   * The frame is read straight into VGPRs: lane l holds samples [64l, 64l + 64) as 64 packed
//     (L, R) dwords (16 global_load_dwordx4 per lane; every 128-B line is used whole by 8
//     consecutive loads of the wave).  They are issued as soon as the previous frame's last pass
//     is done, so the loads run under that frame's descriptor stores and the ticket round trip.
//   * One pass per candidate (encoder.zig:329-350 samples, fixed.zig:85-167 bestOrder) computes
//     for every order q = 0..4 and every 16-sample group (the finest Rice partitions) the sum of
//     |e_q| (rice.zig:288-340) and the max / min of e_q -- the escape widths of the chosen order
//     without a second residual pass (the largest zigzag of a group is that of its max or its min).
//     The sums are taken on the unshifted samples: every sample of a subframe is a multiple of
//     2^w (w = its wasted bits, encoder.zig:556-570), so the differences, sums and extremes of the
//     shifted samples are exactly these shifted right by w, and bestOrder's argmin is the same.
//     The OR for w comes from the same pass (L and R: one OR of the packed words).
//   * CONSTANT (encoder.zig:495-500): all samples equal <=> the order-1 sum is 0.
//   * The Rice search is k_analyze's (closed-form parameter per partition, all 9 orders).
//   * The stereo choice (encoder.zig:441-452) and the frame header are uniform per wave; the exact
//     bits of the two written subframes (frame_writer.zig:299-372) are a second pass over them.
// The descriptor, frame size and decision records are byte-for-byte those of k_analyze.
// Frames come from per-XCD queues (8 counters: one device-scope atomic per frame would cap the
// queue near 88 dequeues/us, MI355X_MICROARCH.md "dequeue").
#pragma once
// (included inside namespace fg)

// per-XCD frame queue (items = frames; xcd_ticket's channel-half variant hands out 2 per frame)
__device__ __forceinline__ uint32_t xcd_ticket_frames(uint32_t *q, uint32_t n_frames) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 7u;
    for (uint32_t i = 0; i < 8u; i++) {
        const uint32_t y = (x + i) & 7u;
        const uint32_t f0 = (uint32_t)(((uint64_t)n_frames * y) >> 3);
        const uint32_t f1 = (uint32_t)(((uint64_t)n_frames * (y + 1u)) >> 3);
        if (f1 == f0) continue;
        const uint32_t t = atomicAdd(&q[y], 1u);
        if (t < f1 - f0) return f0 + t;
    }
    return 0xFFFFFFFFu;
}

// sample j of the lane's packed (L low, R high) words
__device__ __forceinline__ uint32_t raw_at(const uint32_t (&rq)[64], int j) { return rq[j]; }

// candidate sample from a packed word: 0 L, 1 R, 2 mid = (L + R) >> 1, 3 side = L - R
template <int CAND>
__device__ __forceinline__ int32_t cand_x(uint32_t w) {
    const int32_t L = (int32_t)(w << 16) >> 16, R = (int32_t)w >> 16;
    if constexpr (CAND == 0) return L;
    else if constexpr (CAND == 1) return R;
    else if constexpr (CAND == 2) return (L + R) >> 1;
    else return L - R;
}

// The candidate sample of a packed word; the compiler forms SDWA operations (sign-extended 16-bit
// halves as operands): L and R one v_add_u32_sdwa with the bias folded in, side two ops, mid two
// (the sum kept opaque: otherwise (L + R) >> 1 is narrowed to a five-op 16-bit average).  Inline
// asm is avoided here: the hazard recognizer pads every asm statement with s_nop.  Returns the
// sample; *b0 = sample + 0x7FFFFFFF.
template <int CAND>
__device__ __forceinline__ int32_t cand_sdwa(uint32_t w, uint32_t kb, uint32_t *b0) {
    const int32_t L = (int32_t)(w << 16) >> 16, R = (int32_t)w >> 16;
    int32_t x;
    if constexpr (CAND == 0) x = L;
    else if constexpr (CAND == 1) x = R;
    else if constexpr (CAND == 2) {
        int32_t t = L + R;
        asm volatile("" : "+v"(t));
        x = t >> 1;
    } else x = L - R;
    *b0 = (uint32_t)x + kb;
    return x;
}

// a * b + c on 24-bit signed operands: v_mad_i32_i24 (full rate; v_mul_lo_u32 is quarter rate)
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) { return __mul24(a, b) + c; }

__device__ __forceinline__ uint32_t max3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Per-order, per-group sums of |e_q| (S) and zigzag widths: the max / min of the biased
// e_q + 0x7FFFFFFF of a 16-sample group are reduced at the group's end to the bit length of its
// largest zigzag, five bits per order in Wp[g] (bits 5q .. 5q + 4; <= 23).  Lane 0's e_q[j] for
// j < q are warm-up samples and do not count (fixed.zig:102-127).
struct Pass1 {
    uint32_t S[5][4];
    uint32_t Wp[4];
    uint32_t ov;  // OR of the candidate's samples (mid / side; L, R use the packed words' OR)
};

// the packed words as values the optimiser cannot see through: without it the extractions common
// to the candidates (L and R of all 64 words) are computed once and held live across the
// candidates' passes (128 VGPRs, spilled)
// (single dwords, not uint4 tuples: an asm that rewrites a tuple's components makes the compiler
// rebuild the tuple, a second copy of all 64)
__device__ __forceinline__ void opaque_raw(uint32_t (&rq)[64]) {
#pragma unroll
    for (int t = 0; t < 64; t++) asm volatile("" : "+v"(rq[t]));
}

template <int CAND>
__device__ __forceinline__ void pass1(const uint32_t (&rq)[64], uint32_t l, Pass1 &P) {
    const uint32_t KB = 0x7FFFFFFFu;
    // the previous lane's last four samples (lane 0: zeros, its warm-up terms are masked)
    const uint32_t u1 = (uint32_t)shr1(cand_x<CAND>(raw_at(rq, 63))), u2 = (uint32_t)shr1(cand_x<CAND>(raw_at(rq, 62)));
    const uint32_t u3 = (uint32_t)shr1(cand_x<CAND>(raw_at(rq, 61))), u4 = (uint32_t)shr1(cand_x<CAND>(raw_at(rq, 60)));
    uint32_t pb0 = u1 + KB;
    uint32_t pb1 = (u1 - u2) + KB;
    uint32_t pb2 = (u1 - 2u * u2 + u3) + KB;
    uint32_t pb3 = (u1 - 3u * u2 + 3u * u3 - u4) + KB;
    uint32_t ov = 0;
    const bool z = (l == 0);
    const uint32_t kbv = KB;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint32_t S0 = 0, S1 = 0, S2 = 0, S3 = 0, S4 = 0;
        uint32_t mx[5] = {0u, 0u, 0u, 0u, 0u}, bp[5] = {0u, 0u, 0u, 0u, 0u};
        uint32_t mn[5] = {~0u, ~0u, ~0u, ~0u, ~0u};
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
            const int j = 16 * g + jj;
            uint32_t b0;
            const int32_t x = cand_sdwa<CAND>(raw_at(rq, j), kbv, &b0);
            if constexpr (CAND >= 2) ov |= (uint32_t)x;
            const uint32_t n0 = sad_u32(b0, KB, S0);
            const uint32_t n1 = sad_u32(b0, pb0, S1);
            const uint32_t b1 = (pb0 ^ KB) + b0;
            const uint32_t n2 = sad_u32(b1, pb1, S2);
            const uint32_t b2 = (pb1 ^ KB) + b1;
            const uint32_t n3 = sad_u32(b2, pb2, S3);
            const uint32_t b3 = (pb2 ^ KB) + b2;
            const uint32_t n4 = sad_u32(b3, pb3, S4);
            const uint32_t b4 = (pb3 ^ KB) + b3;
            const uint32_t bq[5] = {b0, b1, b2, b3, b4};
            if (j < 4) {  // lane 0: e_q[j] for j < q does not count
                S0 = n0;
                S1 = !(z && j < 1) ? n1 : S1;
                S2 = !(z && j < 2) ? n2 : S2;
                S3 = !(z && j < 3) ? n3 : S3;
                S4 = !z ? n4 : S4;
#pragma unroll
                for (int q = 0; q < 5; q++) {
                    const bool warm = z && j < q;
                    mx[q] = max(mx[q], warm ? 0u : bq[q]);
                    mn[q] = min(mn[q], warm ? ~0u : bq[q]);
                }
            } else if (jj & 1) {
                // the extremes of a pair of samples in one v_max3 / v_min3 each (inline asm: kept
                // as serial chains, not trees that hold many samples' differences live)
                S0 = n0; S1 = n1; S2 = n2; S3 = n3; S4 = n4;
#pragma unroll
                for (int q = 0; q < 5; q++) {
                    mx[q] = max3_u32(mx[q], bp[q], bq[q]);
                    mn[q] = min3_u32(mn[q], bp[q], bq[q]);
                }
            } else {
                S0 = n0; S1 = n1; S2 = n2; S3 = n3; S4 = n4;
#pragma unroll
                for (int q = 0; q < 5; q++) bp[q] = bq[q];
            }
            pb0 = b0; pb1 = b1; pb2 = b2; pb3 = b3;
            if (jj & 1) __builtin_amdgcn_sched_barrier(0);
        }
        P.S[0][g] = S0; P.S[1][g] = S1; P.S[2][g] = S2; P.S[3][g] = S3; P.S[4][g] = S4;
        uint32_t wp = 0;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const uint32_t za = zigzag32((int32_t)(mx[q] - KB)), zb = zigzag32((int32_t)(mn[q] - KB));
            wp |= bitlen32(max(za, zb)) << (5 * q);
        }
        // pinned here: sunk to its only use (the non-CONSTANT branch) the group's ten extremes
        // would stay live through the rest of the pass
        asm volatile("" : "+v"(wp));
        // (the same for the OR: deferred to its use it holds the group's samples live)
        if constexpr (CAND >= 2) asm volatile("" : "+v"(ov));
        P.Wp[g] = wp;
        __builtin_amdgcn_sched_barrier(0);  // one group's temporaries live at a time
    }
    P.ov = ov;
}

// V: register budget -- 1: 168 VGPRs, 3 waves per SIMD, no spills; 2: 128 VGPRs, 4 waves per SIMD
// (a few long-lived values spilled).  Instantiated in the 16-bit fixed-prediction unit only.
template <int V>
__global__ void __launch_bounds__(64, V == 2 ? 4 : 3) k_ana1(EncodeArgs a) {
    if (a.enc_prio) __builtin_amdgcn_s_setprio(1);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *par = smem + Ana1Layout::par;
    uint32_t *rec = (uint32_t *)(smem + Ana1Layout::rec);  // [cand][8]: type, waste, order, porder, method, est lo, hi, cval
    uint32_t *hw = (uint32_t *)(smem + Ana1Layout::hdr);
    const uint32_t l0 = lane_id();
    const uint32_t n_jobs = a.n_jobs;
    uint32_t *q8 = a.work_ctr + 8;
    if (blockIdx.x == 0 && l0 == 0) a.work_ctr[2] = a.work_ctr[3] = 0u;  // the pack kernel's queues

    auto ticket = [&]() -> uint32_t {
        uint32_t t = 0;
        if (l0 == 0) t = xcd_ticket_frames(q8, n_jobs);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
    };
    auto load_raw = [&](uint32_t (&rq)[64], uint64_t off, uint32_t l) {
        const uint4 *src = (const uint4 *)(a.pcm + off) + 16u * l;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const uint4 v = src[t];
            rq[4 * t] = v.x; rq[4 * t + 1] = v.y; rq[4 * t + 2] = v.z; rq[4 * t + 3] = v.w;
        }
    };

    uint32_t jidx = ticket();
    FrameJob job{};
    uint32_t rq[64];
    if (jidx < n_jobs) {
        job = a.jobs[jidx];
        load_raw(rq, job.pcm_off, l0);
    }
    uint32_t nxt = ticket();
    FrameJob jn{};
    if (nxt < n_jobs) jn = a.jobs[nxt];
    uint32_t nn_t = 0;

    while (jidx < n_jobs) {
        const uint32_t l = opaque(l0);
        // the packed words' OR: the wasted bits of L (low halves) and R (high halves)
        uint32_t orw = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) orw |= raw_at(rq, j);
        orw = wave_or32(orw);

        // ---- the four candidates (encoder.zig:352-439): decision + Rice parameters each, in
        // sequence (one specialised pass per candidate; the raw words are re-opaqued before each)
        auto candidate = [&](auto CT) {
            constexpr uint32_t c = decltype(CT)::value;
            __builtin_amdgcn_sched_barrier(0);
            opaque_raw(rq);
            Pass1 P;
            pass1<c>(rq, l, P);
            const uint32_t bd = a.bits + (c == 3u ? 1u : 0u);
            uint32_t o32 = c == 0 ? (orw & 0xFFFFu) : c == 1 ? (orw >> 16) : wave_or32(P.ov);
            const uint32_t w = (o32 == 0) ? bd : (uint32_t)__builtin_ctz(o32);
            const uint32_t bps = bd - w;
            uint64_t T[5];
#pragma unroll
            for (int q = 0; q < 5; q++) {
                const uint32_t r = row_sum32(P.S[q][0] + P.S[q][1] + P.S[q][2] + P.S[q][3]);
                T[q] = (uint64_t)rdl(r, 0) + rdl(r, 16) + rdl(r, 32) + rdl(r, 48);
            }
            uint32_t type, order = 0, porder = 0, method = 0;
            uint64_t est;
            int32_t cval = 0;
            if (bps == 0) {  // all zero (encoder.zig:495-497)
                type = 0;
                est = 0;
            } else if (T[1] == 0) {  // all equal (encoder.zig:498-500)
                type = 0;
                est = bps;
                cval = cand_x<c>(rdl(raw_at(rq, 0), 0)) >> w;
            } else {
                type = 1;
                est = (uint64_t)kBlock * bps;  // VERBATIM (encoder.zig:503-511)
                // bestOrder's first minimum (fixed.zig:164); the shifted sums are these >> w
                uint32_t k = 0;
#pragma unroll
                for (int q = 1; q < 5; q++)
                    if (T[q] < T[k]) k = q;
                // the chosen order's group sums and widths of the shifted samples: a zigzag of
                // e / 2^w is the zigzag of e shifted right by w (e a multiple of 2^w)
                uint32_t S8[4], W8[4];
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    uint32_t s = P.S[0][g];
#pragma unroll
                    for (int q = 1; q < 5; q++) s = k == (uint32_t)q ? P.S[q][g] : s;
                    const uint32_t wb = (P.Wp[g] >> (5u * k)) & 31u;
                    S8[g] = s >> w;
                    W8[g] = wb > w ? wb - w : 0u;
                }
                const uint32_t capp = bps > 16 ? 30u : 14u;
                const uint32_t maxp = capp < a.max_param ? capp : a.max_param;
                uint32_t best_o, best_m;
                const uint64_t best = rice_search16(S8, W8, k, a.max_part_order, maxp, par + 512u * c, l, best_o, best_m);
                if (best < est) {  // FIXED iff strictly below the verbatim estimate (encoder.zig:538)
                    type = 2;
                    est = best;
                    order = k;
                    porder = best_o;
                    method = best_m;
                }
            }
            if (l == 0) {
                uint32_t *rc = rec + 8u * c;
                rc[0] = type; rc[1] = w; rc[2] = order; rc[3] = porder; rc[4] = method;
                rc[5] = (uint32_t)est; rc[6] = (uint32_t)(est >> 32); rc[7] = (uint32_t)cval;
            }
        };
        candidate(ic<0>{});
        candidate(ic<1>{});
        candidate(ic<2>{});
        candidate(ic<3>{});
        opaque_raw(rq);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- stereo decision (encoder.zig:441-452): first minimum of L+R, L+S, S+R, M+S
        uint64_t e[4];
#pragma unroll
        for (int c = 0; c < 4; c++)
            e[c] = (uint64_t)__builtin_amdgcn_readfirstlane((int)rec[8 * c + 5]) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)rec[8 * c + 6]) << 32);
        const uint64_t sum0 = e[0] + e[1], sum1 = e[0] + e[3], sum2 = e[3] + e[1], sum3 = e[2] + e[3];
        uint32_t b = 0;
        uint64_t sb = sum0;
        if (sum1 < sb) { b = 1; sb = sum1; }
        if (sum2 < sb) { b = 2; sb = sum2; }
        if (sum3 < sb) { b = 3; sb = sum3; }
        const uint32_t channel_code = b == 0 ? 1u : b + 7u;
        // written pairs (encoder.zig:263-268): LR {0,1}, LS {0,3}, SR {3,1}, MS {2,3}
        const uint32_t cs0 = (b == 0 || b == 1) ? 0u : (b == 2 ? 3u : 2u);
        const uint32_t cs1 = (b == 0 || b == 2) ? 1u : 3u;

        // ---- frame header (frame_writer.zig:151-265) on lane 0
        if (l == 0) {
            hw[0] = hw[1] = hw[2] = hw[3] = 0;
            hw[4] = write_frame_header(hw, job.number, a.bits, channel_code, (uint32_t)kBlock, a.sample_rate);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- exact bits of each lane's segment of the two written subframes (pass A of
        // frame_writer.zig:269-372), then their descriptors
        uint8_t *fd = a.desc + (uint64_t)job.slot * a.desc_stride;
        uint32_t sub_bits0 = 0, sub_bits1 = 0;
#pragma unroll 1
        for (uint32_t s = 0; s < 2u; s++) {
            const uint32_t c = s ? cs1 : cs0;
            const uint32_t *rc = rec + 8u * c;
            const uint32_t type = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc[0]);
            const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc[1]);
            const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc[2]);
            const uint32_t o = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc[3]);
            const uint32_t method = (uint32_t)__builtin_amdgcn_readfirstlane((int)rc[4]);
            const uint32_t bd = a.bits + (c == 3u ? 1u : 0u);
            const uint32_t bps = bd - w;
            const uint8_t *pp = par + 512u * c + (1u << o);
            uint32_t seg = 0;
            if (type == 0) {
                seg = (l == 0) ? 8u + bd : 0u;
            } else if (type == 1) {
                seg = 64u * bps + ((l == 0) ? 8u + w : 0u);
            } else {
                const uint32_t param_len = 4u + method;
                if (l == 0) seg = 8u + w + k * bps + 6u + param_len + ((pp[0] & 0x80u) ? 5u : 0u);
                const uint32_t sh = 12u - o, psz = 4096u >> o;
                uint32_t pq[4];
#pragma unroll
                for (int g = 0; g < 4; g++) pq[g] = pp[(l * 64u + 16u * (uint32_t)g) >> sh];
                // the candidate's shifted samples: x = (lo + beta * hi) >> gam (gam includes w)
                const uint32_t o1 = c == 1u ? 16u : 0u;
                const int32_t beta = c == 2u ? 1 : (c == 3u ? -1 : 0);
                const uint32_t gam = w + (c == 2u ? 1u : 0u);
                auto xs = [&](uint32_t wd) -> int32_t {
                    const int32_t lo = __builtin_amdgcn_sbfe((int32_t)wd, o1, 16u);
                    return mad24((int32_t)wd >> 16, beta, lo) >> gam;
                };
                // residual e = x - sum c_i x[-i] (fixed.zig:12-18 COEFF_SCALAR), 24-bit MACs
                const int32_t c1 = k == 1 ? -1 : k == 2 ? -2 : k == 3 ? -3 : k == 4 ? -4 : 0;
                const int32_t c2 = k == 2 ? 1 : k == 3 ? 3 : k == 4 ? 6 : 0;
                const int32_t c3 = k == 3 ? -1 : k == 4 ? -4 : 0;
                const int32_t c4 = k == 4 ? 1 : 0;
                int32_t q1 = shr1(xs(raw_at(rq, 63))), q2 = shr1(xs(raw_at(rq, 62)));
                int32_t q3 = shr1(xs(raw_at(rq, 61))), q4 = shr1(xs(raw_at(rq, 60)));
                uint32_t qa[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < 64; j++) {
                    const int32_t x = xs(raw_at(rq, j));
                    const int32_t r = mad24(q4, c4, mad24(q3, c3, mad24(q2, c2, mad24(q1, c1, x))));
                    q4 = q3; q3 = q2; q2 = q1; q1 = x;
                    const bool warm = j < 4 && l == 0 && (uint32_t)j < k;
                    const uint32_t zz = zigzag32(r);
                    qa[j >> 4] = add_chain(qa[j >> 4], warm ? 0u : (zz >> (pq[j >> 4] & 31u)));
                    if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const uint32_t p = pq[g], i = l * 64u + 16u * (uint32_t)g;
                    const bool esc = (p & 0x80u) != 0;
                    const uint32_t cnt = 16u - ((g == 0 && l == 0) ? k : 0u);  // warm-ups: lane 0, j < k
                    seg += esc ? cnt * (p & 0x7Fu) : qa[g] + cnt * (1u + p);
                    if (i != 0 && (i & (psz - 1u)) == 0) seg += param_len + (esc ? 5u : 0u);
                }
            }
            const uint32_t sbits = wave_sum32(seg);
            if (s) sub_bits1 = sbits;
            else sub_bits0 = sbits;
            // ---- the subframe's descriptor (SubDesc, as k_analyze writes it)
            SubDesc *sd = (SubDesc *)(fd + sizeof(FrameDesc)) + s;
            sd->lane_bits[l] = seg;
            if (type >= 2) {
                const uint32_t np = 1u << o;
                for (uint32_t j = l; j < np; j += 64) sd->params[j] = pp[j];
            }
            if (l == 0) {
                const int32_t cv = (int32_t)rc[7];
                // (SubDesc is 8-byte aligned: the second of a frame's two sits at 600 mod 16 = 8)
                uint2 *sd2 = (uint2 *)sd;
                sd2[0] = make_uint2(type | (w << 8) | (bd << 16) | (k << 24), o | (method << 8) | (c << 16));
                sd2[1] = make_uint2(sbits, (uint32_t)kLpcPrec);  // bits, lpc_prec (lpc_shift 0 above)
                sd->cval = (int64_t)cv;
            }
        }
        // the next frame's samples: raw is dead from here (its loads run under the stores below);
        // the ticket of the frame after next first, so waiting for its value never waits for them
        if (l0 == 0) nn_t = xcd_ticket_frames(q8, n_jobs);
        if (nxt < n_jobs) load_raw(rq, jn.pcm_off, l);

        // ---- frame descriptor + exact frame size
        const uint32_t hb = (uint32_t)__builtin_amdgcn_readfirstlane((int)hw[4]);
        if (l == 0) {
            const uint32_t total = 8u * hb + sub_bits0 + sub_bits1;
            const uint32_t fbytes = ((total + 7u) >> 3) + 2u;
            if (fbytes + 16u > a.image_bytes) atomicOr(a.err, 1u);  // the pack kernel's image bound
            a.frame_bytes[job.slot] = fbytes;
            FrameDesc *f = (FrameDesc *)fd;
            f->hdr_bytes = hb;
            f->total_bits = total;
            f->channel_code = channel_code;
            f->n_out = 2;
            f->hdr[0] = hw[0];
            f->hdr[1] = hw[1];
            f->hdr[2] = hw[2];
            f->hdr[3] = hw[3];
        }

        // ---- optional decision records (parity tests)
        if (a.records) {
            FrameRec *fr = a.records + job.slot;
            for (uint32_t c = 0; c < 4u; c++) {
                const uint32_t *rc = rec + 8u * c;
                const uint32_t type = rc[0], o = rc[3];
                SubRec *sr = &fr->cand[c];
                if (l == 0) {
                    sr->type = (uint8_t)type;
                    sr->waste = (uint8_t)rc[1];
                    sr->bits = (uint8_t)(a.bits + (c == 3u ? 1u : 0u));
                    sr->order = (uint8_t)rc[2];
                    sr->part_order = (uint8_t)o;
                    sr->method = (uint8_t)rc[4];
                    sr->written = (c == cs0 || c == cs1) ? 1 : 0;
                    sr->pad = 0;
                    sr->pad2 = 0;
                    sr->estimate = (uint64_t)rc[5] | ((uint64_t)rc[6] << 32);
                    sr->constant = (int64_t)(int32_t)rc[7];
                    sr->lpc_precision = 0;
                    sr->lpc_shift = 0;
                }
                if (l < 32u) sr->lpc_coefs[l] = 0;
                const uint32_t np = 1u << o;
                const uint8_t *pp = par + 512u * c + (1u << o);
                for (uint32_t j = l; j < 256u; j += 64) sr->params[j] = (type >= 2 && j < np) ? pp[j] : 0;
            }
            if (l == 0) {
                fr->channel_code = channel_code;
                fr->n_cand = 4;
                fr->frame_bytes = ((8u * hb + sub_bits0 + sub_bits1 + 7u) >> 3) + 2u;
                fr->pad = 0;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // LDS reads above before the next frame's writes
        jidx = nxt;
        job = jn;
        nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)nn_t);
        if (nxt < n_jobs) jn = a.jobs[nxt];
    }
}
