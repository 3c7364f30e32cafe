// fg_fused.hpp -- the pack phase of the fused single-pass encode of full 16-bit stereo frames
// (k_analyze<2, 16, true, 256, 2, 0, FP = true>; included by fg_device.hpp inside namespace fg).
//
// The split encode analyses a frame (k_analyze), writes its descriptor to HBM, scans the frame
// sizes, and a second kernel (k_pack4) stages the PCM again, reloads the descriptor and packs.  The
// fused kernel packs each frame in the workgroup that analysed it, from the PCM still staged in
// LDS and the decisions still in LDS / registers, and gets its byte offset from an in-kernel
// exclusive scan over the frame slots (decoupled look-back, Merrill & Garland): the PCM is read
// once and no descriptor makes a round trip through memory (frame_writer.zig:269-372 restated,
// as in k_pack4 / k_packw).
#pragma once

// status word of a frame slot for the in-kernel scan: 0 = size not known yet, kStAgg | bytes = the
// frame's own size, kStInc | bytes = the bytes of every slot up to and including it
constexpr uint64_t kStAgg = 1ull << 62, kStInc = 2ull << 62, kStVal = (1ull << 62) - 1ull;

__device__ __forceinline__ void st_publish(uint64_t *st, uint64_t slot, uint64_t v) {
    __hip_atomic_store(st + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t st_load(const uint64_t *st, uint64_t idx) {
    return __hip_atomic_load(st + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of the frame sizes before slot s, by one wave: windows of 64 predecessors (lane
// l reads slot s - 1 - l - 64 k), summing sizes back to the nearest inclusive prefix; slots before
// 0 read as an inclusive 0.  Every slot's size is published as soon as it is known (full frames by
// their workgroup right after the analysis, before any wait; short frames by the tail analysis
// launched before), and a workgroup waits only on slots whose tickets were taken before its own,
// i.e. by workgroups already running: the wait is bounded.  A spin budget ends it regardless
// (error word bit 0), so a fault shows as an error, never as a hung device.
__device__ __noinline__ uint64_t frame_lookback(const uint64_t *st, uint32_t s, uint32_t l, uint32_t *err) {
    uint64_t acc = 0;
    int64_t base = (int64_t)s - 1;
    uint32_t spins = 0;
    while (true) {
        const int64_t idx = base - (int64_t)l;
        const uint64_t v = idx >= 0 ? st_load(st, (uint64_t)idx) : kStInc;
        const uint64_t inc = __ballot((v >> 62) == 2u);
        const uint64_t rdy = __ballot((v >> 62) != 0u);
        const uint32_t fi = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        const uint64_t need = fi >= 63u ? ~0ull : ((2ull << fi) - 1ull);  // lanes 0..fi
        if ((rdy & need) != need) {
            if (++spins > (1u << 22)) {
                if (l == 0) atomicOr(err, 1u);
                return acc;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        acc += wave_sum64((uint32_t)l <= fi ? (v & kStVal) : 0ull);
        if (fi < 64u) return acc;
        base -= 64;
    }
}

// The written subframes' fields, published in misc by their analysis waves (slot s = 0, 1):
// misc[40 + s] bits, [44 + s] candidate, [46 + s] type | waste << 8 | bd << 16 | order << 24,
// [48 + s] porder | method << 8, [50 + 2 s], [51 + 2 s] the CONSTANT value; misc[18] header bytes,
// misc[32..35] header words.  lbits[64 s + j] = bits of 64-sample segment j of subframe s (the
// analysis kernel's exact pass A).  par + cand * par_stride = the candidate's Rice parameters.
//
// Wave w packs half w & 1 of written subframe w >> 1; lane l its 32 samples [2048 (w & 1) + 32 l,
// +32) and the 4 before them, read from the interleaved staging (fg_layout.hpp: sample i at dword
// 272 (i >> 8) + 4 ((i >> 6) & 3) + 16 ((i & 63) >> 2) + (i & 3)).  Then the staging becomes the
// frame image: zeroed, codes ORed in at their bit offsets, CRC-16 (table-free fold), stored at the
// offset of the look-back.  Returns the frame's byte offset (uniform).
__device__ __forceinline__ void fused_pack(const EncodeArgs &a, uint32_t *stg, uint32_t *misc, const uint32_t *lbits,
                                           const uint8_t *par, uint32_t par_stride, uint32_t slot, uint32_t total_bits,
                                           uint32_t tid, uint32_t wave, uint32_t l) {
    constexpr uint32_t NT = 256, NW = 4;
    const uint32_t sfi = wave >> 1, hq = wave & 1u;
    const uint32_t Lb = (total_bits + 7u) >> 3, fbytes = Lb + 2u;
    const bool fits = fbytes + 16u <= a.image_bytes;  // uniform (else the analysis flagged it)
    const uint32_t cand = misc[44 + sfi], sdw = misc[46 + sfi], pw = misc[48 + sfi];
    const uint32_t type = sdw & 255u, w = (sdw >> 8) & 255u, bd = (sdw >> 16) & 255u, k = sdw >> 24;
    const uint32_t o = pw & 255u, method = pw >> 8;
    const uint32_t bps = bd - w;
    const uint32_t i0 = 2048u * hq + 32u * l;
    const uint8_t *pp = par + cand * par_stride + ((1u << o) - 1u);
    uint32_t pq[2];
#pragma unroll
    for (int g = 0; g < 2; g++) pq[g] = pp[(i0 + 16u * g) >> (12u - o)];
    uint32_t sub_start = 8u * misc[18];
    if (sfi) sub_start += misc[40];
    const uint32_t hbase = wave_sum32((hq && l < 32u) ? lbits[64u * sfi + l] : 0u);
    const uint32_t hdrw = misc[32u + (tid & 3u)];
    const int64_t cval = (int64_t)(((uint64_t)misc[51 + 2 * sfi] << 32) | misc[50 + 2 * sfi]);

    // ---- samples i0 - 4 .. i0 + 31 of the candidate (raw (L, R) dwords)
    uint32_t raw[36];
    {
        const uint32_t ch = i0 >> 6, g0 = (i0 & 63u) >> 2;
        const uint32_t *cb = stg + 272u * (ch >> 2) + 4u * (ch & 3u);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint4 v = *(const uint4 *)(cb + 16u * (g0 + (uint32_t)t));
            raw[4 + 4 * t] = v.x; raw[5 + 4 * t] = v.y; raw[6 + 4 * t] = v.z; raw[7 + 4 * t] = v.w;
        }
        const uint32_t chp = g0 ? ch : ch - 1u;
        const uint32_t *hp = stg + 272u * (chp >> 2) + 4u * (chp & 3u) + 16u * (g0 ? g0 - 1u : 15u);
        const uint4 hv = i0 ? *(const uint4 *)hp : make_uint4(0, 0, 0, 0);
        raw[0] = hv.x; raw[1] = hv.y; raw[2] = hv.z; raw[3] = hv.w;
    }
    int32_t x[36];
    auto unpack = [&](auto KD) {
        constexpr uint32_t KND = decltype(KD)::value;
#pragma unroll
        for (int i = 0; i < 36; i++) {
            const int32_t L = (int32_t)(raw[i] << 16) >> 16, R = (int32_t)raw[i] >> 16;
            x[i] = KND == 0 ? L : KND == 1 ? R : KND == 2 ? (L + R) >> 1 : L - R;
        }
    };
    if (cand == 0) unpack(ic<0>{});
    else if (cand == 1) unpack(ic<1>{});
    else if (cand == 2) unpack(ic<2>{});
    else unpack(ic<3>{});
    bar_lds();  // staging dead: it becomes the frame image
    uint32_t *img = stg;
    const uint32_t Wz = (fbytes + 3u) / 4u + 2u;
    if (fits)
        for (uint32_t i = tid; i < Wz; i += NT) img[i] = 0;

    // ---- waste shift, residuals, this lane's code lengths (as k_packw at SPL = 32)
    if (type != 0 && w != 0) {
#pragma unroll
        for (int i = 0; i < 36; i++) x[i] >>= w;
    }
    const bool first = (hq == 0) && (l == 0);
    const uint32_t param_len = 4u + method;
    uint32_t r[32];
    auto resid = [&](auto KO) {
        constexpr uint32_t K = decltype(KO)::value;
#pragma unroll
        for (int i = 0; i < 32; i++) {
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
    const uint32_t nwarm = (first && type == 2) ? k : 0u;
    auto warm_at = [&](int j) -> bool { return j < 4 && (uint32_t)j < nwarm; };
    uint32_t len = 0;
    if (first) {
        const uint32_t p0 = pq[0];
        if (type == 0) len = 8u + bd;
        else if (type == 1) len = 8u + w;
        else len = 8u + w + k * bps + 6u + param_len + ((p0 & 0x80u) ? 5u : 0u);
    }
    if (type == 1) {
        len += 32u * bps;
    } else if (type == 2) {
        const uint32_t psz = 4096u >> o;
#pragma unroll
        for (int g = 0; g < 2; g++) {
            const uint32_t p = pq[g], ig = i0 + 16u * g;
            const bool esc = (p & 0x80u) != 0;
            const uint32_t pr = esc ? 0u : p, cl = esc ? (p & 0x7Fu) : pr + 1u;
            if (ig != 0 && (ig & (psz - 1u)) == 0) len += param_len + (esc ? 5u : 0u);
            uint32_t qs = 0, nc = 16;
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                const int j = 16 * g + jj;
                const bool wm = warm_at(j);
                qs = add_chain(qs, wm ? 0u : (zigzag32((int32_t)r[j]) >> pr));
                if (j < 4) nc -= wm ? 1u : 0u;
            }
            len += (esc ? 0u : qs) + nc * cl;
        }
    }
    const uint32_t lane_off = wave_incl_scan32(len) - len;
    bar_lds();  // image zeroed
    if (fits && tid < 4 && hdrw) atomicOr(&img[tid], hdrw);

    // ---- codes into the image at their bit offsets
    if (fits) {
        uint32_t pos = sub_start + hbase + lane_off;
        const uint64_t mask = ~0ull >> (64 - (bps ? bps : 1u));
        if (first) {
            AtomicWriter bw;
            bw.init(img, pos);
            if (type == 0) {  // writeConstantSubframe: 0x00, value << waste in bd bits
                bw.put(0, 8);
                bw.put(((uint64_t)cval << w) & (~0ull >> (64 - bd)), bd);
            } else {
                const uint32_t tc = (type == 1) ? 1u : (8u | k);
                bw.put((tc << 1) | (w ? 1u : 0u), 8);
                if (w) bw.put(1, w);
                if (type == 2) {
#pragma unroll
                    for (int j = 0; j < 4; j++)  // warm-up samples
                        if ((uint32_t)j < k) bw.put((uint64_t)(int64_t)x[4 + j] & mask, bps);
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
        if (type == 1) {
#pragma unroll
            for (int j = 0; j < 32; j++) {
                put_or2(img, pos, (uint64_t)(int64_t)x[4 + j] & mask, bps);
                pos += bps;
            }
        } else if (type == 2) {
            const uint32_t psz = 4096u >> o;
            const uint32_t esc_code = (0x0Fu | (method << 4)) << 5;
            const uint32_t img_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)img;
#pragma unroll
            for (int g = 0; g < 2; g++) {
                __builtin_amdgcn_sched_barrier(0);
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
                    if (j < 4) {
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

    // ---- CRC-16 (table-free fold, see k_pack4) and, on wave 0, the frame's byte offset
    const uint32_t W4 = Lb >> 2;
    const uint32_t H = max((W4 + 2u * NT - 1u) / (2u * NT), 1u);
    if (fits) {
        const uint32_t crc_pw = a.crc_pow4[(min(H, a.crc_hmax4) - 1u) * NT + tid];
        const int32_t Z = (int32_t)(NT * 2u * H) - (int32_t)W4;
        const int32_t va = (int32_t)(tid * 2u * H) - Z;
        uint32_t contrib = crc_lane_q(img, va, 2u * H, crc_pw);
        contrib = wave_xor32(contrib);
        if (l == 0) misc[wave] = contrib;
    }
    if (wave == 0) {
        const uint64_t D = frame_lookback(a.status, slot, l, a.err);
        if (l == 0) {
            st_publish(a.status, slot, kStInc | (D + fbytes));
            const_cast<uint64_t *>(a.offsets)[slot] = D;
            misc[24] = (uint32_t)D;
            misc[25] = (uint32_t)(D >> 32);
        }
    }
    bar_lds();
    if (fits && tid == 0) {
        uint32_t qp = 0;
        for (uint32_t i = 0; i < NW; i++) qp ^= misc[i];
        uint32_t crc = crc_from_q(qp);
        for (uint32_t b = W4 * 4u; b < Lb; b++) crc = crc_byte_v(crc, (img[b >> 2] >> (24 - 8 * (b & 3))) & 255u);
        put_bits(img, Lb * 8u, crc, 16);
    }
    bar_lds();
    const uint64_t D = ((uint64_t)misc[25] << 32) | misc[24];
    if (fits) {
        if (D + fbytes > a.out_cap) {
            if (tid == 0) atomicOr(a.err, 2u);
        } else {
            store_frame16(img, a.out, D, fbytes, tid, NT);
        }
    }
}
