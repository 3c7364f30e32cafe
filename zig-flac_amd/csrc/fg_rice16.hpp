// fg_rice16.hpp -- rice.calcParams (rice.zig:87-107, 248-405) for full 4096-sample frames of 16-bit
// input, shared by k_analyze (fixed prediction) and k_ana1.  Included by fg_device.hpp inside
// namespace fg (uses its wave helpers and rice_choose).
#pragma once

// rice.zig:343-405 for one partition of a full frame: len = 2^L - kwl samples (kwl: the warm-up
// samples inside it, nonzero only for partition 0; L uniform, kwl < 2^(L-1)), sum S of |residual|
// (< 2^32: 16-bit input), zigzag width W.  The closed-form parameter of rice_choose with the
// products of the cost model as shifts (and 24-bit products by kwl): the generic version's
// per-lane lengths made every product a 32-bit multiply.  Returns param (0x80|W = escape).
__device__ __forceinline__ uint32_t rice_pow2(uint32_t S, uint32_t L, uint32_t kwl, uint32_t W, uint32_t maxp,
                                              uint32_t *cost) {
    const uint32_t len = (1u << L) - kwl, two = 2u * len;
    uint32_t p;
    if (S <= ((len + 1u) >> 1)) {
        p = 0;
    } else if (S <= two) {
        p = 1;
    } else {
        const uint32_t m0 = bitlen32(S) - (L + (kwl ? 1u : 2u));  // bitlen(S) - bitlen(2 len)
        p = m0 + 1u + ((S >> m0) > two ? 1u : 0u);
    }
    if (p > maxp - 1u) p = maxp - 1u;
    const uint32_t f = (p == 0) ? len + (S << 1)
                                : ((1u + p) << L) - __umul24(1u + p, kwl) + (S >> (p - 1u)) - (len >> 1);
    const uint32_t esc = (W <= 31u) ? 5u + (W << L) - __umul24(W, kwl) : ~0u;
    if (f < esc) {
        *cost = f;
        return p;
    }
    *cost = esc;
    return 0x80u | W;
}

// rice.calcParams for one residual set of a full 4096-sample frame, partitions held as k_analyze's
// FULL path holds them: lane l owns the four 16-sample groups of order 8 (sums S8, zigzag widths
// W8; 32-bit sums: 16-bit input).  Parameters of order o go to pb[(1 << o) + j] (4-byte aligned
// rows: the order-8 parameters of a lane are one dword store); returns the estimate, best_o /
// best_m the partition order and method (rice.zig:248-405).
// The per-order totals are summed two orders per dword: each partition costs at most its escape
// code (5 + 23 len, 16-bit input), so a 16-lane row's sum of one order stays below 2^16.
__device__ __forceinline__ uint64_t rice_search16(const uint32_t (&S8)[4], const uint32_t (&W8)[4], uint32_t kw,
                                                  uint32_t P, uint32_t maxp, uint8_t *pb, uint32_t l, uint32_t &best_o,
                                                  uint32_t &best_m) {
    const uint32_t S7a = S8[0] + S8[1], S7b = S8[2] + S8[3];
    const uint32_t W7a = max(W8[0], W8[1]), W7b = max(W8[2], W8[3]);
    const uint32_t S6 = S7a + S7b;
    const uint32_t W6 = max(W7a, W7b);
    uint32_t Sl[4], Wl[4];
    {
        uint32_t Sg = S6, Wg = W6;
        Sg += dpp<DPP_XOR1>(Sg); Wg = max(Wg, dpp<DPP_XOR1>(Wg)); Sl[0] = Sg; Wl[0] = Wg;
        Sg += dpp<DPP_XOR2>(Sg); Wg = max(Wg, dpp<DPP_XOR2>(Wg)); Sl[1] = Sg; Wl[1] = Wg;
        Sg += dpp<DPP_HMIRROR>(Sg); Wg = max(Wg, dpp<DPP_HMIRROR>(Wg)); Sl[2] = Sg; Wl[2] = Wg;
        Sg += dpp<DPP_MIRROR>(Sg); Wg = max(Wg, dpp<DPP_MIRROR>(Wg)); Sl[3] = Sg; Wl[3] = Wg;
    }
    const uint32_t kw0 = (l == 0) ? kw : 0u;  // warm-ups inside the lane's first partition
    uint32_t cst[9];
    uint32_t fv = 0;  // bit o: some partition of order o uses a parameter > 14 (method FIVE)
    auto five = [&](uint32_t p) { return (p < 0x80u && p > 14u) ? 1u : 0u; };
    // orders 8, 7, 6: partitions within the lane
    {
        uint32_t c, cc = 0, pk = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t p = rice_pow2(S8[q], 4u, q == 0 ? kw0 : 0u, W8[q], maxp, &c);
            cc += c;
            fv |= five(p) << 8;
            pk |= p << (8 * q);
        }
        *(uint32_t *)(pb + 256u + 4u * l) = pk;
        cst[8] = cc;
        uint32_t p0 = rice_pow2(S7a, 5u, kw0, W7a, maxp, &c);
        cc = c;
        const uint32_t p1 = rice_pow2(S7b, 5u, 0u, W7b, maxp, &c);
        cc += c;
        fv |= (five(p0) | five(p1)) << 7;
        *(uint16_t *)(pb + 128u + 2u * l) = (uint16_t)(p0 | (p1 << 8));
        cst[7] = cc;
        p0 = rice_pow2(S6, 6u, kw0, W6, maxp, &c);
        cst[6] = c;
        fv |= five(p0) << 6;
        pb[64u + l] = (uint8_t)p0;
    }
    // orders 5..2: a partition spans 2^g lanes (the butterfly value); its first lane stores it
#pragma unroll
    for (int o = 5; o >= 2; o--) {
        const int g = 6 - o;
        const bool lead = (l & ((1u << g) - 1u)) == 0;
        uint32_t c;
        const uint32_t p = rice_pow2(Sl[g - 1], 12u - o, kw0, Wl[g - 1], maxp, &c);
        cst[o] = lead ? c : 0u;
        fv |= (lead ? five(p) : 0u) << o;
        if (lead) pb[(1u << o) + (l >> g)] = (uint8_t)p;
    }
    // per-order totals: row sums two orders per dword, then the four rows (uniform)
    uint64_t tots[9];
    {
        const uint32_t v0 = row_sum32(cst[8] | (cst[7] << 16)), v1 = row_sum32(cst[6] | (cst[5] << 16));
        const uint32_t v2 = row_sum32(cst[4] | (cst[3] << 16)), v3 = row_sum32(cst[2]);
        auto rows = [&](uint32_t x, int sh) -> uint64_t {
            return (uint64_t)((rdl(x, 0) >> sh) & 0xFFFFu) + ((rdl(x, 16) >> sh) & 0xFFFFu) +
                   ((rdl(x, 32) >> sh) & 0xFFFFu) + ((rdl(x, 48) >> sh) & 0xFFFFu);
        };
        tots[8] = rows(v0, 0); tots[7] = rows(v0, 16);
        tots[6] = rows(v1, 0); tots[5] = rows(v1, 16);
        tots[4] = rows(v2, 0); tots[3] = rows(v2, 16);
        tots[2] = rows(v3, 0);
        fv = maxp > 15u ? wave_or32(fv) : 0u;
    }
    // orders 1, 0: uniform (the four row sums)
    {
        const uint32_t r0 = rdl(Sl[3], 0), r1 = rdl(Sl[3], 16), r2 = rdl(Sl[3], 32), r3 = rdl(Sl[3], 48);
        const uint32_t m0 = rdl(Wl[3], 0), m1 = rdl(Wl[3], 16), m2 = rdl(Wl[3], 32), m3 = rdl(Wl[3], 48);
        uint32_t c0, c1, c2;
        const uint32_t p10 = rice_pow2(r0 + r1, 11u, kw, max(m0, m1), maxp, &c0);
        const uint32_t p11 = rice_pow2(r2 + r3, 11u, 0u, max(m2, m3), maxp, &c1);
        // (the whole frame's sum can pass 2^32: 4096 residuals of up to 2^20, the generic 64-bit form)
        const uint32_t p00 = rice_choose((uint64_t)r0 + r1 + r2 + r3, 4096u - kw, max(max(m0, m1), max(m2, m3)),
                                         maxp, &c2);
        if (l == 0) {
            pb[2] = (uint8_t)p10;
            pb[3] = (uint8_t)p11;
            pb[1] = (uint8_t)p00;
        }
        tots[1] = (uint64_t)c0 + c1;
        tots[0] = c2;
        if (maxp > 15u) fv |= ((five(p10) | five(p11)) << 1) | five(p00);
    }
    uint64_t best = ~0ull;
    best_o = 0;
    best_m = 0;
#pragma unroll
    for (int o = 0; o < 9; o++) {
        const uint32_t f5 = (fv >> o) & 1u;
        const uint64_t tot = tots[o] + ((uint64_t)(4u + f5) << o);
        if ((uint32_t)o <= P && tot <= best) {  // ascending, "<=": the higher order wins ties (rice.zig:271)
            best = tot;
            best_o = (uint32_t)o;
            best_m = f5;
        }
    }
    return best;
}

