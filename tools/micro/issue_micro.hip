// issue_micro.hip -- VALU issue throughput on gfx950 for the integer forms the analysis kernels
// are built from (tools only): v_add_u32, v_sad_u32, v_xad_u32, v_max3_u32, v_add_u32_sdwa,
// v_mul_u32_u24, at 1..8 waves per SIMD, 8 independent chains per lane.  Reports wave-instructions
// per SIMD-cycle from the in-kernel clock (s_memtime / s_memrealtime x 100 MHz), so DVFS is
// factored out: 0.5 = one wave64 VALU instruction every 2 cycles (the SIMD-32 peak).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int KIND>
__global__ void __launch_bounds__(64) k(const unsigned *in, unsigned *out, unsigned long long *clk, int iters) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned a[8], b[8];
    const unsigned kk = (unsigned)__builtin_amdgcn_readfirstlane((int)in[5]);
    const unsigned long long mask = __builtin_amdgcn_ballot_w64((in[t & 1023] & 1u) != 0);
#pragma unroll
    for (int i = 0; i < 8; i++) { a[i] = in[(t + 8 * i) & 1023]; b[i] = in[(t * 3 + i) & 1023]; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const unsigned x = b[(i + r) & 7];
                // inline asm: one instruction each, nothing folded across the unrolled loop
                if constexpr (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 1) asm volatile("v_sad_u32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(b[i]));
                else if constexpr (KIND == 2) asm volatile("v_xad_u32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(b[i]));
                else if constexpr (KIND == 3) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(x), "v"(b[i]));
                else if constexpr (KIND == 4)
                    asm volatile("v_add_u32_sdwa %0, sext(%1), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"
                                 : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 5) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(b[i]));
                // encoding vs operand count: VOP3 forms with two VGPR sources, VOP2 forms
                else if constexpr (KIND == 6) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 7) asm volatile("v_sad_u32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "s"(kk));
                else if constexpr (KIND == 8) asm volatile("v_xad_u32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(x), "s"(kk));
                else if constexpr (KIND == 9) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 10) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 11) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(x), "v"(b[i]));
                else if constexpr (KIND == 12) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 13) asm volatile("v_sub_u32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 14) asm volatile("v_lshrrev_b32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 15) asm volatile("v_ashrrev_i32_e32 %0, 3, %0" : "+v"(a[i]));
                else if constexpr (KIND == 16) asm volatile("v_ffbh_u32_e32 %0, %1" : "=v"(a[i]) : "v"(a[i] ^ x));
                // an explicit SGPR-pair lane mask (round 4 read an uninitialised vcc: 0.061, an artefact)
                else if constexpr (KIND == 17) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(x), "s"(mask));
                else if constexpr (KIND == 18) asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 19) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a[i]));
                else if constexpr (KIND == 20) asm volatile("v_add_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
                else if constexpr (KIND == 21) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 22) asm volatile("v_lshl_or_b32 %0, %1, 3, %0" : "+v"(a[i]) : "v"(x));
                else if constexpr (KIND == 23) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(a[i]), "v"(x) : "vcc");
                else asm volatile("v_min_i32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
            }
        b[0] ^= a[7];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= a[i];
    out[t] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}


// 64-bit and f64 forms (the LPC kernels' MACs, Levinson-Durbin, 64-bit sums): KIND 0 v_mad_i64_i32,
// 1 v_mad_u64_u32, 2 v_fma_f64, 3 v_mul_f64, 4 v_add_f64, 5 64-bit add as v_add_co_u32 +
// v_addc_co_u32 (2 instructions), 6 v_alignbit_b32, 7 v_mul_hi_i32, 8 v_lshlrev_b64,
// 9 v_sub_co_u32 + v_subb_co_u32 (2 instructions), 10 v_mul_lo_u32
template <int KIND>
__global__ void __launch_bounds__(64) k2(const unsigned *in, unsigned *out, unsigned long long *clk, int iters) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long a[8];
    double d[8];
    unsigned b[8], u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        b[i] = in[(t * 3 + i) & 1023];
        u[i] = in[(t + 8 * i) & 1023];
        a[i] = ((unsigned long long)b[i] << 20) ^ u[i];
        d[i] = (double)u[i] * 1e-9;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const unsigned x = b[(i + r) & 7];
                unsigned y = x;
                if constexpr (KIND == 0) asm volatile("v_mad_i64_i32 %0, s[100:101], %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(u[i]) : "s100", "s101");
                else if constexpr (KIND == 1) asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(u[i]) : "s100", "s101");
                else if constexpr (KIND == 2) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[i]) : "v"(d[(i + r) & 7]), "v"(d[i]));
                else if constexpr (KIND == 3) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + r) & 7]));
                else if constexpr (KIND == 4) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + r) & 7]));
                else if constexpr (KIND == 5)
                    asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, 0, %2, vcc" : "+v"(u[i]), "+v"(y), "+v"(b[i]) : : "vcc");
                else if constexpr (KIND == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(u[i]) : "v"(x));
                else if constexpr (KIND == 7) asm volatile("v_mul_hi_i32 %0, %0, %1" : "+v"(u[i]) : "v"(x));
                else if constexpr (KIND == 8) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(a[i]));
                else if constexpr (KIND == 9)
                    asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_subb_co_u32 %2, vcc, %2, 0, vcc" : "+v"(u[i]), "+v"(y), "+v"(b[i]) : : "vcc");
                else asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(x));
                (void)y;
            }
        b[0] ^= u[7] ^ (unsigned)a[7] ^ (unsigned)(long long)d[7];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= u[i] ^ b[i] ^ (unsigned)a[i] ^ (unsigned)(long long)d[i];
    out[t] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int KIND, bool K2 = false>
void run(const char *name, unsigned *din, unsigned *dout, unsigned long long *dclk, int wps) {
    const int cus = 256, blocks = cus * 4 * wps, iters = 2000;
    auto kern = K2 ? k2<KIND> : k<KIND>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, din, dout, dclk, 10);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, din, dout, dclk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long clk[2];
    (void)hipMemcpy(clk, dclk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;  // in-kernel clock
    const double instr = (double)blocks * iters * 16 * 8;                 // wave-instructions (ops per lane)
    const double per_simd_cycle = instr / (cus * 4.0) / (ms * 1e-3 * ghz * 1e9);
    printf("%-10s waves/SIMD %d: %.3f ms, clock %.2f GHz, %.3f wave-instr per SIMD-cycle\n", name, wps, ms, ghz,
           per_simd_cycle);
}

int main() {
    unsigned *din, *dout;
    unsigned long long *dclk;
    (void)hipMalloc(&din, 4096 * 4);
    (void)hipMalloc(&dout, 256 * 4 * 8 * 64 * 4);
    (void)hipMalloc(&dclk, 16);
    unsigned h[1024];
    for (int i = 0; i < 1024; i++) h[i] = rand();
    (void)hipMemcpy(din, h, 4096, hipMemcpyHostToDevice);
    const int ws[] = {4, 8};
    for (int w : ws) {
        run<0>("v_add", din, dout, dclk, w);
        run<1>("v_sad", din, dout, dclk, w);
        run<2>("v_xad", din, dout, dclk, w);
        run<3>("v_max3", din, dout, dclk, w);
        run<4>("add_sdwa", din, dout, dclk, w);
        run<5>("mad_u24", din, dout, dclk, w);
        run<6>("add_e64", din, dout, dclk, w);
        run<7>("sad_s", din, dout, dclk, w);
        run<8>("xad_s", din, dout, dclk, w);
        run<9>("max_e32", din, dout, dclk, w);
        run<10>("mul_u24", din, dout, dclk, w);
        run<11>("add3", din, dout, dclk, w);
        run<12>("xor_e32", din, dout, dclk, w);
        run<13>("sub_e32", din, dout, dclk, w);
        run<14>("lshr_e32", din, dout, dclk, w);
        run<15>("ashr_imm", din, dout, dclk, w);
        run<16>("ffbh", din, dout, dclk, w);
        run<17>("cndmask", din, dout, dclk, w);
        run<18>("or_e32", din, dout, dclk, w);
        run<19>("bfe_u32", din, dout, dclk, w);
        run<20>("add_dpp", din, dout, dclk, w);
        run<21>("mul_lo", din, dout, dclk, w);
        run<22>("lshl_or", din, dout, dclk, w);
        run<23>("cmp_e32", din, dout, dclk, w);
        run<24>("min_i32", din, dout, dclk, w);
        run<0, true>("mad_i64_i32", din, dout, dclk, w);
        run<1, true>("mad_u64_u32", din, dout, dclk, w);
        run<2, true>("fma_f64", din, dout, dclk, w);
        run<3, true>("mul_f64", din, dout, dclk, w);
        run<4, true>("add_f64", din, dout, dclk, w);
        run<5, true>("add64(2 ins)", din, dout, dclk, w);
        run<6, true>("alignbit", din, dout, dclk, w);
        run<7, true>("mul_hi_i32", din, dout, dclk, w);
        run<8, true>("lshl_b64", din, dout, dclk, w);
        run<9, true>("sub64(2 ins)", din, dout, dclk, w);
        run<10, true>("mul_lo(k2)", din, dout, dclk, w);
    }
    return 0;
}
