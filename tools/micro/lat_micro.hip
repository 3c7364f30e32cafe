// lat_micro.hip -- dependent-issue latency of the VALU forms an MD5 step uses on gfx950
// (tools only): one wave per SIMD, one long dependent chain per lane, s_memtime around it.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(64) k(uint32_t *out, uint32_t seed, int iters, unsigned long long *cyc) {
    uint32_t x = seed + threadIdx.x, y = seed * 3u + 1u, z = seed ^ 0x55u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 32; r++) {
            if constexpr (OP == 0) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(y));
            if constexpr (OP == 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
            if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
            if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe4" : "+v"(x) : "v"(y), "v"(z));
            if constexpr (OP == 4) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(y));
            if constexpr (OP == 5) asm volatile("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(x));
            if constexpr (OP == 6) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
            if constexpr (OP == 7) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 8) asm volatile("v_add_lshl_u32 %0, %0, %1, 3" : "+v"(x) : "v"(y));
            if constexpr (OP == 9) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    uint32_t *o;
    unsigned long long *c, h;
    hipMalloc(&o, 1024 * 64 * 4);
    hipMalloc(&c, 8);
    const char *names[10] = {"v_add_u32 (VOP2)", "v_add3_u32", "v_alignbit_b32", "v_bitop3_b32", "v_xor_b32 (VOP2)",
                             "v_lshlrev_b32 (VOP2)", "v_bfi_b32", "v_lshl_add_u32", "v_add_lshl_u32", "v_xad_u32"};
    const int iters = 2000;
    for (int op = 0; op < 10; op++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
#define L(N) if (op == N) hipLaunchKernelGGL(k<N>, dim3(1024), dim3(64), 0, 0, o, 7u, iters, c);
            L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9)
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
            if (rep == 1)
                printf("%-22s %.2f ns per dependent op (event), s_memtime %.2f ticks/op\n", names[op],
                       ms * 1e6 / (iters * 32.0), (double)h / (iters * 32.0));
        }
    }
    return 0;
}
