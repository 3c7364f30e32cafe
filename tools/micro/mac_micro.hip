// mac_micro.hip -- throughput of the multiply-accumulate forms an LPC residual
// pass could use on gfx950 (tools only): i64 += i32*i32 (v_mad_i64_i32),
// f64 fma, u32 mul_lo, i32 24-bit mad.  8 independent accumulators per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void __launch_bounds__(256) k(const int *in, long long *out, int iters) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    int x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = in[(t * 8 + i) & 1023];
    if constexpr (KIND == 0) {
        long long acc[8] = {};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int r = 0; r < 8; r++)
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] += (long long)x[i] * (long long)x[(i + r) & 7];
            x[0] ^= (int)acc[7];
        }
        long long s = 0;
        for (int i = 0; i < 8; i++) s += acc[i];
        out[t] = s;
    } else if constexpr (KIND == 1) {
        double acc[8] = {}, xd[8];
        for (int i = 0; i < 8; i++) xd[i] = (double)x[i];
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int r = 0; r < 8; r++)
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = __builtin_fma(xd[i], xd[(i + r) & 7], acc[i]);
            xd[0] += acc[7] * 1e-30;
        }
        double s = 0;
        for (int i = 0; i < 8; i++) s += acc[i];
        out[t] = (long long)s;
    } else if constexpr (KIND == 2) {
        unsigned acc[8] = {};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int r = 0; r < 8; r++)
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] += (unsigned)x[i] * (unsigned)x[(i + r) & 7];
            x[0] ^= acc[7];
        }
        long long s = 0;
        for (int i = 0; i < 8; i++) s += acc[i];
        out[t] = s;
    } else {
        int acc[8] = {};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int r = 0; r < 8; r++)
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = __mul24(x[i], x[(i + r) & 7]) + acc[i];
            x[0] ^= acc[7];
        }
        long long s = 0;
        for (int i = 0; i < 8; i++) s += acc[i];
        out[t] = s;
    }
}

int main() {
    int *in;
    long long *out;
    hipMalloc(&in, 4096 * 4);
    hipMemset(in, 1, 4096 * 4);
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    hipMalloc(&out, (size_t)blocks * threads * 8);
    const char *names[4] = {"i64 += i32*i32", "f64 fma", "u32 mul_lo+add", "i24 mul+add"};
    for (int kind = 0; kind < 4; kind++) {
        auto launch = [&]() {
            if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
            if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
            if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
            if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
        };
        launch();
        hipDeviceSynchronize();
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double macs = (double)blocks * threads * iters * 64;
        printf("%-18s %8.3f ms  %8.1f G MAC/s  (%.2f cyc/wave-MAC/SIMD at 2.4 GHz)\n", names[kind], ms,
               macs / ms / 1e6, (256.0 * 4 * 2.4e9) / (macs / 64 / (ms * 1e-3)));
    }
    return 0;
}
