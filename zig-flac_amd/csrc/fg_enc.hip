// fg_enc.hip -- one instantiation set of the analysis + pack kernels, compiled once
// per (PCM sample bytes FG_B, LPC taps FG_LPW) by the Makefile so the variants
// build in parallel: FG_B = 1..4 (8/16/24/32-bit), FG_LPW = 0 (fixed prediction,
// the reference), 8 or 12 (LPC search, build-defined).
#include "fg_device.hpp"

#if !defined(FG_B) || !defined(FG_LPW)
#error "FG_B and FG_LPW must be defined"
#endif
#define FG_CLS (FG_B == 4 ? 32 : (FG_B == 3 ? 24 : 16))
#define FG_CAT2(a, b, c) a##b##_l##c
#define FG_CAT(a, b, c) FG_CAT2(a, b, c)

namespace fg {
hipError_t FG_CAT(launch_stage_b, FG_B, FG_LPW)(int stage, const EncodeArgs &a, bool full, uint32_t threads,
                                                uint32_t lds, hipStream_t st) {
    return launch_stage_b<FG_B, FG_CLS, FG_LPW>(stage, a, full, threads, lds, st);
}
}  // namespace fg
