// fg_enc_b1.hip -- analysis + pack kernels for 1-byte PCM samples (8-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_stage_b1(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_stage_b<1, 16>(stage, a, full, threads, lds, st);
}
}  // namespace fg
