// fg_enc_b2.hip -- analysis + pack kernels for 2-byte PCM samples (16-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_stage_b2(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_stage_b<2, 16>(stage, a, full, threads, lds, st);
}
}  // namespace fg
