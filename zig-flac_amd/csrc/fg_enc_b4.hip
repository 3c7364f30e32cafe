// fg_enc_b4.hip -- analysis + pack kernels for 4-byte PCM samples (32-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_stage_b4(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_stage_b<4, 32>(stage, a, full, threads, lds, st);
}
}  // namespace fg
