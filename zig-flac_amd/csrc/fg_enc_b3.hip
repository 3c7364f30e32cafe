// fg_enc_b3.hip -- analysis + pack kernels for 3-byte PCM samples (24-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_stage_b3(int stage, const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_stage_b<3, 24>(stage, a, full, threads, lds, st);
}
}  // namespace fg
