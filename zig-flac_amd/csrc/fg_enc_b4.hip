// fg_enc_b4.hip -- frame-encode kernels for 4-byte PCM samples (32-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_encode_b4(const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_encode_b<4, 32>(a, full, threads, lds, st);
}
}  // namespace fg
