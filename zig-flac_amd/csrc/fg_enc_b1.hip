// fg_enc_b1.hip -- frame-encode kernels for 1-byte PCM samples (8-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_encode_b1(const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_encode_b<1, 16>(a, full, threads, lds, st);
}
}  // namespace fg
