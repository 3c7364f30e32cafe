// fg_enc_b2.hip -- frame-encode kernels for 2-byte PCM samples (16-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_encode_b2(const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_encode_b<2, 16>(a, full, threads, lds, st);
}
}  // namespace fg
