// fg_enc_b3.hip -- frame-encode kernels for 3-byte PCM samples (24-bit).
#include "fg_device.hpp"

namespace fg {
hipError_t launch_encode_b3(const EncodeArgs &a, bool full, uint32_t threads, uint32_t lds, hipStream_t st) {
    return launch_encode_b<3, 24>(a, full, threads, lds, st);
}
}  // namespace fg
