// placeholder replaced by the HIP backend
#include "encoder_iface.h"
#include <stdexcept>
namespace sk {
EncoderBackend* create_hip_backend(const h264::EncoderConfig&, int) {
    throw std::runtime_error("HIP backend not built");
}
}
