// placeholder until the HIP JPEG backend lands
#include "encoder_iface.h"
#include <stdexcept>
namespace sk {
EncoderBackend* create_hip_jpeg_backend(const jpeg::JpegConfig&, int) {
    throw std::runtime_error("HIP JPEG backend not built");
}
}
