// Fused MFMA forward+backward — placeholder until the CDNA4 kernel lands.
#include "ncf_internal.h"

namespace ncf {

bool fused_supported(const ncf_shape_t&) { return false; }

hipError_t launch_fb_fused(const ncf_shape_t&, const WsLayout&, void*, const float*, const float*, const int32_t*,
                           const int32_t*, const float*, int64_t, float, int*, int*, hipStream_t) {
    return hipErrorNotSupported;
}

}  // namespace ncf
