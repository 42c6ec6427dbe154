// band.hip -- dispatch of the typed band kernels (render_nn.h,
// render_bil.h, render_lds.h) by value type.
#include "render_lds.h"

namespace gsky {

void launch_band_kernels(const RenderArgs &a, int vt, bool mask, int n_items, hipStream_t s) {
  switch (vt) {
    case GSKYHIP_INT16: launch_band_i16(a, mask, n_items, s); break;
    case GSKYHIP_UINT16: launch_band_u16(a, mask, n_items, s); break;
    case GSKYHIP_FLOAT32: launch_band_f32(a, mask, n_items, s); break;
    case GSKYHIP_SIGNEDBYTE: launch_band_i8(a, mask, n_items, s); break;
    default: launch_band_u8(a, mask, n_items, s); break;
  }
}

}  // namespace gsky
