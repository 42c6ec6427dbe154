// band_u8.hip -- the band kernels of value type uint8_t (one TU per type):
// render_nn_kernel (nearest neighbour), render_lds_kernel (bilinear with a
// mask layer or typed RGBA).
#include "render_nn.h"

namespace gsky {
void launch_band_u8(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_band_t<uint8_t>(a, mask, n_items, s);
}
}  // namespace gsky
