// band_f32.hip -- the band kernels of value type float (one TU per type):
// render_nn_kernel (nearest neighbour), render_lds_kernel (bilinear with a
// mask layer or typed RGBA) and render_bil_kernel (bilinear float canvases).
#include "render_bil.h"
#include "render_nn.h"

namespace gsky {
void launch_band_f32(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_band_t<float>(a, mask, n_items, s);
}
}  // namespace gsky
