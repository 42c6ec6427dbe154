// render_lds_f32.hip -- band kernels of float (one TU per value type).
#include "render_bil.h"
#include "render_nn_stage.h"

namespace gsky {
void launch_lds_f32(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_band_t<float>(a, mask, n_items, s);
}
}  // namespace gsky
