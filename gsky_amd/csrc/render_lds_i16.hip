// render_lds_i16.hip -- band kernels of int16_t (one TU per value type).
#include "render_nn_stage.h"

namespace gsky {
void launch_lds_i16(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_band_t<int16_t>(a, mask, n_items, s);
}
}  // namespace gsky
