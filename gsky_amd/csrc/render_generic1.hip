// render_generic1.hip -- the NOUT=1 generic render kernels (single namespace: palette/grey).
#include "render_generic.h"

namespace gsky {
void dispatch_render_1(const RenderArgs &a, int resample, bool mask, dim3 grid, bool general_only,
                       hipStream_t s) {
  dispatch_render_t<1>(a, resample, mask, grid, general_only, s);
}
}  // namespace gsky
