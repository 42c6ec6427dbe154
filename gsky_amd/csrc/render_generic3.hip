// render_generic3.hip -- the NOUT=3 generic render kernels (RGB).
#include "render_generic.h"

namespace gsky {
void dispatch_render_3(const RenderArgs &a, int resample, bool mask, dim3 grid, bool general_only,
                       hipStream_t s) {
  dispatch_render_t<3>(a, resample, mask, grid, general_only, s);
}
}  // namespace gsky
