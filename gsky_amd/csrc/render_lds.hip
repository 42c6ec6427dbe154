// render_lds.hip -- dispatch of the typed band kernels (render_nn.h, render_lds.h).
#include <cstdlib>

#include "render_lds.h"

namespace gsky {

void launch_lds_kernels(const RenderArgs &a0, int vt, bool mask, int n_items, hipStream_t s) {
  // GSKYHIP_LDS_STAGE=1 stages the source windows in LDS; the default gathers
  // from HBM, measured faster on C2 and C5 (profiles/r02_ab_*.jsonl).  Results
  // are identical either way.
  RenderArgs a = a0;
  const char *st = getenv("GSKYHIP_LDS_STAGE");
  a.lds_stage = st ? atoi(st) : 0;
  const char *fl = getenv("GSKYHIP_LDS_FLAGS");
  a.lds_flags = fl ? atoi(fl) : 0;
  // NN work goes to render_nn_kernel unless GSKYHIP_NN_KERNEL=0 (A/B);
  // GSKYHIP_NN_SHAPE picks its pixels x rows per lane (render_nn.h)
  const char *nk = getenv("GSKYHIP_NN_KERNEL");
  a.nn_kernel = nk ? atoi(nk) : 1;
  const char *ns = getenv("GSKYHIP_NN_SHAPE");
  // 5: 4 x 1 strided at 8 waves / SIMD, masked kernel too (r02z10/z11: C2 1.83 vs 1.85 ms, C5 0.58 vs 0.66 ms
  // for 4 x 2); 4: the same with the masked kernel at 4 x 2
  a.nn_shape = ns ? atoi(ns) : 5;
  const char *np = getenv("GSKYHIP_NN_PROBE");   // timing-only probes (wrong images): never set in production
  a.nn_probe = np ? atoi(np) : 0;
  const char *nw = getenv("GSKYHIP_NN_WPE");
  a.nn_wpe = nw ? atoi(nw) : 0;
  const char *rp = getenv("GSKYHIP_NN_RPW");
  a.nn_rpw = rp ? atoi(rp) : 4;
  const char *nw2 = getenv("GSKYHIP_NN_WIDE");
  a.nn_wide = nw2 ? atoi(nw2) : 1;
  const char *ne = getenv("GSKYHIP_NN_EXPRESS");
  a.nn_express = ne ? atoi(ne) : 1;
  const char *bk = getenv("GSKYHIP_BIL_KERNEL");
  a.bil_kernel = bk ? atoi(bk) : 5;   // 4 x 1, lane pixels 64 columns apart (r02z6: 1.31-1.34 vs 1.35 ms for 1)
  const char *ng = getenv("GSKYHIP_NN_GEN");
  a.nn_gen = ng ? atoi(ng) : 2;   // render_nn_kernel unless GSKYHIP_NN_GEN=3 (render_nn2_kernel, A/B: measured 2-4 % slower)
  const char *nl = getenv("GSKYHIP_NN_LUT");
  a.nn_lut = nl ? atoi(nl) : 0;   // A/B knob (1: clamped-value LUT; measured 2 % slower on C2, r02z3)
  const char *nsd = getenv("GSKYHIP_NN_STRIDE");
  a.nn_stride = nsd ? atoi(nsd) : 1;   // lane pixels 64 columns apart (0: consecutive; A/B r02z4/5: C2 -2 %, C5 -12 %)
  const char *nx = getenv("GSKYHIP_NN_XCD");
  a.nn_xcd = nx ? atoi(nx) : 0;   // linear item order by default (A/B, profiles/r02g_ab_*.jsonl)
  switch (vt) {
    case GSKYHIP_INT16: launch_lds_i16(a, mask, n_items, s); break;
    case GSKYHIP_UINT16: launch_lds_u16(a, mask, n_items, s); break;
    case GSKYHIP_FLOAT32: launch_lds_f32(a, mask, n_items, s); break;
    case GSKYHIP_SIGNEDBYTE: launch_lds_i8(a, mask, n_items, s); break;
    default: launch_lds_u8(a, mask, n_items, s); break;
  }
}

}  // namespace gsky
