// stages.hip -- the reference's operator boundaries as standalone kernels:
// RasterMerger fold over FlexRasters (tile_merger.go:38-503), ComputeMask
// (314-445), utils.Scale (raster_scaler.go:30-346), the legacy RasterScaler
// (tile_scaler.go:17-112) and the EncodePNG pixel loop (ogc_encoders.go:86-133).
// Elementwise / HBM-bound: one lane per 4 values, 16-byte accesses where the
// element width allows.
#include "gsky_device.h"
#include "stages.h"

namespace gsky {

__device__ __forceinline__ Val load_typed(const void *p, int dtype, long idx) {
  Val v;
  switch (dtype) {
    case GSKYHIP_SIGNEDBYTE: v.i = ((const int8_t *)p)[idx]; break;
    case GSKYHIP_BYTE: v.i = ((const uint8_t *)p)[idx]; break;
    case GSKYHIP_INT16: v.i = ((const int16_t *)p)[idx]; break;
    case GSKYHIP_UINT16: v.i = ((const uint16_t *)p)[idx]; break;
    default: v.u = ((const uint32_t *)p)[idx]; break;
  }
  return v;
}
__device__ __forceinline__ void store_typed(void *p, int dtype, long idx, Val v) {
  switch (dtype) {
    case GSKYHIP_SIGNEDBYTE: case GSKYHIP_BYTE: ((uint8_t *)p)[idx] = (uint8_t)v.i; break;
    case GSKYHIP_INT16: case GSKYHIP_UINT16: ((uint16_t *)p)[idx] = (uint16_t)v.i; break;
    default: ((uint32_t *)p)[idx] = v.u; break;
  }
}

__device__ __forceinline__ bool mask_bit_s(const MaskSpecS &m, int dtype, int32_t v) {
  if (m.has_value) {
    int32_t a = v & m.value;
    switch (dtype) {
      case GSKYHIP_SIGNEDBYTE: return (int8_t)a > 0;
      case GSKYHIP_INT16: return (int16_t)a > 0;
      case GSKYHIP_BYTE: return (uint8_t)a > 0;
      default: return (uint16_t)a > 0;
    }
  }
  for (int j = 0; j < m.n_tests; j++) {
    int32_t a = v & m.filt[j];
    bool eq;
    switch (dtype) {
      case GSKYHIP_SIGNEDBYTE: eq = (int8_t)a == (int8_t)m.want[j]; break;
      case GSKYHIP_INT16: eq = (int16_t)a == (int16_t)m.want[j]; break;
      case GSKYHIP_BYTE: eq = (uint8_t)a == (uint8_t)m.want[j]; break;
      default: eq = (uint16_t)a == (uint16_t)m.want[j]; break;
    }
    if (eq) return true;
  }
  return false;
}

// ---------------------------------------------------------------- merge fold
// One canvas (namespace): every pixel folds the ordered entries that cover it.
__global__ __launch_bounds__(256) void merge_fold_kernel(const FlexEntry *e, int n, int width,
                                                         int height, int canvas_dtype,
                                                         double canvas_nodata, MaskSpecS ms,
                                                         void *canvas) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)width * height) return;
  const int x = (int)(idx % width), y = (int)(idx / width);
  Val c = go_conv_to(canvas_nodata, canvas_dtype);
  for (int k = 0; k < n; k++) {
    const FlexEntry &r = e[k];
    const int ic = x - r.off_x, ir = y - r.off_y;
    if (ic < 0 || ir < 0 || ic >= r.data_w || ir >= r.data_h) continue;
    const long iSrc = (long)ir * r.data_w + ic;
    const Val v = load_typed(r.data, r.dtype, iSrc);
    const Val nd = go_conv_to(r.nodata, r.dtype);
    const bool isf = r.dtype == GSKYHIP_FLOAT32;
    if (val_eq(v, nd, isf)) continue;
    if (r.mask_data) {
      if (iSrc >= r.mask_len) continue;  // host rejects this case beforehand
      const Val mv = load_typed(r.mask_data, r.mask_dtype, iSrc);
      if (mask_bit_s(ms, r.mask_dtype, mv.i)) continue;
    }
    if (r.fill_mode && !val_eq(c, nd, isf)) continue;
    c = v;
  }
  store_typed(canvas, canvas_dtype, idx, c);
}

// ---------------------------------------------------------------- ComputeMask
__global__ void compute_mask_kernel(const void *data, int dtype, long n, MaskSpecS ms, uint8_t *out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = mask_bit_s(ms, dtype, load_typed(data, dtype, i).i) ? 1 : 0;
}

// ---------------------------------------------------------------- Scale
__device__ double go_log10_s(double x);

__device__ __forceinline__ uint8_t scale_one(const ScaleC &k, Val v) {
  if (k.dtype == GSKYHIP_FLOAT32) {
    float value = v.f;
    if (value == k.noData.f) return 0xFF;
    if (k.colour_scale > 0) {
      double d = (double)value;
      if (!(d == k.nodata64)) {
        if (k.colour_scale == 1) d = go_log10_s(d);
        if (isinf(d) || d != d) d = k.nodata64;
      }
      if (d == k.nodata64) return 0xFF;
      value = (float)d;
    }
    value += k.off.f;
    if (value > k.clp.f) value = k.clp.f;
    if (value < 0.0f) value = 0.0f;
    return go_f32_u8(value * k.sc);
  }
  int32_t value = v.i;
  if (value == k.noData.i) return 0xFF;
  switch (k.dtype) {
    case GSKYHIP_SIGNEDBYTE: value = (int8_t)(value + k.off.i); break;
    case GSKYHIP_BYTE: value = (uint8_t)(value + k.off.i); break;
    case GSKYHIP_INT16: value = (int16_t)(value + k.off.i); break;
    default: value = (uint16_t)(value + k.off.i); break;
  }
  if (value > k.clp.i) value = k.clp.i;
  if (value < 0) value = 0;
  return go_f32_u8((float)value * k.sc);
}

__device__ double go_log_s(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (x != x || x == INFINITY) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 1.41421356237309504880168872420969808 / 2) { f1 *= 2; ki--; }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}
__device__ double go_log10_s(double x) {
  int e;
  double frac = frexp(x, &e);
  double l2;
  if (frac == 0.5) l2 = (double)(e - 1);
  else l2 = go_log_s(frac) * (1.0 / 0.693147180559945309417232121458176568) + (double)e;
  return l2 * 0.301029995663981195213738894724493026768189881462108541310;
}

__device__ __forceinline__ int32_t fenc_s(float f) {
  int32_t i = __float_as_int(f);
  return i ^ ((i >> 31) & 0x7FFFFFFF);
}
__device__ __forceinline__ float fdec_s(int32_t i) { return __int_as_float(i ^ ((i >> 31) & 0x7FFFFFFF)); }

// Auto-scale reduction: min/max over valid (normalised) values.
__global__ __launch_bounds__(256) void scale_minmax_kernel(const void *data, int dtype, long n,
                                                           double nodata, int colour_scale,
                                                           int32_t *mm /* mn, mx, p0v, p0 */) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float mn = INFINITY, mx = -INFINITY;
  if (i < n) {
    const Val v = load_typed(data, dtype, i);
    bool valid = true;
    float f;
    if (dtype == GSKYHIP_FLOAT32) {
      f = v.f;
      if (f == (float)nodata) valid = false;
      else if (colour_scale > 0) {
        double d = (double)f;
        if (!(d == nodata)) {
          if (colour_scale == 1) d = go_log10_s(d);
          if (isinf(d) || d != d) d = nodata;
        }
        if (d == nodata) valid = false;
        f = (float)d;
      }
    } else {
      f = (float)v.i;
      if (v.i == go_conv_to(nodata, dtype).i) valid = false;
    }
    if (valid) {
      if (i == 0) { mm[2] = 1; mm[3] = __float_as_int(f); }
      if (f == f) { mn = f; mx = f; }
    }
  }
  int32_t emn = fenc_s(mn), emx = fenc_s(mx);
  for (int o = 32; o > 0; o >>= 1) {
    emn = min(emn, __shfl_xor(emn, o, 64));
    emx = max(emx, __shfl_xor(emx, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    if (emn != fenc_s(INFINITY)) atomicMin(&mm[0], emn);
    if (emx != fenc_s(-INFINITY)) atomicMax(&mm[1], emx);
  }
}

__global__ void scale_finalize_kernel(ScaleC *k, const int32_t *mm, int autom) {
  if (!autom) return;
  float minVal, maxVal;
  if (mm[2]) {
    const float p0 = __int_as_float(mm[3]);
    if (p0 != p0) { minVal = p0; maxVal = p0; }
    else { minVal = fdec_s(mm[0]); maxVal = fdec_s(mm[1]); }
  } else {
    minVal = fminf(0.0f, fdec_s(mm[0]));
    maxVal = fmaxf(0.0f, fdec_s(mm[1]));
  }
  if (minVal == maxVal) maxVal += 0.1f;
  k->sc = 254.0f / (maxVal - minVal);
  if (k->dtype == GSKYHIP_FLOAT32) {
    k->off.f = -minVal;
    k->clp.f = maxVal + k->off.f;
  } else {
    const float dfOffset = -minVal;
    k->off = go_conv_to((double)dfOffset, k->dtype);
    k->clp = go_conv_to((double)(maxVal + dfOffset), k->dtype);
  }
}

__global__ __launch_bounds__(256) void scale_apply_kernel(void *data, int dtype, long n, const ScaleC *kp,
                                                          uint8_t *out, int inplace_byte) {
  const ScaleC k = *kp;
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= n) return;
  uint8_t b[4];
#pragma unroll
  for (int q = 0; q < 4; q++) b[q] = (i0 + q < n) ? scale_one(k, load_typed(data, dtype, i0 + q)) : 0;
  if (i0 + 3 < n && ((((uintptr_t)(out + i0)) & 3) == 0)) {
    *(uint32_t *)(out + i0) = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
  } else {
    for (int q = 0; q < 4 && i0 + q < n; q++) out[i0 + q] = b[q];
  }
  if (inplace_byte)
    for (int q = 0; q < 4 && i0 + q < n; q++) ((uint8_t *)data)[i0 + q] = b[q];
}

// processor/tile_scaler.go:17-112
__global__ void scale_legacy_kernel(void *data, int dtype, long n, double nodata, double offset,
                                    double scale, double clip, uint8_t *out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (dtype) {
    case GSKYHIP_BYTE: {
      uint8_t value = ((uint8_t *)data)[i];
      uint8_t o;
      if (value == go_u8(nodata)) o = 0xFF;
      else {
        const uint8_t clp = go_u8(clip);
        if (value > clp) value = clp;
        o = go_u8((double)value * scale);
      }
      ((uint8_t *)data)[i] = o;
      out[i] = o;
      break;
    }
    case GSKYHIP_INT16: {
      int16_t value = ((int16_t *)data)[i];
      if (value == go_i16(nodata)) { out[i] = 0xFF; break; }
      const int16_t clp = go_i16(clip);
      if (value > clp) value = clp;
      if (value < 0) value = 0;
      out[i] = go_f32_u8((float)value * 254.0f / (float)clp);
      break;
    }
    case GSKYHIP_UINT16: {
      uint16_t value = ((uint16_t *)data)[i];
      if (value == go_u16(nodata)) { out[i] = 0xFF; break; }
      const uint16_t clp = go_u16(clip);
      if (value > clp) value = clp;
      out[i] = go_f32_u8((float)value * 254.0f / (float)clp);
      break;
    }
    case GSKYHIP_FLOAT32: {
      float value = ((float *)data)[i];
      if (value == (float)nodata) { out[i] = 0xFF; break; }
      value += (float)go_u8(offset);
      if (value > (float)clip) value = (float)clip;
      if (value < 0) value = 0;
      out[i] = go_f32_u8(value * (float)scale);
      break;
    }
    default: break;
  }
}

// EncodePNG pixel loop (ogc_encoders.go:86-133)
__global__ __launch_bounds__(256) void encode_rgba_kernel(const uint8_t *b0, const uint8_t *b1,
                                                          const uint8_t *b2, int nbands, long npx,
                                                          const uint32_t *ramp, uint32_t *rgba) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npx) return;
  uint32_t o = 0;
  if (nbands == 1) {
    const uint8_t v = b0[i];
    if (v != 0xFF) o = ramp ? ramp[v] : (0xFF000000u | ((uint32_t)v << 16) | ((uint32_t)v << 8) | v);
  } else {
    const uint8_t r = b0[i], g = b1[i], b = b2[i];
    if (r != 0xFF || g != 0xFF || b != 0xFF) o = 0xFF000000u | ((uint32_t)b << 16) | ((uint32_t)g << 8) | r;
  }
  rgba[i] = o;
}

}  // namespace gsky

// ======================================================================== host
namespace gsky {

static inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

int launch_merge_fold(const FlexEntry *entries_host, int n, int width, int height, int canvas_dtype,
                      double canvas_nodata, const MaskSpecS &ms, void *canvas, hipStream_t s) {
  const int64_t npx = (int64_t)width * height;
  if (npx <= 0) return 0;
  FlexEntry *d = nullptr;
  const size_t bytes = sizeof(FlexEntry) * (size_t)(n > 0 ? n : 1);
  if (hipMallocAsync((void **)&d, bytes, s) != hipSuccess) return GSKYHIP_E_HIP;
  if (n > 0 && hipMemcpyAsync(d, entries_host, sizeof(FlexEntry) * n, hipMemcpyHostToDevice, s) != hipSuccess)
    return GSKYHIP_E_HIP;
  hipLaunchKernelGGL(merge_fold_kernel, dim3(blocks_for(npx, 256)), dim3(256), 0, s, d, n, width, height,
                     canvas_dtype, canvas_nodata, ms, canvas);
  const bool launched = hipGetLastError() == hipSuccess;
  const bool freed = hipFreeAsync(d, s) == hipSuccess;
  return launched && freed ? 0 : GSKYHIP_E_HIP;
}

int launch_compute_mask(const void *data, int dtype, int64_t n, const MaskSpecS &ms, uint8_t *out,
                        hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(compute_mask_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, data, dtype, (long)n,
                     ms, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

ScaleC host_scale_consts(int dtype, double nodata, const gskyhip_scale_params &sp) {
  ScaleC k;
  k.dtype = dtype;
  k.colour_scale = sp.colour_scale;
  k.nodata64 = nodata;
  float sc = (float)sp.scale;                                  // raster_scaler.go:31-38
  if (sc <= 0.0f) sc = (sp.clip <= 0.0) ? 1.0f : (float)(254.0f / (float)sp.clip);
  k.sc = sc;
  k.noData = go_conv_to(nodata, dtype);
  if (dtype == GSKYHIP_FLOAT32) {
    k.off.f = (float)sp.offset;
    k.clp.f = (float)sp.clip;
  } else {
    k.off = go_conv_to(sp.offset, dtype);
    k.clp = go_conv_to(sp.clip, dtype);
  }
  return k;
}

int launch_scale(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params &sp,
                 uint8_t *out, hipStream_t s) {
  if (!(dtype == GSKYHIP_SIGNEDBYTE || dtype == GSKYHIP_BYTE || dtype == GSKYHIP_INT16 ||
        dtype == GSKYHIP_UINT16 || dtype == GSKYHIP_FLOAT32))
    return GSKYHIP_E_TYPE;                                     // raster_scaler.go:329-331
  if (n <= 0) return 0;
  const bool autom = sp.scale == 0.0 && sp.clip == 0.0 && sp.offset == 0.0;
  struct Buf { ScaleC k; int32_t mm[4]; };
  Buf h;
  h.k = host_scale_consts(dtype, nodata, sp);
  h.mm[0] = 0x7F800000;                     // fenc(+inf)
  h.mm[1] = (int32_t)(0xFF800000u ^ 0x7FFFFFFFu);  // fenc(-inf)
  h.mm[2] = 0;
  h.mm[3] = 0;
  Buf *d = nullptr;
  if (hipMallocAsync((void **)&d, sizeof(Buf), s) != hipSuccess) return GSKYHIP_E_HIP;
  if (hipMemcpyAsync(d, &h, sizeof(Buf), hipMemcpyHostToDevice, s) != hipSuccess) {
    (void)hipFreeAsync(d, s);
    return GSKYHIP_E_HIP;
  }
  if (autom) {
    hipLaunchKernelGGL(scale_minmax_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, data, dtype, (long)n,
                       nodata, sp.colour_scale, d->mm);
    hipLaunchKernelGGL(scale_finalize_kernel, dim3(1), dim3(1), 0, s, &d->k, d->mm, 1);
  }
  hipLaunchKernelGGL(scale_apply_kernel, dim3(blocks_for((n + 3) / 4, 256)), dim3(256), 0, s, data, dtype,
                     (long)n, &d->k, out, dtype == GSKYHIP_BYTE ? 1 : 0);
  const bool launched = hipGetLastError() == hipSuccess;
  const bool freed = hipFreeAsync(d, s) == hipSuccess;
  const bool synced = hipStreamSynchronize(s) == hipSuccess;   // host staging struct `h` must outlive the copy
  return launched && freed && synced ? 0 : GSKYHIP_E_HIP;
}

int launch_scale_legacy(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params &sp,
                        uint8_t *out, hipStream_t s) {
  if (!(dtype == GSKYHIP_BYTE || dtype == GSKYHIP_INT16 || dtype == GSKYHIP_UINT16 ||
        dtype == GSKYHIP_FLOAT32))
    return GSKYHIP_E_TYPE;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_legacy_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, data, dtype, (long)n,
                     nodata, sp.offset, sp.scale, sp.clip, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_encode_rgba(const uint8_t *b0, const uint8_t *b1, const uint8_t *b2, int nbands, int64_t npx,
                       const uint8_t *ramp, uint8_t *rgba, hipStream_t s) {
  if (nbands != 1 && nbands != 3) return GSKYHIP_E_ARG;
  if (npx <= 0) return 0;
  hipLaunchKernelGGL(encode_rgba_kernel, dim3(blocks_for(npx, 256)), dim3(256), 0, s, b0, b1, b2, nbands,
                     (long)npx, (const uint32_t *)ramp, (uint32_t *)rgba);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
