/*
 * gsky_oracle.c -- CPU restatement of GSKY's raster hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gsky_oracle.h).  Built with
 * -O2 -ffp-contract=off so every double expression rounds exactly as the
 * x86-64 SSE2 code of the reference (Go gc / GDAL built without -mfma).
 *
 * Reference citations are file:line under chuc92man/gsky; [ext] marks the
 * restated algorithm of an un-vendored dependency (GDAL 3.0.1, PROJ 6.1.1,
 * Go 1.12 runtime/strconv/math).
 */
#define _GNU_SOURCE
#include "gsky_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

int oracle_type_size(int dtype) {
    switch (dtype) {
    case OR_BYTE: case OR_SIGNEDBYTE: return 1;
    case OR_UINT16: case OR_INT16: return 2;
    case OR_UINT32: case OR_INT32: case OR_FLOAT32: return 4;
    case OR_FLOAT64: return 8;
    default: return 0;
    }
}

/* ======================================================================== */
/* Go 1.12 amd64 conversions [ext]: float -> int{8,16}/uint{8,16} is        */
/* CVTTSD2SL / CVTTSS2SL to int32 (NaN or out of range -> 0x80000000)       */
/* followed by truncation to the narrow type.                               */
/* ======================================================================== */
static int32_t go_cvtt32(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int32_t)x;
}
int8_t   or_go_f64_i8(double v)  { return (int8_t)(uint8_t)(uint32_t)go_cvtt32(v); }
uint8_t  or_go_f64_u8(double v)  { return (uint8_t)(uint32_t)go_cvtt32(v); }
int16_t  or_go_f64_i16(double v) { return (int16_t)(uint16_t)(uint32_t)go_cvtt32(v); }
uint16_t or_go_f64_u16(double v) { return (uint16_t)(uint32_t)go_cvtt32(v); }
int8_t   or_go_f32_i8(float v)   { return or_go_f64_i8((double)v); }
uint8_t  or_go_f32_u8(float v)   { return or_go_f64_u8((double)v); }
int16_t  or_go_f32_i16(float v)  { return or_go_f64_i16((double)v); }
uint16_t or_go_f32_u16(float v)  { return or_go_f64_u16((double)v); }

/* GDALCopyWord(double -> T) [ext, gdal_priv_templates.hpp]: integer targets
 * round half away from zero and saturate, NaN -> 0; float32 saturates at
 * +-FLT_MAX (infinities kept). */
static double gdal_round_clamp(double v, double lo, double hi) {
    if (isnan(v)) return 0.0;
    double r = v >= 0.0 ? v + 0.5 : v - 0.5;
    if (r > hi) r = hi;
    if (r < lo) r = lo;
    return trunc(r);
}
void or_gdal_copy_word(double v, int dtype, void *out) {
    switch (dtype) {
    case OR_BYTE: case OR_SIGNEDBYTE: { uint8_t o = (uint8_t)gdal_round_clamp(v, 0, 255); memcpy(out, &o, 1); break; }
    case OR_UINT16: { uint16_t o = (uint16_t)gdal_round_clamp(v, 0, 65535); memcpy(out, &o, 2); break; }
    case OR_INT16: { int16_t o = (int16_t)gdal_round_clamp(v, -32768, 32767); memcpy(out, &o, 2); break; }
    case OR_UINT32: { uint32_t o = (uint32_t)gdal_round_clamp(v, 0, 4294967295.0); memcpy(out, &o, 4); break; }
    case OR_INT32: { int32_t o = (int32_t)gdal_round_clamp(v, -2147483648.0, 2147483647.0); memcpy(out, &o, 4); break; }
    case OR_FLOAT32: {
        float o;
        if (isinf(v)) o = (float)v;
        else if (v > FLT_MAX) o = FLT_MAX;
        else if (v < -FLT_MAX) o = -FLT_MAX;
        else o = (float)v;
        memcpy(out, &o, 4); break;
    }
    case OR_FLOAT64: memcpy(out, &v, 8); break;
    default: break;
    }
}

/* ======================================================================== */
/* Go math.Log / Log10 [ext: Go 1.12 math/log.go, log10.go; the amd64        */
/* assembly runs the same FreeBSD sequence].                                */
/* ======================================================================== */
static double go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    if (isnan(x) || (isinf(x) && x > 0)) return x;
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
static double go_log2(double x) {
    int e;
    double frac = frexp(x, &e);
    if (frac == 0.5) return (double)(e - 1);
    return go_log(frac) * (1.0 / 0.693147180559945309417232121458176568) + (double)e;
}
static double go_log10(double x) {
    /* Ln2/Ln10 is an exact Go constant expression rounded once to float64. */
    return go_log2(x) * 0.301029995663981195213738894724493026768189881462108541310;
}

/* utils/raster_scaler.go:15-28 normalise() */
static double go_normalise(double val, int colour_scale, double nodata) {
    if (val == nodata) return val;
    double v = val;
    if (colour_scale == 1) v = go_log10(val); /* ColourLogScale, utils/config.go:34 */
    if (isinf(v) || isnan(v)) v = nodata;
    return v;
}

/* ======================================================================== */
/* utils/raster_scaler.go:30-332  scale()                                   */
/* ======================================================================== */
#define SCALE_INT_CASE(T, CONV32, CONV64)                                          \
    do {                                                                           \
        T *d = (T *)data;                                                          \
        T noData = CONV64(nodata);                                                 \
        T off = CONV64(offset);                                                    \
        T clp = CONV64(clip);                                                      \
        if (autom) {                                                               \
            float minVal = 0.0f, maxVal = 0.0f;                                    \
            for (int64_t i = 0; i < n; i++) {                                      \
                T value = d[i];                                                    \
                if (value == noData) continue;                                     \
                float val = (float)value;                                          \
                if (i == 0) { minVal = val; maxVal = val; }                        \
                else { if (val < minVal) minVal = val; if (val > maxVal) maxVal = val; } \
            }                                                                      \
            if (minVal == maxVal) maxVal += 0.1f;                                  \
            sc = 254.0f / (maxVal - minVal);                                       \
            float dfOffset = -minVal;                                              \
            off = CONV32(dfOffset);                                                \
            clp = CONV32(maxVal + dfOffset);                                       \
        }                                                                          \
        for (int64_t i = 0; i < n; i++) {                                          \
            T value = d[i];                                                        \
            if (value == noData) { out[i] = 0xFF; continue; }                      \
            value = (T)(value + off);                                              \
            if (value > clp) value = clp;                                          \
            if (value < 0) value = 0;                                              \
            out[i] = or_go_f32_u8((float)value * sc);                              \
        }                                                                          \
    } while (0)

int oracle_scale(void *data, int dtype, int64_t n, double nodata,
                 double offset, double scale, double clip, int colour_scale,
                 uint8_t *out) {
    float sc = (float)scale;                               /* 31 */
    if (sc <= 0.0f) {
        if (clip <= 0.0) sc = 1.0f;
        else sc = (float)(254.0f / (float)clip);           /* 36 */
    }
    const int autom = (scale == 0.0 && clip == 0.0 && offset == 0.0);
    switch (dtype) {
    case OR_SIGNEDBYTE: SCALE_INT_CASE(int8_t, or_go_f32_i8, or_go_f64_i8); return 0;   /* 41-94 */
    case OR_BYTE: {                                                                       /* 96-148 */
        /* scaled in place: the input raster is overwritten */
        SCALE_INT_CASE(uint8_t, or_go_f32_u8, or_go_f64_u8);
        memcpy(data, out, (size_t)n);
        return 0;
    }
    case OR_INT16: SCALE_INT_CASE(int16_t, or_go_f32_i16, or_go_f64_i16); return 0;     /* 150-203 */
    case OR_UINT16: SCALE_INT_CASE(uint16_t, or_go_f32_u16, or_go_f64_u16); return 0;   /* 205-258 */
    case OR_FLOAT32: {                                                                    /* 260-327 */
        float *d = (float *)data;
        float noData = (float)nodata;
        float off = (float)offset;
        float clp = (float)clip;
        if (autom) {
            float minVal = 0.0f, maxVal = 0.0f;
            for (int64_t i = 0; i < n; i++) {
                float value = d[i];
                if (value == noData) continue;
                if (colour_scale > 0) {
                    double v = go_normalise((double)value, colour_scale, nodata);
                    if (v == nodata) continue;
                    value = (float)v;
                }
                if (i == 0) { minVal = value; maxVal = value; }
                else { if (value < minVal) minVal = value; if (value > maxVal) maxVal = value; }
            }
            if (minVal == maxVal) maxVal += 0.1f;
            sc = 254.0f / (maxVal - minVal);
            off = -minVal;
            clp = maxVal + off;
        }
        for (int64_t i = 0; i < n; i++) {
            float value = d[i];
            if (value == noData) { out[i] = 0xFF; continue; }
            if (colour_scale > 0) {
                double v = go_normalise((double)value, colour_scale, nodata);
                if (v == nodata) { out[i] = 0xFF; continue; }
                value = (float)v;
            }
            value += off;
            if (value > clp) value = clp;
            if (value < 0.0f) value = 0.0f;
            out[i] = or_go_f32_u8(value * sc);
        }
        return 0;
    }
    default:
        return -1;
    }
}

/* processor/tile_scaler.go:17-112 (no callers in the reference) */
int oracle_scale_legacy(void *data, int dtype, int64_t n, double nodata,
                        double offset, double scale, double clip, uint8_t *out) {
    switch (dtype) {
    case OR_BYTE: {                                           /* 22-40 */
        uint8_t *d = (uint8_t *)data;
        uint8_t noData = or_go_f64_u8(nodata);
        uint8_t clp = or_go_f64_u8(clip);
        for (int64_t i = 0; i < n; i++) {
            uint8_t value = d[i];
            if (value == noData) { d[i] = 0xFF; }
            else {
                if (value > clp) value = clp;
                d[i] = or_go_f64_u8((double)value * scale);
            }
            out[i] = d[i];
        }
        return 0;
    }
    case OR_INT16: {                                          /* 42-62 */
        int16_t *d = (int16_t *)data;
        int16_t noData = or_go_f64_i16(nodata);
        int16_t clp = or_go_f64_i16(clip);
        for (int64_t i = 0; i < n; i++) {
            int16_t value = d[i];
            if (value == noData) { out[i] = 0xFF; continue; }
            if (value > clp) value = clp;
            if (value < 0) value = 0;
            out[i] = or_go_f32_u8((float)value * 254.0f / (float)clp);
        }
        return 0;
    }
    case OR_UINT16: {                                         /* 64-84 */
        uint16_t *d = (uint16_t *)data;
        uint16_t noData = or_go_f64_u16(nodata);
        uint16_t clp = or_go_f64_u16(clip);
        for (int64_t i = 0; i < n; i++) {
            uint16_t value = d[i];
            if (value == noData) { out[i] = 0xFF; continue; }
            if (value > clp) value = clp;
            out[i] = or_go_f32_u8((float)value * 254.0f / (float)clp);
        }
        return 0;
    }
    case OR_FLOAT32: {                                        /* 86-108 */
        float *d = (float *)data;
        float noData = (float)nodata;
        float sc = (float)scale;
        uint8_t off = or_go_f64_u8(offset);
        float clp = (float)clip;
        for (int64_t i = 0; i < n; i++) {
            float value = d[i];
            if (value == noData) { out[i] = 0xFF; continue; }
            value += (float)off;
            if (value > clp) value = clp;
            if (value < 0) value = 0;
            out[i] = or_go_f32_u8(value * sc);
        }
        return 0;
    }
    default:
        return -1;
    }
}

/* ======================================================================== */
/* utils/palette.go:11-69                                                    */
/* ======================================================================== */
static uint8_t interp_u8(uint8_t a, uint8_t b, long i, long section) {
    /* Go int arithmetic, truncating division, uint8 wrap (palette.go:11-13) */
    long q = (i * ((long)b - (long)a)) / section;
    return (uint8_t)(a + (uint8_t)q);
}

int oracle_gradient_palette(const uint8_t *colours, int n, int interpolate, uint8_t *ramp) {
    if (interpolate) {
        if (n < 2) return -1;
        int bins = n - 1;
        int sectionLength = 256 / bins;
        if (sectionLength == 0) return -1;  /* Go: integer divide by zero panic (palette.go:12) */
        int bonus = 256 - sectionLength * bins;
        int index = 0;
        for (int section = 0; section < bins; section++) {
            const uint8_t *a = colours + 4 * section, *b = colours + 4 * (section + 1);
            int cnt = sectionLength + (section < bonus ? 1 : 0);
            for (int i = 0; i < cnt; i++) {
                uint8_t *o = ramp + 4 * index;
                o[0] = interp_u8(a[0], b[0], i, sectionLength);
                o[1] = interp_u8(a[1], b[1], i, sectionLength);
                o[2] = interp_u8(a[2], b[2], i, sectionLength);
                o[3] = a[3];                           /* alpha of the lower colour (22) */
                index++;
            }
        }
    } else {
        if (n < 1) return -1;
        int bins = n;
        int sectionLength = 256 / bins;
        int bonus = 256 - sectionLength * bins;
        int index = 0;
        for (int section = 0; section < bins; section++) {
            int cnt = sectionLength + (section < bonus ? 1 : 0);
            for (int i = 0; i < cnt; i++) {
                memcpy(ramp + 4 * index, colours + 4 * section, 4);
                index++;
            }
        }
    }
    return 0;
}

int oracle_encode_rgba(const uint8_t *const *bands, int nbands, int w, int h,
                       const uint8_t *ramp, uint8_t *rgba) {
    const int64_t npx = (int64_t)w * h;
    memset(rgba, 0, (size_t)npx * 4);                  /* image.NewRGBA */
    if (nbands == 1) {
        const uint8_t *b = bands[0];
        for (int64_t i = 0; i < npx; i++) {
            uint8_t v = b[i];
            if (v == 0xFF) continue;
            if (ramp) memcpy(rgba + 4 * i, ramp + 4 * v, 4);          /* 94-100 */
            else { rgba[4*i] = v; rgba[4*i+1] = v; rgba[4*i+2] = v; rgba[4*i+3] = 0xFF; } /* 102-112 */
        }
        return 0;
    }
    if (nbands == 3) {                                                  /* 115-133 */
        for (int64_t i = 0; i < npx; i++) {
            if (bands[0][i] != 0xFF || bands[1][i] != 0xFF || bands[2][i] != 0xFF) {
                rgba[4*i] = bands[0][i]; rgba[4*i+1] = bands[1][i];
                rgba[4*i+2] = bands[2][i]; rgba[4*i+3] = 0xFF;
            }
        }
        return 0;
    }
    return -1;                                                          /* 135-136 */
}

/* ======================================================================== */
/* processor/tile_merger.go                                                 */
/* ======================================================================== */
uint32_t oracle_fnv32a(const char *s, size_t n) {     /* Go hash/fnv New32a [ext] */
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; i++) { h ^= (uint8_t)s[i]; h *= 16777619u; }
    return h;
}

/* strconv.ParseUint / ParseInt (base 2) of Go 1.12 [ext], errors ignored by
 * the caller exactly as tile_merger.go:332-431 does (value returned anyway). */
static uint64_t go_parse_uint2(const char *s, int bits) {
    uint64_t maxVal = (bits >= 64) ? UINT64_MAX : ((1ull << bits) - 1);
    if (!s || !*s) return 0;
    uint64_t n = 0;
    const uint64_t cutoff = UINT64_MAX / 2 + 1;
    for (const char *p = s; *p; p++) {
        int d;
        char c = *p;
        if (c >= '0' && c <= '9') d = c - '0';
        else if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') d = (c | 0x20) - 'a' + 10;
        else return 0;
        if (d >= 2) return 0;
        if (n >= cutoff) return maxVal;
        n *= 2;
        uint64_t n1 = n + (uint64_t)d;
        if (n1 < n || n1 > maxVal) return maxVal;
        n = n1;
    }
    return n;
}
static int64_t go_parse_int2(const char *s, int bits) {
    if (!s || !*s) return 0;
    int neg = 0;
    if (*s == '+') s++;
    else if (*s == '-') { neg = 1; s++; }
    /* ParseUint with a syntax error -> 0 */
    uint64_t maxVal = (1ull << bits) - 1;
    uint64_t un;
    {
        if (!*s) return 0;
        uint64_t n = 0; int syntax = 0, range = 0;
        for (const char *p = s; *p; p++) {
            char c = *p; int d;
            if (c >= '0' && c <= '9') d = c - '0';
            else if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') d = (c | 0x20) - 'a' + 10;
            else { syntax = 1; break; }
            if (d >= 2) { syntax = 1; break; }
            if (n >= UINT64_MAX / 2 + 1) { n = maxVal; range = 1; break; }
            n *= 2;
            uint64_t n1 = n + (uint64_t)d;
            if (n1 < n || n1 > maxVal) { n = maxVal; range = 1; break; }
            n = n1;
        }
        if (syntax) return 0;
        (void)range;
        un = n;
    }
    uint64_t cutoff = 1ull << (bits - 1);
    if (!neg && un >= cutoff) return (int64_t)(cutoff - 1);
    if (neg && un > cutoff) return -(int64_t)cutoff;
    int64_t r = (int64_t)un;
    return neg ? -r : r;
}

int oracle_compute_mask(const void *data, int dtype, int64_t n,
                        const char *value, const char *const *bit_tests,
                        int n_bit_tests, uint8_t *out) {
    const int has_value = value && *value;
    if (!has_value) {                                    /* 315-323 */
        if (n_bit_tests == 0) return -1;
        if (n_bit_tests % 2 != 0) return -1;
    }
#define MASK_CASE(T, UNSIGNED_VALUE, PARSE_BITS, POSITIVE)                                \
    do {                                                                                   \
        const T *d = (const T *)data;                                                      \
        if (has_value) {                                                                   \
            T mv = UNSIGNED_VALUE ? (T)go_parse_uint2(value, PARSE_BITS)                   \
                                  : (T)go_parse_int2(value, PARSE_BITS);                   \
            for (int64_t i = 0; i < n; i++) { T a = (T)(d[i] & mv); out[i] = POSITIVE(a); } \
        } else {                                                                           \
            for (int64_t i = 0; i < n; i++) {                                              \
                out[i] = 0;                                                                \
                for (int j = 0; j < n_bit_tests; j += 2) {                                 \
                    T f = (T)go_parse_int2(bit_tests[j], PARSE_BITS);                      \
                    T v = (T)go_parse_int2(bit_tests[j + 1], PARSE_BITS);                  \
                    if ((T)(d[i] & f) == v) { out[i] = 1; break; }                          \
                }                                                                          \
            }                                                                              \
        }                                                                                  \
    } while (0)
#define POS_SIGNED(a) ((a) > 0 ? 1 : 0)
#define POS_UNSIGNED(a) ((a) > 0 ? 1 : 0)
    switch (dtype) {
    case OR_SIGNEDBYTE: MASK_CASE(int8_t, 1, 8, POS_SIGNED); return 0;   /* 328-354 */
    case OR_BYTE: MASK_CASE(uint8_t, 1, 8, POS_UNSIGNED); return 0;      /* 355-381 */
    case OR_INT16: MASK_CASE(int16_t, 0, 16, POS_SIGNED); return 0;      /* 382-410: ParseInt */
    case OR_UINT16: MASK_CASE(uint16_t, 1, 16, POS_UNSIGNED); return 0;  /* 411-439 */
    default: return -2;                                                   /* 440-442 */
    }
}

static void init_nodata(void *buf, int dtype, double nodata, int64_t n) {   /* 227-279 */
    switch (dtype) {
    case OR_SIGNEDBYTE: { int8_t f = or_go_f64_i8(nodata); for (int64_t i = 0; i < n; i++) ((int8_t *)buf)[i] = f; break; }
    case OR_BYTE: { uint8_t f = or_go_f64_u8(nodata); for (int64_t i = 0; i < n; i++) ((uint8_t *)buf)[i] = f; break; }
    case OR_INT16: { int16_t f = or_go_f64_i16(nodata); for (int64_t i = 0; i < n; i++) ((int16_t *)buf)[i] = f; break; }
    case OR_UINT16: { uint16_t f = or_go_f64_u16(nodata); for (int64_t i = 0; i < n; i++) ((uint16_t *)buf)[i] = f; break; }
    case OR_FLOAT32: { float f = (float)nodata; for (int64_t i = 0; i < n; i++) ((float *)buf)[i] = f; break; }
    default: break;
    }
}

/* MergeMaskedRaster tile_merger.go:38-225 */
static int merge_masked_raster(const oracle_flex_raster *r, oracle_canvas *cv,
                               const uint8_t *mask, int64_t mask_len) {
    if (r->dtype != cv->dtype) return -4;  /* the reference would reinterpret bytes */
    if ((int64_t)r->data_w * r->data_h > mask_len) return -3; /* Go would panic */
    const int fill = r->timestamp < cv->timestamp;
#define MERGE_CASE(T, NODATA)                                                       \
    do {                                                                            \
        T *canvas = (T *)cv->data;                                                  \
        const T *data = (const T *)r->data;                                         \
        T nodata = NODATA;                                                          \
        int64_t iSrc = 0;                                                           \
        for (int ir = 0; ir < r->data_h; ir++) {                                    \
            for (int ic = 0; ic < r->data_w; ic++) {                                \
                T val = data[iSrc];                                                 \
                int64_t iDst = (int64_t)(ir + r->off_y) * r->width + ic + r->off_x; \
                if (fill) {                                                         \
                    if (val != nodata && !mask[iSrc] && canvas[iDst] == nodata)     \
                        canvas[iDst] = val;                                         \
                } else {                                                            \
                    if (val != nodata && !mask[iSrc]) canvas[iDst] = val;           \
                }                                                                   \
                iSrc++;                                                             \
            }                                                                       \
        }                                                                           \
    } while (0)
    switch (r->dtype) {
    case OR_SIGNEDBYTE: MERGE_CASE(int8_t, or_go_f64_i8(r->nodata)); break;
    case OR_BYTE: MERGE_CASE(uint8_t, or_go_f64_u8(r->nodata)); break;
    case OR_INT16: MERGE_CASE(int16_t, or_go_f64_i16(r->nodata)); break;
    case OR_UINT16: MERGE_CASE(uint16_t, or_go_f64_u16(r->nodata)); break;
    case OR_FLOAT32: MERGE_CASE(float, (float)r->nodata); break;
    default: return -5;                                               /* 221-223 */
    }
    if (!fill) cv->timestamp = r->timestamp;
    return 0;
}

typedef struct { double key; int first; } stack_key;
static int cmp_key_desc(const void *a, const void *b) {
    double x = ((const stack_key *)a)->key, y = ((const stack_key *)b)->key;
    return (x > y) ? -1 : (x < y) ? 1 : 0;
}

int oracle_merge_batch(const oracle_flex_raster *rasters, int n,
                       int mask_ns, const char *mask_value,
                       const char *const *bit_tests, int n_bit_tests,
                       int mask_inclusive, oracle_canvas *canvases, int n_ns) {
    int rc = 0;
    double *stamp = (double *)malloc(sizeof(double) * (n > 0 ? n : 1));
    int *in_stack = (int *)calloc(n > 0 ? n : 1, sizeof(int));
    uint8_t **masks = (uint8_t **)calloc(n > 0 ? n : 1, sizeof(uint8_t *));
    int64_t *mask_len = (int64_t *)calloc(n > 0 ? n : 1, sizeof(int64_t));
    stack_key *keys = (stack_key *)malloc(sizeof(stack_key) * (n > 0 ? n : 1));
    int nkeys = 0;
    /* tile_merger.go:468-492 */
    for (int i = 0; i < n; i++) {
        const oracle_flex_raster *r = &rasters[i];
        stamp[i] = r->timestamp + (double)r->polygon_hash;
        if (mask_ns >= 0 && r->ns == mask_ns) {
            int64_t len = (int64_t)r->data_w * r->data_h;
            masks[i] = (uint8_t *)malloc(len > 0 ? len : 1);
            mask_len[i] = len;
            rc = oracle_compute_mask(r->data, r->dtype, len, mask_value, bit_tests, n_bit_tests, masks[i]);
            if (rc) goto done;
            if (!mask_inclusive) continue;
        }
        in_stack[i] = 1;
        int found = 0;
        for (int k = 0; k < nkeys; k++) if (keys[k].key == stamp[i]) { found = 1; break; }
        if (!found) { keys[nkeys].key = stamp[i]; keys[nkeys].first = i; nkeys++; }
    }
    /* ProcessRasterStack 281-312: keys sorted descending */
    qsort(keys, nkeys, sizeof(stack_key), cmp_key_desc);
    for (int k = 0; k < nkeys; k++) {
        const double key = keys[k].key;
        /* maskMap[geoStamp]: last mask raster stored under that key wins */
        const uint8_t *mask = NULL; int64_t mlen = 0;
        for (int i = 0; i < n; i++)
            if (masks[i] && stamp[i] == key) { mask = masks[i]; mlen = mask_len[i]; }
        for (int i = 0; i < n; i++) {
            if (!in_stack[i] || stamp[i] != key) continue;
            const oracle_flex_raster *r = &rasters[i];
            if (r->ns < 0 || r->ns >= n_ns) { rc = -6; goto done; }
            oracle_canvas *cv = &canvases[r->ns];
            if (!cv->created) {                                      /* 291-297 */
                cv->created = 1;
                cv->dtype = r->dtype;
                cv->nodata = r->nodata;
                cv->timestamp = 0;
                init_nodata(cv->data, r->dtype, r->nodata, (int64_t)r->width * r->height);
            }
            uint8_t *zero = NULL;
            const uint8_t *m = mask; int64_t ml = mlen;
            if (!m) {                                               /* 300-302 */
                ml = (int64_t)r->height * r->width;
                zero = (uint8_t *)calloc(ml > 0 ? ml : 1, 1);
                m = zero;
            }
            rc = merge_masked_raster(r, cv, m, ml);
            free(zero);
            if (rc) goto done;
        }
    }
done:
    for (int i = 0; i < n; i++) free(masks[i]);
    free(masks); free(mask_len); free(stamp); free(in_stack); free(keys);
    return rc;
}

/* ======================================================================== */
/* Projections [ext: PROJ 6.1.1 pj_fwd/pj_inv wrappers, merc.cpp (webmerc),   */
/* aea.cpp, gn_sinu.cpp; GDAL 3 traditional GIS axis order].                */
/* ======================================================================== */
#define OR_HALFPI 1.57079632679489661923
#define OR_PI 3.14159265358979323846
#define OR_TWOPI 6.2831853071795864769
#define OR_FORTPI 0.78539816339744830962
#define OR_D2R 0.017453292519943295769236907684886
#define OR_R2D (1.0 / 0.017453292519943295769236907684886)

static double adjlon(double lon) {
    if (fabs(lon) < OR_PI + 1e-12) return lon;
    lon += OR_PI;
    lon -= OR_TWOPI * floor(lon / OR_TWOPI);
    lon -= OR_PI;
    return lon;
}
static double pj_qsfn(double sinphi, double e, double one_es) {
    if (e >= 1.0e-7) {
        double con = e * sinphi;
        double div1 = 1.0 - con * con;
        double div2 = 1.0 + con;
        if (div1 == 0.0 || div2 == 0.0) return HUGE_VAL;
        return one_es * (sinphi / div1 - (.5 / e) * log((1. - con) / div2));
    }
    return sinphi + sinphi;
}
static double pj_msfn(double sinphi, double cosphi, double es) {
    return cosphi / sqrt(1. - es * sinphi * sinphi);
}
static double aea_phi1(double qs, double Te, double Tone_es) {
    double Phi = asin(.5 * qs);
    if (Te < 1.0e-7) return Phi;
    int i = 15;
    double dphi;
    do {
        double sinpi = sin(Phi), cospi = cos(Phi);
        double con = Te * sinpi;
        double com = 1. - con * con;
        dphi = .5 * com * com / cospi *
               (qs / Tone_es - sinpi / com + .5 / Te * log((1. - con) / (1. + con)));
        Phi += dphi;
    } while (fabs(dphi) > 1.0e-10 && --i);
    return i ? Phi : HUGE_VAL;
}

static void set_ellps(oracle_crs *c, double a, double rf) {
    c->a = a;
    c->ra = 1.0 / a;
    if (rf == 0.0) { c->es = 0.0; }
    else { double f = 1.0 / rf; c->es = 2 * f - f * f; }
    c->e = sqrt(c->es);
    c->one_es = 1.0 - c->es;
}

static int aea_setup(oracle_crs *c) {
    double phi1 = c->phi1, phi2 = c->phi2;
    if (fabs(phi1 + phi2) < 1e-10) return -1;
    double sinphi = sin(phi1), cosphi = cos(phi1);
    c->n = sinphi;
    int secant = fabs(phi1 - phi2) >= 1e-10;
    if (c->es > 0.) {
        double m1 = pj_msfn(sinphi, cosphi, c->es);
        double ml1 = pj_qsfn(sinphi, c->e, c->one_es);
        if (secant) {
            double s2 = sin(phi2), c2 = cos(phi2);
            double m2 = pj_msfn(s2, c2, c->es);
            double ml2 = pj_qsfn(s2, c->e, c->one_es);
            if (ml2 == ml1) return -1;
            c->n = (m1 * m1 - m2 * m2) / (ml2 - ml1);
        }
        c->ec = 1. - .5 * c->one_es * log((1. - c->e) / (1. + c->e)) / c->e;
        c->c = m1 * m1 + c->n * ml1;
        c->dd = 1. / c->n;
        c->rho0 = c->dd * sqrt(c->c - c->n * pj_qsfn(sin(c->phi0), c->e, c->one_es));
    } else {
        if (secant) c->n = .5 * (c->n + sin(phi2));
        double n2 = c->n + c->n;
        c->c = cosphi * cosphi + n2 * sinphi;
        c->dd = 1. / c->n;
        c->rho0 = c->dd * sqrt(c->c - n2 * sin(c->phi0));
    }
    return 0;
}

/* ---- tmerc.cpp (PROJ 6.1.1), the exact ellipsoidal algorithm [ext] ------
 * Poder / Engsager: geodetic <-> Gaussian latitude by a trigonometric series,
 * Gaussian <-> complementary spherical by spherical trigonometry, spherical
 * <-> ellipsoidal (N, E) by a complex trigonometric series; all series of
 * 6th order in the third flattening n (the Krueger series), summed by
 * Clenshaw.  Restated from the published algorithm; pinned by the
 * known-answer points of tests/test_tmerc.py.  Coefficient k of each series
 * is n^(k+1) * (c[0] + n * (c[1] + ...)): the rational coefficients below. */
typedef struct { int len; double c[6]; } or_poly;
static const or_poly OR_CGB[6] = {
    {6, {2, -2 / 3.0, -2, 116 / 45.0, 26 / 45.0, -2854 / 675.0}},
    {5, {7 / 3.0, -8 / 5.0, -227 / 45.0, 2704 / 315.0, 2323 / 945.0}},
    {4, {56 / 15.0, -136 / 35.0, -1262 / 105.0, 73814 / 2835.0}},
    {3, {4279 / 630.0, -332 / 35.0, -399572 / 14175.0}},
    {2, {4174 / 315.0, -144838 / 6237.0}},
    {1, {601676 / 22275.0}}};
static const or_poly OR_CBG[6] = {
    {6, {-2, 2 / 3.0, 4 / 3.0, -82 / 45.0, 32 / 45.0, 4642 / 4725.0}},
    {5, {5 / 3.0, -16 / 15.0, -13 / 9.0, 904 / 315.0, -1522 / 945.0}},
    {4, {-26 / 15.0, 34 / 21.0, 8 / 5.0, -12686 / 2835.0}},
    {3, {1237 / 630.0, -12 / 5.0, -24832 / 14175.0}},
    {2, {-734 / 315.0, 109598 / 31185.0}},
    {1, {444337 / 155925.0}}};
static const or_poly OR_UTG[6] = {
    {6, {-0.5, 2 / 3.0, -37 / 96.0, 1 / 360.0, 81 / 512.0, -96199 / 604800.0}},
    {5, {-1 / 48.0, -1 / 15.0, 437 / 1440.0, -46 / 105.0, 1118711 / 3870720.0}},
    {4, {-17 / 480.0, 37 / 840.0, 209 / 4480.0, -5569 / 90720.0}},
    {3, {-4397 / 161280.0, 11 / 504.0, 830251 / 7257600.0}},
    {2, {-4583 / 161280.0, 108847 / 3991680.0}},
    {1, {-20648693 / 638668800.0}}};
static const or_poly OR_GTU[6] = {
    {6, {0.5, -2 / 3.0, 5 / 16.0, 41 / 180.0, -127 / 288.0, 7891 / 37800.0}},
    {5, {13 / 48.0, -3 / 5.0, 557 / 1440.0, 281 / 630.0, -1983433 / 1935360.0}},
    {4, {61 / 240.0, -103 / 140.0, 15061 / 26880.0, 167603 / 181440.0}},
    {3, {49561 / 161280.0, -179 / 168.0, 6601661 / 7257600.0}},
    {2, {34729 / 80640.0, -3418889 / 1995840.0}},
    {1, {212378941 / 319334400.0}}};

/* n^(k+1) * poly in the nesting order of setup_exact (innermost first). */
static void or_series(const or_poly *P, double n, double *out, int utg_gtu) {
    double np = n;
    for (int k = 0; k < 6; k++) {
        /* setup_exact's powers: cgb / cbg step np by n each k; utg / gtu use
         * n (k = 0), then n^2 for k = 0..1's second term onwards */
        if (utg_gtu) np = k == 0 ? n : k == 1 ? n * n : np * n;
        else if (k > 0) np *= n;
        double h = P[k].c[P[k].len - 1];
        for (int j = P[k].len - 2; j >= 0; j--) h = P[k].c[j] + n * h;
        out[k] = np * h;
    }
}

static double or_gatg(const double *p1, int len, double B) {
    double h = 0, h1, h2 = 0, cos_2B = 2 * cos(2 * B);
    const double *p = p1 + len;
    h1 = *--p;
    while (p - p1) { h = -h2 + cos_2B * h1 + *--p; h2 = h1; h1 = h; }
    return B + h * sin(2 * B);
}

static double or_clens(const double *a, int size, double arg_r) {
    const double *p = a + size;
    double r = 2 * cos(arg_r), hr1 = 0, hr = *--p, hr2;
    while (a - p) { hr2 = hr1; hr1 = hr; hr = -hr2 + r * hr1 + *--p; }
    return sin(arg_r) * hr;
}

static void or_clenS(const double *a, int size, double ar, double ai, double *R, double *I) {
    const double *p = a + size;
    double sr = sin(ar), cr = cos(ar), sh = sinh(ai), ch = cosh(ai);
    double r = 2 * cr * ch, i = -2 * sr * sh;
    double hr = *--p, hi = 0, hr1 = 0, hi1 = 0, hr2, hi2;
    while (a - p) {
        hr2 = hr1; hi2 = hi1; hr1 = hr; hi1 = hi;
        hr = -hr2 + r * hr1 - i * hi1 + *--p;
        hi = -hi2 + i * hr1 + r * hi1;
    }
    r = sr * ch; i = cr * sh;
    *R = r * hr - i * hi;
    *I = r * hi + i * hr;
}

static int tmerc_setup(oracle_crs *c) {
    if (!(c->es > 0)) return -1;
    c->kind = OR_CRS_TMERC;
    double f = c->es / (1 + sqrt(1 - c->es));
    double n = f / (2 - f);
    or_series(OR_CGB, n, c->tm_cgb, 0);
    or_series(OR_CBG, n, c->tm_cbg, 0);
    or_series(OR_UTG, n, c->tm_utg, 1);
    or_series(OR_GTU, n, c->tm_gtu, 1);
    double n2 = n * n;
    c->tm_qn = c->k0 / (1 + n) * (1 + n2 * (1 / 4.0 + n2 * (1 / 64.0 + n2 / 256.0)));
    double Z = or_gatg(c->tm_cbg, 6, c->phi0);
    c->tm_zb = -c->tm_qn * (Z + or_clens(c->tm_gtu, 6, 2 * Z));
    return 0;
}

static int utm_setup(oracle_crs *c, int zone, int south) {   /* utm.cpp */
    if (zone < 1 || zone > 60) return -1;
    c->lam0 = (zone - .5) * OR_PI / 30. - OR_PI;
    c->phi0 = 0; c->k0 = 0.9996; c->x0 = 500000; c->y0 = south ? 10000000 : 0;
    return tmerc_setup(c);
}

/* ---- lcc.cpp (PROJ 6.1.1), ellipsoidal [ext] -----------------------------
 * Snyder 15-1..15-11 as PROJ states them: t(phi) = pj_tsfn, m(phi) =
 * pj_msfn, the inverse latitude by pj_phi2's fixed-point iteration. */
static double or_tsfn(double phi, double sinphi, double e) {
    sinphi *= e;
    return tan(.5 * (OR_HALFPI - phi)) / pow((1. - sinphi) / (1. + sinphi), .5 * e);
}

static int lcc_setup(oracle_crs *c) {
    if (!(c->es > 0)) return -1;
    c->kind = OR_CRS_LCC;
    if (fabs(c->phi1 + c->phi2) < 1e-10) return -1;
    double sinphi = sin(c->phi1), cosphi = cos(c->phi1);
    c->n = sinphi;
    double m1 = cosphi / sqrt(1. - c->es * sinphi * sinphi);
    double ml1 = or_tsfn(c->phi1, sinphi, c->e);
    if (fabs(c->phi1 - c->phi2) >= 1e-10) {
        sinphi = sin(c->phi2);
        c->n = log(m1 / (cos(c->phi2) / sqrt(1. - c->es * sinphi * sinphi)));
        c->n /= log(ml1 / or_tsfn(c->phi2, sinphi, c->e));
    }
    c->c = c->rho0 = m1 * pow(ml1, -c->n) / c->n;
    c->rho0 *= fabs(fabs(c->phi0) - OR_HALFPI) < 1e-10 ? 0. : pow(or_tsfn(c->phi0, sin(c->phi0), c->e), c->n);
    return 0;
}

/* ---- stere.cpp (PROJ 6.1.1), polar aspects on an ellipsoid [ext] ----------
 * Snyder 21-33..21-40: rho = akm1 t(phi) about the pole phi0 = +-pi/2;
 * |lat_ts| = pi/2 puts k0 at the pole, else true scale on lat_ts. */
static int stere_polar_setup(oracle_crs *c, int south, int has_ts, double lat_ts) {
    if (!(c->es > 0)) return -1;
    c->kind = OR_CRS_STERE_POLAR;
    c->phi0 = south ? -OR_HALFPI : OR_HALFPI;
    c->phi1 = fabs(has_ts ? lat_ts : OR_HALFPI);
    if (fabs(c->phi1 - OR_HALFPI) < 1e-10) {
        c->c = 2. * c->k0 / sqrt(pow(1 + c->e, 1 + c->e) * pow(1 - c->e, 1 - c->e));
    } else {
        double s1 = sin(c->phi1);
        c->c = cos(c->phi1) / or_tsfn(c->phi1, s1, c->e);
        c->c /= sqrt(1. - (c->e * s1) * (c->e * s1));
    }
    return 0;
}

static double param_of(const char *s, const char *key, double dflt, int *found) {
    const char *p = s;
    size_t kl = strlen(key);
    while ((p = strstr(p, key)) != NULL) {
        if ((p == s || p[-1] == ' ' || p[-1] == '+') && p[kl] == '=') {
            if (found) *found = 1;
            return strtod(p + kl + 1, NULL);
        }
        p += kl;
    }
    if (found) *found = 0;
    return dflt;
}

int oracle_crs_init(oracle_crs *c, const char *spec) {
    memset(c, 0, sizeof(*c));
    c->k0 = 1.0;
    if (!spec) return -1;
    if (!strcasecmp(spec, "EPSG:4326")) { c->kind = OR_CRS_LONGLAT; set_ellps(c, 6378137.0, 298.257223563); return 0; }
    if (!strcasecmp(spec, "EPSG:3857") || !strcasecmp(spec, "EPSG:900913")) {
        c->kind = OR_CRS_WEBMERC; set_ellps(c, 6378137.0, 0.0); return 0;
    }
    if (!strcasecmp(spec, "EPSG:3577")) {
        c->kind = OR_CRS_AEA; set_ellps(c, 6378137.0, 298.257222101);
        c->lam0 = 132.0 * OR_D2R; c->phi0 = 0.0; c->phi1 = -18.0 * OR_D2R; c->phi2 = -36.0 * OR_D2R;
        return aea_setup(c);
    }
    if (!strcasecmp(spec, "SR-ORG:6842") || !strcasecmp(spec, "MODIS")) {
        c->kind = OR_CRS_SINU; set_ellps(c, 6371007.181, 0.0); return 0;
    }
    if (!strcasecmp(spec, "EPSG:4283")) { c->kind = OR_CRS_LONGLAT; set_ellps(c, 6378137.0, 298.257222101); return 0; }
    if (!strncasecmp(spec, "EPSG:", 5)) {      /* UTM / MGA zones */
        int code = atoi(spec + 5);
        if (code > 32600 && code <= 32660) { set_ellps(c, 6378137.0, 298.257223563); return utm_setup(c, code - 32600, 0); }
        if (code > 32700 && code <= 32760) { set_ellps(c, 6378137.0, 298.257223563); return utm_setup(c, code - 32700, 1); }
        if (code >= 28348 && code <= 28358) { set_ellps(c, 6378137.0, 298.257222101); return utm_setup(c, code - 28300, 1); }
        if (code >= 7846 && code <= 7859) { set_ellps(c, 6378137.0, 298.257222101); return utm_setup(c, code - 7800, 1); }
        if (code == 3031 || code == 3976) {
            set_ellps(c, 6378137.0, 298.257223563);
            return stere_polar_setup(c, 1, 1, (code == 3031 ? -71.0 : -70.0) * OR_D2R);
        }
        if (code == 3413) {
            set_ellps(c, 6378137.0, 298.257223563);
            c->lam0 = -45.0 * OR_D2R;
            return stere_polar_setup(c, 0, 1, 70.0 * OR_D2R);
        }
        if (code == 32661 || code == 32761) {
            set_ellps(c, 6378137.0, 298.257223563);
            c->k0 = 0.994; c->x0 = c->y0 = 2000000.0;
            return stere_polar_setup(c, code == 32761, 0, 0.0);
        }
        if (code == 3112 || code == 7845) {
            set_ellps(c, 6378137.0, 298.257222101);
            c->phi1 = -18.0 * OR_D2R; c->phi2 = -36.0 * OR_D2R; c->phi0 = 0.0; c->lam0 = 134.0 * OR_D2R;
            return lcc_setup(c);
        }
    }
    if (strstr(spec, "+proj=")) {
        int f = 0;
        double a = param_of(spec, "+a", 0, &f);
        double R = param_of(spec, "+R", 0, NULL);
        double rf = param_of(spec, "+rf", 0, NULL);
        int has_a = f;
        if (strstr(spec, "+ellps=GRS80")) { a = 6378137.0; rf = 298.257222101; has_a = 1; }
        else if (strstr(spec, "+ellps=WGS84") || strstr(spec, "+datum=WGS84")) { a = 6378137.0; rf = 298.257223563; has_a = 1; }
        if (R > 0) { a = R; rf = 0; has_a = 1; }
        if (!has_a) { a = 6378137.0; rf = 298.257223563; }
        c->lam0 = param_of(spec, "+lon_0", 0, NULL) * OR_D2R;
        c->phi0 = param_of(spec, "+lat_0", 0, NULL) * OR_D2R;
        c->x0 = param_of(spec, "+x_0", 0, NULL);
        c->y0 = param_of(spec, "+y_0", 0, NULL);
        if (strstr(spec, "+proj=longlat") || strstr(spec, "+proj=latlong")) {
            c->kind = OR_CRS_LONGLAT; set_ellps(c, a, rf); return 0;
        }
        if (strstr(spec, "+proj=webmerc") ||
            (strstr(spec, "+proj=merc") && R > 0)) {
            c->kind = OR_CRS_WEBMERC; set_ellps(c, a, 0.0); return 0;
        }
        if (strstr(spec, "+proj=aea")) {
            c->kind = OR_CRS_AEA; set_ellps(c, a, rf);
            c->phi1 = param_of(spec, "+lat_1", 0, NULL) * OR_D2R;
            c->phi2 = param_of(spec, "+lat_2", 0, NULL) * OR_D2R;
            return aea_setup(c);
        }
        if (strstr(spec, "+proj=sinu")) { c->kind = OR_CRS_SINU; set_ellps(c, a, rf == 0 ? 0 : rf); if (c->es != 0) return -1; return 0; }
        if (strstr(spec, "+proj=utm")) {
            int fz = 0;
            double zone = param_of(spec, "+zone", 0, &fz);
            set_ellps(c, a, rf);
            if (!fz || zone != floor(zone)) return -1;
            return utm_setup(c, (int)zone, strstr(spec, "+south") != NULL);
        }
        if (strstr(spec, "+proj=lcc")) {
            int f1 = 0, f2 = 0, f0 = 0, fk = 0;
            set_ellps(c, a, rf);
            c->phi1 = param_of(spec, "+lat_1", 0, &f1) * OR_D2R;
            c->phi2 = param_of(spec, "+lat_2", 0, &f2) * OR_D2R;
            param_of(spec, "+lat_0", 0, &f0);
            if (!f2) { c->phi2 = c->phi1; if (!f0) c->phi0 = c->phi1; }
            c->k0 = param_of(spec, "+k_0", 1.0, &fk);
            if (!fk) c->k0 = param_of(spec, "+k", 1.0, NULL);
            return lcc_setup(c);
        }
        if (strstr(spec, "+proj=ups")) {
            set_ellps(c, a, rf);
            c->k0 = 0.994; c->x0 = c->y0 = 2000000.0; c->lam0 = 0;
            return stere_polar_setup(c, strstr(spec, "+south") != NULL, 0, 0.0);
        }
        if (strstr(spec, "+proj=stere ") || (strlen(spec) >= 11 && !strcmp(spec + strlen(spec) - 11, "+proj=stere"))) {
            int fts = 0, fk = 0;
            double ts = param_of(spec, "+lat_ts", 0, &fts) * OR_D2R;
            set_ellps(c, a, rf);
            if (fabs(fabs(c->phi0) - OR_HALFPI) >= 1e-10) return -1;
            c->k0 = param_of(spec, "+k_0", 1.0, &fk);
            if (!fk) c->k0 = param_of(spec, "+k", 1.0, NULL);
            return stere_polar_setup(c, c->phi0 < 0, fts, ts);
        }
        if ((strstr(spec, "+proj=tmerc") || strstr(spec, "+proj=etmerc")) && !strstr(spec, "+approx")) {
            int fk = 0;
            set_ellps(c, a, rf);
            c->k0 = param_of(spec, "+k_0", 1.0, &fk);
            if (!fk) c->k0 = param_of(spec, "+k", 1.0, NULL);
            return tmerc_setup(c);
        }
    }
    return -1;
}

static int crs_equal(const oracle_crs *a, const oracle_crs *b) {
    return memcmp(a, b, sizeof(*a)) == 0;
}

/* inverse: CRS coordinates -> (lam, phi) radians.  pj_inv wrapper. */
static int crs_inverse(const oracle_crs *c, double x, double y, double *lam, double *phi) {
    if (x == HUGE_VAL || y == HUGE_VAL) return 0;
    if (c->kind == OR_CRS_LONGLAT) {            /* unitconvert deg -> rad */
        *lam = x * OR_D2R; *phi = y * OR_D2R; return 1;
    }
    double xn = (x * 1.0 - c->x0) * c->ra;
    double yn = (y * 1.0 - c->y0) * c->ra;
    double l, p;
    switch (c->kind) {
    case OR_CRS_WEBMERC:                        /* merc.cpp s_inverse */
        p = OR_HALFPI - 2. * atan(exp(-yn / c->k0));
        l = xn / c->k0;
        break;
    case OR_CRS_AEA: {                          /* aea.cpp e_inverse */
        double rho;
        yn = c->rho0 - yn;
        if ((rho = hypot(xn, yn)) != 0.0) {
            if (c->n < 0.) { rho = -rho; xn = -xn; yn = -yn; }
            p = rho / c->dd;
            if (c->es > 0.) {
                p = (c->c - p * p) / c->n;
                if (fabs(c->ec - fabs(p)) > 1e-7) {
                    if ((p = aea_phi1(p, c->e, c->one_es)) == HUGE_VAL) return 0;
                } else {
                    p = p < 0. ? -OR_HALFPI : OR_HALFPI;
                }
            } else {
                p = (c->c - p * p) / (c->n + c->n);
                if (fabs(p) <= 1.) p = asin(p);
                else p = p < 0. ? -OR_HALFPI : OR_HALFPI;
            }
            l = atan2(xn, yn) / c->n;
        } else {
            l = 0.;
            p = c->n > 0. ? OR_HALFPI : -OR_HALFPI;
        }
        break;
    }
    case OR_CRS_SINU:                           /* gn_sinu.cpp s_inverse, m=0 n=1 */
        p = yn;
        l = xn / cos(yn);
        break;
    case OR_CRS_LCC: {                          /* lcc.cpp e_inverse */
        double X = xn / c->k0, Y = c->rho0 - yn / c->k0;
        double rho = hypot(X, Y);
        if (rho != 0.) {
            if (c->n < 0.) { rho = -rho; X = -X; Y = -Y; }
            double ts = pow(rho / c->c, 1. / c->n), Phi = OR_HALFPI - 2. * atan(ts), dphi;
            int i = 15;
            do {
                double con = c->e * sin(Phi);
                dphi = OR_HALFPI - 2. * atan(ts * pow((1. - con) / (1. + con), .5 * c->e)) - Phi;
                Phi += dphi;
            } while (fabs(dphi) > 1.0e-10 && --i);
            if (i <= 0) return 0;
            p = Phi;
            l = atan2(X, Y) / c->n;
        } else {
            l = 0.;
            p = c->n > 0. ? OR_HALFPI : -OR_HALFPI;
        }
        break;
    }
    case OR_CRS_STERE_POLAR: {                  /* stere.cpp e_inverse, S_POLE / N_POLE */
        double sg = c->phi0 < 0 ? -1. : 1.;     /* south: work on the mirrored (north) problem */
        double ts = hypot(xn, yn) / c->c;
        double Phi = OR_HALFPI + 2. * atan(ts), prev;   /* PROJ's start: sin() equals the sphere's */
        int i = 8, done = 0;
        while (i--) {
            prev = Phi;
            double es = c->e * sin(prev);
            Phi = OR_HALFPI - 2. * atan(ts * pow((1. - es) / (1. + es), .5 * c->e));
            if (fabs(prev - Phi) < 1e-10) { done = 1; break; }
        }
        if (!done) return 0;
        p = sg * Phi;
        l = (xn == 0. && yn == 0.) ? 0. : atan2(xn, sg > 0 ? -yn : yn);
        break;
    }
    case OR_CRS_TMERC: {                        /* tmerc.cpp exact_e_inv */
        double Cn = (yn - c->tm_zb) / c->tm_qn, Ce = xn / c->tm_qn, dCn, dCe;
        if (!(fabs(Ce) <= 2.623395162778)) return 0;   /* 150 degrees */
        or_clenS(c->tm_utg, 6, 2 * Cn, 2 * Ce, &dCn, &dCe);
        Cn += dCn;
        Ce += dCe;
        Ce = atan(sinh(Ce));
        double sCn = sin(Cn), cCn = cos(Cn), sCe = sin(Ce), cCe = cos(Ce);
        Ce = atan2(sCe, cCe * cCn);
        Cn = atan2(sCn * cCe, hypot(sCe, cCe * cCn));
        p = or_gatg(c->tm_cgb, 6, Cn);
        l = Ce;
        break;
    }
    default:
        return 0;
    }
    if (l == HUGE_VAL || p == HUGE_VAL || isnan(l) || isnan(p)) return 0;
    l = l + c->lam0;
    l = adjlon(l);
    *lam = l; *phi = p;
    return 1;
}

/* forward: (lam, phi) radians -> CRS coordinates.  pj_fwd wrapper. */
static int crs_forward(const oracle_crs *c, double lam, double phi, double *x, double *y) {
    if (c->kind == OR_CRS_LONGLAT) {            /* unitconvert rad -> deg */
        *x = lam * OR_R2D; *y = phi * OR_R2D; return 1;
    }
    double t = (phi < 0 ? -phi : phi) - OR_HALFPI;
    if (t > 1e-12 || lam > 10 || lam < -10) return 0;
    if (phi > OR_HALFPI) phi = OR_HALFPI;
    if (phi < -OR_HALFPI) phi = -OR_HALFPI;
    lam = lam - c->lam0;
    lam = adjlon(lam);
    double xn, yn;
    switch (c->kind) {
    case OR_CRS_WEBMERC:                        /* merc.cpp s_forward */
        if (fabs(fabs(phi) - OR_HALFPI) <= 1.e-10) return 0;
        xn = c->k0 * lam;
        yn = c->k0 * log(tan(OR_FORTPI + .5 * phi));
        break;
    case OR_CRS_AEA: {                          /* aea.cpp e_forward */
        double rho = c->c - (c->es > 0. ? c->n * pj_qsfn(sin(phi), c->e, c->one_es)
                                        : (c->n + c->n) * sin(phi));
        if (rho < 0.) return 0;
        rho = c->dd * sqrt(rho);
        lam *= c->n;
        xn = rho * sin(lam);
        yn = c->rho0 - rho * cos(lam);
        break;
    }
    case OR_CRS_SINU:                           /* gn_sinu.cpp s_forward, m=0 n=1 */
        xn = lam * cos(phi);
        yn = phi;
        break;
    case OR_CRS_LCC: {                          /* lcc.cpp e_forward */
        double rho;
        if (fabs(fabs(phi) - OR_HALFPI) < 1.e-10) {
            if (phi * c->n <= 0.) return 0;
            rho = 0.;
        } else {
            rho = c->c * pow(or_tsfn(phi, sin(phi), c->e), c->n);
        }
        double L = lam * c->n;
        xn = c->k0 * (rho * sin(L));
        yn = c->k0 * (c->rho0 - rho * cos(L));
        break;
    }
    case OR_CRS_STERE_POLAR: {                  /* stere.cpp e_forward, S_POLE / N_POLE */
        double sg = c->phi0 < 0 ? -1. : 1.;
        double rho = c->c * or_tsfn(sg * phi, sg * sin(phi), c->e);
        xn = rho * sin(lam);
        yn = -sg * rho * cos(lam);
        break;
    }
    case OR_CRS_TMERC: {                        /* tmerc.cpp exact_e_fwd */
        double Cn = or_gatg(c->tm_cbg, 6, phi), dCn, dCe;
        double sCn = sin(Cn), cCn = cos(Cn), sCe = sin(lam), cCe = cos(lam);
        Cn = atan2(sCn, cCe * cCn);
        double Ce = atan2(sCe * cCn, hypot(sCn, cCn * cCe));
        Ce = asinh(tan(Ce));
        or_clenS(c->tm_gtu, 6, 2 * Cn, 2 * Ce, &dCn, &dCe);
        Cn += dCn;
        Ce += dCe;
        if (!(fabs(Ce) <= 2.623395162778)) return 0;
        yn = c->tm_qn * Cn + c->tm_zb;
        xn = c->tm_qn * Ce;
        break;
    }
    default:
        return 0;
    }
    if (isnan(xn) || isnan(yn) || isinf(xn) || isinf(yn)) return 0;
    *x = 1.0 * (c->a * xn + c->x0);
    *y = 1.0 * (c->a * yn + c->y0);
    return 1;
}

int oracle_crs_transform(const oracle_crs *src, const oracle_crs *dst, double *x, double *y) {
    if (crs_equal(src, dst)) return 1;
    double lam, phi;
    if (!crs_inverse(src, *x, *y, &lam, &phi)) return 0;
    return crs_forward(dst, lam, phi, x, y);
}

/* ======================================================================== */
/* GDAL GenImgProj / Approx transformers [ext: gdaltransformer.cpp 3.0.1]     */
/* ======================================================================== */
static void inv_geot(const double *gt, double *o) {   /* GDALInvGeoTransform */
    if (gt[2] == 0.0 && gt[4] == 0.0 && gt[1] != 0.0 && gt[5] != 0.0) {
        o[0] = -gt[0] / gt[1];
        o[1] = 1.0 / gt[1];
        o[2] = 0.0;
        o[3] = -gt[3] / gt[5];
        o[4] = 0.0;
        o[5] = 1.0 / gt[5];
        return;
    }
    double det = gt[1] * gt[5] - gt[2] * gt[4];
    double inv_det = 1.0 / det;
    o[0] = (gt[2] * gt[3] - gt[0] * gt[5]) * inv_det;
    o[3] = (-gt[1] * gt[3] + gt[0] * gt[4]) * inv_det;
    o[1] = gt[5] * inv_det;
    o[4] = -gt[4] * inv_det;
    o[2] = -gt[2] * inv_det;
    o[5] = gt[1] * inv_det;
}

/* ---- GDAL 3.0.1 geolocation-array transformer (alg/gdalgeoloc.cpp) [ext]
 * selected by warp.go:128-141 (createGeoLocTransformer, 52-67) for requests
 * with GeoLocOpts (tile_grpc.go:338-350).  Restated from the published
 * algorithm; parity unpinned (GDAL absent).
 *   GeoLocLoadFullData: X / Y bands as double; one-row X and Y bands form a
 *     regular grid (X per column, Y per row).
 *   GeoLocGenerateBackMap: extent of the valid points (X nodata excluded),
 *     pixel size sqrt(area / (nx * ny * 1.3)), a grid of ceil(extent / size)
 *     + 1 cells whose origin is half a cell outside the extent; every point
 *     splatted bilinearly onto the 4 cells around it with its source
 *     pixel / line (i * STEP + OFFSET); cells of weight > 0.25 averaged,
 *     the rest -1; 3 hole-filling sweeps, a hole taking the mean of its set
 *     4-neighbours (cells filled in a sweep are used from the next one).
 *   GDALGeoLocTransform: pixel/line -> georef by bilinear interpolation of
 *     the arrays (nearest square extended beyond them, nodata corners
 *     falling back to the edge / corner rules); georef -> pixel/line by
 *     bilinear interpolation of the backmap where its 4 cells are set, else
 *     its nearest cell. */
int oracle_geoloc_init(oracle_geoloc *g, const double *xb, int xw, int xh, const double *yb, int yw, int yh,
                       int has_nodata, double nodata_x, double pixel_offset, double line_offset,
                       double pixel_step, double line_step) {
    memset(g, 0, sizeof(*g));
    const int regular = xh == 1 && yh == 1;
    const int nx = xw, ny = regular ? yw : xh;
    if (nx <= 0 || ny <= 0 || (!regular && (yw != xw || yh != xh))) return 3;
    g->nx = nx; g->ny = ny;
    g->gx = (double *)malloc(sizeof(double) * (size_t)nx * ny);
    g->gy = (double *)malloc(sizeof(double) * (size_t)nx * ny);
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
            g->gx[(size_t)j * nx + i] = regular ? xb[i] : xb[(size_t)j * nx + i];
            g->gy[(size_t)j * nx + i] = regular ? yb[j] : yb[(size_t)j * nx + i];
        }
    g->has_nodata = has_nodata; g->nodata_x = nodata_x;
    g->pixel_offset = pixel_offset; g->line_offset = line_offset;
    g->pixel_step = pixel_step; g->line_step = line_step;
    /* the backmap */
    double mnx = 0, mxx = 0, mny = 0, mxy = 0;
    int any = 0;
    for (long i = (long)nx * ny - 1; i >= 0; i--) {
        const double X = g->gx[i], Y = g->gy[i];
        if (has_nodata && X == nodata_x) continue;
        if (!any) { mnx = mxx = X; mny = mxy = Y; any = 1; continue; }
        if (X < mnx) mnx = X;
        if (X > mxx) mxx = X;
        if (Y < mny) mny = Y;
        if (Y > mxy) mxy = Y;
    }
    const double size = sqrt((mxx - mnx) * (mxy - mny) / ((double)nx * ny * 1.3));
    if (!(size > 0.0) || isinf(size)) return 3;
    const double fw = ceil((mxx - mnx) / size) + 1, fh = ceil((mxy - mny) / size) + 1;
    if (!(fw > 0 && fw < 4194304.0) || !(fh > 0 && fh < 4194304.0) || fw * fh > 4.0e9) return 3;
    const int bw = (int)fw, bh = (int)fh;
    const double x0 = mnx - size / 2.0, y0 = mxy + size / 2.0;
    g->bw = bw; g->bh = bh;
    g->bgt[0] = x0; g->bgt[1] = size; g->bgt[2] = 0.0; g->bgt[3] = y0; g->bgt[4] = 0.0; g->bgt[5] = -size;
    const size_t nc = (size_t)bw * bh;
    g->bmx = (float *)calloc(nc, sizeof(float));
    g->bmy = (float *)calloc(nc, sizeof(float));
    float *w = (float *)calloc(nc, sizeof(float));
    for (int iy = 0; iy < ny; iy++)
        for (int ix = 0; ix < nx; ix++) {
            const size_t k = (size_t)iy * nx + ix;
            if (has_nodata && g->gx[k] == nodata_x) continue;
            const double cx = (g->gx[k] - x0) / size - 0.5, cy = (y0 - g->gy[k]) / size - 0.5;
            const int c0 = (int)floor(cx), r0 = (int)floor(cy);
            const double ax = cx - c0, ay = cy - r0;
            const double p = ix * pixel_step + pixel_offset, l = iy * line_step + line_offset;
            const double wt[4] = {(1.0 - ax) * (1.0 - ay), ax * (1.0 - ay), (1.0 - ax) * ay, ax * ay};
            for (int q = 0; q < 4; q++) {
                const int c = c0 + (q & 1), r = r0 + (q >> 1);
                if (c < 0 || c >= bw || r < 0 || r >= bh) continue;
                const size_t o = (size_t)r * bw + c;
                g->bmx[o] += (float)(p * wt[q]);
                g->bmy[o] += (float)(l * wt[q]);
                w[o] += (float)wt[q];
            }
        }
    for (size_t o = 0; o < nc; o++) {
        if (w[o] > 0.25f) { g->bmx[o] /= w[o]; g->bmy[o] /= w[o]; w[o] = 4.0f; }
        else { g->bmx[o] = -1.0f; g->bmy[o] = -1.0f; w[o] = 0.0f; }
    }
    for (int pass = 0; pass < 3; pass++) {
        const float mark = (float)(3 - pass);
        size_t set = 0;
        for (int r = 0; r < bh; r++)
            for (int c = 0; c < bw; c++) {
                const size_t o = (size_t)r * bw + c;
                if (g->bmx[o] >= 0) { set++; continue; }
                const long nb[4] = {c > 0 ? (long)o - 1 : -1, c + 1 < bw ? (long)o + 1 : -1,
                                    r > 0 ? (long)o - bw : -1, r + 1 < bh ? (long)o + bw : -1};
                double sx = 0.0, sy = 0.0;
                int n = 0;
                for (int q = 0; q < 4; q++)
                    if (nb[q] >= 0 && w[nb[q]] > mark) { sx += g->bmx[nb[q]]; sy += g->bmy[nb[q]]; n++; }
                if (n) { g->bmx[o] = (float)(sx / n); g->bmy[o] = (float)(sy / n); w[o] = mark; }
            }
        if (set == nc) break;
    }
    free(w);
    return 0;
}

void oracle_geoloc_free(oracle_geoloc *g) {
    free(g->gx); free(g->gy); free(g->bmx); free(g->bmy);
    memset(g, 0, sizeof(*g));
}

static int geoloc_fwd(const oracle_geoloc *g, double *x, double *y) {
    if (*x == HUGE_VAL || *y == HUGE_VAL) return 0;
    const double gp = (*x - g->pixel_offset) / g->pixel_step, gl = (*y - g->line_offset) / g->line_step;
    int ix = go_cvtt32(gp), iy = go_cvtt32(gl);
    if (ix < 0) ix = 0;
    if (ix > g->nx - 1) ix = g->nx - 1;
    if (iy < 0) iy = 0;
    if (iy > g->ny - 1) iy = g->ny - 1;
    const size_t k = (size_t)iy * g->nx + ix;
    const double *X = g->gx + k, *Y = g->gy + k;
    const int nx = g->nx;
    const double nd = g->nodata_x;
    if (g->has_nodata && X[0] == nd) return 0;
    const double u = gp - ix, v = gl - iy;
    if (ix + 1 < g->nx && iy + 1 < g->ny && (!g->has_nodata || (X[1] != nd && X[nx] != nd && X[nx + 1] != nd))) {
        *x = (1 - v) * (X[0] + u * (X[1] - X[0])) + v * (X[nx] + u * (X[nx + 1] - X[nx]));
        *y = (1 - v) * (Y[0] + u * (Y[1] - Y[0])) + v * (Y[nx] + u * (Y[nx + 1] - Y[nx]));
    } else if (ix + 1 < g->nx && (!g->has_nodata || X[1] != nd)) {
        *x = X[0] + u * (X[1] - X[0]);
        *y = Y[0] + u * (Y[1] - Y[0]);
    } else if (iy + 1 < g->ny && (!g->has_nodata || X[nx] != nd)) {
        *x = X[0] + v * (X[nx] - X[0]);
        *y = Y[0] + v * (Y[nx] - Y[0]);
    } else {
        *x = X[0];
        *y = Y[0];
    }
    return 1;
}

static int geoloc_inv(const oracle_geoloc *g, double *x, double *y) {
    if (*x == HUGE_VAL || *y == HUGE_VAL) return 0;
    const double cx = (*x - g->bgt[0]) / g->bgt[1] - 0.5, cy = (*y - g->bgt[3]) / g->bgt[5] - 0.5;
    if (!(cx > -0.5 && cy > -0.5 && cx < g->bw - 0.5 && cy < g->bh - 0.5)) return 0;
    const int c = (int)floor(cx), r = (int)floor(cy);
    const long bw = g->bw;
    if (c >= 0 && r >= 0 && c + 1 < g->bw && r + 1 < g->bh) {
        const size_t o = (size_t)r * bw + c;
        const float *MX = g->bmx + o, *MY = g->bmy + o;
        if (MX[0] >= 0 && MX[1] >= 0 && MX[bw] >= 0 && MX[bw + 1] >= 0) {
            const double u = cx - c, v = cy - r;
            *x = (1 - u) * (1 - v) * MX[0] + u * (1 - v) * MX[1] + (1 - u) * v * MX[bw] + u * v * MX[bw + 1];
            *y = (1 - u) * (1 - v) * MY[0] + u * (1 - v) * MY[1] + (1 - u) * v * MY[bw] + u * v * MY[bw + 1];
            return 1;
        }
    }
    const size_t o = (size_t)floor(cy + 0.5) * bw + (size_t)floor(cx + 0.5);
    if (g->bmx[o] < 0) return 0;
    *x = g->bmx[o];
    *y = g->bmy[o];
    return 1;
}

typedef struct {
    oracle_crs src, dst;
    int reproject;
    double src_gt[6], src_igt[6], dst_gt[6], dst_igt[6];
    const oracle_geoloc *gl;   /* geolocation arrays in place of src_gt, or NULL */
} gip_t;

static void gip_init(gip_t *t, const oracle_crs *src, const oracle_crs *dst,
                     const double *src_gt, const double *dst_gt) {
    memset(t, 0, sizeof(*t));
    t->src = *src;
    if (dst) t->dst = *dst;
    t->reproject = dst && !crs_equal(src, dst);
    memcpy(t->src_gt, src_gt, 6 * sizeof(double));
    memcpy(t->dst_gt, dst_gt, 6 * sizeof(double));
    inv_geot(t->src_gt, t->src_igt);
    inv_geot(t->dst_gt, t->dst_igt);
}

/* GDALGenImgProjTransform for one point. */
static int gip_point(const gip_t *t, int dst_to_src, double *x, double *y) {
    const double *g1 = dst_to_src ? t->dst_gt : t->src_gt;
    const double *g2 = dst_to_src ? t->src_igt : t->dst_igt;
    double X, Y;
    if (t->gl && !dst_to_src) {
        X = *x; Y = *y;
        if (!geoloc_fwd(t->gl, &X, &Y)) return 0;
    } else {
        X = g1[0] + *x * g1[1] + *y * g1[2];
        Y = g1[3] + *x * g1[4] + *y * g1[5];
    }
    if (t->reproject) {
        const oracle_crs *from = dst_to_src ? &t->dst : &t->src;
        const oracle_crs *to = dst_to_src ? &t->src : &t->dst;
        if (!oracle_crs_transform(from, to, &X, &Y)) return 0;
    }
    if (t->gl && dst_to_src) {
        *x = X; *y = Y;
        return geoloc_inv(t->gl, x, y);
    }
    *x = g2[0] + X * g2[1] + Y * g2[2];
    *y = g2[3] + X * g2[4] + Y * g2[5];
    return 1;
}
static int gip_transform(const gip_t *t, int dst_to_src, int n, double *x, double *y, int *ok) {
    for (int i = 0; i < n; i++) ok[i] = gip_point(t, dst_to_src, &x[i], &y[i]);
    return 1;
}

/* GDALApproxTransformInternal (3.0.1) with dfMaxError = 0.125. */
static int approx_internal(const gip_t *t, int dst2src, int nPoints, double *x, double *y,
                           int *ok, const double *xs, const double *ys) {
    const int nMiddle = (nPoints - 1) / 2;
    const double dfDeltaX = (xs[2] - xs[0]) / (x[nPoints - 1] - x[0]);
    const double dfDeltaY = (ys[2] - ys[0]) / (x[nPoints - 1] - x[0]);
    const double dfError = fabs((xs[0] + dfDeltaX * (x[nMiddle] - x[0])) - xs[1]) +
                           fabs((ys[0] + dfDeltaY * (x[nMiddle] - x[0])) - ys[1]);
    if (dfError > 0.125) {
        double xM[3] = {x[(nMiddle - 1) / 2], x[nMiddle - 1], x[nMiddle + (nPoints - nMiddle - 1) / 2]};
        double yM[3] = {y[(nMiddle - 1) / 2], y[nMiddle - 1], y[nMiddle + (nPoints - nMiddle - 1) / 2]};
        const int base1 = nMiddle <= 5 || y[0] != y[nMiddle - 1] || y[0] != y[(nMiddle - 1) / 2] ||
                          x[0] == x[nMiddle - 1] || x[0] == x[(nMiddle - 1) / 2];
        const int base2 = nPoints - nMiddle <= 5 || y[nMiddle] != y[nPoints - 1] ||
                          y[nMiddle] != y[nMiddle + (nPoints - nMiddle - 1) / 2] ||
                          x[nMiddle] == x[nPoints - 1] ||
                          x[nMiddle] == x[nMiddle + (nPoints - nMiddle - 1) / 2];
        int s2[3] = {0, 0, 0};
        int bSuccess = 0;
        if (!base1 && !base2) {
            bSuccess = gip_transform(t, dst2src, 3, xM, yM, s2);
        } else if (!base1) {
            bSuccess = gip_transform(t, dst2src, 2, xM, yM, s2);
            s2[2] = 1;
        } else if (!base2) {
            bSuccess = gip_transform(t, dst2src, 1, xM + 2, yM + 2, s2 + 2);
            s2[0] = 1; s2[1] = 1;
        }
        if (!bSuccess || !s2[0] || !s2[1] || !s2[2]) {
            bSuccess = gip_transform(t, dst2src, nMiddle - 1, x + 1, y + 1, ok + 1);
            bSuccess &= gip_transform(t, dst2src, nPoints - nMiddle - 2, x + nMiddle + 1,
                                      y + nMiddle + 1, ok + nMiddle + 1);
            x[0] = xs[0]; y[0] = ys[0]; ok[0] = 1;
            x[nMiddle] = xs[1]; y[nMiddle] = ys[1]; ok[nMiddle] = 1;
            x[nPoints - 1] = xs[2]; y[nPoints - 1] = ys[2]; ok[nPoints - 1] = 1;
            return bSuccess;
        }
        double x2[3], y2[3];
        if (!base1) {
            x2[0] = xs[0]; y2[0] = ys[0];
            x2[1] = xM[0]; y2[1] = yM[0];
            x2[2] = xM[1]; y2[2] = yM[1];
            bSuccess = approx_internal(t, dst2src, nMiddle, x, y, ok, x2, y2);
        } else {
            bSuccess = gip_transform(t, dst2src, nMiddle - 1, x + 1, y + 1, ok + 1);
            x[0] = xs[0]; y[0] = ys[0]; ok[0] = 1;
        }
        if (!bSuccess) return 0;
        if (!base2) {
            x2[0] = xs[1]; y2[0] = ys[1];
            x2[1] = xM[2]; y2[1] = yM[2];
            x2[2] = xs[2]; y2[2] = ys[2];
            bSuccess = approx_internal(t, dst2src, nPoints - nMiddle, x + nMiddle, y + nMiddle,
                                       ok + nMiddle, x2, y2);
        } else {
            bSuccess = gip_transform(t, dst2src, nPoints - nMiddle - 2, x + nMiddle + 1,
                                     y + nMiddle + 1, ok + nMiddle + 1);
            x[nMiddle] = xs[1]; y[nMiddle] = ys[1]; ok[nMiddle] = 1;
            x[nPoints - 1] = xs[2]; y[nPoints - 1] = ys[2]; ok[nPoints - 1] = 1;
        }
        return bSuccess;
    }
    for (int i = nPoints - 1; i >= 0; i--) {
        const double dfDist = x[i] - x[0];
        y[i] = ys[0] + dfDeltaY * dfDist;
        x[i] = xs[0] + dfDeltaX * dfDist;
        ok[i] = 1;
    }
    return 1;
}

/* GDALApproxTransform (3.0.1) */
static int approx_transform(const gip_t *t, int dst2src, int nPoints, double *x, double *y, int *ok) {
    const int nMiddle = (nPoints - 1) / 2;
    if (y[0] != y[nPoints - 1] || y[0] != y[nMiddle] || x[0] == x[nPoints - 1] ||
        x[0] == x[nMiddle] || nPoints <= 5)
        return gip_transform(t, dst2src, nPoints, x, y, ok);
    double x2[3] = {x[0], x[nMiddle], x[nPoints - 1]};
    double y2[3] = {y[0], y[nMiddle], y[nPoints - 1]};
    int s2[3];
    gip_transform(t, dst2src, 3, x2, y2, s2);
    if (!s2[0] || !s2[1] || !s2[2]) return gip_transform(t, dst2src, nPoints, x, y, ok);
    return approx_internal(t, dst2src, nPoints, x, y, ok, x2, y2);
}

void oracle_approx_row(const oracle_crs *src, const oracle_crs *dst,
                       const double src_geot[6], const double dst_geot[6],
                       int n, double *x, double *y, int *success) {
    gip_t t;
    gip_init(&t, src, dst, src_geot, dst_geot);
    approx_transform(&t, 1, n, x, y, success);
}

/* GDALSuggestedWarpOutput2_MustAdjustFor{Right,Bottom}Border [ext] */
static int must_adjust(const gip_t *t, const double *ext, int np, int nl, double psx, double psy, int right) {
    double ax[21], ay[21];
    int s1[21], s2[21];
    int ns = 0;
    for (double r = 0.0; r <= 1.01; r += 0.05) {
        if (r > 0.99) r = 1.0;
        if (right) { ax[ns] = ext[2]; ay[ns] = ext[3] - psy * r * nl; }
        else { ax[ns] = ext[0] + psx * r * np; ay[ns] = ext[1]; }
        ns++;
    }
    gip_transform(t, 1, ns, ax, ay, s1);
    gip_transform(t, 0, ns, ax, ay, s2);
    int bad = 0, k = 0;
    for (double r = 0.0; r <= 1.01; r += 0.05) {
        double ex = right ? ext[2] : ext[0] + psx * r * np;
        double ey = right ? ext[3] - psy * r * nl : ext[1];
        if (!s1[k] || !s2[k] || fabs(ax[k] - ex) > psx || fabs(ay[k] - ey) > psy) bad++;
        k++;
    }
    return bad == ns;
}

/* GDALSuggestedWarpOutput2 [ext: gdaltransformer.cpp 3.0.1], nOptions = 0,
 * with the transformer GDALGenImgProjTransform (warp.go:154). */
static int suggested_warp_output(const gip_t *t, int nInX, int nInY, double *gt_out,
                                 int *pnPixels, int *pnLines, double *ext) {
    enum { NSTEPS = 20 };
    double px[(NSTEPS + 1) * (NSTEPS + 1)], py[(NSTEPS + 1) * (NSTEPS + 1)];
    int ok[(NSTEPS + 1) * (NSTEPS + 1)];
    const double dfStep = 1.0 / NSTEPS;
    int ns = 0;
    for (int i = 0; i <= NSTEPS; i++) {
        const double r = (i == NSTEPS) ? 1.0 : i * dfStep;
        px[ns] = r * nInX; py[ns] = 0.0; ns++;          /* top    */
        px[ns] = r * nInX; py[ns] = nInY; ns++;         /* bottom */
        px[ns] = 0.0; py[ns] = r * nInY; ns++;          /* left   */
        px[ns] = nInX; py[ns] = r * nInY; ns++;         /* right  */
    }
    gip_transform(t, 0, ns, px, py, ok);
    int failed = 0;
    for (int i = 0; i < ns; i++) if (!ok[i]) failed++;
    if (failed > 0) {                                    /* fall back to a full grid */
        ns = 0;
        for (int iy = 0; iy <= NSTEPS; iy++) {
            const double ry = (iy == NSTEPS) ? 1.0 : iy * dfStep;
            for (int ix = 0; ix <= NSTEPS; ix++) {
                const double rx = (ix == NSTEPS) ? 1.0 : ix * dfStep;
                px[ns] = rx * nInX; py[ns] = ry * nInY; ns++;
            }
        }
        gip_transform(t, 0, ns, px, py, ok);
    }
    double minX = 0, minY = 0, maxX = 0, maxY = 0;
    int got = 0;
    for (int i = 0; i < ns; i++) {
        if (!ok[i]) continue;
        if (!got) { minX = maxX = px[i]; minY = maxY = py[i]; got = 1; }
        else {
            if (px[i] < minX) minX = px[i];
            if (py[i] < minY) minY = py[i];
            if (px[i] > maxX) maxX = px[i];
            if (py[i] > maxY) maxY = py[i];
        }
    }
    if (!got) return -1;
    double dX = 0, dY = 0;
    if (ok[0] && ok[ns - 1]) { dX = px[ns - 1] - px[0]; dY = py[ns - 1] - py[0]; }
    if (dX == 0.0 || dY == 0.0) { dX = maxX - minX; dY = maxY - minY; }
    const double diag = sqrt(dX * dX + dY * dY);
    const double ps = diag / sqrt((double)nInX * nInX + (double)nInY * nInY);
    const double dfPixels = (maxX - minX) / ps;
    const double dfLines = (maxY - minY) / ps;
    if (!(dfPixels <= 2147483646.0 && dfLines <= 2147483646.0)) return -1;
    *pnPixels = (int)(dfPixels + 0.5);
    *pnLines = (int)(dfLines + 0.5);
    double psx = ps, psy = ps;
    static const double ratios[5] = {0.000, 0.001, 0.010, 0.100, 1.000};
    for (int k = 0; k < 5; k++) {
        const double tryx = psx - psx * ratios[k] / *pnPixels;
        double e[4] = {minX, maxY - (*pnLines) * psy, minX + (*pnPixels) * tryx, maxY};
        if (!must_adjust(t, e, *pnPixels, *pnLines, tryx, psy, 1)) { psx = tryx; break; }
    }
    for (int k = 0; k < 5; k++) {
        const double tryy = psy - psy * ratios[k] / *pnLines;
        double e[4] = {minX, maxY - (*pnLines) * tryy, minX + (*pnPixels) * psx, maxY};
        if (!must_adjust(t, e, *pnPixels, *pnLines, psx, tryy, 0)) { psy = tryy; break; }
    }
    maxX = minX + (*pnPixels) * psx;
    minY = maxY - (*pnLines) * psy;
    ext[0] = minX; ext[1] = minY; ext[2] = maxX; ext[3] = maxY;
    gt_out[0] = minX; gt_out[1] = psx; gt_out[2] = 0.0;
    gt_out[3] = maxY; gt_out[4] = 0.0; gt_out[5] = -psy;
    return 0;
}

int oracle_suggested_warp_output(const oracle_granule *g, const oracle_crs *src,
                                 const oracle_crs *dst, const double src_geot[6],
                                 const double dst_geot[6], double geot_out[6],
                                 int *n_pixels, int *n_lines, double extent[4]) {
    gip_t t;
    gip_init(&t, src, dst, src_geot ? src_geot : g->geot, dst_geot);
    return suggested_warp_output(&t, g->xsize, g->ysize, geot_out, n_pixels, n_lines, extent);
}

static int round_coord(double coord, int maxExtent) {     /* warp.go:69-80 */
    int c;
    if (coord < 0) c = 0;
    else {
        c = (int)(coord + 1e-10);
        if (c > maxExtent - 1) c = maxExtent - 1;
    }
    return c;
}

static double read_as_double(const void *base, int dtype, int64_t idx) {
    switch (dtype) {
    case OR_BYTE: return ((const uint8_t *)base)[idx];
    case OR_SIGNEDBYTE: return ((const int8_t *)base)[idx];
    case OR_UINT16: return ((const uint16_t *)base)[idx];
    case OR_INT16: return ((const int16_t *)base)[idx];
    case OR_UINT32: return ((const uint32_t *)base)[idx];
    case OR_INT32: return ((const int32_t *)base)[idx];
    case OR_FLOAT32: return ((const float *)base)[idx];
    case OR_FLOAT64: return ((const double *)base)[idx];
    default: return 0;
    }
}

/* GWKBilinearResample4Sample [ext: gdalwarpkernel.cpp] with validity from
 * the band nodata (UNIFIED_SRC_NODATA); returns 1 and *out when density > 0. */
static int bilinear_sample(const void *band, int dtype, int nx, int ny, int has_nodata,
                           double nodata, double sx, double sy, double *out) {
    int iSrcX = (int)floor(sx - 0.5);
    int iSrcY = (int)floor(sy - 0.5);
    double rX = 1.5 - (sx - iSrcX);
    double rY = 1.5 - (sy - iSrcY);
    if (iSrcX == -1) { iSrcX = 0; rX = 1; }
    if (iSrcY == -1) { iSrcY = 0; rY = 1; }
    double accR = 0.0, accDiv = 0.0;
    const int xs[4] = {iSrcX, iSrcX + 1, iSrcX, iSrcX + 1};
    const int ys[4] = {iSrcY, iSrcY, iSrcY + 1, iSrcY + 1};
    const double w[4] = {rX * rY, (1.0 - rX) * rY, rX * (1.0 - rY), (1.0 - rX) * (1.0 - rY)};
    for (int k = 0; k < 4; k++) {
        if (xs[k] < 0 || xs[k] >= nx || ys[k] < 0 || ys[k] >= ny) continue;
        double v = read_as_double(band, dtype, (int64_t)ys[k] * nx + xs[k]);
        if (has_nodata && (v == nodata || (isnan(nodata) && isnan(v)))) continue;
        accDiv += w[k];
        accR += v * w[k];
    }
    if (accDiv == 1.0) { *out = accR; return 1; }
    if (accDiv < 0.00001) return 0;
    *out = accR / accDiv;
    return 1;
}

int oracle_warp_geoloc(const oracle_granule *g, const oracle_crs *src,
                       const oracle_crs *dst, const double dst_geot[6],
                       int dst_w, int dst_h, int resample, const oracle_geoloc *gl,
                       void **out_buf, int *out_size, int32_t bbox[4],
                       double *nodata, int *dtype, int *bytes_read) {
    *bytes_read = 0;
    double srcGeot[6];
    memcpy(srcGeot, g->geot, sizeof(srcGeot));
    gip_t t;
    gip_init(&t, src, dst, srcGeot, dst_geot);                  /* warp.go:130 / 136 */
    t.gl = gl;
    double geotOut[6], ext[4];
    int nPixels = 0, nLines = 0;
    const int err = suggested_warp_output(&t, g->xsize, g->ysize, geotOut, &nPixels, &nLines, ext);

    /* overview pick, warp.go:156-198 (never with geolocation arrays, 158) */
    const void *band = g->data;
    int bandX = g->xsize, bandY = g->ysize;
    if (!gl && err == 0 && g->n_ovr > 0) {
        const double targetRatio = 1.0 / geotOut[1];
        if (targetRatio > 1.0) {
            const int srcXSize = g->xsize, srcYSize = g->ysize;
            int iOvr = -1;
            for (; iOvr < g->n_ovr - 1; iOvr++) {
                double ovrRatio = 1.0;
                if (iOvr >= 0) ovrRatio = (double)srcXSize / g->ovr_xsize[iOvr];
                const double nextOvrRatio = (double)srcXSize / g->ovr_xsize[iOvr + 1];
                if (ovrRatio < targetRatio && nextOvrRatio > targetRatio) break;
                const double diff = ovrRatio - targetRatio;
                if (diff > -1e-1 && diff < 1e-1) break;
            }
            if (iOvr >= 0) {
                band = g->ovr_data[iOvr];
                bandX = g->ovr_xsize[iOvr];
                bandY = g->ovr_ysize[iOvr];
                srcGeot[1] *= srcXSize / (double)bandX;
                srcGeot[2] *= srcXSize / (double)bandX;
                srcGeot[4] *= srcYSize / (double)bandY;
                srcGeot[5] *= srcYSize / (double)bandY;
                gip_init(&t, src, dst, srcGeot, dst_geot);
            }
        }
    }

    /* window, warp.go:200-217 */
    int dstXOff = 0, dstYOff = 0, dstXSize = dst_w, dstYSize = dst_h;
    if (err == 0) {
        const int minX = round_coord(ext[0], dstXSize);
        const int minY = round_coord(ext[1], dstYSize);
        const int maxX = round_coord(ext[2] + 0.5, dstXSize);
        const int maxY = round_coord(ext[3] + 0.5, dstYSize);
        dstXOff = minX; dstYOff = minY;
        dstXSize = maxX - minX + 1;
        dstYSize = maxY - minY + 1;
    }

    /* data types, warp.go:232-247 */
    const int srcType = g->dtype;
    int outType = srcType;
    const int supported = srcType == OR_BYTE || srcType == OR_INT16 || srcType == OR_UINT16 ||
                          srcType == OR_FLOAT32;
    if (!supported) outType = OR_FLOAT32;
    const int dsz = oracle_type_size(outType);
    *out_size = dstXSize * dstYSize * dsz;
    uint8_t *buf = (uint8_t *)malloc(*out_size > 0 ? *out_size : 1);
    *nodata = g->nodata;
    uint8_t fillv[8];
    or_gdal_copy_word(g->nodata, outType, fillv);
    for (int64_t i = 0; i < (int64_t)dstXSize * dstYSize; i++) memcpy(buf + i * dsz, fillv, dsz);

    /* per-row approximate transform + gather, warp.go:249-345 */
    double *dx = (double *)malloc(sizeof(double) * 2 * (dstXSize > 0 ? dstXSize : 1));
    double *dy = (double *)malloc(sizeof(double) * (dstXSize > 0 ? dstXSize : 1));
    int *ok = (int *)malloc(sizeof(int) * (dstXSize > 0 ? dstXSize : 1));
    for (int i = 0; i < dstXSize; i++) dx[dstXSize + i] = i + 0.5 + dstXOff;
    const int has_nodata = g->nodata != -1e10;
    /* bytesRead bookkeeping, warp.go:221-231, 259-260, 278-332, 347 */
    const int bx = g->block_x > 0 ? g->block_x : bandX;   /* default: one scanline of the level */
    const int by = g->block_y > 0 ? g->block_y : 1;
    const int nXBlocks = (bandX + bx - 1) / bx, nYBlocks = (bandY + by - 1) / by;
    int bCache = -1, nBlocksRead = 0;
    uint8_t *seen = NULL;
    for (int iy = 0; iy < dstYSize; iy++) {
        memcpy(dx, dx + dstXSize, dstXSize * sizeof(double));
        const double dfY = iy + 0.5 + dstYOff;
        for (int i = 0; i < dstXSize; i++) dy[i] = dfY;
        approx_transform(&t, 1, dstXSize, dx, dy, ok);
        for (int i = 0; i < dstXSize; i++) {
            if (!ok[i]) continue;
            uint8_t *o = buf + ((int64_t)iy * dstXSize + i) * dsz;
            if (resample == 1) {
                double v;
                if (!bilinear_sample(band, srcType, bandX, bandY, has_nodata, g->nodata, dx[i], dy[i], &v))
                    continue;
                if (outType == OR_FLOAT32) { float f = (float)v; memcpy(o, &f, 4); }
                else or_gdal_copy_word(floor(v + 0.5), outType, o);
                continue;
            }
            if (dx[i] < 0 || dy[i] < 0) continue;
            if (dx[i] + 1.0e-10 >= 2147483647.0 || dy[i] + 1.0e-10 >= 2147483647.0) continue;
            const int iSrcX = (int)(dx[i] + 1.0e-10);
            const int iSrcY = (int)(dy[i] + 1.0e-10);
            if (iSrcX >= bandX || iSrcY >= bandY) continue;
            if (bCache == -1) {      /* stride of the first two usable columns of this row */
                int prev = -1, curr = -1;
                for (int j = i; j < dstXSize; j++) {
                    if (!ok[j] || dx[j] < 0 || dx[j] + 1.0e-10 >= 2147483647.0) continue;
                    const int sxj = (int)(dx[j] + 1.0e-10);
                    if (sxj >= bandX) continue;
                    if (prev < 0) prev = sxj;
                    else { curr = sxj; break; }
                }
                if (prev >= 0 && curr < prev) curr = prev;
                const int stride = curr - prev;
                bCache = stride >= 0 && stride < bx;
                if (bCache) seen = (uint8_t *)calloc((size_t)nXBlocks * nYBlocks, 1);
            }
            if (!bCache) nBlocksRead++;
            else {
                const int64_t blk = (int64_t)(iSrcX / bx) + (int64_t)(iSrcY / by) * nXBlocks;
                if (!seen[blk]) { seen[blk] = 1; nBlocksRead++; }
            }
            const int64_t sidx = (int64_t)iSrcY * bandX + iSrcX;
            if (supported) memcpy(o, (const uint8_t *)band + sidx * dsz, dsz);
            else or_gdal_copy_word(read_as_double(band, srcType, sidx), OR_FLOAT32, o);
        }
    }
    free(dx); free(dy); free(ok); free(seen);
    *bytes_read = (int32_t)(uint32_t)(uint64_t)((int64_t)bx * by * oracle_type_size(srcType) * nBlocksRead);
    bbox[0] = dstXOff; bbox[1] = dstYOff; bbox[2] = dstXSize; bbox[3] = dstYSize;
    if (outType == OR_BYTE && g->signed_byte) outType = OR_SIGNEDBYTE;    /* 354-359 */
    *dtype = outType;
    *out_buf = buf;
    return 0;
}

int oracle_warp(const oracle_granule *g, const oracle_crs *src,
                const oracle_crs *dst, const double dst_geot[6],
                int dst_w, int dst_h, int resample,
                void **out_buf, int *out_size, int32_t bbox[4],
                double *nodata, int *dtype, int *bytes_read) {
    return oracle_warp_geoloc(g, src, dst, dst_geot, dst_w, dst_h, resample, NULL, out_buf, out_size, bbox,
                              nodata, dtype, bytes_read);
}

/* ======================================================================== */
/* Tile pipeline for the CPU baseline                                       */
/* ======================================================================== */
typedef struct {
    const oracle_granule *granules; const oracle_crs *src_crs;
    const double *ts; const uint32_t *ph; const int32_t *ns;
    const oracle_crs *dst; const oracle_tile *tiles; int n_tiles;
    const int32_t *pair_granule; int resample;
    int mask_ns; const char *mask_value; int mask_inclusive; int n_ns;
    const oracle_scale_params *sp; const uint8_t *ramp; uint8_t *rgba_out;
    int max_w, max_h;            /* output slot of every tile (row stride max_w) */
    uint8_t *canvas_out;         /* optional typed canvases, n_tiles x n_out x max_h*max_w*4 B */
    int32_t *created_out;        /* optional n_tiles x 3 flags */
    int next; int err; pthread_mutex_t mu;
} render_job;

static int render_one(render_job *j, int ti) {
    const oracle_tile *tile = &j->tiles[ti];
    const int npairs = tile->pair_end - tile->pair_begin;
    const int64_t npx = (int64_t)tile->width * tile->height;
    oracle_flex_raster *fr = (oracle_flex_raster *)calloc(npairs > 0 ? npairs : 1, sizeof(*fr));
    void **bufs = (void **)calloc(npairs > 0 ? npairs : 1, sizeof(void *));
    int rc = 0;
    for (int p = 0; p < npairs; p++) {
        const int gi = j->pair_granule[tile->pair_begin + p];
        int sz, dt, br; int32_t bb[4]; double nd;
        rc = oracle_warp(&j->granules[gi], &j->src_crs[gi], j->dst, tile->dst_geot,
                         tile->width, tile->height, j->resample, &bufs[p], &sz, bb, &nd, &dt, &br);
        if (rc) goto out;
        fr[p].data = bufs[p]; fr[p].data_w = bb[2]; fr[p].data_h = bb[3];
        fr[p].width = tile->width; fr[p].height = tile->height;
        fr[p].off_x = bb[0]; fr[p].off_y = bb[1]; fr[p].dtype = dt; fr[p].ns = j->ns[gi];
        fr[p].nodata = nd; fr[p].timestamp = j->ts[gi]; fr[p].polygon_hash = j->ph[gi];
    }
    {
        oracle_canvas cv[4];
        void *cbuf[4];
        memset(cv, 0, sizeof(cv));
        for (int k = 0; k < j->n_ns; k++) { cbuf[k] = malloc((size_t)npx * 8); cv[k].data = cbuf[k]; }
        const char *bt[1] = {NULL};
        rc = oracle_merge_batch(fr, npairs, j->mask_ns, j->mask_value, bt, 0, j->mask_inclusive, cv, j->n_ns);
        const int64_t slot = (int64_t)j->max_w * j->max_h;
        uint8_t *rgba = (uint8_t *)malloc((size_t)npx * 4);
        if (!rc) {
            /* output namespaces exclude the mask layer */
            const uint8_t *bands[3];
            uint8_t *sb[3] = {NULL, NULL, NULL};
            int nb = 0, missing = 0;
            for (int k = 0; k < j->n_ns && nb < 3; k++) {
                if (k == j->mask_ns) continue;
                sb[nb] = (uint8_t *)malloc((size_t)npx);
                if (j->created_out) j->created_out[(int64_t)ti * 3 + nb] = cv[k].created;
                if (cv[k].created && j->canvas_out) {     /* tile_merger.go:562-652 typed canvas */
                    const int tsz = oracle_type_size(cv[k].dtype);
                    uint8_t *dst = j->canvas_out + ((int64_t)ti * (j->n_ns - (j->mask_ns >= 0 ? 1 : 0)) + nb) * slot * 4;
                    for (int r = 0; r < tile->height; r++)
                        memcpy(dst + (int64_t)r * j->max_w * tsz, (const uint8_t *)cv[k].data + (int64_t)r * tile->width * tsz,
                               (size_t)tile->width * tsz);
                }
                if (!cv[k].created) { missing = 1; }
                else oracle_scale(cv[k].data, cv[k].dtype, npx, cv[k].nodata, j->sp->offset,
                                  j->sp->scale, j->sp->clip, j->sp->colour_scale, sb[nb]);
                bands[nb] = sb[nb];
                nb++;
            }
            if (missing) memset(rgba, 0, (size_t)npx * 4);
            else rc = oracle_encode_rgba(bands, nb, tile->width, tile->height, j->ramp, rgba);
            for (int k = 0; k < 3; k++) free(sb[k]);
            if (!rc && j->rgba_out) {
                uint8_t *o = j->rgba_out + (int64_t)ti * slot * 4;
                for (int r = 0; r < tile->height; r++)
                    memcpy(o + (int64_t)r * j->max_w * 4, rgba + (int64_t)r * tile->width * 4, (size_t)tile->width * 4);
            }
        }
        free(rgba);
        for (int k = 0; k < j->n_ns; k++) free(cbuf[k]);
    }
out:
    for (int p = 0; p < npairs; p++) free(bufs[p]);
    free(bufs); free(fr);
    return rc;
}

static void *render_worker(void *arg) {
    render_job *j = (render_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int ti = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (ti >= j->n_tiles) break;
        int rc = render_one(j, ti);
        if (rc) { pthread_mutex_lock(&j->mu); if (!j->err) j->err = rc; pthread_mutex_unlock(&j->mu); }
    }
    return NULL;
}

int oracle_render_tiles2(const oracle_granule *granules, const oracle_crs *src_crs,
                         const double *ts, const uint32_t *ph, const int32_t *ns,
                         int n_granules, const oracle_crs *dst,
                         const oracle_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int resample,
                         int mask_ns, const char *mask_value, int mask_inclusive,
                         int n_ns, const oracle_scale_params *sp,
                         const uint8_t *ramp, uint8_t *rgba_out, int max_w, int max_h,
                         uint8_t *canvas_out, int32_t *created_out, int n_threads) {
    (void)n_granules;
    if (n_ns > 4) return -7;
    for (int t = 0; t < n_tiles; t++)
        if (tiles[t].width <= 0 || tiles[t].height <= 0 || tiles[t].width > max_w || tiles[t].height > max_h) return -1;
    render_job j = {granules, src_crs, ts, ph, ns, dst, tiles, n_tiles, pair_granule, resample,
                    mask_ns, mask_value, mask_inclusive, n_ns, sp, ramp, rgba_out, max_w, max_h,
                    canvas_out, created_out, 0, 0, PTHREAD_MUTEX_INITIALIZER};
    if (n_threads < 1) n_threads = 1;
    if (n_threads == 1) { render_worker(&j); return j.err; }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * n_threads);
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, render_worker, &j);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    free(th);
    return j.err;
}

int oracle_render_tiles(const oracle_granule *granules, const oracle_crs *src_crs,
                        const double *ts, const uint32_t *ph, const int32_t *ns,
                        int n_granules, const oracle_crs *dst,
                        const oracle_tile *tiles, int n_tiles,
                        const int32_t *pair_granule, int resample,
                        int mask_ns, const char *mask_value, int mask_inclusive,
                        int n_ns, const oracle_scale_params *sp,
                        const uint8_t *ramp, uint8_t *rgba_out, int n_threads) {
    int mw = 1, mh = 1;
    for (int t = 0; t < n_tiles; t++) {
        if (tiles[t].width > mw) mw = tiles[t].width;
        if (tiles[t].height > mh) mh = tiles[t].height;
    }
    return oracle_render_tiles2(granules, src_crs, ts, ph, ns, n_granules, dst, tiles, n_tiles, pair_granule,
                                resample, mask_ns, mask_value, mask_inclusive, n_ns, sp, ramp, rgba_out, mw, mh,
                                NULL, NULL, n_threads);
}

/* ======================================================================== */
/* worker/gdalprocess/drill.go:90-227 readData                               */
/* ======================================================================== */
static void band_mean(const float *d, const uint8_t *mask, int npx, float nodata,
                      float lo, float hi, int pixel_count, double *v, int32_t *c) {
    float sum = 0.0f;
    int32_t total = 0;
    for (int i = 0; i < npx; i++) {                       /* 153-170 */
        if (mask[i] == 255 && d[i] != nodata) {
            const float val = d[i];
            if (pixel_count != 0) total++;
            if (val < lo || val > hi) continue;
            if (pixel_count == 0) { sum += val; total++; }
            else sum += 1.0f;
        }
    }
    if (total > 0) { *v = (double)(sum / (float)total); *c = total; }   /* 172-177 */
    else { *v = 0; *c = 0; }
}

int oracle_drill_read_data(const float *data, int nbands, int count_x, int count_y,
                           const uint8_t *mask, float nodata, float clip_lower,
                           float clip_upper, int pixel_count, int band_strides,
                           double *out_value, int32_t *out_count) {
    const int npx = count_x * count_y;
    if (band_strides <= 0) band_strides = 1;             /* 110-112 */
    int nrow = 0;
    for (int ibBgn = 0; ibBgn < nbands; ibBgn += band_strides) {   /* 128 */
        int ibEnd = ibBgn + band_strides;
        if (ibEnd > nbands) ibEnd = nbands;
        int bandsRead[2] = {ibBgn, ibEnd - 1};
        const int eff = band_strides == 1 ? 1 : 2;
        double bv[2]; int32_t bc[2];
        for (int ib = 0; ib < eff; ib++)
            band_mean(data + (int64_t)bandsRead[ib] * npx, mask, npx, nodata, clip_lower,
                      clip_upper, pixel_count, &bv[ib], &bc[ib]);
        out_value[nrow] = bv[0]; out_count[nrow] = bc[0]; nrow++;          /* 195 */
        if (band_strides > 2 && eff > 1) {                                  /* 197-214 */
            const double beta = (bv[1] - bv[0]) / (double)(band_strides - 1);
            const double cnt = round((double)(bc[0] + bc[1]) / 2.0);
            for (int ip = 1; ip < band_strides - 1; ip++) {
                out_value[nrow] = bv[0] + (double)ip * beta;
                out_count[nrow] = (int32_t)cnt;
                nrow++;
            }
        }
        if (eff > 1) { out_value[nrow] = bv[1]; out_count[nrow] = bc[1]; nrow++; }   /* 216-218 */
    }
    return nrow;
}

void oracle_drill_merge(const double *values, const int32_t *counts,
                        int n_files, int n_dates, double *out) {
    for (int d = 0; d < n_dates; d++) {                    /* drill_merger.go:79-93 */
        double total = 0.0;
        long count = 0;
        for (int f = 0; f < n_files; f++) {
            double v = values[(int64_t)f * n_dates + d];
            if (!isnan(v)) { total += v * (double)counts[(int64_t)f * n_dates + d]; count += counts[(int64_t)f * n_dates + d]; }
        }
        out[d] = (!isnan(total) && count > 0) ? total / (double)count : NAN;
    }
}

/* ======================================================================== */
/* worker/gdalprocess/drill.go:363-423 getDrillFileDescriptor + 275-327      */
/* createMask, with GDAL 3.0.1's rasterizer (alg/llrasterize.cpp             */
/* GDALdllImageFilledPolygon + GDALdllImageLineAllTouched, ALL_TOUCHED=TRUE) */
/* restated [ext], after OGR_G_Buffer(g, 0, 30) as GEOS 3.7.2 computes it  */
/* (rings_buffer0 below).                                                    */
/* ======================================================================== */
typedef struct { double *x, *y; int *part_size, *part_poly; int n_parts, n_pts, cap_pts, cap_parts, n_polys; } or_rings;

static void rings_push(or_rings *r, double x, double y) {
    if (r->n_pts == r->cap_pts) {
        r->cap_pts = r->cap_pts ? 2 * r->cap_pts : 64;
        r->x = (double *)realloc(r->x, sizeof(double) * r->cap_pts);
        r->y = (double *)realloc(r->y, sizeof(double) * r->cap_pts);
    }
    r->x[r->n_pts] = x; r->y[r->n_pts] = y; r->n_pts++;
    r->part_size[r->n_parts - 1]++;
}
static void rings_new_part(or_rings *r) {
    if (r->n_parts == r->cap_parts) {
        r->cap_parts = r->cap_parts ? 2 * r->cap_parts : 8;
        r->part_size = (int *)realloc(r->part_size, sizeof(int) * r->cap_parts);
        r->part_poly = (int *)realloc(r->part_poly, sizeof(int) * r->cap_parts);
    }
    r->part_poly[r->n_parts] = r->n_polys;
    r->part_size[r->n_parts++] = 0;
}
static void rings_free(or_rings *r) {
    free(r->x); free(r->y); free(r->part_size); free(r->part_poly); memset(r, 0, sizeof(*r));
}

/* Nested JSON arrays of numbers: depth of the first '[' below `p` decides
 * the level of a ring (Polygon 3 = [ring][pt][xy], MultiPolygon 4). */
static const char *skip_ws(const char *p) { while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') p++; return p; }

static const char *parse_coords(const char *p, int depth, int ring_depth, or_rings *r) {
    p = skip_ws(p);
    if (*p != '[') return NULL;
    p++;
    if (depth == ring_depth - 1) r->n_polys++;  /* a polygon: its first ring is the shell */
    if (depth == ring_depth) rings_new_part(r);
    if (depth == ring_depth + 1) {               /* a point [x, y(, z)] */
        char *e;
        const double x = strtod(p, &e);
        if (e == p) return NULL;
        p = skip_ws(e);
        if (*p != ',') return NULL;
        p++;
        const double y = strtod(p, &e);
        if (e == p) return NULL;
        p = skip_ws(e);
        while (*p == ',') {        /* a third (z) coordinate is ignored */
            p++;
            strtod(p, &e);
            if (e == p) return NULL;
            p = skip_ws(e);
        }
        if (*p != ']') return NULL;
        rings_push(r, x, y);
        return p + 1;
    }
    p = skip_ws(p);
    if (*p == ']') return p + 1;
    for (;;) {
        p = parse_coords(p, depth + 1, ring_depth, r);
        if (!p) return NULL;
        p = skip_ws(p);
        if (*p == ',') { p++; continue; }
        if (*p == ']') return p + 1;
        return NULL;
    }
}

/* The geometry of a GeoJSON Feature or a bare Polygon / MultiPolygon. */
static int parse_geojson(const char *js, or_rings *r) {
    const char *g = strstr(js, "\"geometry\"");
    const char *base = g ? g : js;
    const char *mp = strstr(base, "\"MultiPolygon\"");
    const char *pg = strstr(base, "\"Polygon\"");
    const char *c = strstr(base, "\"coordinates\"");
    if (!c || (!mp && !pg)) return -1;
    c = strchr(c, ':');
    if (!c) return -1;
    const int ring_depth = mp ? 2 : 1;            /* depth (from 0) at which rings start */
    if (!parse_coords(c + 1, 0, ring_depth, r)) return -1;
    return r->n_parts > 0 ? 0 : -1;
}

/* ---- OGR_G_Buffer(g, 0, 30) (drill.go:364-367) as GEOS 3.7.2 computes a
 * zero-distance polygon buffer [ext, parity unpinned: GEOS is absent]:
 * every ring (repeated points removed; a shell under 3 points drops its
 * polygon, a ring under 4 points is skipped) is a curve whose sides carry a
 * depth step: +1 across it from the right to the left for a shell that
 * CGAlgorithms::isCCW calls counter-clockwise (interior left) or a hole it
 * calls clockwise, -1 otherwise.  The curves are noded (crossings, touches,
 * collinear overlaps), equal edges merged with their steps added, and the
 * result is the region of depth >= 1 (depth 0 far outside): its boundary
 * edges, interior on their right.  Here the depth at a point is the step-
 * weighted winding number over all edges, brute force; a polygon already
 * valid keeps its vertices (rings turned interior-right).  An empty result
 * keeps the rings as drawn (drill.go:366). */
typedef struct { double ax, ay, bx, by; int q, ring; } or_seg;

/* sign of (b - a) x (c - a): the double value when it clears its rounding
 * bound, else the differences exactly (two-diff) and the products and their
 * difference in double-double arithmetic -- the product's predicate, so the
 * two agree on every degenerate configuration */
static void or_two_diff(double a, double b, double *hi, double *lo) {
    const double s = a - b, bb = s - a;
    *hi = s; *lo = (a - (s - bb)) - (b + bb);
}
static void or_dd_mul(double ah, double al, double bh, double bl, double *hi, double *lo) {
    const double p = ah * bh;
    const double e = fma(ah, bh, -p) + (ah * bl + al * bh);
    *hi = p + e; *lo = e - (*hi - p);
}
static int or_orient(double ax, double ay, double bx, double by, double cx, double cy) {
    if ((cx == ax && cy == ay) || (cx == bx && cy == by)) return 0;
    const double l = (bx - ax) * (cy - ay), r = (by - ay) * (cx - ax);
    const double det = l - r, bound = 1e-15 * (fabs(l) + fabs(r));
    if (det > bound) return 1;
    if (det < -bound) return -1;
    if (l == 0 && r == 0) return 0;
    double d1h, d1l, d2h, d2l, d3h, d3l, d4h, d4l, ph, pl, qh, ql;
    or_two_diff(bx, ax, &d1h, &d1l); or_two_diff(cy, ay, &d2h, &d2l);
    or_two_diff(by, ay, &d3h, &d3l); or_two_diff(cx, ax, &d4h, &d4l);
    or_dd_mul(d1h, d1l, d2h, d2l, &ph, &pl);
    or_dd_mul(d3h, d3l, d4h, d4l, &qh, &ql);
    const double s = ph - qh, bb = s - ph;
    const double e = ((ph - (s - bb)) - (qh + bb)) + pl - ql;
    const double v = s + e;
    return (v > 0) - (v < 0);
}

/* CGAlgorithms::isCCW: the turn at the first highest vertex of a closed ring */
static int or_ring_ccw(const double *x, const double *y, int n) {
    int hi = 0, last = n - 1;
    for (int i = 1; i <= last; i++) if (y[i] > y[hi]) hi = i;
    int a = hi, b = hi;
    do { a = a == 0 ? last : a - 1; } while (x[a] == x[hi] && y[a] == y[hi] && a != hi);
    do { b = (b + 1) % last; } while (x[b] == x[hi] && y[b] == y[hi] && b != hi);
    if ((x[a] == x[hi] && y[a] == y[hi]) || (x[b] == x[hi] && y[b] == y[hi]) || (x[a] == x[b] && y[a] == y[b])) return 0;
    const int o = or_orient(x[a], y[a], x[hi], y[hi], x[b], y[b]);
    return o == 0 ? x[a] > x[b] : o > 0;
}

/* Sunday's winding rule, one edge, weight q */
static int or_wind(const or_seg *e, double px, double py) {
    if (e->ay <= py) return (e->by > py && or_orient(e->ax, e->ay, e->bx, e->by, px, py) > 0) ? e->q : 0;
    return (e->by <= py && or_orient(e->ax, e->ay, e->bx, e->by, px, py) < 0) ? -e->q : 0;
}

/* depth just right of edge k: the other edges' winding at its midpoint plus
 * its own share.  Edge sets of 48 or more that are wider than tall are cast
 * in the frame (x, y) -> (y, -x), as the product does (its rays then run
 * across the short side); the winding numbers agree off the edges. */
static int or_depth_right_raw(const or_seg *s, int n, int k) {
    const double mx = 0.5 * (s[k].ax + s[k].bx), my = 0.5 * (s[k].ay + s[k].by);
    int d = 0;
    for (int f = 0; f < n; f++) if (f != k) d += or_wind(&s[f], mx, my);
    if (s[k].ay == s[k].by) return s[k].ax < s[k].bx ? d - s[k].q : d;   /* d = depth above */
    return s[k].by < s[k].ay ? d - s[k].q : d;
}
static int or_turned(const or_seg *s, int n) {
    if (n < 48) return 0;
    double x0 = HUGE_VAL, x1 = -HUGE_VAL, y0 = HUGE_VAL, y1 = -HUGE_VAL;
    for (int k = 0; k < n; k++) {
        x0 = fmin(x0, fmin(s[k].ax, s[k].bx)); x1 = fmax(x1, fmax(s[k].ax, s[k].bx));
        y0 = fmin(y0, fmin(s[k].ay, s[k].by)); y1 = fmax(y1, fmax(s[k].ay, s[k].by));
    }
    return x1 - x0 > y1 - y0;
}
static or_seg *or_turn(const or_seg *s, int n) {
    or_seg *t = (or_seg *)malloc(sizeof(or_seg) * (n > 0 ? n : 1));
    for (int k = 0; k < n; k++) {
        or_seg e = {s[k].ay, -s[k].ax, s[k].by, -s[k].bx, s[k].q, s[k].ring};
        t[k] = e;
    }
    return t;
}

static int on_open_seg(double ax, double ay, double bx, double by, double px, double py) {
    if ((px == ax && py == ay) || (px == bx && py == by)) return 0;
    return fmin(ax, bx) <= px && px <= fmax(ax, bx) && fmin(ay, by) <= py && py <= fmax(ay, by);
}

typedef struct { double x, y; } or_pt;
typedef struct { or_pt *p; int n, cap; } or_ptlist;
static void ptl_push(or_ptlist *l, double x, double y) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 4; l->p = (or_pt *)realloc(l->p, sizeof(or_pt) * l->cap); }
    l->p[l->n].x = x; l->p[l->n].y = y; l->n++;
}
static int pt_lt(double ax, double ay, double bx, double by) { return ax < bx || (ax == bx && ay < by); }
static int cmp_seg_key(const void *u, const void *v) {
    const or_seg *a = (const or_seg *)u, *b = (const or_seg *)v;
    if (pt_lt(a->ax, a->ay, b->ax, b->ay)) return -1;
    if (pt_lt(b->ax, b->ay, a->ax, a->ay)) return 1;
    if (pt_lt(a->bx, a->by, b->bx, b->by)) return -1;
    if (pt_lt(b->bx, b->by, a->bx, a->by)) return 1;
    return 0;
}
static const or_seg *g_sort_seg;
static int cmp_by_xmin(const void *u, const void *v) {
    const or_seg *a = &g_sort_seg[*(const int *)u], *b = &g_sort_seg[*(const int *)v];
    const double x = fmin(a->ax, a->bx), y = fmin(b->ax, b->bx);
    return (x > y) - (x < y);
}
static double g_dx, g_dy, g_ox, g_oy;
static int cmp_along(const void *u, const void *v) {
    const or_pt *a = (const or_pt *)u, *b = (const or_pt *)v;
    const double s = (a->x - g_ox) * g_dx + (a->y - g_oy) * g_dy, t = (b->x - g_ox) * g_dx + (b->y - g_oy) * g_dy;
    if (s != t) return (s > t) - (s < t);
    return pt_lt(a->x, a->y, b->x, b->y) ? -1 : pt_lt(b->x, b->y, a->x, a->y) ? 1 : 0;
}

static void rings_buffer0(or_rings *r) {
    /* the curves */
    int cap = r->n_pts + 8, ns = 0, ncurves = 0;
    or_seg *s = (or_seg *)malloc(sizeof(or_seg) * cap);
    int *cstart = (int *)malloc(sizeof(int) * (r->n_parts + 1)), *cq = (int *)malloc(sizeof(int) * (r->n_parts + 1));
    double *cx = (double *)malloc(sizeof(double) * (r->n_pts + 1)), *cy = (double *)malloc(sizeof(double) * (r->n_pts + 1));
    int skip = 0;
    for (int k = 0, off = 0; k < r->n_parts; off += r->part_size[k++]) {
        const int shell = k == 0 || r->part_poly[k] != r->part_poly[k - 1];
        int n = 0;
        for (int i = 0; i < r->part_size[k]; i++)
            if (n == 0 || cx[n - 1] != r->x[off + i] || cy[n - 1] != r->y[off + i]) { cx[n] = r->x[off + i]; cy[n] = r->y[off + i]; n++; }
        if (shell) skip = n < 3;
        if (skip) continue;
        if (n > 0 && (cx[0] != cx[n - 1] || cy[0] != cy[n - 1])) { cx[n] = cx[0]; cy[n] = cy[0]; n++; }
        if (n < 4) continue;
        const int q = (shell ? 1 : -1) * (or_ring_ccw(cx, cy, n) ? 1 : -1);
        cstart[ncurves] = ns; cq[ncurves] = q;
        for (int i = 0; i + 1 < n; i++) {
            or_seg e = {cx[i], cy[i], cx[i + 1], cy[i + 1], q, ncurves};
            s[ns++] = e;
        }
        ncurves++;
    }
    cstart[ncurves] = ns;
    free(cx); free(cy);
    if (ns == 0) { free(s); free(cstart); free(cq); return; }

    /* noding: pairs from a sweep in x */
    or_ptlist *sp = (or_ptlist *)calloc(ns, sizeof(or_ptlist));
    int *ord = (int *)malloc(sizeof(int) * ns), split = 0, overlap = 0, touch = 0;
    for (int i = 0; i < ns; i++) ord[i] = i;
    g_sort_seg = s;
    qsort(ord, ns, sizeof(int), cmp_by_xmin);
    for (int u = 0; u < ns; u++) {
        for (int v = u + 1; v < ns && fmin(s[ord[v]].ax, s[ord[v]].bx) <= fmax(s[ord[u]].ax, s[ord[u]].bx); v++) {
            const int i = ord[u] < ord[v] ? ord[u] : ord[v], j = ord[u] < ord[v] ? ord[v] : ord[u];
            const or_seg *a = &s[i], *b = &s[j];
            if (fmax(a->ay, a->by) < fmin(b->ay, b->by) || fmax(b->ay, b->by) < fmin(a->ay, a->by)) continue;
            const int o1 = or_orient(b->ax, b->ay, b->bx, b->by, a->ax, a->ay), o2 = or_orient(b->ax, b->ay, b->bx, b->by, a->bx, a->by);
            const int o3 = or_orient(a->ax, a->ay, a->bx, a->by, b->ax, b->ay), o4 = or_orient(a->ax, a->ay, a->bx, a->by, b->bx, b->by);
            if (!o1 && !o2 && !o3 && !o4) {
                const int alongx = fabs(a->bx - a->ax) >= fabs(a->by - a->ay);
                const double a0 = alongx ? fmin(a->ax, a->bx) : fmin(a->ay, a->by), a1 = alongx ? fmax(a->ax, a->bx) : fmax(a->ay, a->by);
                const double b0 = alongx ? fmin(b->ax, b->bx) : fmin(b->ay, b->by), b1 = alongx ? fmax(b->ax, b->bx) : fmax(b->ay, b->by);
                if (fmin(a1, b1) > fmax(a0, b0)) overlap = 1;
                if (on_open_seg(a->ax, a->ay, a->bx, a->by, b->ax, b->ay)) { ptl_push(&sp[i], b->ax, b->ay); split = 1; }
                if (on_open_seg(a->ax, a->ay, a->bx, a->by, b->bx, b->by)) { ptl_push(&sp[i], b->bx, b->by); split = 1; }
                if (on_open_seg(b->ax, b->ay, b->bx, b->by, a->ax, a->ay)) { ptl_push(&sp[j], a->ax, a->ay); split = 1; }
                if (on_open_seg(b->ax, b->ay, b->bx, b->by, a->bx, a->by)) { ptl_push(&sp[j], a->bx, a->by); split = 1; }
                continue;
            }
            if (o1 * o2 < 0 && o3 * o4 < 0) {
                /* both segments lesser point first, the lesser segment first: every
                 * copy of a segment meets a third one at the same point */
                double s0x = a->ax, s0y = a->ay, s1x = a->bx, s1y = a->by, t0x = b->ax, t0y = b->ay, t1x = b->bx, t1y = b->by, tmp;
                if (pt_lt(s1x, s1y, s0x, s0y)) { tmp = s0x; s0x = s1x; s1x = tmp; tmp = s0y; s0y = s1y; s1y = tmp; }
                if (pt_lt(t1x, t1y, t0x, t0y)) { tmp = t0x; t0x = t1x; t1x = tmp; tmp = t0y; t0y = t1y; t1y = tmp; }
                if (pt_lt(t0x, t0y, s0x, s0y) || (t0x == s0x && t0y == s0y && pt_lt(t1x, t1y, s1x, s1y))) {
                    tmp = s0x; s0x = t0x; t0x = tmp; tmp = s0y; s0y = t0y; t0y = tmp;
                    tmp = s1x; s1x = t1x; t1x = tmp; tmp = s1y; s1y = t1y; t1y = tmp;
                }
                const double dx = s1x - s0x, dy = s1y - s0y, ex = t1x - t0x, ey = t1y - t0y;
                const double kk = ((t0x - s0x) * ey - (t0y - s0y) * ex) / (dx * ey - dy * ex);
                double px = s0x + kk * dx, py = s0y + kk * dy;
                px = fmin(fmax(px, fmax(fmin(a->ax, a->bx), fmin(b->ax, b->bx))), fmin(fmax(a->ax, a->bx), fmax(b->ax, b->bx)));
                py = fmin(fmax(py, fmax(fmin(a->ay, a->by), fmin(b->ay, b->by))), fmin(fmax(a->ay, a->by), fmax(b->ay, b->by)));
                ptl_push(&sp[i], px, py); ptl_push(&sp[j], px, py);
                split = 1;
                continue;
            }
            if (!o3 && on_open_seg(a->ax, a->ay, a->bx, a->by, b->ax, b->ay)) { ptl_push(&sp[i], b->ax, b->ay); split = 1; }
            if (!o4 && on_open_seg(a->ax, a->ay, a->bx, a->by, b->bx, b->by)) { ptl_push(&sp[i], b->bx, b->by); split = 1; }
            if (!o1 && on_open_seg(b->ax, b->ay, b->bx, b->by, a->ax, a->ay)) { ptl_push(&sp[j], a->ax, a->ay); split = 1; }
            if (!o2 && on_open_seg(b->ax, b->ay, b->bx, b->by, a->bx, a->by)) { ptl_push(&sp[j], a->bx, a->by); split = 1; }
            const int shares = (a->ax == b->ax && a->ay == b->ay) || (a->ax == b->bx && a->ay == b->by) ||
                               (a->bx == b->ax && a->by == b->ay) || (a->bx == b->bx && a->by == b->by);
            const int len = a->ring == b->ring ? cstart[a->ring + 1] - cstart[a->ring] : 0;
            if (shares && !(a->ring == b->ring && (j - i == 1 || j - i == len - 1))) touch = 1;
        }
    }
    free(ord);

    int done = 0;
    if (!split && !overlap && !touch) {            /* valid: keep the vertices, interior right */
        int ok = 1;
        int *flip = (int *)malloc(sizeof(int) * ncurves);
        or_seg *ts = or_turned(s, ns) ? or_turn(s, ns) : NULL;
        for (int c = 0; c < ncurves && ok; c++) {
            const int dr = or_depth_right_raw(ts ? ts : s, ns, cstart[c]), dl = dr + cq[c];
            ok = (dr == 1 && dl == 0) || (dr == 0 && dl == 1);
            flip[c] = dl == 1;
        }
        free(ts);
        if (ok) {
            or_rings out;
            memset(&out, 0, sizeof(out));
            for (int c = 0; c < ncurves; c++) {
                rings_new_part(&out);
                const int a = cstart[c], b = cstart[c + 1];
                if (!flip[c]) { for (int k = a; k < b; k++) rings_push(&out, s[k].ax, s[k].ay); rings_push(&out, s[b - 1].bx, s[b - 1].by); }
                else { for (int k = b - 1; k >= a; k--) rings_push(&out, s[k].bx, s[k].by); rings_push(&out, s[a].ax, s[a].ay); }
            }
            rings_free(r);
            *r = out;
            done = 1;
        }
        free(flip);
    }
    if (!done) {
        /* noded edges in canonical direction (lesser point first), merged */
        int ne = 0, ecap = ns + 16;
        or_seg *e = (or_seg *)malloc(sizeof(or_seg) * ecap);
        for (int k = 0; k < ns; k++) {
            g_ox = s[k].ax; g_oy = s[k].ay; g_dx = s[k].bx - s[k].ax; g_dy = s[k].by - s[k].ay;
            if (sp[k].n) qsort(sp[k].p, sp[k].n, sizeof(or_pt), cmp_along);
            double px = s[k].ax, py = s[k].ay;
            for (int t = 0; t <= sp[k].n; t++) {
                const double qx = t < sp[k].n ? sp[k].p[t].x : s[k].bx, qy = t < sp[k].n ? sp[k].p[t].y : s[k].by;
                if (qx == px && qy == py) continue;
                if (ne == ecap) { ecap *= 2; e = (or_seg *)realloc(e, sizeof(or_seg) * ecap); }
                if (pt_lt(px, py, qx, qy)) { or_seg x = {px, py, qx, qy, s[k].q, -1}; e[ne++] = x; }
                else { or_seg x = {qx, qy, px, py, -s[k].q, -1}; e[ne++] = x; }
                px = qx; py = qy;
            }
        }
        qsort(e, ne, sizeof(or_seg), cmp_seg_key);
        int nu = 0;
        for (int k = 0; k < ne; k++) {
            if (nu && !cmp_seg_key(&e[nu - 1], &e[k])) e[nu - 1].q += e[k].q;
            else e[nu++] = e[k];
        }
        int m = 0;
        for (int k = 0; k < nu; k++) if (e[k].q) e[m++] = e[k];
        /* result edges, directed interior-right */
        or_seg *res = (or_seg *)malloc(sizeof(or_seg) * (m + 1));
        int nr = 0;
        or_seg *te = or_turned(e, m) ? or_turn(e, m) : NULL;
        for (int k = 0; k < m; k++) {
            const int dr = or_depth_right_raw(te ? te : e, m, k), dl = dr + e[k].q;
            if (dr >= 1 && dl <= 0) { or_seg x = {e[k].ax, e[k].ay, e[k].bx, e[k].by, 0, 0}; res[nr++] = x; }
            else if (dl >= 1 && dr <= 0) { or_seg x = {e[k].bx, e[k].by, e[k].ax, e[k].ay, 0, 0}; res[nr++] = x; }
        }
        free(te);
        if (nr) {                                  /* chain them into closed rings */
            or_rings out;
            memset(&out, 0, sizeof(out));
            char *used = (char *)calloc(nr, 1);
            for (int k0 = 0; k0 < nr; k0++) {
                if (used[k0]) continue;
                rings_new_part(&out);
                rings_push(&out, res[k0].ax, res[k0].ay);
                int k = k0;
                for (;;) {
                    used[k] = 1;
                    rings_push(&out, res[k].bx, res[k].by);
                    if (res[k].bx == res[k0].ax && res[k].by == res[k0].ay) break;
                    int nxt = -1;
                    for (int t = 0; t < nr && nxt < 0; t++)
                        if (!used[t] && res[t].ax == res[k].bx && res[t].ay == res[k].by) nxt = t;
                    if (nxt < 0) { rings_push(&out, res[k0].ax, res[k0].ay); break; }
                    k = nxt;
                }
            }
            free(used);
            rings_free(r);
            *r = out;
        }
        free(res);
        free(e);
    }
    for (int k = 0; k < ns; k++) free(sp[k].p);
    free(sp); free(s); free(cstart); free(cq);
}

static int point_in_rings(const or_rings *r, double px, double py) {   /* even-odd over all rings */
    int inside = 0, off = 0;
    for (int k = 0; k < r->n_parts; k++) {
        const int n = r->part_size[k];
        for (int i = 0, j = n - 1; i < n; j = i++) {
            const double xi = r->x[off + i], yi = r->y[off + i], xj = r->x[off + j], yj = r->y[off + j];
            if ((yi > py) != (yj > py) && px < (xj - xi) * (py - yi) / (yj - yi) + xi) inside = !inside;
        }
        off += n;
    }
    return inside;
}

/* Envelope of (rings intersect [x0,x1]x[y0,y1]): vertices inside, edge /
 * side crossings, rectangle corners inside the polygon.  0 = empty. */
static int intersection_envelope(const or_rings *r, double x0, double y0, double x1, double y1, double env[4]) {
    double mnx = HUGE_VAL, mny = HUGE_VAL, mxx = -HUGE_VAL, mxy = -HUGE_VAL;
    int any = 0;
#define OR_ADD(px, py)                       \
    do {                                     \
        const double _x = (px), _y = (py);   \
        any = 1;                             \
        mnx = _x < mnx ? _x : mnx;           \
        mxx = _x > mxx ? _x : mxx;           \
        mny = _y < mny ? _y : mny;           \
        mxy = _y > mxy ? _y : mxy;           \
    } while (0)
    int off = 0;
    for (int k = 0; k < r->n_parts; k++) {
        const int n = r->part_size[k];
        for (int i = 0; i < n; i++) {
            const double ax = r->x[off + i], ay = r->y[off + i];
            if (ax >= x0 && ax <= x1 && ay >= y0 && ay <= y1) OR_ADD(ax, ay);
            const int j = (i + 1) % n;
            const double bx = r->x[off + j], by = r->y[off + j];
            const double xs[2] = {x0, x1}, ys[2] = {y0, y1};
            for (int s = 0; s < 2; s++) {
                const double X = xs[s];
                if ((ax - X) * (bx - X) <= 0 && ax != bx) {
                    const double y = ay + (X - ax) * (by - ay) / (bx - ax);
                    if (y >= y0 && y <= y1) OR_ADD(X, y);
                }
                const double Y = ys[s];
                if ((ay - Y) * (by - Y) <= 0 && ay != by) {
                    const double x = ax + (Y - ay) * (bx - ax) / (by - ay);
                    if (x >= x0 && x <= x1) OR_ADD(x, Y);
                }
            }
        }
        off += n;
    }
    const double cx[4] = {x0, x1, x1, x0}, cy[4] = {y0, y0, y1, y1};
    for (int k = 0; k < 4; k++) if (point_in_rings(r, cx[k], cy[k])) OR_ADD(cx[k], cy[k]);
#undef OR_ADD
    if (!any) return 0;
    env[0] = mnx; env[1] = mny; env[2] = mxx; env[3] = mxy;
    return 1;
}

static double fmt6(double v) {    /* Go fmt "%f" then OGR's parse: 6 decimals */
    char buf[64];
    snprintf(buf, sizeof(buf), "%.6f", v);
    return strtod(buf, NULL);
}

static void burn(uint8_t *m, int w, int h, int x, int y) { if (x >= 0 && x < w && y >= 0 && y < h) m[(int64_t)y * w + x] = 255; }

static int cmp_int(const void *a, const void *b) { const int x = *(const int *)a, y = *(const int *)b; return (x > y) - (x < y); }

/* GDALdllImageFilledPolygon (GDAL 3.0.1 alg/llrasterize.cpp). */
static void filled_polygon(const or_rings *r, uint8_t *m, int w, int h) {
    const int n = r->n_pts;
    if (!r->n_parts || n == 0) return;
    int *ints = (int *)malloc(sizeof(int) * (n + 1));
    double dminy = r->y[0], dmaxy = r->y[0];
    for (int i = 1; i < n; i++) { if (r->y[i] < dminy) dminy = r->y[i]; if (r->y[i] > dmaxy) dmaxy = r->y[i]; }
    int miny = (int)dminy, maxy = (int)dmaxy;
    if (miny < 0) miny = 0;
    if (maxy >= h) maxy = h - 1;
    const int minx = 0, maxx = w - 1;
    for (int y = miny; y <= maxy; y++) {
        int partoffset = 0, part = 0, nints = 0;
        const double dy = y + 0.5;
        for (int i = 0; i < n; i++) {
            if (i == partoffset + r->part_size[part]) { partoffset += r->part_size[part]; part++; }
            int ind1, ind2;
            if (i == partoffset) { ind1 = partoffset + r->part_size[part] - 1; ind2 = partoffset; }
            else { ind1 = i - 1; ind2 = i; }
            double dy1 = r->y[ind1], dy2 = r->y[ind2];
            if ((dy1 < dy && dy2 < dy) || (dy1 > dy && dy2 > dy)) continue;
            double dx1, dx2;
            if (dy1 < dy2) { dx1 = r->x[ind1]; dx2 = r->x[ind2]; }
            else if (dy1 > dy2) { dy2 = r->y[ind1]; dy1 = r->y[ind2]; dx2 = r->x[ind1]; dx1 = r->x[ind2]; }
            else {   /* horizontal: bottom segments filled separately, top ones skipped */
                if (r->x[ind1] > r->x[ind2]) {
                    const int hx1 = (int)floor(r->x[ind2] + 0.5), hx2 = (int)floor(r->x[ind1] + 0.5);
                    if (hx1 > maxx || hx2 <= minx) continue;
                    for (int x = hx1 < 0 ? 0 : hx1; x <= hx2 - 1 && x <= maxx; x++) burn(m, w, h, x, y);
                }
                continue;
            }
            if (dy < dy2 && dy >= dy1) {
                const double intersect = (dy - dy1) * (dx2 - dx1) / (dy2 - dy1) + dx1;
                ints[nints++] = (int)floor(intersect + 0.5);
            }
        }
        qsort(ints, nints, sizeof(int), cmp_int);
        for (int i = 0; i + 1 < nints; i += 2) {
            if (ints[i] <= maxx && ints[i + 1] > minx) {
                int xs = ints[i], xe = ints[i + 1] - 1;
                if (xs > xe) continue;
                if (xs < 0) xs = 0;
                if (xe >= w) xe = w - 1;
                for (int x = xs; x <= xe; x++) burn(m, w, h, x, y);
            }
        }
    }
    free(ints);
}

/* GDALdllImageLineAllTouched (GDAL 3.0.1), burn value only. */
static void line_all_touched(const or_rings *r, uint8_t *m, int w, int h) {
    for (int k = 0, n = 0; k < r->n_parts; n += r->part_size[k++]) {
        for (int j = 1; j < r->part_size[k]; j++) {
            double dfX = r->x[n + j - 1], dfY = r->y[n + j - 1];
            double dfXEnd = r->x[n + j], dfYEnd = r->y[n + j];
            if ((dfY < 0.0 && dfYEnd < 0.0) || (dfY > h && dfYEnd > h) || (dfX < 0.0 && dfXEnd < 0.0) ||
                (dfX > w && dfXEnd > w))
                continue;
            if (dfX > dfXEnd) { double t = dfX; dfX = dfXEnd; dfXEnd = t; t = dfY; dfY = dfYEnd; dfYEnd = t; }
            if (floor(dfX) == floor(dfXEnd) || fabs(dfX - dfXEnd) < .01) {       /* vertical */
                if (dfYEnd < dfY) { const double t = dfY; dfY = dfYEnd; dfYEnd = t; }
                const int iX = (int)floor(dfXEnd);
                int iY = (int)floor(dfY), iYEnd = (int)floor(dfYEnd);
                if (iX < 0 || iX >= w) continue;
                if (iY < 0) iY = 0;
                if (iYEnd >= h) iYEnd = h - 1;
                for (; iY <= iYEnd; iY++) burn(m, w, h, iX, iY);
                continue;
            }
            if (floor(dfY) == floor(dfYEnd) || fabs(dfY - dfYEnd) < .01) {       /* horizontal */
                if (dfXEnd < dfX) { double t = dfX; dfX = dfXEnd; dfXEnd = t; }
                int iX = (int)floor(dfX);
                const int iY = (int)floor(dfY);
                int iXEnd = (int)floor(dfXEnd);
                if (iY < 0 || iY >= h) continue;
                if (iX < 0) iX = 0;
                if (iXEnd >= w) iXEnd = w - 1;
                for (; iX <= iXEnd; iX++) burn(m, w, h, iX, iY);
                continue;
            }
            const double dfSlope = (dfYEnd - dfY) / (dfXEnd - dfX);              /* general */
            if (dfXEnd > w) { dfYEnd -= (dfXEnd - w) * dfSlope; dfXEnd = w; }
            if (dfX < 0.0) { dfY += (0.0 - dfX) * dfSlope; dfX = 0.0; }
            if (dfYEnd > dfY) {
                if (dfY < 0.0) { dfX += (0.0 - dfY) / dfSlope; dfY = 0.0; }
                if (dfYEnd >= h) { dfXEnd += (dfYEnd - h) / dfSlope; dfYEnd = h; }
            } else {
                if (dfY >= h) { dfX += (h - dfY) / dfSlope; dfY = h; }
                if (dfYEnd < 0.0) { dfXEnd -= (dfYEnd - 0) / dfSlope; dfYEnd = 0.0; }
            }
            while (dfX >= 0.0 && dfX < dfXEnd) {
                const int iX = (int)floor(dfX), iY = (int)floor(dfY);
                if (iY >= 0 && iY < h) burn(m, w, h, iX, iY);
                double dfStepX = floor(dfX + 1.0) - dfX;
                double dfStepY = dfStepX * dfSlope;
                if ((int)floor(dfY + dfStepY) == iY) {
                    dfX += dfStepX; dfY += dfStepY;
                } else if (dfSlope < 0) {
                    dfStepY = iY - dfY;
                    if (dfStepY > -0.000000001) dfStepY = -0.000000001;
                    dfStepX = dfStepY / dfSlope;
                    dfX += dfStepX; dfY += dfStepY;
                } else {
                    dfStepY = (iY + 1) - dfY;
                    if (dfStepY < 0.000000001) dfStepY = 0.000000001;
                    dfStepX = dfStepY / dfSlope;
                    dfX += dfStepX; dfY += dfStepY;
                }
            }
        }
    }
}

int oracle_drill_descriptor(const char *geometry_json, const oracle_crs *ds_crs, const double geot[6],
                            int xsize, int ysize, int32_t win[4], uint8_t **mask_out) {
    *mask_out = NULL;
    or_rings r;
    memset(&r, 0, sizeof(r));
    if (parse_geojson(geometry_json, &r)) { rings_free(&r); return -1; }
    rings_buffer0(&r);                              /* drill.go:364-367 */
    if (ds_crs) {                                   /* drill.go:371-380: WGS84 lon/lat -> dataset SRS */
        oracle_crs wgs;
        oracle_crs_init(&wgs, "EPSG:4326");
        for (int i = 0; i < r.n_pts; i++)
            if (!oracle_crs_transform(&wgs, ds_crs, &r.x[i], &r.y[i])) { rings_free(&r); return -1; }
    }
    /* envelopePolygon (drill.go:329-361): corners through the geotransform, "%f" */
    const double ulX = fmt6(geot[0] + 0 * geot[1] + 0 * geot[2]), ulY = fmt6(geot[3] + 0 * geot[4] + 0 * geot[5]);
    const double lrX = fmt6(geot[0] + xsize * geot[1] + ysize * geot[2]);
    const double lrY = fmt6(geot[3] + xsize * geot[4] + ysize * geot[5]);
    double env[4];
    if (!intersection_envelope(&r, fmin(ulX, lrX), fmin(ulY, lrY), fmax(ulX, lrX), fmax(ulY, lrY), env)) {
        rings_free(&r);
        return -2;
    }
    double igt[6];
    inv_geot(geot, igt);
    const double offMinX = igt[0] + env[0] * igt[1] + env[1] * igt[2], offMinY = igt[3] + env[0] * igt[4] + env[1] * igt[5];
    const double offMaxX = igt[0] + env[2] * igt[1] + env[3] * igt[2], offMaxY = igt[3] + env[2] * igt[4] + env[3] * igt[5];
    int32_t offX = go_cvtt32(fmin(offMinX, offMaxX)), offY = go_cvtt32(fmin(offMinY, offMaxY));
    int32_t cX = go_cvtt32(fmax(offMinX, offMaxX)) - offX, cY = go_cvtt32(fmax(offMinY, offMaxY)) - offY;
    if (cX == 0) cX++;
    if (cY == 0) cY++;
    if (offX < 0) offX = 0;
    if (offY < 0) offY = 0;
    win[0] = offX; win[1] = offY; win[2] = cX; win[3] = cY;
    if (cX <= 0 || cY <= 0) { rings_free(&r); return -2; }
    /* createMask (drill.go:275-327): MEM raster at the window, burn 255 ALL_TOUCHED */
    double mgt[6], migt[6];
    memcpy(mgt, geot, sizeof(mgt));
    mgt[0] += mgt[1] * (double)offX;
    mgt[3] += mgt[5] * (double)offY;
    inv_geot(mgt, migt);
    for (int i = 0; i < r.n_pts; i++) {
        const double X = r.x[i], Y = r.y[i];
        r.x[i] = migt[0] + X * migt[1] + Y * migt[2];
        r.y[i] = migt[3] + X * migt[4] + Y * migt[5];
    }
    uint8_t *m = (uint8_t *)calloc((size_t)cX * cY, 1);
    line_all_touched(&r, m, cX, cY);
    filled_polygon(&r, m, cX, cY);
    rings_free(&r);
    *mask_out = m;
    return 0;
}
