/*
 * gsky_oracle.h -- CPU restatement of GSKY's raster hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product in gsky_amd/.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product never links it.
 *
 * Every function restates one reference function (file:line under
 * chuc92man/gsky) or, where the reference delegates to GDAL 3.0.1 / PROJ
 * 6.1.1 / Go 1.12 (none of which is vendored or installable here), the
 * published algorithm of that dependency.  Pinning:
 *   - oracle_scale: pinned by the 18 TestScale known-answer cases
 *     (utils/raster_scaler_test.go:18-151), transcribed in tests/.
 *   - palette / merge / mask / RGBA fill: pinned by hand-derived KATs
 *      only -- "parity unpinned" against a running reference.
 *   - warp (GDAL approx transformer, SuggestedWarpOutput2, PROJ formulas) and
 *     drill: parity unpinned (no reference test covers them; GDAL/PROJ absent).
 */
#ifndef GSKY_ORACLE_H
#define GSKY_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GDALDataType codes as carried by warp.go:428-431, plus 100 = SignedByte
 * (warp.go:354-359). */
enum {
    OR_BYTE = 1, OR_UINT16 = 2, OR_INT16 = 3, OR_UINT32 = 4, OR_INT32 = 5,
    OR_FLOAT32 = 6, OR_FLOAT64 = 7, OR_SIGNEDBYTE = 100
};

int oracle_type_size(int dtype);

/* ---- Go 1.12 amd64 numeric conversions ------------------- */
int8_t   or_go_f64_i8(double v);
uint8_t  or_go_f64_u8(double v);
int16_t  or_go_f64_i16(double v);
uint16_t or_go_f64_u16(double v);
int8_t   or_go_f32_i8(float v);
uint8_t  or_go_f32_u8(float v);
int16_t  or_go_f32_i16(float v);
uint16_t or_go_f32_u16(float v);

/* GDALCopyWords(double -> dtype) of one value: round half away from zero,
 * saturate, NaN -> 0 for integer targets.  Writes sizeof(dtype) bytes. */
void or_gdal_copy_word(double v, int dtype, void *out);

/* ---- utils/raster_scaler.go --------------------------------------------- */
/* scale() raster_scaler.go:30-332 for one raster of n values.  For OR_BYTE the
 * reference scales in place (134-148): `data` is then modified too.
 * Returns 0, or -1 for an unimplemented type (raster_scaler.go:329-331). */
int oracle_scale(void *data, int dtype, int64_t n, double nodata,
                 double offset, double scale, double clip, int colour_scale,
                 uint8_t *out);

/* processor/tile_scaler.go:17-112 (dead "legacy" scaler). */
int oracle_scale_legacy(void *data, int dtype, int64_t n, double nodata,
                        double offset, double scale, double clip, uint8_t *out);

/* ---- utils/palette.go:27-69 ---------------------------------------------- */
/* colours: n x RGBA; ramp: 256 x RGBA.  Returns -1 when n is too small. */
int oracle_gradient_palette(const uint8_t *colours, int n, int interpolate,
                            uint8_t *ramp);

/* EncodePNG pixel loop, ogc_encoders.go:82-134 (png.Encode excluded).
 * nbands 1 (ramp may be NULL = grey) or 3.  rgba: w*h*4, fully written. */
int oracle_encode_rgba(const uint8_t *const *bands, int nbands, int w, int h,
                       const uint8_t *ramp, uint8_t *rgba);

/* ---- processor/tile_merger.go -------------------------------------------- */
uint32_t oracle_fnv32a(const char *s, size_t n);

/* ComputeMask tile_merger.go:314-445.  value: base-2 string or NULL/"";
 * bit_tests: pairs of base-2 strings.  out: n bytes (0/1).
 * Returns 0, -1 (bad mask spec), -2 (type cannot hold a bit mask). */
int oracle_compute_mask(const void *data, int dtype, int64_t n,
                        const char *value, const char *const *bit_tests,
                        int n_bit_tests, uint8_t *out);

/* One warped granule as assembled by tile_grpc.go:228-241 (FlexRaster). */
typedef struct {
    const void *data;       /* DataWidth*DataHeight values of dtype        */
    int32_t data_w, data_h; /* window size                                  */
    int32_t width, height;  /* full tile                                    */
    int32_t off_x, off_y;   /* window offset in the tile                    */
    int32_t dtype;
    int32_t ns;             /* namespace id                                 */
    double nodata;
    double timestamp;
    uint32_t polygon_hash;  /* fnv32a(Polygon), tile_merger.go:473-475      */
    int32_t _pad;
} oracle_flex_raster;

/* Canvas per namespace (tile_merger.go:291-297). */
typedef struct {
    void *data;             /* caller-owned width*height*8 byte buffer      */
    int32_t created;        /* 1 once a raster of this namespace was merged */
    int32_t dtype;
    double nodata;
    double timestamp;
} oracle_canvas;

/* RasterMerger.Run for one input batch (tile_merger.go:447-503 ->
 * ProcessRasterStack 281-312 -> MergeMaskedRaster 38-225).
 * mask_ns: namespace id of the mask layer or -1; mask spec as ComputeMask;
 * mask_inclusive: r.Mask.Inclusive.  canvases: n_ns entries, pre-zeroed
 * (created = 0).  Returns 0 or a negative error. */
int oracle_merge_batch(const oracle_flex_raster *rasters, int n,
                       int mask_ns, const char *mask_value,
                       const char *const *bit_tests, int n_bit_tests,
                       int mask_inclusive, oracle_canvas *canvases, int n_ns);

/* ---- projections (PROJ 6.1.1 formulas, restated) ------------------------ */
enum { OR_CRS_LONGLAT = 0, OR_CRS_WEBMERC = 1, OR_CRS_AEA = 2, OR_CRS_SINU = 3, OR_CRS_TMERC = 4, OR_CRS_LCC = 5, OR_CRS_STERE_POLAR = 6 };

typedef struct {
    int32_t kind;
    int32_t _pad;
    double a, ra, es, e, one_es;
    double lam0, phi0, phi1, phi2, x0, y0, k0;
    /* aea constants (lcc: n, c, rho0) */
    double n, c, dd, rho0, ec;
    /* tmerc (PROJ 6 exact: Poder / Engsager) constants */
    double tm_qn, tm_zb;
    double tm_cgb[6], tm_cbg[6], tm_utg[6], tm_gtu[6];
} oracle_crs;

/* spec: "EPSG:4326", "EPSG:4283", "EPSG:3857", "EPSG:3577", "EPSG:900913",
 * the UTM / MGA zones "EPSG:326zz" / "327zz" / "283zz" / "78zz", the GA
 * Lambert "EPSG:3112" / "7845",
 * "SR-ORG:6842" / "MODIS" (sinusoidal R=6371007.181), or a proj4 string
 * (+proj=longlat|merc|webmerc|aea|sinu|tmerc|utm|lcc ...).  Returns 0 or -1. */
int oracle_crs_init(oracle_crs *crs, const char *spec);

/* Whole transformation src CRS -> dst CRS for one point (degrees for
 * longlat, metres otherwise).  Returns 1 on success. */
int oracle_crs_transform(const oracle_crs *src, const oracle_crs *dst,
                         double *x, double *y);

/* ---- worker/gdalprocess/warp.go ------------------------------------------ */
#define OR_MAX_OVR 12
typedef struct {
    const void *data;          /* xsize*ysize of dtype, row-major          */
    int32_t dtype;
    int32_t xsize, ysize;
    int32_t signed_byte;       /* PIXELTYPE=SIGNEDBYTE metadata            */
    double geot[6];
    double nodata;             /* GDALGetRasterNoDataValue (-1e10 if unset) */
    int32_t n_ovr;
    int32_t _pad;
    const void *ovr_data[OR_MAX_OVR];
    int32_t ovr_xsize[OR_MAX_OVR];
    int32_t ovr_ysize[OR_MAX_OVR];
    int32_t block_x, block_y;    /* GDALGetBlockSize (0: xsize x 1), bytesRead only */
} oracle_granule;

/* warp_operation_fast (warp.go:82-382) over an in-memory granule.
 * dst may be NULL (no reprojection, warp.go:143-148).  resample: 0 nearest
 * (the reference), 1 bilinear (GDAL GRA_Bilinear semantics).
 * *out_buf is malloc'd here (caller frees), like warp.go:244/573-574.
 * Returns 0 / 3 (transformer failed), as warp.go:103-140. */
int oracle_warp(const oracle_granule *g, const oracle_crs *src,
                const oracle_crs *dst, const double dst_geot[6],
                int dst_w, int dst_h, int resample,
                void **out_buf, int *out_size, int32_t bbox[4],
                double *nodata, int *dtype, int *bytes_read);

/* GDAL 3.0.1 geolocation-array transformer (GDALCreateGeoLocTransformer,
 * called by warp.go:52-67 for GeoLocOpts requests): the X / Y bands as
 * double (xh == yh == 1: a regular grid), the X band's nodata, the
 * PIXEL/LINE OFFSET/STEP options; builds the backmap.  Returns 0 or 3. */
typedef struct {
    double *gx, *gy;             /* ny x nx */
    int nx, ny, has_nodata;
    double nodata_x, pixel_offset, line_offset, pixel_step, line_step;
    float *bmx, *bmy;            /* backmap bh x bw */
    int bw, bh;
    double bgt[6];
} oracle_geoloc;
int oracle_geoloc_init(oracle_geoloc *g, const double *x_band, int xw, int xh, const double *y_band, int yw,
                       int yh, int has_nodata, double nodata_x, double pixel_offset, double line_offset,
                       double pixel_step, double line_step);
void oracle_geoloc_free(oracle_geoloc *g);

/* oracle_warp with the geolocation transformer as the source side
 * (warp.go:134-140; no overview, 158); gl NULL = oracle_warp. */
int oracle_warp_geoloc(const oracle_granule *g, const oracle_crs *src,
                       const oracle_crs *dst, const double dst_geot[6],
                       int dst_w, int dst_h, int resample, const oracle_geoloc *gl,
                       void **out_buf, int *out_size, int32_t bbox[4],
                       double *nodata, int *dtype, int *bytes_read);

/* GDALSuggestedWarpOutput2 restatement: extent in dst pixel space plus the
 * suggested geotransform.  Returns 0 on success (CE_None). */
int oracle_suggested_warp_output(const oracle_granule *g, const oracle_crs *src,
                                 const oracle_crs *dst, const double src_geot[6],
                                 const double dst_geot[6], double geot_out[6],
                                 int *n_pixels, int *n_lines, double extent[4]);

/* GDALApproxTransform (dst->src, max error 0.125) over one row of points,
 * exposed for tests. x,y: n values in/out; success: n ints. */
void oracle_approx_row(const oracle_crs *src, const oracle_crs *dst,
                       const double src_geot[6], const double dst_geot[6],
                       int n, double *x, double *y, int *success);

/* ---- tile pipeline used by the CPU baseline ----------------------------- */
typedef struct {
    double dst_geot[6];
    int32_t width, height;
    int32_t pair_begin, pair_end; /* into pair_granule[]                   */
} oracle_tile;

typedef struct {
    double offset, scale, clip;
    int32_t colour_scale;
    int32_t _pad;
} oracle_scale_params;

/* Renders tiles like serveWMS GetMap: per (tile, granule) warp -> FlexRaster
 * -> merge -> Scale -> EncodePNG RGBA fill.  Granule k carries timestamp
 * ts[k], polygon hash ph[k] and namespace ns[k]; its CRS is src_crs[k].
 * rgba_out: n_tiles * width*height*4.  Uses n_threads pthreads over tiles.
 * Returns 0 or the first error. */
int oracle_render_tiles(const oracle_granule *granules, const oracle_crs *src_crs,
                        const double *ts, const uint32_t *ph, const int32_t *ns,
                        int n_granules, const oracle_crs *dst,
                        const oracle_tile *tiles, int n_tiles,
                        const int32_t *pair_granule, int resample,
                        int mask_ns, const char *mask_value, int mask_inclusive,
                        int n_ns, const oracle_scale_params *sp,
                        const uint8_t *ramp, uint8_t *rgba_out, int n_threads);

/* The same with tiles of mixed sizes: every tile t lands in an output slot
 * of max_h x max_w (row stride max_w) -- rgba_out n_tiles*max_h*max_w*4
 * (may be NULL), canvas_out (may be NULL) n_tiles x n_out x max_h*max_w*4
 * bytes receiving the typed merged canvases of the rendered namespaces
 * (tile_merger.go:562-652), created_out (may be NULL) n_tiles x 3 flags. */
int oracle_render_tiles2(const oracle_granule *granules, const oracle_crs *src_crs,
                         const double *ts, const uint32_t *ph, const int32_t *ns,
                         int n_granules, const oracle_crs *dst,
                         const oracle_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int resample,
                         int mask_ns, const char *mask_value, int mask_inclusive,
                         int n_ns, const oracle_scale_params *sp,
                         const uint8_t *ramp, uint8_t *rgba_out, int max_w, int max_h,
                         uint8_t *canvas_out, int32_t *created_out, int n_threads);

/* ---- worker/gdalprocess/drill.go:90-227 readData -------------------------- */
/* data: band-sequential float32 [nbands][count_y*count_x] already read as in
 * GDALDatasetRasterIO (drill.go:141-142).  mask: count_x*count_y (255 = in).
 * Only bandStrides == 1 semantic per read band; band_strides > 1 handled by
 * the caller-visible interpolation (197-214) via `band_strides`.
 * out_value/out_count: n_rows entries (n_rows returned). decile_count must be
 * 0 here (deciles are SURVEY 8f "next"). */
int oracle_drill_read_data(const float *data, int nbands, int count_x, int count_y,
                           const uint8_t *mask, float nodata, float clip_lower,
                           float clip_upper, int pixel_count, int band_strides,
                           double *out_value, int32_t *out_count);

/* getDrillFileDescriptor + createMask (worker/gdalprocess/drill.go:363-423,
 * 275-327): the request geometry (GeoJSON Feature or Polygon / MultiPolygon,
 * WGS84 lon/lat) -> dataset SRS (ds_crs NULL: no projection, no transform)
 * -> intersection envelope with the "%f"-formatted file envelope -> window
 * {offX, offY, countX, countY} (Go int32 truncations) and the ALL_TOUCHED
 * mask (GDAL 3.0.1 GDALdllImageLineAllTouched + GDALdllImageFilledPolygon,
 * burn 255) in *mask_out (malloc'd countX*countY, caller frees).
 * Returns 0, -1 unparsable geometry, -2 empty intersection. */
int oracle_drill_descriptor(const char *geometry_json, const oracle_crs *ds_crs, const double geot[6],
                            int xsize, int ysize, int32_t win[4], uint8_t **mask_out);

/* drill_merger.go:79-93: per date weighted mean over files. values/counts:
 * n_files x n_dates.  out: n_dates (NaN where count == 0). */
void oracle_drill_merge(const double *values, const int32_t *counts,
                        int n_files, int n_dates, double *out);

#ifdef __cplusplus
}
#endif
#endif
