/*
 * gskyhip.h -- C-ABI of the MI355X-native GSKY raster hot path.
 *
 * libgskyhip.so (gsky_amd/libgskyhip.so) implements GSKY's per-request
 * raster hot path on gfx950 with hand-written HIP kernels:
 *   warp (reprojection + nearest/bilinear resampling)
 *   -> nodata-aware time-ordered mosaic (merge, masks)
 *   -> byte scaling -> palette / RGBA fill
 * and the drill (zonal) reduction.
 *
 * Every entry point names the reference interface it replaces
 * (chuc92man/gsky file:line).  Signatures use plain C types and pointers only.
 * "dev" pointers are HIP device pointers (hipMalloc / torch CUDA tensors);
 * `stream` is a hipStream_t passed as void* (NULL = default stream).
 * Batch entry points are asynchronous on `stream` and never allocate,
 * synchronise or copy to the host, so they can be captured in a hipGraph.
 *
 * Error codes: 0 OK; >0 follow the reference where one exists
 * (warp.go:103-140: 1 open failed, 2 band failed, 3 transformer failed);
 * negative values are GSKYHIP_E_* below.
 */
#ifndef GSKYHIP_H
#define GSKYHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes -------------------------------------------------------- */
#define GSKYHIP_OK 0
#define GSKYHIP_E_ARG (-1)         /* bad argument / size                     */
#define GSKYHIP_E_TYPE (-2)        /* raster type not implemented             */
#define GSKYHIP_E_HIP (-3)         /* HIP runtime error                       */
#define GSKYHIP_E_CRS (-4)         /* unsupported CRS                          */
#define GSKYHIP_E_MASK (-5)        /* bad mask spec (tile_merger.go:315-323)   */
#define GSKYHIP_E_NOGPU (-6)       /* no HIP device                            */
#define GSKYHIP_E_RANGE (-7)       /* index out of range (Go would panic)      */
#define GSKYHIP_E_XFORM (-8)       /* GDALSuggestedWarpOutput() failed         */
#define GSKYHIP_E_SERVICE (-9)     /* per-node service unreachable / protocol  */

/* ---- raster data types: GDALDataType codes (warp.go:428-431) + 100 ------- */
#define GSKYHIP_BYTE 1
#define GSKYHIP_UINT16 2
#define GSKYHIP_INT16 3
#define GSKYHIP_UINT32 4
#define GSKYHIP_INT32 5
#define GSKYHIP_FLOAT32 6
#define GSKYHIP_FLOAT64 7
#define GSKYHIP_SIGNEDBYTE 100     /* warp.go:354-359 */

/* ---- coordinate reference systems --------------------------------------- */
#define GSKYHIP_CRS_LONGLAT 0      /* EPSG:4326, traditional GIS order, deg   */
#define GSKYHIP_CRS_WEBMERC 1      /* EPSG:3857                                 */
#define GSKYHIP_CRS_AEA 2          /* EPSG:3577 (GDA94 / Australian Albers)    */
#define GSKYHIP_CRS_SINU 3         /* MODIS sinusoidal, sphere R=6371007.181    */
#define GSKYHIP_CRS_TMERC 4        /* Transverse Mercator, ellipsoidal: UTM     *
                                    * (EPSG:326zz / 327zz), GDA94 / GDA2020 MGA *
                                    * (EPSG:283zz / 78zz), +proj=tmerc / utm    */
#define GSKYHIP_CRS_LCC 5          /* Lambert Conformal Conic, ellipsoidal, 1SP *
                                    * or 2SP: GDA94 / GDA2020 GA Lambert        *
                                    * (EPSG:3112 / 7845), +proj=lcc; constants   *
                                    * in n, c, rho0                              */
#define GSKYHIP_CRS_STERE_POLAR 6  /* polar stereographic, ellipsoidal: EPSG:3031 *
                                    * / 3413 / 3976, UPS 32661 / 32761,          *
                                    * +proj=stere +lat_0=+-90 / +proj=ups; akm1  *
                                    * in c, |lat_ts| in phi1                     */

typedef struct {
    int32_t kind;
    int32_t _pad;
    double a, ra, es, e, one_es;
    double lam0, phi0, phi1, phi2, x0, y0, k0;
    double n, c, dd, rho0, ec;      /* aea constants                           */
    /* tmerc (Poder / Engsager, 6th order): normalised meridian quadrant,
     * northing of the origin latitude, and the trigonometric series
     * Gaussian <-> geodetic latitude (cgb, cbg) and ellipsoidal <->
     * spherical northing / easting (utg, gtu)                                */
    double tm_qn, tm_zb;
    double tm_cgb[6], tm_cbg[6], tm_utg[6], tm_gtu[6];
} gskyhip_crs;

/* Parse an SRS as handed over by gsky-ows (tile_grpc.go:127-136 exports the
 * request CRS as WKT): WKT with a top-level AUTHORITY["EPSG",...], "EPSG:n",
 * a proj4 string, or "MODIS".  Returns 0 or GSKYHIP_E_CRS. */
int gskyhip_crs_from_srs(const char *srs, gskyhip_crs *out);

/* The coordinate transformation of the warp's GenImgProj transformer between
 * two parsed CRSs (PROJ pj_inv of src, then pj_fwd of dst; the
 * OGRCoordinateTransformation step of warp.go:130), on the host with the same
 * functions the kernels run: x[i], y[i] in place, ok[i] = 1 or 0 (the
 * transform failed; x / y then undefined).  Returns 0 or GSKYHIP_E_ARG. */
int gskyhip_crs_transform(const gskyhip_crs *src, const gskyhip_crs *dst, int n, double *x, double *y,
                          int32_t *ok);

/* ---- granules (the HBM-resident stand-in for an opened GDAL dataset) ----- */
#define GSKYHIP_MAX_OVR 12
typedef struct {
    const void *data;            /* dev: ysize x xsize of dtype, row-major   */
    int32_t dtype;               /* GSKYHIP_* (Byte for SignedByte data)       */
    int32_t xsize, ysize;
    int32_t signed_byte;         /* PIXELTYPE=SIGNEDBYTE                        */
    double geot[6];              /* GDALGetGeoTransform                          */
    double nodata;               /* GDALGetRasterNoDataValue (-1e10 if unset)   */
    int32_t has_nodata;
    int32_t crs;                 /* index into the CRS table of the call        */
    int32_t n_ovr;
    int32_t ns;                  /* namespace slot of this granule (merge)      */
    const void *ovr_data[GSKYHIP_MAX_OVR];  /* dev, finest first (GDALGetOverview) */
    int32_t ovr_xsize[GSKYHIP_MAX_OVR];
    int32_t ovr_ysize[GSKYHIP_MAX_OVR];
    double timestamp;            /* GeoTileGranule.TimeStamp                     */
    uint32_t polygon_hash;       /* fnv32a(GeoTileGranule.Polygon)               */
    int32_t block_x, block_y;    /* GDALGetBlockSize of the band (0: xsize x 1);  *
                                  * only bytesRead (warp.go:347) depends on it    */
    int32_t geoloc;              /* 0; k > 0: the k-th geolocation transformer of *
                                  * the call (the drop-in's GeoLocOpts requests) */
} gskyhip_granule;

/* One output tile of a GetMap batch.  Granules of the tile are
 * pair_granule[pair_begin..pair_end) in indexer / gRPC fan-out order
 * (tile_grpc.go:200-289). */
typedef struct {
    double dst_geot[6];          /* BBox2Geot (tile_grpc.go:380-382)             */
    int32_t width, height;
    int32_t pair_begin, pair_end;
} gskyhip_tile;

/* Scale parameters, utils.ScaleParams (raster_scaler.go:8-13). */
typedef struct {
    double offset, scale, clip;
    int32_t colour_scale;
    int32_t _pad;
} gskyhip_scale_params;

/* Mask layer, utils.Mask (utils/config.go:73-80).  `ns` is the namespace slot
 * whose rasters are the mask (Mask.ID == NameSpace); -1 = no mask.  value is
 * the base-2 Mask.Value string (may be NULL); bit_tests pairs. */
#define GSKYHIP_MAX_BIT_TESTS 8
typedef struct {
    int32_t ns;
    int32_t inclusive;
    int32_t n_bit_tests;         /* number of strings in bit_tests (even)        */
    int32_t _pad;
    const char *value;
    const char *bit_tests[GSKYHIP_MAX_BIT_TESTS];
} gskyhip_mask;

/* ---- native granule ingest ------------------------- */
/* What GDALOpenEx + GDALGetGeoTransform / GetRasterNoDataValue / GetOverview
 * report for a GeoTIFF (warp.go:89-101, 156-198, 246): classic TIFF and
 * BigTIFF, striped or tiled, chunky or planar, none / LZW / Deflate /
 * PackBits, predictors 1-3, 8-64 bit samples.  epsg: ProjectedCSTypeGeoKey
 * or GeographicTypeGeoKey, -1 for a user-defined sinusoidal on the MODIS
 * sphere, 0 when unknown.  nodata -1e10 when GDAL_NODATA is absent (the
 * value GDALGetRasterNoDataValue returns, warp.go:246). */
typedef struct {
    int32_t xsize, ysize, n_bands, dtype;
    int32_t signed_byte, block_x, block_y;
    int32_t compression, predictor, planar;
    int32_t epsg, has_nodata, n_ovr, _pad;
    double geot[6];
    double nodata;
    int32_t ovr_xsize[GSKYHIP_MAX_OVR], ovr_ysize[GSKYHIP_MAX_OVR];
} gskyhip_raster_info;

int gskyhip_geotiff_info(const char *path, gskyhip_raster_info *info);
/* Band `band` (1-based) of level `level` (0 = full resolution, k = overview
 * k) row-major into HOST memory (no device work; out_bytes >= x*y*size). */
int gskyhip_geotiff_read_host(const char *path, int band, int level, void *out, int64_t out_bytes);
/* The same into device memory: blocks decompressed by host threads into
 * pinned staging, one H2D copy, placed row-major on the GPU; returns after
 * the copy (the staging buffer is freed). */
int gskyhip_geotiff_read(const char *path, int band, int level, void *dev_out, int64_t out_bytes, void *stream);
/* Decode every level of (path, band) into HBM owned by the library and
 * register it for warp_operation_fast (freed by gskyhip_unregister_all).
 * warp_operation_fast does this itself for an unregistered *.tif / *.tiff
 * path, as GDALOpenEx would open it.  Returns 0, 1 (open failed), 2 (no such
 * band) or GSKYHIP_E_*. */
int gskyhip_register_geotiff(const char *path, int band);
/* netCDF classic (CDF-1/2/5) the way the GSKY_netCDF driver presents it
 * (libs/gdal/frmts/gsky_netcdf/netcdfdataset.cpp): path "NETCDF:file:var"
 * or a file holding one data variable; band = index along the leading
 * dimension of a 3-D variable (band_query, netcdfdataset.cpp:6994-7021);
 * geotransform from the coordinate variables (3504-3655, y increasing ->
 * rows returned north first); nodata from _FillValue / missing_value. */
int gskyhip_netcdf_info(const char *path, gskyhip_raster_info *info);
int gskyhip_netcdf_read_host(const char *path, int band, void *out, int64_t out_bytes);
/* The dataset SRS GSKY_netCDF reports for the srs_cf open option
 * (warp.go:95, netcdfdataset.cpp:7023-7025, 3661-3720): srs_cf = 0 -- the
 * grid mapping's GDAL WKT (spatial_ref / crs_wkt) when it names an EPSG
 * code, else the CF grid-mapping attributes; srs_cf = 1 -- the CF attributes
 * only.  out: "EPSG:<n>", a PROJ string, "" (none: the warp takes WGS84) or
 * "?" (a CF mapping outside the supported projections). */
int gskyhip_netcdf_srs(const char *path, int srs_cf, char *out, int cap);
int gskyhip_netcdf_read(const char *path, int band, void *dev_out, int64_t out_bytes, void *stream);
/* Decode (path, band) into library-owned HBM and register it; what
 * warp_operation_fast does itself for an unregistered netCDF path. */
int gskyhip_register_netcdf(const char *path, int band);

/* ---- drop-in for the cgo entry point of the worker ----------------------- */
/* Registers an HBM-resident granule under (path, band) so that the drop-in
 * below can find it (it replaces GDALOpenEx in warp.go:89-101; GeoTIFF files
 * the library decodes itself: gskyhip_register_geotiff above).  `g->data`
 * etc. must stay valid until unregistered. */
int gskyhip_register_granule(const char *path, int band, const gskyhip_granule *g,
                             const char *srs);
int gskyhip_unregister_all(void);

/* Same signature, ownership and return codes as
 *   int warp_operation_fast(const char *srcFilePath, char *srcProjRef,
 *       double *srcGeot, const char **geoLocOpts, const char *dstProjRef,
 *       double *dstGeot, int dstXImageSize, int dstYImageSize, int band,
 *       int srsCf, void **dstBuf, int *dstBufSize, int *dstBbox,
 *       double *noData, GDALDataType *dType, int *bytesRead)
 * (worker/gdalprocess/warp.go:82).  *dstBuf is host memory from malloc(); the
 * caller frees it with free() (warp.go:573-574).  srcGeot, when given, may be
 * overwritten by the overview pick (warp.go:186-189).  geoLocOpts (a
 * NULL-terminated GDAL geolocation option list, warp.go:128-141) selects the
 * geolocation-array transformer; 3 only when the options are incomplete or
 * their X / Y datasets cannot be read (createGeoLocTransformer fails,
 * warp.go:134-140).  Nearest-neighbour, like the reference.
 * Lookup (warp.go:89-118): "NETCDF:..." / "*.nc" paths are opened per band
 * (band_query) and read as band 1, i.e. (path, band) is looked up; other
 * paths: unregistered path -> 1, registered path without that band -> 2.
 * *bytesRead = block bytes x blocks read, with the reference's block-cache
 * heuristic (warp.go:278-347) over the granule's block_x x block_y. */
int warp_operation_fast(const char *srcFilePath, char *srcProjRef, double *srcGeot,
                        const char **geoLocOpts, const char *dstProjRef, double *dstGeot,
                        int dstXImageSize, int dstYImageSize, int band, int srsCf,
                        void **dstBuf, int *dstBufSize, int *dstBbox, double *noData,
                        int *dType, int *bytesRead);

/* ---- batched GetMap path (the MI355X hot path) --------------------------- */
/* Workspace bytes needed by gskyhip_render_tiles / gskyhip_warp_windows for
 * n_tiles tiles with n_pairs pairs whose tiles are at most max_tile_height
 * rows. */
int64_t gskyhip_render_workspace_size(int n_tiles, int n_pairs, int max_tile_height);

#define GSKYHIP_RESAMPLE_NEAREST 0
#define GSKYHIP_RESAMPLE_BILINEAR 1

/* Warp + merge + scale + palette for a batch of tiles, replacing per tile:
 * gRPC warp fan-out (tile_grpc.go:200-289 -> warp.go:82-382), RasterMerger
 * (tile_merger.go:447-738), utils.Scale (raster_scaler.go:334) and the
 * EncodePNG pixel loop (ogc_encoders.go:82-134).
 *   granules, crs_table, tiles, pair_granule: dev arrays.
 *   out_ns[0..n_out_ns): HOST array of namespace slots rendered
 *     (ConfigPayLoad.NameSpaces order; 1 = palette/grey, 3 = RGB).
 *   mask, sp: HOST structs.
 *   ramp: dev 256x4 RGBA (GradientRGBAPalette) or NULL for grey.
 *   rgba_out: dev n_tiles x height x width x 4.
 *   canvas_out: optional dev buffer n_tiles x n_out_ns x height x width x 4
 *     bytes receiving the typed merged canvases (tile_merger.go:562-652), or NULL.
 *   auto_scale (Offset = Scale = Clip = 0) needs canvas_out.
 *   workspace: dev, gskyhip_render_workspace_size bytes. */
int gskyhip_render_tiles(const gskyhip_granule *granules, int n_granules,
                         const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                         const gskyhip_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int n_pairs,
                         int max_tile_width, int max_tile_height,
                         const int32_t *out_ns, int n_out_ns,
                         const gskyhip_mask *mask, int resample,
                         const gskyhip_scale_params *sp, const uint8_t *ramp,
                         uint8_t *rgba_out, void *canvas_out,
                         void *workspace, int64_t workspace_bytes, void *stream);

/* The same call split in phases: 1 = planning kernels only (windows,
 * merge order, row plans into `workspace`), 2 = render kernels only (needs
 * a phase-1 call with identical arguments before it on the stream),
 * 0 = both (= gskyhip_render_tiles).  rgba_out may be NULL: typed canvases
 * only (WCS GetCoverage, FusionUnscale: ows.go:728), canvas_out required. */
int gskyhip_render_tiles_phase(int phase, const gskyhip_granule *granules, int n_granules,
                               const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                               const gskyhip_tile *tiles, int n_tiles,
                               const int32_t *pair_granule, int n_pairs,
                               int max_tile_width, int max_tile_height,
                               const int32_t *out_ns, int n_out_ns,
                               const gskyhip_mask *mask, int resample,
                               const gskyhip_scale_params *sp, const uint8_t *ramp,
                               uint8_t *rgba_out, void *canvas_out,
                               void *workspace, int64_t workspace_bytes, void *stream);

/* The same with a hint: value_types = OR of GSKYHIP_VT_* over the value types
 * the batch's stack granules warp to (Byte/SignedByte/Int16/UInt16/Float32;
 * granules of a non-inclusive mask layer excluded), 0 = unknown.  With exactly
 * one type, one NN palette/grey namespace, RGBA output and no auto-scale the
 * batch runs the typed LDS-staged band kernel (the MI355X fast path); every
 * other combination runs the generic kernels.  Results are identical. */
#define GSKYHIP_VT_BYTE 1u
#define GSKYHIP_VT_SIGNEDBYTE 2u
#define GSKYHIP_VT_INT16 4u
#define GSKYHIP_VT_UINT16 8u
#define GSKYHIP_VT_FLOAT32 16u
int gskyhip_render_tiles_typed(int phase, uint32_t value_types, const gskyhip_granule *granules,
                               int n_granules, const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                               const gskyhip_tile *tiles, int n_tiles,
                               const int32_t *pair_granule, int n_pairs,
                               int max_tile_width, int max_tile_height,
                               const int32_t *out_ns, int n_out_ns,
                               const gskyhip_mask *mask, int resample,
                               const gskyhip_scale_params *sp, const uint8_t *ramp,
                               uint8_t *rgba_out, void *canvas_out,
                               void *workspace, int64_t workspace_bytes, void *stream);

/* WCS GetCoverage (ows.go:815-1150): the chunk tiles rendered as typed
 * canvases (FusionUnscale, ows.go:728: no Scale / RGBA) of the first
 * namespace, each written straight into ONE coverage image at its chunk
 * offset -- tile t's row r lands at coverage_out + (tile_offsets[t] + r *
 * row_stride) elements -- instead of per-tile slots, so no assembly copy
 * follows.  tile_offsets: dev int64 per tile; the coverage's value type is
 * the canvas type (value_types hint as gskyhip_render_tiles_typed). */
int gskyhip_render_coverage(int phase, uint32_t value_types, const gskyhip_granule *granules,
                            int n_granules, const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                            const gskyhip_tile *tiles, int n_tiles, const int32_t *pair_granule,
                            int n_pairs, int max_tile_width, int max_tile_height, int resample,
                            const gskyhip_scale_params *sp, const int64_t *tile_offsets,
                            int64_t row_stride, void *coverage_out, void *workspace,
                            int64_t workspace_bytes, void *stream);

/* Warped windows only (the FlexRasters of tile_grpc.go:228-241): for pair p
 * (tile t, granule g) writes window bbox[4*p..] = {xoff,yoff,w,h} and the
 * window data (dtype of warp.go:232-243) into win_out + p*win_stride bytes. */
int gskyhip_warp_windows(const gskyhip_granule *granules, int n_granules,
                         const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                         const gskyhip_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int n_pairs,
                         int max_tile_width, int max_tile_height, int resample,
                         int32_t *bbox_out, int32_t *dtype_out, double *nodata_out,
                         void *win_out, int64_t win_stride,
                         void *workspace, int64_t workspace_bytes, void *stream);

/* ComputeReprojectExtent (worker/gdalprocess/warp.go:433-487, the worker's
 * "extent" operation), batched over n granules: for granule i,
 * GDALSuggestedWarpOutput of its GenImgProj transformer to crs_table[dst_crs]
 * (no destination dataset: destination georeferenced coordinates; dst_crs
 * -1 = the granule's own CRS), then its request's pixel counts
 *   out[2i]   = nPixels = int((bbox[2] - bbox[0] + xRes/2) / xRes)
 *   out[2i+1] = nLines  = int((bbox[3] - bbox[1] + yRes/2) / yRes)
 * with bbox = dst_bbox[4i..4i+3] (the request's DstGeot[0..3]) and xRes /
 * yRes the suggested geotransform's gt[1] / |gt[5]|.  status[i] = 0, or
 * GSKYHIP_E_XFORM where the reference returns "GDALSuggestedWarpOutput()
 * failed".  granules, crs_table, dst_bbox, out and status are device
 * pointers; asynchronous on `stream`. */
int gskyhip_compute_reproject_extent(const gskyhip_granule *granules, int n, const gskyhip_crs *crs_table,
                                     int n_crs, int dst_crs, const double *dst_bbox, int32_t *out,
                                     int32_t *status, void *stream);

/* ---- per-node warp service (SURVEY 8b threading contract, 8f row 1) ------
 * The reference runs N = NumCPU single-threaded gsky-gdal-process workers per
 * node (grpc-server/main.go:58, gdal-process/main.go:115-123; pool.go:19-74
 * and process.go:108-160 spawn, feed and kill them).  One daemon per GPU
 * (gskyhipd = gskyhip_service_run) owns the HIP context and the HBM-resident
 * granules; a worker whose environment has GSKYHIP_SERVICE=<socket> sends
 * each warp_operation_fast call there over a Unix socket and never touches
 * the GPU, so N workers share one context and a SIGKILLed worker leaves no
 * device state.  The daemon keeps two batches in flight: whenever requests
 * are queued and a batch slot is free it plans and warps up to `max_batch`
 * of them in one launch set (while the other batch is still on the GPU it may
 * first wait up to `window_us` for the batch to grow; with the GPU idle it
 * dispatches at once).  Each worker thread passes a sealed memfd reply arena
 * with its first request; the daemon registers it with HIP and the warp
 * kernel writes the window straight into it (GSKYHIP_SVC_DIRECT=0 in the
 * daemon's environment: staged in HBM and copied instead).  All pointers are
 * host. */
int gskyhip_service_run(const char *socket_path, int max_batch, int window_us);   /* blocks until shutdown */
int gskyhip_service_register_granule(const char *socket_path, const char *path, int band,
                                     const gskyhip_granule *g, const void *data, const void *const *ovr_data,
                                     const char *srs);   /* data / ovr_data: host arrays, uploaded by the daemon */
int gskyhip_service_unregister_all(const char *socket_path);
/* stats[4]: warp requests served, batches run, largest batch, registered granules */
int gskyhip_service_stats(const char *socket_path, int64_t *stats);
/* the same and, at [4], nanoseconds the dispatcher spent preparing and
 * launching batches, at [5] the summed residence of requests (enqueued ->
 * answer ready), at [6..8] the warp batches' launch, wait for the GPU and
 * staged window read-back (ns), at [9] replies whose window the GPU wrote into
 * the worker's arena, at [10] replies whose window was copied; the first
 * n_stats values are written (0 past what the daemon reports) */
int gskyhip_service_stats_n(const char *socket_path, int64_t *stats, int n_stats);
int gskyhip_service_shutdown(const char *socket_path);

/* Band-math on merged canvases (processor/tile_merger.go:523-731): evaluate
 * `expr` (govaluate subset: ?: || && == != < <= > >= + - * / % ** unary - ! +,
 * numbers, the variable names, parentheses; float32 per element) over the
 * canvases of one axis -- var_names[k] names canvases[k] (dev, n_px values
 * of dtypes[k], nodata nodatas[k]) -- into out (dev float32 n_px).  A pixel
 * where any variable equals its nodata, or whose result is not finite,
 * becomes out_nodata (the first namespace's nodata); an expression without
 * variables fills every valid pixel.  GSKYHIP_E_ARG: parse error / unknown
 * variable (govaluate's errors); GSKYHIP_E_TYPE: canvas type. */
#define GSKYHIP_BANDMATH_MAX_VARS 8
int gskyhip_band_math(const char *expr, const char *const *var_names, const void *const *canvases,
                      const int32_t *dtypes, const double *nodatas, int n_vars, int64_t n_px, double out_nodata,
                      float *out, void *stream);

/* ---- standalone stages (the reference's own operator boundaries) -------- */
/* FlexRaster (tile_types.go:95-106) as flat fields; data is dev. */
typedef struct {
    const void *data;
    int32_t data_w, data_h, width, height, off_x, off_y;
    int32_t dtype, ns;
    double nodata, timestamp;
    uint32_t polygon_hash;
    int32_t _pad;
} gskyhip_flex_raster;

/* RasterMerger.Run for one batch (tile_merger.go:447-503 ->
 * ProcessRasterStack 281-312 -> MergeMaskedRaster 38-225 / ComputeMask
 * 314-445).  rasters: HOST array (ordering metadata); their data: dev.
 * canvases: n_ns dev buffers of width*height*4 bytes (typed by the first
 * raster of each namespace); created/dtype/nodata: host outputs per ns. */
int gskyhip_merge_rasters(const gskyhip_flex_raster *rasters, int n,
                          const gskyhip_mask *mask, void *const *canvases, int n_ns,
                          int32_t *created, int32_t *dtype, double *nodata, void *stream);

/* utils.Scale for one raster (raster_scaler.go:30-332): data dev (n values),
 * out dev (n bytes).  Byte input is scaled in place like the reference. */
int gskyhip_scale(void *data, int dtype, int64_t n, double nodata,
                  const gskyhip_scale_params *sp, uint8_t *out, void *stream);

/* processor.RasterScaler.Run (tile_scaler.go:17-112, dead in the reference). */
int gskyhip_scale_legacy(void *data, int dtype, int64_t n, double nodata,
                         const gskyhip_scale_params *sp, uint8_t *out, void *stream);

/* GradientRGBAPalette (utils/palette.go:27-69): colours host n x RGBA,
 * ramp host 256 x RGBA. */
int gskyhip_gradient_palette(const uint8_t *colours, int n, int interpolate, uint8_t *ramp);

/* EncodePNG pixel loop (ogc_encoders.go:86-133): bands dev (1 or 3), ramp
 * dev or NULL, rgba dev w*h*4. */
int gskyhip_encode_rgba(const uint8_t *const *bands, int nbands, int w, int h,
                        const uint8_t *ramp, uint8_t *rgba, void *stream);

/* ComputeMask (tile_merger.go:314-445): data dev, out dev (n bytes 0/1). */
int gskyhip_compute_mask(const void *data, int dtype, int64_t n, const gskyhip_mask *mask,
                         uint8_t *out, void *stream);

/* ---- output codecs ------------------------------------------------------ */
/* png.Encode of EncodePNG (utils/ogc_encoders.go:139; Go 1.12 image/png) for
 * a batch of RGBA tiles in HBM, e.g. the rgba_out of gskyhip_render_tiles:
 *   rgba: dev, tile t row y at rgba + t*tile_stride + y*row_stride (bytes);
 *   sizes: HOST int32 2 per tile {width, height} (<= max_w, max_h);
 *   png_out: HOST, png_capacity bytes per tile (>= gskyhip_png_bound(w, h));
 *   png_sizes: HOST int64 per tile, the PNG's length.
 * Colour type RGB when every alpha is 0xff else RGBA (NRGBA bytes), Go's
 * per-row filter choice, 32 KiB IDAT chunks (see encode.hip: the filtered
 * rows are Go's bytes; the zlib stream is deflated on the GPU -- LZ77 at run
 * / pixel / row / diagonal distances, per-tile Huffman codes -- so its bytes
 * are neither zlib's nor Go's compress/flate, parity unpinned).
 * n_threads host threads frame the PNGs; `stream` runs the GPU passes. */
int64_t gskyhip_png_workspace_size(int n_tiles, int max_w, int max_h);
int64_t gskyhip_png_bound(int width, int height);
int gskyhip_encode_png(const uint8_t *rgba, int n_tiles, int max_w, int max_h, int64_t tile_stride,
                       int64_t row_stride, const int32_t *sizes, void *workspace, int64_t workspace_bytes,
                       uint8_t *png_out, int64_t png_capacity, int64_t *png_sizes, int n_threads, void *stream);

/* EncodeGdalOpen + EncodeGdal for format "geotiff" (utils/ogc_encoders.go:
 * 277-450) of one WCS coverage held in HBM: a BigTIFF with the reference's
 * creation options COMPRESS=PACKBITS, TILED=YES, BIGTIFF=YES,
 * INTERLEAVE=BAND, BLOCKXSIZE / BLOCKYSIZE (ows.go passes 1024 x 256),
 * PIXELTYPE=SIGNEDBYTE for int8; the geotransform (ModelPixelScale +
 * ModelTiepoint, ModelTransformation when rotated), EPSG code as GeoKeys,
 * per-band long_name (GDAL_METADATA) and nodata (GDAL_NODATA: GeoTIFF holds
 * one, the last band's value), Photometric RGB for 3 or 4 Byte bands (the 4th
 * an associated alpha), MinIsBlack otherwise.  A band whose name starts with
 * "EmptyTile" is skipped as EncodeGdal skips it (ogc_encoders.go:364): no
 * nodata, no long_name, its pointer may be NULL and its samples are the
 * dataset nodata (0 without one).
 *   bands: HOST array of n_bands dev pointers, each height x width samples of
 *     dtype (GSKYHIP_BYTE / SIGNEDBYTE / INT16 / UINT16 / FLOAT32), row-major;
 *   geot: HOST 6 doubles (GDAL order); epsg <= 0 writes no GeoKeys;
 *   nodata, names: HOST n_bands each, or NULL;
 *   block_x, block_y: multiples of 16;
 *   workspace: dev, gskyhip_geotiff_workspace_size bytes;
 *   out: HOST, capacity >= gskyhip_geotiff_bound bytes; *size = file length.
 * PackBits runs on the GPU (one thread per tile row, libtiff encodes tiled
 * PackBits row by row); the framing on the host.  The bytes are a valid
 * GeoTIFF of the same samples, tags and keys GDAL writes, not GDAL's file
 * byte for byte (tag set and tile order differ: parity on decoded content). */
int64_t gskyhip_geotiff_workspace_size(int width, int height, int n_bands, int dtype, int block_x, int block_y);
int64_t gskyhip_geotiff_bound(int width, int height, int n_bands, int dtype, int block_x, int block_y);
int gskyhip_encode_geotiff(const void *const *bands, int n_bands, int dtype, int width, int height,
                           const double *geot, int epsg, const double *nodata, const char *const *names,
                           int block_x, int block_y, void *workspace, int64_t workspace_bytes, uint8_t *out,
                           int64_t capacity, int64_t *size, void *stream);

/* EncodeGdalOpen + EncodeGdal for format "netcdf" (utils/ogc_encoders.go:
 * 263-301, creation options COMPRESS=DEFLATE, ZLEVEL=6; ows.go:1172) of one
 * WCS coverage held in HBM: the netCDF-4 classic-model file GDAL 3.0.1's
 * netCDF driver creates for those options -- one variable per band
 * ("Band1", ...) with long_name = names[k] and _FillValue = nodata[k] (an
 * "EmptyTile" band skipped as EncodeGdal skips it), chunks of one row,
 * shuffle + deflate at zlevel, rows bottom-up with increasing y (GDAL's
 * WRITE_BOTTOMUP default), x / y (lon / lat) coordinate variables at pixel
 * centres, the "crs" grid mapping (CF attributes of `epsg`, spatial_ref
 * naming the EPSG code, GeoTransform).  Byte is NC_BYTE + _Unsigned "true",
 * UInt16 widens to NC_INT (the classic model has no unsigned types).
 *   bands: HOST array of n_bands dev pointers, height x width of dtype;
 *   out: HOST, capacity >= gskyhip_netcdf_bound bytes; *size = file length.
 * The rows are deflated by n_threads host threads after one copy of each
 * band to the host.  Parity with GDAL's bytes unpinned (no netCDF / HDF5
 * library here): checked by reading the file back (gskyhip_netcdf_read_host). */
int64_t gskyhip_netcdf_bound(int width, int height, int n_bands, int dtype);
int gskyhip_encode_netcdf(const void *const *bands, int n_bands, int dtype, int width, int height,
                          const double *geot, int epsg, const double *nodata, const char *const *names, int zlevel,
                          int n_threads, uint8_t *out, int64_t capacity, int64_t *size, void *stream);
/* The same from HOST bands (EncodeGdal's rasters are host memory in the
 * reference): no device involved. */
int gskyhip_encode_netcdf_host(const void *const *bands, int n_bands, int dtype, int width, int height,
                               const double *geot, int epsg, const double *nodata, const char *const *names,
                               int zlevel, int n_threads, uint8_t *out, int64_t capacity, int64_t *size);

/* ---- drill (WPS zonal statistics) --------------------------------------- */
/* readData (worker/gdalprocess/drill.go:90-227), mean / pixel-count mode,
 * decileCount = 0, for a batch of polygons over one time stack.
 *   stack: dev float32, time-innermost layout [y][x][t] of an
 *     xsize x ysize x n_bands stack, t fastest, t padded to t_stride >= n_bands
 *     (xsize * ysize < 2^31).
 *   win: dev int32 4 per polygon {off_x, off_y, count_x, count_y}
 *     (DrillFileDescriptor, drill.go:25-29); pixels of a window outside the
 *     stack count as outside the mask.
 *   mask_off: dev int64 per polygon, byte offset into masks (dev uint8,
 *     255 = in, row-major count_x*count_y); the polygons' mask regions must
 *     not overlap and every region must lie inside [0, mask_bytes).
 *   bands: HOST int32 list of 1-based band numbers (the reference's
 *     `bands []int32`), or NULL for 1..n_bands (n_list ignored).
 *   band_strides as drill.go:110-219.  Rows per polygon =
 *     gskyhip_drill_rows(n_list, band_strides).
 *   mode 0: reference summation order, means bit-exact; mode 1: wave-split
 *     reduction (float32 partials over 1024-pixel segments, combined in
 *     float64), within 1e-5 relative of mode 0, not bound by the largest polygon.
 *   out_value: dev f64, out_count: dev i32, n_polys x rows.
 *   workspace: dev, gskyhip_drill_workspace_size bytes. */
int gskyhip_drill_rows(int n_bands, int band_strides);
int64_t gskyhip_drill_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides,
                                     int mode);
int gskyhip_drill_batch(const float *stack, int xsize, int ysize, int n_bands, int t_stride,
                        const int32_t *win, const int64_t *mask_off, const uint8_t *masks,
                        int n_polys, int64_t mask_bytes, const int32_t *bands, int n_list,
                        float nodata, float clip_lower, float clip_upper, int pixel_count,
                        int band_strides, int mode, double *out_value, int32_t *out_count,
                        void *workspace, int64_t workspace_bytes, void *stream);
/* computeDeciles (worker/gdalprocess/drill.go:229-273; decileCount > 0,
 * bandStrides 1) for the same batch as gskyhip_drill_batch: per polygon and
 * selected band the in-mask, non-nodata values (no clipping) and the
 * reference's decile_count picks of their ascending order, found by radix
 * selection (no sort).
 *   totals: dev int32 n_polys x n_list, the out_count of the mean pass
 *     (gskyhip_drill_batch, same bands, band_strides 1): deciles only where
 *     total > 0, zeros elsewhere (drill.go:179-191);
 *   out: dev float32 n_polys x n_list x decile_count (decile_count <= 16);
 *   status: dev int32 n_polys x n_list -- 0, 1 (total 0: the reference's
 *     Count-0 zeros), GSKYHIP_E_RANGE (the reference indexes past the values
 *     and panics: len % (dc+1) == 0 with len == dc+1);
 *   band_chunk: bands per pass (workspace scales with mask_bytes x band_chunk). */
int64_t gskyhip_drill_deciles_workspace_size(int n_polys, int64_t mask_bytes, int band_chunk);
int gskyhip_drill_deciles(const float *stack, int xsize, int ysize, int n_bands, int t_stride,
                          const int32_t *win, const int64_t *mask_off, const uint8_t *masks, int n_polys,
                          int64_t mask_bytes, const int32_t *bands, int n_list, float nodata, int decile_count,
                          int band_chunk, const int32_t *totals, float *out, int32_t *status, void *workspace,
                          int64_t workspace_bytes, void *stream);

/* readData complete (worker/gdalprocess/drill.go:90-227), one call per
 * batch of polygons over one time stack -- what DrillDataset (drill.go:33-88)
 * calls after getDrillFileDescriptor: readData(ds, bands, geom, bandStrides,
 * decileCount, pixelCount, clipUpper, clipLower).  Mean / pixel-count
 * (pixel_count), decile_count >= 0 (<= 16), band_strides >= 1 with the
 * reference's bound-band reads and interpolated rows (every column, counts
 * math.Round of the two bounds' mean).  Arguments as gskyhip_drill_batch;
 * out_value (dev f64) / out_count (dev i32): n_polys x rows x (1 +
 * decile_count) = Result.TimeSeries (Value, Count) row-major with Shape
 * [rows, 1 + decile_count], rows = gskyhip_drill_rows(n_list, band_strides);
 * status: dev int32 per polygon, 0 or GSKYHIP_E_RANGE where computeDeciles
 * would panic (the reference's gsky-gdal-process dies; the request fails). */
int64_t gskyhip_drill_read_data_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides,
                                               int decile_count, int mode);
int gskyhip_drill_read_data(const float *stack, int xsize, int ysize, int n_bands, int t_stride,
                            const int32_t *win, const int64_t *mask_off, const uint8_t *masks, int n_polys,
                            int64_t mask_bytes, const int32_t *bands, int n_list, float nodata,
                            float clip_lower, float clip_upper, int pixel_count, int band_strides,
                            int decile_count, int mode, double *out_value, int32_t *out_count,
                            int32_t *status, void *workspace, int64_t workspace_bytes, void *stream);

/* Round-1 form (bands 1..n_bands, mode 0): sizes and allocates its workspace
 * itself (one synchronous read-back of win / mask_off). */
int gskyhip_drill(const float *stack, int xsize, int ysize, int n_bands, int t_stride,
                  const int32_t *win, const int64_t *mask_off, const uint8_t *masks,
                  int n_polys, float nodata, float clip_lower, float clip_upper,
                  int pixel_count, int band_strides, double *out_value,
                  int32_t *out_count, void *stream);

/* getDrillFileDescriptor + createMask (drill.go:363-423, 275-327) for n
 * request geometries against one dataset (HOST function, no device work):
 *   geometries: GeoJSON (a Feature or a bare Polygon / MultiPolygon) in
 *     WGS84 lon/lat, as GeoRPCGranule.Geometry; first repaired as
 *     OGR_G_Buffer(g, 0, 30) does it (drill.go:364-367, GEOS 3.7.2's
 *     zero-distance buffer: self-intersecting / overlapping rings become the
 *     region of depth >= 1; an empty buffer keeps the rings as drawn);
 *   dataset_srs: the dataset's SRS (NULL / "" = no projection: no transform);
 *   geot, xsize, ysize: the dataset's geotransform and size.
 * Per polygon: win_out[4*i..] = {off_x, off_y, count_x, count_y} with the
 * reference's int32 truncations, status_out[i] = 0, GSKYHIP_E_ARG (geometry
 * not parsable), GSKYHIP_E_CRS (transform failed) or GSKYHIP_E_RANGE (the
 * polygon misses the file; window 0).  mask_off_out[i] = byte offset of its
 * mask (16-byte aligned, polygon order), *mask_bytes_out = total bytes.
 * masks_out: NULL sizes only; else a HOST buffer of *mask_bytes_out bytes
 * that receives the ALL_TOUCHED masks (255 = burnt) -- the layout
 * gskyhip_drill_batch takes (copy it to the device). */
int gskyhip_drill_descriptors(const char *const *geometries, int n, const char *dataset_srs,
                              const double *geot, int xsize, int ysize, int32_t *win_out,
                              int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_out,
                              int32_t *status_out);

/* DrillMerger weighted mean (drill_merger.go:79-93): values/counts dev
 * n_files x n_dates, out dev n_dates (NaN where no count). */
/* The same descriptors with the ALL_TOUCHED masks rasterized on the GPU
 * straight into masks_dev (dev, mask_bytes: call once with masks_dev NULL to
 * size it), one workgroup per polygon (edges, then scanlines) -- the
 * expressions of the host rasterizer, bit-identical masks.  win_out,
 * mask_off_out, mask_bytes_out, status_out are host arrays as above. */
int gskyhip_drill_descriptors_device(const char *const *geometries, int n, const char *dataset_srs,
                                     const double *geot, int xsize, int ysize, int32_t *win_out,
                                     int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_dev,
                                     int32_t *status_out, void *stream);

/* Device memory supplier of gskyhip_drill_masks_device: returns at least
 * `bytes` of device memory (or NULL), owned by the caller (cgo: a hipMalloc
 * wrapper; Python: a torch tensor kept alive by the caller). */
typedef void *(*gskyhip_alloc_fn)(void *ctx, int64_t bytes);

/* gskyhip_drill_descriptors_device in one pass (getDrillFileDescriptor +
 * createMask, drill.go:363-423 / 275-327, for a whole WPS request): every
 * polygon described once on up to 16 host threads, then alloc(alloc_ctx,
 * *mask_bytes_out) supplies the mask buffer (returned in *masks_dev_out) and
 * the masks are rasterized into it on `stream`.  GSKYHIP_E_HIP if alloc
 * returns NULL. */
int gskyhip_drill_masks_device(const char *const *geometries, int n, const char *dataset_srs, const double *geot,
                               int xsize, int ysize, int32_t *win_out, int64_t *mask_off_out,
                               int64_t *mask_bytes_out, gskyhip_alloc_fn alloc, void *alloc_ctx,
                               uint8_t **masks_dev_out, int32_t *status_out, void *stream);
/* The same with the n geometries packed NUL-separated in one buffer of
 * packed_bytes (every string NUL-terminated inside it). */
int gskyhip_drill_masks_device_packed(const char *packed, int64_t packed_bytes, int n, const char *dataset_srs,
                                      const double *geot, int xsize, int ysize, int32_t *win_out,
                                      int64_t *mask_off_out, int64_t *mask_bytes_out, gskyhip_alloc_fn alloc,
                                      void *alloc_ctx, uint8_t **masks_dev_out, int32_t *status_out, void *stream);
/* Test hook: the GeoJSON number parser of the drill descriptors on n
 * NUL-separated strings packed in `text`; out[i] the value, consumed[i] the
 * characters parsed (strtod semantics). */
int gskyhip_parse_numbers(const char *text, int n, double *out, int32_t *consumed);
int gskyhip_drill_merge(const double *values, const int32_t *counts, int n_files,
                        int n_dates, double *out, void *stream);

/* ---- misc ---------------------------------------------------------------- */
uint32_t gskyhip_fnv32a(const char *s, int64_t n);
const char *gskyhip_version(void);
int gskyhip_device_count(void);
/* Status of the last render call (TilePlan status of every tile, read back
 * synchronously): 0 OK or the first error code; n_tiles of the last call. */
int gskyhip_render_status(void *workspace, int n_tiles, int n_pairs, int max_tile_height, void *stream);

/* Diagnostics of the last plan in `workspace` (synchronous): per tile
 * {status, complex (1: some row needs exact per-pixel transforms or the value
 * types are mixed -> general kernel), common value type (GSKYHIP_* or 0),
 * merged entries}; counters_out (3 ints, may be NULL): leaf-pool entries used,
 * rows split by the approximation recursion, complex tiles.  No reference counterpart (an observability hook). */
int gskyhip_render_tile_info(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int32_t *info_out,
                             int32_t *counters_out, void *stream);

/* Source footprint of every pair of a planned batch: info_out (n_pairs x 8
 * int32) = {granule, picked level width, height, element bytes, x0, y0, x1,
 * y1}: the bounding box [x0, x1) x [y0, y1) at that level of the source
 * pixels the pair's linear rows sample.  For the algorithmic bytes of a
 * batch (bench.py C5).  No reference counterpart (an observability hook). */
int gskyhip_render_pair_info(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int32_t *info_out,
                             void *stream);

/* Algorithmic source bytes of a planned batch (unique
 * source bytes touched at the chosen overview level): bytes_out[0] = the
 * distinct source elements x element bytes that the window pixels of every
 * pair (data and mask rasters) pick by the nearest-neighbour rule of
 * warp.go:271-300; bytes_out[1] = the distinct 128-byte lines holding them
 * x 128.  Counted over each picked level once, however many pairs share it
 * (bench.py C5).  No reference counterpart (an observability hook). */
int gskyhip_render_touched(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int64_t *bytes_out,
                           void *stream);

#ifdef __cplusplus
}
#endif
#endif
