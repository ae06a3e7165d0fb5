/*
 * fv3net_amd — MI355X (gfx950) C ABI for fv3net's per-timestep ML-physics hot path.
 *
 * Plain C, no torch or HIP types: pointers are DEVICE pointers (hipMalloc'd or
 * torch CUDA tensors), `stream` is a hipStream_t passed as void* (NULL = default
 * stream).  Every call is asynchronous on `stream` and returns an int status
 * (FV3_OK = 0); on failure the message is in fv3_last_error() (thread-local).
 * Nothing throws across this boundary.
 *
 * Reference interfaces each entry point replaces (paths under /root/reference):
 *   fv3_mappm*            external/mappm/mappm/mappm.f90:10  (f2py `mappm.mappm(pe1, q1,
 *                         pe2, i1, i2, iv, kord, ptop)`, bound at
 *                         external/vcm/vcm/cubedsphere/regridz.py:273)
 *   fv3_dense_*           the Keras predict of a DenseModel (and of the emulator MLP):
 *                         external/fv3fit/fv3fit/keras/_models/shared/pure_keras.py:112
 *                         (graph built in external/fv3fit/fv3fit/keras/_models/dense.py:234-305)
 *   fv3_regrid_coarsen    external/vcm/vcm/cubedsphere/regridz.py:25-55 + 115-161 fused with
 *                         external/vcm/vcm/cubedsphere/coarsen.py:183-218
 *                         (as orchestrated by coarsen_restarts.py:411-516, 840-887)
 *   fv3_weighted_block_average*, fv3_hydrostatic_balance  the plain area-weighted averages
 *                         and _impose_hydrostatic_balance of coarsen_restarts_on_pressure
 *                         (external/vcm/vcm/cubedsphere/coarsen_restarts.py:152-225, 916-938)
 *   fv3_regrid_coarsen_edge  external/vcm/vcm/cubedsphere/regridz.py:58-112 + 115-161 fused with
 *                         external/vcm/vcm/cubedsphere/coarsen.py:221-271 (D-grid u/v of
 *                         coarsen_restarts.py:460-509)
 *   fv3_interpolate_2d    external/mappm/mappm/interpolate_2d.f90:1-27 (f2py
 *                         mappm.interpolate_2d, vcm/interpolate.py:176-180)
 *   fv3_interpolate_levels  metpy.interpolate.interpolate_1d as called by
 *                         vcm/interpolate.py:148-173 (shared output levels)
 *   fv3_pressure_midpoint_log  vcm/calc/thermo/vertically_dependent.py:153-178
 *   fv3_column_integral,  per-rank partial sums behind
 *   fv3_area_weighted_sums, workflows/prognostic_c48_run/runtime/metrics.py:18-55
 *   fv3_level_sums
 *   fv3_ml_epilogue       the PureMLStepper limiter + diagnostics and the loop's
 *                         fillna/add_tendency/precipitation_sum
 *                         (runtime/steppers/machine_learning.py:239-315, runtime/loop.py:103-219)
 */
#ifndef FV3NET_AMD_H
#define FV3NET_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FV3_OK 0
#define FV3_ERR_INVALID 1     /* bad argument (shape, size, NULL) */
#define FV3_ERR_HIP 2         /* HIP runtime failure */
#define FV3_ERR_UNSUPPORTED 3 /* valid request this build does not implement */

const char* fv3_last_error(void);
int fv3_abi_version(void); /* bumped on any signature change (2: emulator fields in fv3_dense_desc,
                              3: fv3_dense_forward_ex, 4: composites + Adapter,
                              5: per-operand dtypes in fv3_adapter_target, fv3_build_kind,
                              6: fv3_host_register / fv3_host_unregister,
                              7: fv3_plan_*, 8: fv3_copy_to_host, fv3_copy_2d,
                              9: fv3_host_alloc / free / copy, the arena, replace
                                 fv3_host_register / unregister; wind rotation,
                                 fv3_sum_squares, fv3_cos_zenith,
                              10: fv3_step_partials_f64, fv3_fold_rows_repeat,
                              11: the `arith` argument of fv3_mappm_ex / _multi and of the
                                  fused coarsen entries) */
const char* fv3_build_kind(void); /* "product" (fv3net_amd/build.py, no experiment knob compiled in)
                                     or "experiment" (a tools/ variant: results may be invalid) */

/*
 * Column layout of a [level, column] field.  Element (column c, level k) lives at
 *     base[(c / ncol_blk) * blk_stride + k * ld + (c % ncol_blk)]
 * A plain [level][ncol] array is {ncol, ncol, 0}; a (tile, z, y, x) restart or
 * prognostic-state array is {ny*nx, ny*nx, nz*ny*nx}, i.e. the stacked sample
 * index of fv3fit's stack() is a zero-copy view (external/fv3fit/fv3fit/_shared/stacking.py:12-27).
 */
typedef struct {
    int64_t ncol_blk;
    int64_t ld;
    int64_t blk_stride;
} fv3_layout;

/* ---- vertical remap: mappm.f90:10-126 ----------------------------------------
 * pe1 [km+1][ncol] input edge pressures (top -> surface), q1 [km][ncol] layer means,
 * pe2 [kn+1][ncol] output edges, q2 [kn][ncol] result.  float32, column fastest
 * (exactly the Fortran pe1(i,k) order).  iv, kord as in the reference; ptop is
 * accepted and ignored, as in the reference (regridz.py:270).  km >= 4.
 *
 * `arith` selects the remap arithmetic (fv3_mappm_ex, fv3_mappm_multi and the fused
 * coarsen entries; fv3_mappm, the f2py signature, is always FV3_ARITH_EXACT):
 *   FV3_ARITH_EXACT  the reference build's arithmetic: IEEE divisions, no FMA
 *                    contraction, Fortran's order-dependent MAX / MIN -> bit-identical
 *                    to the flang-compiled mappm.f90 for every input, NaNs included;
 *   FV3_ARITH_FAST   north_star's floating-point contract (1e-5 rel): divisions by
 *                    v_rcp_f32 reciprocals, FMA within an expression, hardware MAX / MIN
 *                    (csrc/mappm_core.h).  Same algorithm and limiter logic; finite
 *                    inputs only (a NaN operand of MAX / MIN is dropped, not propagated). */
#define FV3_ARITH_EXACT 0
#define FV3_ARITH_FAST 1
int fv3_mappm(const float* pe1, const float* q1, const float* pe2, float* q2, int64_t ncol,
              int km, int kn, int iv, int kord, float ptop, void* stream);

/* Same with an explicit layout per array (e.g. (tile, z, y, x) data in place). */
int fv3_mappm_ex(const float* pe1, fv3_layout pe1_l, const float* q1, fv3_layout q1_l,
                 const float* pe2, fv3_layout pe2_l, float* q2, fv3_layout q2_l, int64_t ncol,
                 int km, int kn, int iv, int kord, float ptop, int arith, void* stream);

/* n_fields fields remapped onto the same edges: one mappm.mappm call per variable on a
 * shared p_in / p_out, as regrid_vertical is used by coarsen_restarts_on_pressure
 * (external/vcm/vcm/cubedsphere/coarsen_restarts.py:411-516, regridz.py:164-279).
 * q1[f] / q2[f] with layouts q1_l[f] / q2_l[f] (host arrays of n_fields device
 * pointers / layouts).  For kord <= 7 fields go two per streaming pass, sharing the
 * pressure-only arithmetic (csrc/mappm_multi.h); every field's result carries exactly
 * the bits of fv3_mappm_ex on that field alone.  1 <= n_fields <= 64. */
int fv3_mappm_multi(const float* pe1, fv3_layout pe1_l, const float* const* q1, const fv3_layout* q1_l,
                    const float* pe2, fv3_layout pe2_l, float* const* q2, const fv3_layout* q2_l,
                    int n_fields, int64_t ncol, int km, int kn, int iv, int kord, float ptop, int arith,
                    void* stream);

/* ---- dense column model: DenseModel predict graph (dense.py:234-305) ----------
 * inputs -> per-input clip (clip.py:65-83) -> StandardNormLayer (x-mean)/(sigma+eps)
 * (emulation/layers/normalization.py:121-139) -> concat (utils.py:65-86) ->
 * n_hidden x Dense(width, relu) (dense_network.py:59-76) -> one linear Dense(out_nz)
 * per output (dense.py:259-264) -> StandardDenormLayer y*sigma+mean
 * (normalization.py:142-149) -> OutputLimit clamp (output_limit.py:29-47) ->
 * zero mask of clipped levels (clip.py:33-46).  All host pointers; the model
 * copies what it needs to the device at create time and is immutable after. */
typedef struct {
    int n_in;                          /* input variables, <= 16 */
    const int* in_nz;                  /* [n_in] levels per input variable */
    const int* in_clip;                /* [n_in][2] {start, stop} kept levels, or NULL = all */
    const float* in_mean;              /* [k_in] k_in = sum of kept levels */
    const float* in_sigma;             /* [k_in] population std (normalization.py:90-94) */
    float epsilon;                     /* StandardNormLayer epsilon (1e-7) */
    int width;                         /* hidden width, <= 256 */
    int n_hidden;                      /* hidden Dense(relu) layers (= depth - 1), >= 1 */
    const float* const* hidden_kernel; /* [n_hidden] -> [fan_in][width] (Keras kernel order) */
    const float* const* hidden_bias;   /* [n_hidden] -> [width] */
    int n_out;                         /* output variables, <= 16 */
    const int* out_nz;                 /* [n_out] */
    const float* const* out_kernel;    /* [n_out] -> [width][out_nz] */
    const float* const* out_bias;      /* [n_out] -> [out_nz] */
    const float* out_mean;             /* [k_out] StandardDenormLayer mean */
    const float* out_sigma;            /* [k_out] StandardDenormLayer sigma */
    const float* out_min;              /* [k_out] or NULL; -inf = no lower limit */
    const float* out_max;              /* [k_out] or NULL; +inf = no upper limit */
    const float* out_mask;             /* [k_out] or NULL; 0/1 zero-mask of clipped levels */
    /* microphysics-emulator graph extensions (emulation/transforms/transforms.py): */
    const float* in_log_eps;           /* [n_in] or NULL; > 0: input v enters as log(max(x, eps)) */
    const int* out_residual;           /* [n_out] or NULL; r >= 0: output o is written as
                                        * input_r + denormalised output (Difference.backward) */
} fv3_dense_desc;

typedef struct fv3_dense_model fv3_dense_model;

int fv3_dense_create(const fv3_dense_desc* desc, fv3_dense_model** out);
int fv3_dense_destroy(fv3_dense_model* model);
int fv3_dense_k_in(const fv3_dense_model* model);
int fv3_dense_k_out(const fv3_dense_model* model);

/* Profiling hook: when `trace` (device, >= 8 * n_blocks int64) is non-NULL, every
 * forward writes per-block phase timestamps (wall_clock64, 100 MHz) and the CU id.
 * Not for concurrent use; pass NULL to disable (the default). */
int fv3_dense_set_trace(fv3_dense_model* model, long long* trace);

/* Forward over ncol columns.  inputs[v] is input variable v (all of its in_nz[v]
 * levels) with layout in_l[v]; outputs[o] receives out_nz[o] levels.  All
 * layouts must share ncol_blk.  Synchronous-free: enqueued on `stream`. */
int fv3_dense_forward(const fv3_dense_model* model, const float* const* inputs,
                      const fv3_layout* in_l, float* const* outputs, const fv3_layout* out_l,
                      int64_t ncol, void* stream);

/* fv3_dense_forward over float64 inputs read in place: each value is cast to float32
 * (round to nearest) in the kernel's input staging, as the Keras model's input cast
 * does (pure_keras.py:98-118 on a float64 state), so the outputs are bit-identical to
 * casting first.  Exact-f32 arithmetic only; FV3_ERR_UNSUPPORTED for models with
 * residual outputs or without the 8-wave kernel (width < 128, 16-column tiles). */
int fv3_dense_forward_f64in(const fv3_dense_model* model, const double* const* inputs,
                            const fv3_layout* in_l, float* const* outputs, const fv3_layout* out_l,
                            int64_t ncol, void* stream);

/* Forward with an explicit arithmetic:
 *   FV3_DENSE_F32     exact f32 products on v_mfma_f32_16x16x4_f32 (= fv3_dense_forward);
 *   FV3_DENSE_BF16X3  every f32 operand split into bf16 hi + lo, products as
 *                     hi*hi + lo*hi + hi*lo on v_mfma_f32_32x32x16_bf16 with f32
 *                     accumulation (~16 mantissa bits per operand: ~1e-5 rel on the
 *                     reference graphs; BASELINE config #5, bf16 MFMA at 1e-3 rel);
 *   FV3_DENSE_BF16X6  every f32 operand split into bf16 hi + mid + lo (~24 mantissa
 *                     bits), products as the six split terms of order <= 2
 *                     (hi*hi, mid*hi, hi*mid, mid*mid, lo*hi, hi*lo), f32 accumulation:
 *                     f32-level error, within the 1e-5 rel tendency contract.
 * Same graph, layouts and in-place semantics as fv3_dense_forward. */
#define FV3_DENSE_F32 0
#define FV3_DENSE_BF16X3 1
#define FV3_DENSE_BF16X6 2
int fv3_dense_forward_ex(const fv3_dense_model* model, const float* const* inputs,
                         const fv3_layout* in_l, float* const* outputs, const fv3_layout* out_l,
                         int64_t ncol, int precision, void* stream);

/* ---- fused pressure-level coarse-graining (config #3) ----------------------------
 * For every coarse cell (factor x factor fine columns of a tile):
 *   delp_c = sum(delp*area)/sum(area)                     (coarsen.py:183-218)
 *   phalf_f = cumsum([ptop_toa, delp_f]), phalf_c likewise  (vertically_dependent.py:41-66)
 *   f_r = mappm(phalf_f, f, phalf_c_on_f, iv, kord)        (regridz.py:164-279)
 *   w = area if phalf_c[k+1] < phalf_f[km+1] else 0        (regridz.py:150-161)
 *   out = sum(f_r*w)/sum(w) per level                      (coarsen.py:183-218)
 * delp, fields: (tile, km, ny, nx) float32; area (tile, ny, nx); out (tile, km, ny/f, nx/f);
 * delp_out (tile, km, ny/f, nx/f) receives delp_c (area-weighted, not masked).
 * fields/out are HOST arrays of n_fields <= 32 device pointers (passed by value to the
 * kernel, nothing is allocated per call); 4 <= km <= 128, 1 <= factor <= 8, kord <= 7.
 * Arithmetic follows the reference's dtype flow: delp products, delp_c and the phalf
 * cumsums in delp's dtype, area and field sums in float32, block sums in numpy's
 * order for the reshaped coarsen().sum() — bit-exact to oracle/coarsen.py with
 * FV3_ARITH_EXACT; FV3_ARITH_FAST remaps under the tolerance contract (see fv3_mappm). */
int fv3_regrid_coarsen(const float* delp, const float* area, const float* const* fields,
                       float* const* out, int n_fields, float* delp_out, int ntile, int km,
                       int ny, int nx, int factor, int iv, int kord, double ptop_toa,
                       int arith, void* stream);

/* Same with float64 delp (FV3 fv_core restarts store delp in double precision; the
 * pressures are cumulated in float64 either way). */
int fv3_regrid_coarsen_f64(const double* delp, const float* area, const float* const* fields,
                           float* const* out, int n_fields, float* delp_out, int ntile, int km,
                           int ny, int nx, int factor, int iv, int kord, double ptop_toa,
                           int arith, void* stream);

/* Same, with the coarse delp returned in float64 (restart precision, as
 * weighted_block_average(delp, area) gives it in coarsen_restarts.py:480-486). */
int fv3_regrid_coarsen_f64d(const double* delp, const float* area, const float* const* fields,
                            float* const* out, int n_fields, double* delp_out, int ntile, int km,
                            int ny, int nx, int factor, int iv, int kord, double ptop_toa,
                            int arith, void* stream);

/* ---- the rest of coarsen_restarts_on_pressure (coarsen_restarts.py:152-225) -------
 * fv3_weighted_block_average[_f64]: sum(obj * w) / sum(w) over factor x factor blocks
 *   (cubedsphere/coarsen.py:183-218) of n_fields (<= 16) arrays (ntile, nz, ny, nx) with
 *   weights (ntile, ny, nx) float32 -> (ntile, nz, ny/f, nx/f) in the field's dtype;
 *   NaN-skipping sums in numpy's order.  Replaces the plain area-weighted averages of
 *   phis/delp/DZ (coarsen_restarts.py:439, 480-486) and u_srf/v_srf (:890-913).
 * fv3_hydrostatic_balance: _impose_hydrostatic_balance (coarsen_restarts.py:916-938) on
 *   the coarse grid: dz_out = hydrostatic_dz(T, sphum, delp) (vertically_dependent.py:
 *   211-228), phis_out = g * (top height of height_at_interface(dz, phis) + sum dz_out)
 *   (:69-100, 182-186).  T/sphum float32 (tile, km, ny, nx), delp/dz float64, phis
 *   (tile, ny, nx) float64.  dz_out may alias dz. */
int fv3_weighted_block_average(const float* const* fields, float* const* out, int n_fields,
                               const float* weights, int ntile, int nz, int ny, int nx, int factor,
                               void* stream);
int fv3_weighted_block_average_f64(const double* const* fields, double* const* out, int n_fields,
                                   const float* weights, int ntile, int nz, int ny, int nx,
                                   int factor, void* stream);
int fv3_hydrostatic_balance(const float* temperature, const float* sphum, const double* delp,
                            const double* dz, const double* phis, double* dz_out, double* phis_out,
                            int ntile, int km, int ny, int nx, double ptop_toa, void* stream);

/* ---- edge-weighted (D-grid wind) pressure-level coarse-graining ------------------
 * edge 0 ("x", u): fields and spacing (dx) on (y outer = ny+1, x center = nx); coarse
 *   output (tile, km, ny/f + 1, nx/f), coarsened along x, every f-th outer row kept.
 * edge 1 ("y", v): fields and spacing (dy) on (y center = ny, x outer = nx+1); coarse
 *   output (tile, km, ny/f, nx/f + 1), coarsened along y, every f-th outer column kept.
 * Per coarse edge, from its f fine edge points:
 *   delp_e = 0.5*(delp on either side)  (xgcm interp with the cubed-sphere face
 *            connections of cubedsphere/xgcm.py:7-34 for the tile-boundary edges)
 *   delp_c = sum(spacing*delp_e)/sum(spacing)                (coarsen.py:221-271)
 *   phalf_f = cumsum([ptop, delp_e]), phalf_c = cumsum([ptop, delp_c])
 *   f_r = mappm(phalf_f, f, phalf_c, iv, kord); w = spacing if phalf_c[k+1] < phalf_f[km+1]
 *   out = sum(f_r*w)/sum(w)
 * All 6 tiles (ntile == 6), square tiles (ny == nx), an even number of coarse cells per
 * side (the reference's block_upsample_like requires it), 4 <= km <= 128,
 * 1 <= factor <= 8, kord <= 7.  delp (tile, km, n, n); fields/out host arrays of
 * n_fields <= 32 device pointers.  Bit-exact to oracle/coarsen.py
 * coarsen_edges_on_pressure. */
int fv3_regrid_coarsen_edge(const float* delp, const float* spacing, const float* const* fields,
                            float* const* out, int n_fields, int ntile, int km, int ny, int nx,
                            int factor, int edge, int iv, int kord, double ptop_toa, int arith,
                            void* stream);
int fv3_regrid_coarsen_edge_f64(const double* delp, const float* spacing,
                                const float* const* fields, float* const* out, int n_fields,
                                int ntile, int km, int ny, int nx, int factor, int edge, int iv,
                                int kord, double ptop_toa, int arith, void* stream);

/* ---- per-column reductions for stepper diagnostics --------------------------------
 * out[c] = sum_k field[k][c] * delp[k][c] * scale  (vcm mass_integrate,
 * external/vcm/vcm/calc/thermo/vertically_dependent.py:18-22, with scale = 1/g),
 * accumulated in float64, written as float32. */
int fv3_column_integral(const float* field, fv3_layout field_l, const float* delp,
                        fv3_layout delp_l, float* out, int64_t ncol, int km, double scale,
                        void* stream);

/* Area-weighted global partial sums: partial[2*d+0] = sum(area*x_d), partial[2*d+1] =
 * sum(area) in float64, over ncol columns, for n_diag 2-D diagnostics x_d (each [ncol]).
 * Deterministic (fixed reduction tree).  metrics.py:18-24 partials. */
int fv3_area_weighted_sums(const float* const* diags, int n_diag, const float* area,
                           int64_t ncol, double* partial, void* stream);
/* The same over float64 diagnostics and area (the reference's dtype: numpy's
 * area * ds on float64 grid data); same reduction tree. */
int fv3_area_weighted_sums_f64(const double* const* diags, int n_diag, const double* area,
                               int64_t ncol, double* partial, void* stream);

/* Per-level horizontal sums out[k] = sum_c x[k][c] in float64 (fixed reduction tree):
 * the per-rank part of metrics.py:27-32 global_horizontal_sum. */
int fv3_level_sums(const float* x, fv3_layout x_l, int64_t ncol, int nz, double* out, void* stream);
/* The same over a float64 field (summed without a float32 rounding, as numpy sums a
 * float64 DataArray) and over a uint8 flag field (the stepper's
 * specific_humidity_limiter_active, machine_learning.py:301-303, read in place). */
int fv3_level_sums_f64(const double* x, fv3_layout x_l, int64_t ncol, int nz, double* out, void* stream);
int fv3_level_sums_u8(const unsigned char* x, fv3_layout x_l, int64_t ncol, int nz, double* out, void* stream);

/* World-size-invariant global sums (distributed.global_row_sums): partials per grid ROW
 * (row_len contiguous columns; a rank's band of the flattened (tile, y) rows is a run
 * of rows), folded in global row order, so the global result has the same bits for any
 * number of ranks.
 *   fv3_area_weighted_row_sums[_f64]: partial[r*partial_ld + 2d + {0,1}] = (sum_c area*x_d,
 *     sum_c area) over row r of n_diag (rows, row_len) diagnostics, float64;
 *   fv3_level_row_sums_{u8,f64}: out[r*out_ld + k] = sum_c x[k][r][c] of a (nz, rows,
 *     row_len) field whose levels are level_stride elements apart, float64 (the u8 flag
 *     counts are integers, exact in any order);
 *   (the strides let both write into one [nrows][W] buffer for a single exchange)
 *   fv3_fold_rows: out[j] = sum_r rows[r][j].
 * Every sum: lane-strided sequential sums over 64 lanes (column c or row r on lane
 * c % 64, r % 64) then a fixed 64-lane xor butterfly. */
int fv3_area_weighted_row_sums(const float* const* diags, int n_diag, const float* area, int64_t nrows,
                               int row_len, double* partial, int64_t partial_ld, void* stream);
int fv3_area_weighted_row_sums_f64(const double* const* diags, int n_diag, const double* area,
                                   int64_t nrows, int row_len, double* partial, int64_t partial_ld,
                                   void* stream);
int fv3_level_row_sums_u8(const unsigned char* x, int nz, int64_t nrows, int row_len, int64_t level_stride,
                          double* out, int64_t out_ld, void* stream);
int fv3_level_row_sums_f64(const double* x, int nz, int64_t nrows, int row_len, int64_t level_stride,
                           double* out, int64_t out_ld, void* stream);
int fv3_fold_rows(const double* rows, int64_t nrows, int width, double* out, void* stream);
/* One stepper step's per-rank reductions in one launch: fv3_area_weighted_row_sums_f64
 * of the n_diag diagnostics and fv3_level_sums_u8 of the (nz, ncol) limiter flags, each
 * with the bits of its own call (replaces the two launches of
 * runtime/steppers/machine_learning.py:301-303 + runtime/metrics.py:18-32's per-rank
 * part; limiter rows not 16-byte aligned take the two launches). */
int fv3_step_partials_f64(const double* const* diags, int n_diag, const double* area, int64_t nrows, int row_len,
                          double* partial, int64_t partial_ld, const unsigned char* limiter, fv3_layout lim_l,
                          int64_t ncol, int nz, double* level_out, void* stream);
/* A stubbed all-gather and its fold in one launch: rep[t*nrows + r][j] = rows[r][j] for
 * t < times (the bytes `times` ranks' partials move), out[j] = fv3_fold_rows(rep). */
int fv3_fold_rows_repeat(const double* rows, int64_t nrows, int width, int times, double* rep, double* out,
                         void* stream);

/* TimeMask (external/emulation/emulation/_emulate/microphysics.py:37-47): out =
 * state * alpha + emulator * (1 - alpha) over n elements, each product in its array's
 * dtype (float64 when *_f64, else float32) and the sum in the promoted dtype (float64 if
 * either is), as numpy computes it.  out may alias either input. */
int fv3_time_blend(const void* state, int state_f64, const void* emulator, int emulator_f64, void* out,
                   int64_t n, double alpha, void* stream);

/* ---- microphysics emulator hook post-processing (external/emulation) ------------------
 * On the hook's [feature, sample] arrays, contiguous, n elements (or nz x ncol), every
 * array of one dtype (f64 != 0: double, else float); numpy semantics (NaN-propagating
 * maximum/minimum, Python-float constants in the arrays' dtype).
 *   fv3_range_mask            RangeMask (masks.py:23-39)
 *   fv3_classify_one_hot      _get_classify_output (zhao_carr.py:214-219): logits
 *                             [n_class][inner] -> masks [n_class + 1][inner] (uint8), the
 *                             last = masks[positive] | masks[negative]
 *   fv3_zc_infer_gscond_cloud infer_gscond_cloud_from_conservation (zhao_carr.py:72-76)
 *   fv3_zc_squash             squash_water_water_conserving (zhao_carr.py:57-69)
 *   fv3_zc_zero_where         out = class_mask ? 0 : cloud (mask_zero_cloud_classifier_precpd,
 *                             zhao_carr.py:240-247)
 *   fv3_zc_gscond_update      mode FV3_ZC_CLOUD_*: the gscond cloud choice then
 *                             _update_with_net_condensation (zhao_carr.py:79-105, 164-245);
 *                             FV3_ZC_PHASE_DEPENDENT: enforce_conservative_phase_dependent
 *                             with ice_flag from fv3_zc_ice_water_flag (:143-146, 242-245)
 *   fv3_zc_ice_water_flag     ice_water_flag (zhao_carr.py:108-133) of T - offset over
 *                             the last axis of (nrows, z) arrays
 *   fv3_zc_precpd_conservative enforce_conservative_precpd (zhao_carr.py:277-352); precip
 *                             [ncol] float64 in m
 *   fv3_zc_precip_simple      conservative_precip_simple (zhao_carr.py:355-371), precip [ncol] */
#define FV3_ZC_CLOUD_EMULATOR 0     /* enforce_conservative_gscond */
#define FV3_ZC_CLOUD_IDENTICAL 1    /* mask_where_fortran_cloud_identical */
#define FV3_ZC_CLOUD_VANISHES 2     /* mask_where_fortran_cloud_vanishes_gscond */
#define FV3_ZC_CLOUD_CLASS_ZERO 3   /* mask_zero_cloud_classifier (class_mask = zero_cloud) */
#define FV3_ZC_CLOUD_CLASS_NOTEND 4 /* mask_zero_tend_classifier (class_mask = zero_tendency) */
#define FV3_ZC_PHASE_DEPENDENT 5    /* enforce_conservative_phase_dependent */
int fv3_range_mask(const void* x, void* out, int64_t n, double lo, double hi, int has_lo, int has_hi, int f64,
                   void* stream);
int fv3_classify_one_hot(const void* logits, int n_class, int64_t inner, unsigned char* masks, int positive,
                         int negative, int f64, void* stream);
int fv3_zc_infer_gscond_cloud(const void* qc_in, const void* qv_in, const void* qv_gscond, void* qc_out,
                              int64_t n, int f64, void* stream);
int fv3_zc_squash(const void* cloud, const void* humidity, double bound, void* cloud_out, void* humidity_out,
                  int64_t n, int f64, void* stream);
int fv3_zc_zero_where(const unsigned char* class_mask, const void* cloud, void* out, int64_t n, int f64,
                      void* stream);
int fv3_zc_gscond_update(int mode, const void* qc_in, const void* qv_in, const void* t_in,
                         const void* qc_fortran_gscond, const void* qc_emulator, const unsigned char* class_mask,
                         const unsigned char* ice_flag, void* qc_out, void* qv_out, void* t_out, int64_t n,
                         int f64, void* stream);
int fv3_zc_ice_water_flag(const void* temperature, const void* cloud, double offset, void* iw, int64_t nrows,
                          int64_t z, int f64, void* stream);
int fv3_zc_precpd_conservative(const void* qc_gscond, const void* qv_gscond, const void* t_gscond,
                               const void* qc_emulator, const void* qv_emulator, const void* delp, void* qc_out,
                               void* qv_out, void* t_out, double* precip, int nz, int64_t ncol, int f64,
                               void* stream);
int fv3_zc_precip_simple(const void* qv_gscond, const void* qc_gscond, const void* qv_emulator,
                         const void* qc_emulator, const void* delp, void* precip, int nz, int64_t ncol, int f64,
                         void* stream);

/* ---- StandardScaler (external/fv3fit/fv3fit/_shared/scaler.py:36-100) -------------
 * As the PytorchPredictor applies it around its model (fv3fit/pytorch/predict.py:
 * 299-399):  out = float32((x - mean) / std) computed in float64 (x float32, or float64
 * when x_f64), and out = y * std + mean in float64 from the model's float32 y.
 * mean/std are DEVICE float64 arrays of n_params = nz values (per level) or 1 (a 2-D
 * variable).  Bit-identical to numpy's float64 arithmetic. */
int fv3_standard_normalize(const void* x, int x_f64, fv3_layout x_l, const double* mean,
                           const double* std_, int n_params, float* out, fv3_layout out_l,
                           int64_t ncol, int nz, void* stream);
int fv3_standard_denormalize(const float* y, fv3_layout y_l, const double* mean, const double* std_,
                             int n_params, double* out, fv3_layout out_l, int64_t ncol, int nz,
                             void* stream);
/* The same with a float64 result (StandardScaler.normalize's own float64 output,
 * scaler.py:65-68) / from a float64 input (StandardScaler.denormalize, :70-73). */
int fv3_standard_normalize_f64(const void* x, int x_f64, fv3_layout x_l, const double* mean,
                               const double* std_, int n_params, double* out, fv3_layout out_l,
                               int64_t ncol, int nz, void* stream);
int fv3_standard_denormalize_f64(const double* y, fv3_layout y_l, const double* mean, const double* std_,
                                 int n_params, double* out, fv3_layout out_l, int64_t ncol, int nz,
                                 void* stream);

/* ---- ML stepper epilogue: limiter + diagnostics + apply (config #4) --------------
 * One pass per column over everything the prognostic loop does with a (dQ1, dQ2)
 * prediction: the non-negative-humidity limiter (MSE-conserving, machine_learning.py:
 * 77-99, or legacy :67-74), its column diagnostics (:267-303), compute_diagnostics'
 * net moistening / column heating (diagnostics/compute.py:77-106), fillna + filled
 * fraction (loop.py:103-110), add_tendency (loop.py:202-219) and precipitation_sum
 * (diagnostics/compute.py:21-39).  dq1/dq2 are the model's float32 [z][col] outputs;
 * the state arrays and every output are float64 (state_f64 = 1, as the FV3 state is)
 * or float32; all [z][col] arrays share `lay`.  Bit-identical to the reference's
 * dtype flow (oracle/stepper.py).  Outputs may be NULL; temperature_out / sphum_out
 * may alias the inputs (in-place update). */
typedef struct {
    const float* dq1;            /* [z][col] model heating tendency, K/s */
    const float* dq2;            /* [z][col] model moistening tendency, kg/kg/s */
    const void* sphum;           /* [z][col] specific humidity */
    const void* delp;            /* [z][col] pressure thickness, Pa */
    const void* temperature;     /* [z][col] air temperature, K */
    const void* physics_precip;  /* [col] physics precipitation (m), or NULL */
    void* dq1_out;               /* [z][col] limited dQ1 (before fillna), or NULL */
    void* dq2_out;               /* [z][col] limited dQ2, or NULL (with dq1_out) */
    unsigned char* limiter_active; /* [z][col] 1 where the limiter changed dQ2, or NULL */
    void* temperature_out;       /* [z][col] T + fillna(dQ1) dt, or NULL */
    void* sphum_out;             /* [z][col] q + fillna(dQ2) dt, or NULL */
    void* column;                /* [7][column_ld] column diagnostics, or NULL:
                                  * 0 dQ1 limiter heating change (W/m2), 1 dQ2 limiter moistening
                                  * change (kg/m2/s), 2 net moistening, 3 column heating,
                                  * 4 dQ1 filled fraction, 5 dQ2 filled fraction,
                                  * 6 total precipitation (m; only with physics_precip) */
    int64_t column_ld;           /* row stride of `column` (0 = ncol) */
} fv3_epilogue_io;

int fv3_ml_epilogue(const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz, int state_f64,
                    double dt, int mse_conserving, int hydrostatic, void* stream);

/* Same, for a prediction that lacks dQ1 or dQ2 (machine_learning.py:258-259 limits
 * zeros in its place): `flags` holds FV3_EPI_HAS_DQ1 / FV3_EPI_HAS_DQ2 for the tendencies
 * the model predicts; for a missing one pass zeros as dq1/dq2, and the kernel leaves its
 * state variable unchanged and its net moistening / column heating at zero, as
 * compute_diagnostics and add_tendency do (diagnostics/compute.py:84-85, loop.py:202-219).
 * fv3_ml_epilogue is this with both flags. */
#define FV3_EPI_HAS_DQ1 1
#define FV3_EPI_HAS_DQ2 2
int fv3_ml_epilogue_ex(const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz, int state_f64,
                       double dt, int mse_conserving, int hydrostatic, int flags, void* stream);

/* The prediction's other tendencies (runtime/names.py:31-50), one pass per column, every
 * [z][col] array under `lay`; delp / state_out / filled_frac in the state's dtype
 * (state_f64), the tendency float32 (model output):
 *   FV3_TEND_WIND (dQu, dQv): integral[col] (state dtype) = sum_z dQ * delp / g, the
 *     column_integrated_dQ{u,v}_stress of compute_ml_momentum_diagnostics
 *     (diagnostics/compute.py:140-161); filled_out (float64, or NULL) = fillna(dQ) as
 *     prepare_agrid_wind_tendencies hands it on (loop.py:126-145).
 *   FV3_TEND_MASS (dQp): integral[col] (float32) = sum_z 1 * dQp / g, the
 *     net_mass_tendency_due_to_<label> (compute.py:107-115); state_out = delp +
 *     fillna(dQp) * dt (add_tendency, loop.py:202-219), may alias delp.
 * filled_frac[col] = NaN count / nz (loop.py:103-110).  Sums run over z in order, NaN
 * skipped.  Any output may be NULL. */
#define FV3_TEND_WIND 0
#define FV3_TEND_MASS 1
int fv3_tendency_columns(const float* tendency, const void* delp, double* filled_out, void* state_out,
                         void* integral, void* filled_frac, fv3_layout lay, int64_t ncol, int nz,
                         int state_f64, int mode, double dt, void* stream);

/* ---- vertical interpolation to new levels ------------------------------------------
 * Every array is level-major: element (level k, column c) at [k * ld + c].  One thread
 * per column; enqueued on `stream`.
 *
 * interpolate_2d.f90 semantics, float64: out = fill_value, then for each output level the
 * LAST interval k (k = 0..n_in-2) with x_k <= xp < x_k+1 (linear, y_k (1-w) + y_k+1 w,
 * w = (xp - x_k)/(x_k+1 - x_k)), x_k == xp (y_k) or x_k+1 == xp (y_k+1) decides.  xp has
 * n_out levels per column (ld_xp = 0 broadcasts one level set).  Bit-exact to the
 * Fortran. */
int fv3_interpolate_2d(const double* xp, int64_t ld_xp, const double* x, int64_t ld_x,
                       const double* y, int64_t ld_y, double* out, int64_t ld_out, int64_t ncol,
                       int n_in, int n_out, double fill_value, void* stream);

/* metpy.interpolate.interpolate_1d for output `levels` shared by all columns (float64,
 * sorted ascending; reverse != 0 writes level j to n_out-1-j, as metpy does for
 * descending requests).  xp (column coordinate, ascending) and var with their level
 * strides; dtypes = xp_is_f64 | var_is_f64 << 1 (else float32); out float64.
 * Values outside [xp_0, xp_n-1] get fill_value.  numpy's promotion: each difference of
 * column values in its own dtype, the rest in float64. */
int fv3_interpolate_levels(const void* xp, int64_t ld_xp, const void* var, int64_t ld_v, int dtypes,
                           const double* levels, int n_out, int reverse, double* out,
                           int64_t ld_out, int64_t ncol, int n_in, double fill_value, void* stream);

/* pressure_at_midpoint_log: pi = cumsum([ptop, delp]); out = delp / diff(log(pi)), in
 * delp's dtype (0 float32, 1 float64). */
int fv3_pressure_midpoint_log(const void* delp, int dtype, int64_t ld_in, void* out, int64_t ld_out,
                              int64_t ncol, int nz, double ptop, void* stream);

/* ---- composite predictors and the online transformer Adapter ------------------------
 * The arithmetic of the fv3fit composites that nest the build's predictor as a
 * base_model (external/fv3fit/fv3fit/_shared/models.py) and of the prognostic run's
 * second Predictor caller (workflows/prognostic_c48_run/runtime/transformers/fv3fit.py).
 *
 * fv3_member_reduce replaces EnsembleModel.predict's xr.concat(outputs, "member") then
 * .mean / .median(dim="member") (models.py:253-260): n_members contiguous arrays of n
 * elements (float32, or float64 with dtype_f64), NaN-skipping as numpy's nanmean /
 * nanmedian (member order, (low + high) / 2 for the median, NaN where every member is
 * NaN); out may alias nothing.  1..32 members. */
#define FV3_REDUCE_MEAN 0
#define FV3_REDUCE_MEDIAN 1
int fv3_member_reduce(const void* const* members, int n_members, int64_t n, int dtype_f64, int op,
                      void* out, void* stream);

/* ---- out-of-sample composite (OutOfSampleModel, _shared/models.py:340-400) -----------
 * fv3_minmax_scores replaces MinMaxNoveltyDetector.predict
 *   (fv3fit/sklearn/_min_max_novelty_detector.py:86-115): per column, the packed features
 *   (variables in order, levels [z0, z0 + nfeat) of each: packer clip), MinMaxScaler's
 *   X *= scale_; X += min_ in X's dtype (x_f64: any float64 input), and
 *   score = max(max X - 1, 0) + max(-1 * min X, 0) (NaN propagates as in numpy).
 *   score: [ncol] in X's dtype.  1 <= n_vars <= FV3_NOV_MAX_VARS.
 * fv3_taper_columns replaces taper_mask / taper_ramp / taper_decay
 *   (_shared/taper_function.py:6-35; mode FV3_TAPER_*, p0/p1 = cutoff / (ramp_min,
 *   ramp_max) / (threshold, rate)) and OutOfSampleModel.predict's output * taper
 *   (models.py:392-398): taper_out (or NULL) receives the taper values (int64 for the
 *   mask, else the score's dtype); every field is multiplied per column in numpy's
 *   promoted dtype (float64 unless both the field and the taper are float32). */
#define FV3_NOV_MAX_VARS 16
#define FV3_NOV_MAX_FIELDS 16
#define FV3_TAPER_MASK 0
#define FV3_TAPER_RAMP 1
#define FV3_TAPER_DECAY 2
typedef struct {
    const void* data;    /* [level][column] under `layout` */
    fv3_layout layout;
    int data_f64;
    int z0;              /* first kept level */
    int nfeat;           /* kept levels (1 for a 2-D variable) */
} fv3_nov_var;
typedef struct {
    const void* in;      /* [level][column] base-model output */
    fv3_layout in_layout;
    int in_f64;
    void* out;           /* [level][column] tapered output, float64 or float32 (see above) */
    fv3_layout out_layout;
    int nz;
} fv3_taper_field;
int fv3_minmax_scores(const fv3_nov_var* vars, int n_vars, const void* scale, const void* min, int scale_f64,
                      int x_f64, int64_t ncol, void* score, void* stream);
int fv3_taper_columns(const void* score, int score_f64, int64_t ncol, int mode, double p0, double p1,
                      void* taper_out, const fv3_taper_field* fields, int n_fields, void* stream);

/* fv3_scale_levels replaces TaperConfig.apply (_shared/config.py:21-29, TaperedModel
 * models.py:95-100): out[k][c] (float64, contiguous [nz][ncol]) = scale[k] * x(c, k),
 * x float32 or float64 under `lay` with its levels on the taper dimension. */
int fv3_scale_levels(const void* x, int x_f64, fv3_layout lay, const double* scale, int64_t ncol, int nz,
                     double* out, void* stream);

/* fv3_adapter_apply replaces Adapter.predict's arithmetic (transformers/fv3fit.py:66-83) for
 * every state variable updated by tendency predictions: tendency = 0 + p_0 + p_1 + ...
 * (Python's sum), out = state + tendency * dt; with `limit` the specific-humidity target
 * (index sphum_target) and, if temp_target >= 0, the air-temperature target go through
 * non_negative_sphum_mse_conserving (steppers/machine_learning.py:77-99) first.  Every
 * intermediate carries numpy's dtype: a prediction is float32 or float64 (bit p of
 * pred_f64), the sum widens at the first float64 term, Python-float constants take the
 * array's dtype, and out is float64 when the state or the (limited) tendency is
 * (out_f64 must say so: FV3_ERR_INVALID otherwise).  Every array holds n contiguous
 * elements; out may alias state when it has the state's dtype.  limit without a
 * humidity target: FV3_ERR_UNSUPPORTED (the reference's NotImplementedError). */
#define FV3_ADAPTER_MAX_PREDS 8
#define FV3_ADAPTER_MAX_TARGETS 16
typedef struct fv3_adapter_target {
    const void* preds[FV3_ADAPTER_MAX_PREDS]; /* float32, or float64 where pred_f64 has the bit */
    int n_preds;
    const void* state; /* float64 (state_f64) or float32 */
    void* out;         /* float64 (out_f64) or float32 */
    unsigned pred_f64;
    int out_f64;
} fv3_adapter_target;
int fv3_adapter_apply(const fv3_adapter_target* targets, int n_targets, int64_t n, int state_f64, double dt,
                      int limit, int sphum_target, int temp_target, void* stream);

/* Derived variables behind fv3fit's DerivedModel and TransformedPredictor
 * (external/fv3fit/fv3fit/_shared/models.py:110-220, 279-337): the vcm.DerivedMapping
 * (vcm/derived_mapping.py:123-127, 264-410) and vcm.DataTransform (vcm/data_transform.py:
 * 65-323) entries a dQ1/dQ2 model feeds.  Operands are float32 or float64; every numpy
 * intermediate keeps numpy's dtype (Python-float constants take the array's dtype), so the
 * results are bit-identical to the numpy expressions.
 *
 * fv3_derived_elementwise: n contiguous elements per operand (a NULL operand of
 * ADD / SUB after the first is zeros_like of its dtype), out in out_f64's dtype:
 *   ADD / SUB       in0 + in1 + ... / in0 - in1 - ... (left to right, promoted)
 *   IADD            in0 += in1 (promoted arithmetic, stored in in0's dtype)
 *   SCALE           p0 * in0            DIV_SCALAR      in0 / p0
 *   MSE             moist_static_energy_tendency(in0 = Q1, in1 = Q2[, in2 = T])
 *   TEMP_TEND       temperature_tendency(in0 = Qm, in1 = Q2[, in2 = T])  (local.py:317-360)
 *   INCLOUD_TO_GRIDCELL / GRIDCELL_TO_INCLOUD  (clouds.py:7-66): in0 = cloud fraction,
 *                   in1 = condensate, p0 = climit1, p1 = climit2
 *   MUL             in0 * in1           ONE_MINUS_MUL   (1 - in0) * in1
 *   ISCLOSE_ONEHOT  where(isclose(in0, p0, rtol = p1, atol = p2), 1.0, 0.0), float64
 *                   (derived_mapping.py:194-262)
 *   SIGN_PARALLEL   sign(in0 / in1) * abs(in1)  (derived_mapping.py:163-174)
 *   PROJECT         (in0 * in1 + in2 * in3) / p0, p0 in float64 if p1 != 0 else float32
 *                   (derived_mapping.py:177-187; p0 the norm from fv3_sum_squares) */
#define FV3_EW_ADD 1
#define FV3_EW_SUB 2
#define FV3_EW_IADD 3
#define FV3_EW_SCALE 4
#define FV3_EW_DIV_SCALAR 5
#define FV3_EW_MSE 6
#define FV3_EW_TEMP_TEND 7
#define FV3_EW_INCLOUD_TO_GRIDCELL 8
#define FV3_EW_GRIDCELL_TO_INCLOUD 9
#define FV3_EW_MUL 10
#define FV3_EW_ONE_MINUS_MUL 11
#define FV3_EW_ISCLOSE_ONEHOT 12
#define FV3_EW_SIGN_PARALLEL 13
#define FV3_EW_PROJECT 14
int fv3_derived_elementwise(int op, const void* const* in, const int* in_f64, int n_in, void* out, int out_f64,
                            int64_t n, const double* params, int n_params, void* stream);

/* fv3_derived_columns: per column over nz levels ([level][column] under each field's
 * layout; 2-D fields are one level):
 *   MASS_INTEGRAL         out0 = [-]p1 * sum_z nan0(s x delp / g), x = in0, delp = in1,
 *                         s = sign(p0), p1 NaN: no scale, p2 != 0: negated, p3 != 0: numpy's
 *                         pairwise order of a z-last array (nz <= 128; else sequential, as
 *                         numpy reduces a leading or middle axis) (vertically_dependent.py:
 *                         18-22, 279-325)
 *   TENDENCY_TO_FLUX      in0 tendency, in1 delp, in2 TOA net flux (NULL: zeros), in3
 *                         surface upward flux; out0 = interface fluxes (nz levels), out1 =
 *                         downward surface flux, rectified when p0 != 0 (flux_form.py:7-42)
 *   IMPLIED_SURFACE_FLUX  the same inputs; out0 = TOA + up - <in0>, p1 as MASS_INTEGRAL's p3
 *                         (flux_form.py:45-73)
 *   FLUX_TO_TENDENCY      in0 fluxes (nz levels), in1 delp, in2 downward, in3 upward
 *                         surface flux; out0 = -(g diff(flux) / delp) (flux_form.py:76-100) */
typedef struct fv3_field {
    const void* data;
    int f64;
    fv3_layout lay;
} fv3_field;
#define FV3_COL_MASS_INTEGRAL 1
#define FV3_COL_TENDENCY_TO_FLUX 2
#define FV3_COL_IMPLIED_SURFACE_FLUX 3
#define FV3_COL_FLUX_TO_TENDENCY 4
int fv3_derived_columns(int op, const fv3_field* in, int n_in, const fv3_field* out, int n_out, int64_t ncol, int nz,
                        const double* params, int n_params, void* stream);

/* A float32 / float64 operand addressed by element strides over the dims of a result of
 * `ndim` <= FV3_MAX_DIMS dims (stride 0: broadcast along that dim, as xarray aligns
 * operands by dim name). */
#define FV3_MAX_DIMS 6
typedef struct fv3_strided {
    const void* data;
    int f64;
    int64_t stride[FV3_MAX_DIMS];
} fv3_strided;

/* D-grid x/y winds (or wind tendencies) to A-grid eastward/northward
 * (vcm/cubedsphere/rotate.py:9-56 center_and_rotate_xy_winds, coarsen.py:54-75
 * shift_edge_var_to_center; derived_mapping.py:130-160 dQu / dQv / eastward_wind /
 * northward_wind).  The result has `shape` (the centered dims, contiguous outputs):
 *   xc = 0.5 * (x[i + x_stag] + x[i])   (x's dtype; x_stag: the stride of x's staggered
 *   yc = 0.5 * (y[i + y_stag] + y[i])    dim, the edge one past the cell),
 *   eastward  = coeff[0] * xc + coeff[1] * yc,  northward = coeff[2] * xc + coeff[3] * yc
 * coeff = eastward_wind_u_coeff, eastward_wind_v_coeff, northward_wind_u_coeff,
 * northward_wind_v_coeff; numpy's dtype flow (each product in its operands' promoted
 * dtype, the sum in the products'), bit-identical to the numpy expressions.  `eastward` /
 * `northward` may be NULL (not wanted); their dtypes must be the promoted ones. */
int fv3_center_rotate_winds(int ndim, const int64_t* shape, fv3_strided x_wind, int64_t x_stag, fv3_strided y_wind,
                            int64_t y_stag, const fv3_strided* coeff, void* eastward, int east_f64, void* northward,
                            int north_f64, void* stream);

/* sum over the n_arr arrays of n contiguous elements each of x^2, accumulated in float64
 * in a fixed order (deterministic), into *out (device, one double): the square of
 * np.linalg.norm((a, b)) (derived_mapping.py:184). */
int fv3_sum_squares(const void* const* in, const int* in_f64, int n_arr, int64_t n, double* out, void* stream);

/* Cosine of the solar zenith angle (vcm/calc/_zenith_angle.py:54-244, derived_mapping.py:
 * 114-120) over a result of `shape`: lon / lat in degrees (or radians when *_rad != 0:
 * np.rad2deg first, as _ensure_units_of_degrees), the time-dependent terms precomputed
 * on the host per time value into `terms` (device, float64 [4][n_times]: Greenwich mean
 * sidereal time, right ascension, sin and cos of the declination), `time_stride`
 * the element strides of the time index over the result's dims.  float64 out:
 *   sin(lat r) sin(dec) + cos(lat r) cos(dec) cos((gmst + lon r) - ra),  r = pi / 180,
 * lon r / lat r and their sine / cosine in the operand's dtype (numpy's flow). */
int fv3_cos_zenith(int ndim, const int64_t* shape, fv3_strided lon, int lon_rad, fv3_strided lat, int lat_rad,
                   const int64_t* time_stride, const double* terms, int64_t n_times, double* out, void* stream);

/*
 * Host memory of the drop-in call (pure_keras.py:98-118 takes and returns host arrays;
 * csrc/host_memory.cpp).  No reference counterpart: transport only.  The
 * library page-locks only memory it allocates itself (never a caller's array).
 *
 * fv3_host_alloc: a page-locked, page-aligned host block (hipHostMalloc) owned by the
 * library, cached after fv3_host_free for reuse by a later fv3_host_alloc of the same
 * page-rounded size: the arrays a host call hands back, and staging.
 * fv3_host_arena_limit sets the cached bytes kept (default 2 GiB; beyond it blocks are
 * released); fv3_host_arena_cap the live + cached bytes held at most (default 32 GiB:
 * arrays a caller keeps stay page-locked; past the cap fv3_host_alloc returns
 * FV3_ERR_UNSUPPORTED and the caller uses pageable memory).  stats[3]: live bytes,
 * cached bytes, blocks.
 *
 * fv3_host_copy: one host <-> device copy on `stream` (kind 1: host to device, 2: device
 * to host): asynchronous DMA for arena memory; complete on return for any other host
 * memory (the runtime's pageable copy, or waited for when the buffer is page-locked by
 * someone else, e.g. torch pin_memory()).
 */
int fv3_host_alloc(size_t bytes, void** out);
int fv3_host_free(void* ptr);
int fv3_host_arena_limit(size_t cached_bytes);
int fv3_host_arena_cap(size_t total_bytes);
int fv3_host_memory_stats(uint64_t* stats);
int fv3_host_copy(void* dst, const void* src, size_t bytes, int kind, void* stream);

/* Copy `bytes` of device memory into host memory of this library (inside one
 * fv3_host_alloc block) with a kernel on `stream` that stores
 * into the host pages over PCIe, instead of a copy engine: the pipelined host call's out-copies, beside the copy engines' in-copies
 * (DESIGN.md §3.7).  FV3_ERR_UNSUPPORTED when the host range is not such memory or the
 * buffers are not 16-byte aligned (the caller copies with hipMemcpyAsync instead).  No
 * reference counterpart: a transport detail of the drop-in call (pure_keras.py:98-118). */
int fv3_copy_to_host(void* host_dst, const void* dev_src, size_t bytes, void* stream);

/* Pitched copy between host and device on `stream` (hipMemcpy2DAsync): `height` rows of
 * `width` bytes, `spitch` / `dpitch` bytes apart; kind 1 host to device, 2 device to
 * host.  A column band of a [level][column] array, one row per level: the pipelined
 * host call over column bands.  Asynchronous for arena rows (fv3_host_alloc), complete on
 * return otherwise (as fv3_host_copy).  No reference counterpart (transport). */
int fv3_copy_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height, int kind,
                void* stream);

/*
 * Launch plan: a fixed sequence of this library's launches over fixed device buffers,
 * recorded once and issued by one call per timestep (the prognostic loop applies the
 * same state buffers every step; runtime/loop.py:604-628 around
 * runtime/steppers/machine_learning.py:239-309).  Each fv3_plan_add_* takes the
 * arguments of the entry point it names, minus the stream; fv3_plan_run issues them in
 * order on `stream` and returns the first failing status.  Every buffer named must stay
 * allocated while the plan is used; the dense model must outlive the plan.
 */
typedef struct fv3_plan fv3_plan;
int fv3_plan_create(fv3_plan** out);
int fv3_plan_destroy(fv3_plan* plan);
int fv3_plan_size(const fv3_plan* plan);
int fv3_plan_run(const fv3_plan* plan, void* stream);
/* fv3_dense_forward_f64in (inputs_f64 != 0) or fv3_dense_forward_ex at `precision` */
int fv3_plan_add_dense_forward(fv3_plan* plan, const fv3_dense_model* model, const void* const* inputs,
                               const fv3_layout* in_l, float* const* outputs, const fv3_layout* out_l, int64_t ncol,
                               int precision, int inputs_f64);
int fv3_plan_add_ml_epilogue(fv3_plan* plan, const fv3_epilogue_io* io, fv3_layout lay, int64_t ncol, int nz,
                             int state_f64, double dt, int mse_conserving, int hydrostatic, int flags);
int fv3_plan_add_area_weighted_sums_f64(fv3_plan* plan, const double* const* diags, int n_diag, const double* area,
                                        int64_t n, double* out);
int fv3_plan_add_area_weighted_row_sums_f64(fv3_plan* plan, const double* const* diags, int n_diag,
                                            const double* area, int64_t nrows, int row_len, double* partial,
                                            int64_t partial_ld);
int fv3_plan_add_level_sums_u8(fv3_plan* plan, const unsigned char* x, fv3_layout x_l, int64_t ncol, int nz,
                               double* out);
int fv3_plan_add_fold_rows(fv3_plan* plan, const double* rows, int64_t nrows, int width, double* out);
int fv3_plan_add_step_partials_f64(fv3_plan* plan, const double* const* diags, int n_diag, const double* area,
                                   int64_t nrows, int row_len, double* partial, int64_t partial_ld,
                                   const unsigned char* limiter, fv3_layout lim_l, int64_t ncol, int nz,
                                   double* level_out);
int fv3_plan_add_fold_rows_repeat(fv3_plan* plan, const double* rows, int64_t nrows, int width, int times,
                                  double* rep, double* out);
/* device-to-device copy of `bytes` */
int fv3_plan_add_copy(fv3_plan* plan, void* dst, const void* src, size_t bytes);
/* `times` back-to-back copies of `bytes` (a multiple of 4) of src into dst, one launch */
int fv3_plan_add_repeat(fv3_plan* plan, void* dst, const void* src, size_t bytes, int times);

#ifdef __cplusplus
}
#endif
#endif /* FV3NET_AMD_H */
