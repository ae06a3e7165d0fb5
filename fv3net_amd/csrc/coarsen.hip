// fv3net_amd — fused pressure-level coarse-graining (BASELINE config #3) on gfx950.
//
// Replaces, for the masked area-weighted variables of coarsen_restarts_on_pressure
// (external/vcm/vcm/cubedsphere/coarsen_restarts.py:411-516, 840-887):
//   regrid_to_area_weighted_pressure   regridz.py:25-55
//     delp_c = weighted_block_average(delp, area, f)       coarsen.py:183-218
//     _regrid_given_delp                                   regridz.py:115-147
//       block_upsample_like(delp_c)                        coarsen.py:900-938
//       pressure_at_interface (phalf = cumsum([300, delp])) vertically_dependent.py:41-66
//       regrid_vertical -> mappm(p_fine, f, p_coarse, iv, kord)  regridz.py:164-279
//     _mask_weights: area where phalf_c[k+1] < phalf_f[-1]  regridz.py:150-161
//   weighted_block_average(f_regrid, masked_area, f)        coarsen.py:183-218
// in ONE kernel and one pass over each input field.
//
// Mapping: a block is one coarse row segment: f waves, wave dy = fine row dy of the
// coarse row, lane = one of 64 consecutive fine columns (C = 64 / f coarse cells x f),
// so every per-level load is one coalesced 256 B row.  Pass 1 streams delp once:
// each lane keeps its fine phalf cumsum, delp*area is combined over the block per
// level (row sums by cross-lane shuffles, rows through LDS) into delp_c and the
// coarse phalf.  Per field: every lane runs the output-driven streaming mappm
// (PpmCursor, mappm_core.h) on its column with p_in rebuilt from delp; after each
// output level the wave is reconverged, so the masked products are row-summed by
// shuffles right away and only [level][row][cell] partials go to LDS.
//
// Arithmetic follows the reference's dtype flow exactly (oracle/coarsen.py): delp
// products, sums, delp_c and both cumsums in delp's dtype DT (float64 for restart
// data), area and masked-field sums in float32, and every f x f block sum in
// numpy's order for a C-order (.., Y, f, X, f) reshape summed over the two f axes:
// each x-row reduced on its own (sequentially for f < 8, numpy's 8-way pairwise
// kernel for f = 8, which is exactly an xor-shuffle tree over 8 aligned lanes), rows
// then added in y order; NaN terms count as 0 (xarray's NaN-skipping sum).
// Deterministic run to run.
// Roofline: HBM-bound, (79 delp + 79*n_fields + 1 area) * 4 B per fine column read
// once (+ ~(1 + n_fields) * 79 * 4 / f^2 written); delp is re-read per field (L2/MALL).
// Measured VALU-bound like the standalone mappm (the PPM arithmetic with its IEEE
// divisions dominates).
#define FV3_HD __host__ __device__
#include <cstdlib>
#include <type_traits>

#include "blocks.h"
#include "common.h"
#include "mappm_core.h"
#include "mappm_multi.h"

namespace fv3 {
namespace FV3_ARITH_NS {  // kernels named fv3::exact::... / fv3::fast::... in traces
namespace {

constexpr int kMaxLev = 128;
constexpr int kMaxFields = 32;  // field/output pointers travel in the kernel arguments

template <typename DT>
struct CoarsenArgs {
    const DT* delp;
    const float* area;
    const float* fields[kMaxFields];
    float* out[kMaxFields];
    float* delp_out;
    double* delp_out64;  // the coarse delp in float64 (restart precision), or NULL
    int n_fields, ntile, km, ny, nx, f, iv, kord;
    double ptop;
    float* scratch;   // [km][gridDim * blockDim]: each lane's remapped column (input-driven path), or NULL
};

constexpr int kChunk = 16;  // delp*area levels staged per pass-1 round

// the one-field cells kernel's loads as buffer operations at 32-bit offsets (1, default)
// or through 64-bit addresses (0, A/B); the host checks every tile's array spans < 4 GiB.
// One field 0.558 -> 0.546 ms; the two-field pass measured 1.542 -> 1.550 ms with them
// (profiles/r06zr_coarsen_ops_ab.log), so it keeps its addresses (coarsen_bufload<NF>)
#ifndef FV3_COARSEN_BUFLOAD
#define FV3_COARSEN_BUFLOAD 1
#endif
template <int NF>
constexpr bool coarsen_bufload() { return FV3_COARSEN_BUFLOAD && NF == 1; }

// the same row sum across the f lanes of this lane's cell (every lane of the cell
// gets the identical value): f == 8 pairwise == xor tree over aligned 8-lane groups
template <typename T>
__device__ __forceinline__ T row_sum(T v, int f, int base)
{
    if (f == 8) {
        v = v + __shfl_xor(v, 1, 64);
        v = v + __shfl_xor(v, 2, 64);
        v = v + __shfl_xor(v, 4, 64);
        return v;
    }
    T s = __shfl(v, base, 64);
    for (int i = 1; i < f; ++i) s = s + __shfl(v, base + i, 64);
    return s;
}

// fine column of this lane: p_in streamed from a running cumsum of delp (in DT)
template <typename DT>
struct FineCol {
    const float* q;   // field at level 0 of this column
    const DT* dp;     // delp at level 0 of this column
    int64_t plane;    // ny*nx
    const DT* pc;     // coarse phalf[k], k = 0..km (LDS)
    DT ptop, pbot, run;
    int next;         // next fine interface index (0-based) the running sum will produce
    int km, kn;
    const DT* dnx;    // &delp[next]
    DT dl;            // delp[next], loaded one call ahead (its latency overlaps a layer)
    __device__ __forceinline__ void start()
    {
        run = ptop;
        next = 0;
        dnx = dp;
        dl = dp[0];
    }
    __device__ __forceinline__ float q1(int k) const { return q[(int64_t)(k - 1) * plane]; }
    __device__ __forceinline__ float pe1(int k)
    {
        // reference: phalf = cumsum([ptop, delp]) in delp's dtype, cast to float32 by f2py
        if (k == 1) return (float)ptop;
        if (k == km + 1) return (float)pbot;
        while (next < k - 1) {  // interface k-1 (0-based) = ptop + sum delp[0..k-2]
            run = run + dl;
            ++next;
            // unconditional (the last level re-read past the end): no phi on the loaded
            // value, so its wait stays at the next call's use instead of right here
            if (next < km) dnx += plane;
            dl = *dnx;
        }
        return (float)run;
    }
    __device__ __forceinline__ float pe2(int k) const { return (float)pc[k - 1]; }
    __device__ __forceinline__ void emit(int k, float v)
    {
        if (out) out[(int64_t)(k - 1) * ostride] = v;
    }
    __device__ __forceinline__ float next_edge(int k) const { return (k + 1 <= kn + 1) ? pe2(k + 1) : 0.0f; }
    float* out = nullptr;  // this lane's remapped column in the scratch (stride ostride), or NULL
    int64_t ostride = 0;
};

// SCR: the input-driven remap through the per-lane scratch (default); !SCR: the
// scratch-free output-driven cursor.  Separate builds, so the default's register
// allocation does not carry the cursor's.
template <typename DT, bool SCR>
__global__ __launch_bounds__(512) void regrid_coarsen_kernel(CoarsenArgs<DT> a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int f = a.f, km = a.km;
    const int C = 64 / f;                 // coarse cells per wave
    const int lane = threadIdx.x & 63;
    const int dy = threadIdx.x >> 6;      // fine row within the coarse row
    const int nxc = a.nx / f, nyc = a.ny / f;
    const int nseg = (nxc + C - 1) / C;
    int64_t bi = blockIdx.x;
    const int seg = (int)(bi % nseg);
    bi /= nseg;
    const int Y = (int)(bi % nyc);
    const int tile = (int)(bi / nyc);
    const int lc = lane / f;              // cell of this lane (>= C: spare lane)
    const int cell = min(lc, C - 1);
    const int dx = lane - lc * f;
    const int X = seg * C + cell;
    const bool active = lc < C && X < nxc;
    const int base = cell * f;            // first lane of this cell
    const int64_t plane = (int64_t)a.ny * a.nx;
    const int64_t fine = (int64_t)(Y * f + dy) * a.nx + (int64_t)min(X, nxc - 1) * f + (active ? dx : 0);
    const int64_t cplane = (int64_t)nyc * nxc;
    const int64_t crow = (int64_t)Y * nxc + (int64_t)seg * C;  // first coarse cell of this block

    DT* pc = reinterpret_cast<DT*>(smem);            // [C][km+1] coarse phalf
    DT* lpb = pc + C * (km + 1);                     // [f][64] fine surface phalf
    float* lar = reinterpret_cast<float*>(lpb + f * 64);  // [f][64] fine area
    float* asum = lar + f * 64;                      // [C]
    char* rsb = reinterpret_cast<char*>(asum + 64);  // partials: [km][f][C] f32, or [kChunk][f][C] DT
    float* rs = reinterpret_cast<float*>(rsb);
    DT* rsd = reinterpret_cast<DT*>(rsb);

    // ---- pass 1: fine phalf (per lane) and area-weighted coarse delp / phalf ----
    const float area = active ? a.area[(int64_t)tile * plane + fine] : 0.0f;
    lar[dy * 64 + lane] = area;
    __syncthreads();
    if ((int)threadIdx.x < C)  // weights.coarsen().sum(): float32 (area's dtype)
        asum[threadIdx.x] = block_sum<float>(
            f, [&](int j) { return nan0(lar[(j / f) * 64 + (int)threadIdx.x * f + j % f]); });
    const DT* dp = a.delp + (int64_t)tile * km * plane + fine;
    const DT ptop = (DT)a.ptop;
    DT run = ptop;  // fine phalf = cumsum([ptop, delp]) (vertically_dependent.py:62-63)
    for (int k0 = 0; k0 < km; k0 += kChunk) {
        const int nk = min(kChunk, km - k0);
        for (int kk = 0; kk < nk; ++kk) {
            const DT d = active ? dp[(int64_t)(k0 + kk) * plane] : (DT)0;
            run = run + d;
            const DT r = row_sum<DT>(nan0(d * (DT)area), f, base);  // (delp * area) in delp's dtype
            if (active && dx == 0) rsd[(kk * f + dy) * C + cell] = r;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nk * C; i += blockDim.x) {
            const int kk = i / C, c = i - (i / C) * C;
            if (seg * C + c < nxc) {
                DT acc = rsd[(kk * f) * C + c];
                for (int r = 1; r < f; ++r) acc = acc + rsd[(kk * f + r) * C + c];
                const DT dc = acc / (DT)asum[c];  // weighted_block_average (coarsen.py:213-215)
                pc[c * (km + 1) + k0 + kk + 1] = dc;
                if (a.delp_out) a.delp_out[((int64_t)tile * km + k0 + kk) * cplane + crow + c] = (float)dc;
                if (a.delp_out64) a.delp_out64[((int64_t)tile * km + k0 + kk) * cplane + crow + c] = (double)dc;
            }
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < C) {  // coarse phalf = cumsum([ptop, delp_c]), sequential like np.cumsum
        DT* p = pc + threadIdx.x * (km + 1);
        p[0] = ptop;
        for (int k = 0; k < km; ++k) p[k + 1] = p[k] + p[k + 1];
    }
    const DT pbot = run;  // phalf_fine[-1] of this fine column
    lpb[dy * 64 + lane] = pbot;
    __syncthreads();

    // ---- per field: remap every fine column level by level, masked area-weighted mean ----
    const DT* pcc = pc + cell * (km + 1);
    for (int v = 0; v < a.n_fields; ++v) {
        FineCol<DT> col;
        col.q = a.fields[v] + (int64_t)tile * km * plane + fine;
        col.dp = dp;
        col.plane = plane;
        col.pc = pcc;
        col.ptop = ptop;
        col.pbot = pbot;
        col.km = km;
        col.start();
        col.kn = km;
        // _mask_weights (regridz.py:150-161): area where phalf_c_on_f[k+1] < phalf_f[-1]
        // (compared in delp's dtype); the masked area stays float32 (coarsen.py:213-215)
        auto level_sum = [&](int k, float q2) {
            const float w = (pcc[k + 1] < pbot) ? area : 0.0f;
            const float r = row_sum<float>(nan0(q2 * w), f, base);
            if (active && dx == 0) rs[(k * f + dy) * C + cell] = r;
        };
#ifdef FV3_EXP_NOPPM  // experiment only (results invalid): no remap, the field's own level
        for (int k = 0; k < km; ++k) level_sum(k, col.q1(k + 1));
#else
        if constexpr (SCR) {
            // input-driven remap (the streaming mappm, uniform over input layers: every
            // lane ingests layer L together) into this lane's scratch column, then the
            // per-level masked row sums read it back (each lane only its own values)
            const int64_t sstride = (int64_t)gridDim.x * blockDim.x;
            float* const mine = a.scratch + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
            col.out = mine;
            col.ostride = sstride;
            mappm_ppm_column(col, km, km, a.iv, a.kord);
            for (int k = 0; k < km; ++k) level_sum(k, mine[(int64_t)k * sstride]);
        } else {
            // output-driven cursor: no scratch, but the per-lane layer loops diverge
            PpmCursor<FineCol<DT>> cur(col, km, km, a.iv, a.kord);
            for (int k = 0; k < km; ++k) level_sum(k, cur.next());
        }
#endif
        __syncthreads();
        float* o = a.out[v] + (int64_t)tile * km * cplane + crow;
        for (int i = threadIdx.x; i < km * C; i += blockDim.x) {
            const int k = i / C, c = i - (i / C) * C;
            if (seg * C + c < nxc) {
                float num = rs[(k * f) * C + c];
                for (int r = 1; r < f; ++r) num = num + rs[(k * f + r) * C + c];
                const DT pk = pc[c * (km + 1) + k + 1];
                const float den = block_sum<float>(f, [&](int j) {
                    const int l = (j / f) * 64 + c * f + j % f;
                    return (pk < lpb[l]) ? nan0(lar[l]) : 0.0f;
                });
                o[(int64_t)k * cplane + c] = num / den;
            }
        }
        __syncthreads();
    }
}

// ====================================================================================
// Cell-per-wave mapping (default for f >= 2): one 64-lane block holds G = 64 / f^2 whole
// coarse cells (f = 8: one cell, lane = dy * 8 + dx), so every f x f block sum is a
// wave-local reduction and the coarse pressure edges of a cell (its remap targets)
// live in LDS per wave.  No cross-wave barrier anywhere.
//   pass 1: delp streamed once; delp*area of CH levels staged in LDS, then the
//           numpy-order cell sums (rows, then rows in y order) of all CH levels at
//           once (lane = row of (cell, level)), coarse delp and its cumsum;
//           the masked-area denominators of every level (field-independent) once.
//   per field: each lane runs the streaming mappm (remap_layer_fast) on its column;
//           emit(k) applies the level's mask weight and drops nan0(q * w) into a
//           per-wave ring of ring_levels(NF) levels; after every input layer, once all lanes
//           have emitted kcons + NB levels, those NB levels are summed per cell in
//           numpy order (lane = row of (cell, level)) and written.  A lane that runs
//           ring_levels(NF) levels ahead of the slowest (e.g. a much shallower column in a
//           steep cell) writes from then on into a per-lane global column instead
//           (sticky, recorded in LDS); the sums read those entries from there.
// Same arithmetic and order as regrid_coarsen_kernel, so the same bits.
// ====================================================================================

// output levels held per wave and field: 16 for one field; 12 for the two-field pass,
// whose 16-level rings (8.3 KB of LDS per one-wave block) held it to 15 blocks per CU
// against the 16 its registers allow (4 fields 2.29 -> 2.11 ms; 1 field with 12 levels
// 0.757 -> 0.761 ms, so it keeps 16; profiles/r05zzh_coarsen_ring_ab.log).  A lane
// running that many levels ahead of its cell's slowest writes to its global column.
constexpr int ring_levels(int nf) { return nf >= 2 ? 12 : 16; }
// levels per cell-sum batch for a compile-time factor FF (G * CH * FF <= 64), 0: run time
constexpr int cells_batch(int ff) { return ff ? (64 / ((64 / (ff * ff)) * ff) < 8 ? 64 / ((64 / (ff * ff)) * ff) : 8) : 0; }
constexpr int kRingLd = 65;   // ring row stride (floats): rows of one cell read bank-free

typedef __amdgpu_buffer_rsrc_t MRsrc;
__device__ __forceinline__ MRsrc mrsrc(const void* p)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0xffffffffu, 0x00020000);
}
template <typename T>
__device__ __forceinline__ T bload(MRsrc r, uint32_t voff, uint32_t soff)
{
    if constexpr (sizeof(T) == 8)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
    else
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}

// per-level cell sums in numpy's order for nb consecutive levels of G cells:
// val(g, kk, j) = element j = dy * f + dx of cell g at level kk; res(g, kk, sum).
// NBM > 0: a compile-time bound on nb (the layout of NBM levels, levels >= nb skipped),
// so no index needs a division by the run-time nb (a ~10-instruction sequence each);
// G * NBM * f <= 64.  Same sums in the same order either way.
template <typename T, int NBM = 0, typename Val, typename Res>
__device__ __forceinline__ void cell_sums(int lane, int G, int f, int nb, T* rowbuf, Val val, Res res)
{
    const int nbl = NBM ? NBM : nb;  // levels in the row layout
    const int nrow = G * nbl * f;
    for (int i = lane; i < nrow; i += 64) {
        const int dy = i % f, kk = (i / f) % nbl, g = i / (f * nbl);
        if (NBM && kk >= nb) continue;
        const int b = dy * f;
        T r;
        if (f == 8) {
            r = ((val(g, kk, b) + val(g, kk, b + 1)) + (val(g, kk, b + 2) + val(g, kk, b + 3))) +
                ((val(g, kk, b + 4) + val(g, kk, b + 5)) + (val(g, kk, b + 6) + val(g, kk, b + 7)));
        } else {
            r = val(g, kk, b);
            for (int c = 1; c < f; ++c) r = r + val(g, kk, b + c);
        }
        rowbuf[i] = r;
    }
    __syncthreads();
    for (int i = lane; i < G * nbl; i += 64) {
        if (NBM && i % nbl >= nb) continue;
        const T* rr = rowbuf + i * f;  // rows of (cell, level) i = g * nbl + kk
        T acc = rr[0];
        for (int dy = 1; dy < f; ++dy) acc = acc + rr[dy];
        res(i / nbl, i % nbl, acc);
    }
    __syncthreads();
}

template <typename DT, int FF, int NF>
struct CellCtx {
    int lane, f, nb, km, tile, Y, X0, nxc;
    int64_t cplane;
    const DT* pc;       // [G][km+1] coarse phalf
    const float* den;   // [G][km] masked-area sums
    float* ring;        // [NF][ring_levels(NF)][kRingLd]
    const int* ovf;     // [NF][64] first level a lane wrote to its global column (km: none)
    float* rowbuf;      // [64]
    float* scr;         // global columns [NF][km][gridDim * 64], or NULL
    int64_t sstride;    // gridDim * 64
    float* out[NF];     // the fields' outputs

    // sum and write levels [k0, k0 + nb) of every cell of the block, for every field;
    // bit fi of ovm: some lane wrote field fi to its global column (else the ring only)
    __device__ void consume(int k0, int nb_, unsigned ovm) const
    {
        const int gl0 = blockIdx.x * 64;
        const int f = FF ? FF : this->f, ff = f * f, G = 64 / ff;
        for (int fi = 0; fi < NF; ++fi) {
            const float* rg = ring + fi * (ring_levels(NF) * kRingLd);
            const int* ov = ovf + fi * 64;
            const float* sc = scr + (int64_t)fi * km * sstride;
            float* o = out[fi];
            const bool any = (ovm >> fi) & 1u;
            cell_sums<float, cells_batch(FF)>(
                lane, G, f, nb_, rowbuf,
                [&](int g, int kk, int j) {
                    const int l = g * ff + j, k = k0 + kk;
                    if (any && k >= ov[l]) return sc[(int64_t)k * sstride + gl0 + l];
                    return rg[(k % ring_levels(NF)) * kRingLd + l];
                },
                [&](int g, int kk, float num) {
                    const int k = k0 + kk, X = X0 + g;
                    if (X < nxc) o[((int64_t)tile * km + k) * cplane + (int64_t)Y * nxc + X] = num / den[g * km + k];
                });
        }
    }
};

// NF fields of one fine column, for mappm_ppm_columns<NF>: pressure edges from the
// running delp sum (FineCol), q from the NF field arrays at the same element offset
template <typename DT, int FF, int NF>
struct CellCol : FineCol<DT> {
    const CellCtx<DT, FF, NF>* ctx;
    const float* const* fields;  // NF field bases (level 0 of tile 0)
    int64_t off;                 // this lane's element offset (tile, level 0, fine column)
    float area;
    bool active;
    int nemit;   // output levels emitted so far by this lane (every field alike)
    int kcons;   // levels [0, kcons) summed and written (wave-uniform)
    int ovf_k[NF];  // first level this lane sent to its global column (km: none)
    int lim[NF];    // min(ovf_k, kcons + ring_levels): levels from here go to the global column
    int* ovf_lds;
    float* mine;  // this lane's global column (field 0, level 0)
    // coarsen_bufload<NF>: loads as buffer operations: resource over this tile's array
    // (SGPRs), the lane's byte offset (VGPR), the level's byte offset (SGPR): no per-load
    // 64-bit address
    MRsrc rq[NF], rdp;
    uint32_t vq, vdp;  // lane byte offsets in a field / in delp
    uint32_t lbq, lbdp;  // level strides in bytes
    __device__ __forceinline__ float q1(int f, int k) const
    {
        if constexpr (coarsen_bufload<NF>())
            return bload<float>(rq[f], vq, (uint32_t)(k - 1) * lbq);
        else
            return fields[f][off + (int64_t)(k - 1) * this->plane];
    }
    __device__ __forceinline__ float pe1(int k)
    {
        if constexpr (!coarsen_bufload<NF>()) return FineCol<DT>::pe1(k);
        // FineCol::pe1 with the next level read at a uniform level offset
        if (k == 1) return (float)this->ptop;
        if (k == this->km + 1) return (float)this->pbot;
        while (this->next < k - 1) {
            this->run = this->run + this->dl;
            ++this->next;
            const int lv = __builtin_amdgcn_readfirstlane(min(this->next, this->km - 1));  // uniform
            this->dl = bload<DT>(rdp, vdp, (uint32_t)lv * lbdp);
        }
        return (float)this->run;
    }
    // bit fi: some lane has sent field fi to its global column
    __device__ __forceinline__ unsigned ovf_mask() const
    {
        unsigned m = 0;
        for (int fi = 0; fi < NF; ++fi)
            if (__any(ovf_k[fi] < ctx->km)) m |= 1u << fi;
        return m;
    }

    __device__ __forceinline__ void emit(int fi, int k, float v)
    {
        const int k0 = k - 1;
        nemit = k;
        if (!active) return;
        // _mask_weights (regridz.py:150-161): area where phalf_c[k0+1] < phalf_f[-1]
        const float w = (this->pc[k] < this->pbot) ? area : 0.0f;
        const float x = nan0(v * w);
        if (k0 >= lim[fi]) {  // = k0 >= ovf_k[fi] || k0 - kcons >= ring_levels(NF)
            if (ovf_k[fi] > k0) {
                ovf_k[fi] = k0;
                lim[fi] = min(k0, kcons + ring_levels(NF));
                ovf_lds[fi * 64 + ctx->lane] = k0;
            }
            mine[((int64_t)fi * ctx->km + k0) * ctx->sstride] = x;
        } else {
            ctx->ring[fi * (ring_levels(NF) * kRingLd) + ((unsigned)k0 % (unsigned)ring_levels(NF)) * kRingLd + ctx->lane] = x;
        }
    }

    // after every input layer: sum the next NB levels once every lane has emitted them
    __device__ __forceinline__ void layer_done()
    {
        const int nb = FF ? std::min(8, 64 / ((64 / (FF * FF)) * FF)) : ctx->nb;
        if (__all(nemit >= kcons + nb)) {
            __syncthreads();
            ctx->consume(kcons, nb, ovf_mask());
            kcons += nb;
            for (int fi = 0; fi < NF; ++fi) lim[fi] = min(ovf_k[fi], kcons + ring_levels(NF));
        }
    }
};

// the one-field pass's PPM window: register rings (1, mappm_core.h RING, the default on
// the fast arithmetic) or shifting (0, the exact kernels).  Before the buffer loads and
// the compile-time batch freed registers, the rings spilled at 6 waves per SIMD (34 VGPRs
// against 7; 21 with the layer hook once per ring group) and lost, 0.577 -> 0.662 / 0.653
// ms (at 5 waves: 0.612 -> 0.599, still behind 6), profiles/r06zi_ring_ab.log,
// r06zo_coarsen_ring_ab.log; after them (10 VGPRs spilled) they win, 0.546 -> 0.534 ms
// (profiles/r06zr_coarsen_ops_ab.log).  tools/ variant builds set it for A/B.
#ifndef FV3_COARSEN_RING
#ifdef FV3_FAST_ARITH
#define FV3_COARSEN_RING 1
#else
#define FV3_COARSEN_RING 0
#endif
#endif
// pass 1's delp prefetch distance in 8-level chunks (1 default; 2 for A/B)
#ifndef FV3_COARSEN_P1_DEPTH
#define FV3_COARSEN_P1_DEPTH 1
#endif

// one pass of the streaming remap for fields [v0, v0 + NF), then the last levels' sums
template <int NF, typename DT, int FF>
__device__ __forceinline__ void cells_field_group(const CoarsenArgs<DT>& a, int v0, int lane, int f, int nb, int tile,
                                                  int Y, int X0, int nxc, int64_t cplane, const DT* pc,
                                                  const DT* pcg, const float* den, float* ring, int* ovf,
                                                  float* rowf, int64_t off, const DT* dp, int64_t plane, DT ptop,
                                                  DT pbot, float area, bool active, int iv, int kord)
{
    const int km = a.km;
    const int64_t sstride = (int64_t)gridDim.x * 64;
    for (int fi = 0; fi < NF; ++fi) ovf[fi * 64 + lane] = km;
    __syncthreads();
    CellCtx<DT, FF, NF> ctx{lane, f, nb, km, tile, Y, X0, nxc, cplane, pc, den, ring, ovf, rowf, a.scratch, sstride, {}};
    for (int fi = 0; fi < NF; ++fi) ctx.out[fi] = a.out[v0 + fi];
    CellCol<DT, FF, NF> col;
    col.q = nullptr;
    col.dp = dp;
    col.plane = plane;
    col.pc = pcg;
    col.ptop = ptop;
    col.pbot = pbot;
    col.km = km;
    col.kn = km;
    col.start();
    col.ctx = &ctx;
    col.fields = a.fields + v0;
    col.off = off;
    col.area = area;
    col.active = active;
    col.nemit = 0;
    col.kcons = 0;
    for (int fi = 0; fi < NF; ++fi) {
        col.ovf_k[fi] = km;
        col.lim[fi] = min(km, ring_levels(NF));
    }
    col.ovf_lds = ovf;
    col.mine = a.scratch + (int64_t)blockIdx.x * 64 + lane;
    if constexpr (coarsen_bufload<NF>()) {
        const int64_t tbase = (int64_t)tile * km * plane;  // this tile's level 0
        for (int fi = 0; fi < NF; ++fi) col.rq[fi] = mrsrc(a.fields[v0 + fi] + tbase);
        col.rdp = mrsrc(a.delp + tbase);
        col.vq = (uint32_t)(off - tbase) * (uint32_t)sizeof(float);
        col.vdp = (uint32_t)(off - tbase) * (uint32_t)sizeof(DT);
        col.lbq = (uint32_t)plane * (uint32_t)sizeof(float);
        col.lbdp = (uint32_t)plane * (uint32_t)sizeof(DT);
        col.dl = bload<DT>(col.rdp, col.vdp, 0);  // start(): delp[0]
    }
    if constexpr (NF == 1) {
        FirstField<CellCol<DT, FF, NF>> one{col};
        mappm_ppm_column<FirstField<CellCol<DT, FF, NF>>, true, false, (bool)FV3_COARSEN_RING>(one, km, km, iv, kord);
    } else {
        mappm_ppm_columns<NF>(col, km, km, iv, kord);
    }
    __syncthreads();
    const unsigned ovm = col.ovf_mask();
    for (int k0 = col.kcons; k0 < km; k0 += nb) ctx.consume(k0, min(nb, km - k0), ovm);
}

// FF: the coarsening factor at compile time (8, config #3: all index arithmetic folds),
// or 0 (runtime a.f)
// WPE: the waves per SIMD its registers are allocated for (the one-field pass on float32
// delp at 6: 80 VGPRs against 91, a 48-byte spill, see the launch below)
// K1: kord 1 and iv 1 (the reference's default, regridz.py:25) at compile time
template <typename DT, int FF, int NF, int WPE, bool K1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void
regrid_coarsen_cells_kernel(CoarsenArgs<DT> a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int f = FF ? FF : a.f, km = a.km, ff = f * f;
    const int G = 64 / ff;
    const int CH = min(8, 64 / (G * f));  // levels per cell-sum batch (G * CH * f <= 64)
    const int lane = threadIdx.x;
    const int g = lane / ff, j = lane - (lane / ff) * ff;
    const int dy = j / f, dx = j - (j / f) * f;
    const int nxc = a.nx / f, nyc = a.ny / f;
    const int ngrp = (nxc + G - 1) / G;
    // neighbouring cells share delp / field cache lines (f = 8: 32 B of each 128 B row
    // line): give them to the same XCD
    int64_t bi = xcd_swizzle(blockIdx.x, gridDim.x);
    const int grp = (int)(bi % ngrp);
    bi /= ngrp;
    const int Y = (int)(bi % nyc);
    const int tile = (int)(bi / nyc);
    const int X0 = grp * G;
    const int X = X0 + min(g, G - 1);
    const bool active = g < G && X < nxc;
    const int64_t plane = (int64_t)a.ny * a.nx;
    const int64_t fine = (int64_t)(Y * f + (active ? dy : 0)) * a.nx + (int64_t)min(X, nxc - 1) * f + (active ? dx : 0);
    const int64_t cplane = (int64_t)nyc * nxc;
    const int gg = min(g, G - 1);

    DT* pc = reinterpret_cast<DT*>(smem);                   // [G][km+1]
    DT* lpb = pc + G * (km + 1);                              // [64] fine surface phalf
    DT* buf = lpb + 64;                                       // [CH][kRingLd] pass-1 staging ...
    float* ring = reinterpret_cast<float*>(buf);              // ... aliased by the rings [NF][ring_levels(NF)][kRingLd]
    char* after = reinterpret_cast<char*>(buf) + std::max(sizeof(DT) * CH * kRingLd, sizeof(float) * NF * ring_levels(NF) * kRingLd);
    DT* rowd = reinterpret_cast<DT*>(after);                  // [64] row sums (DT)
    float* rowf = reinterpret_cast<float*>(rowd + 64);        // [64] row sums (f32)
    float* lar = rowf + 64;                                   // [64] fine area
    float* asum = lar + 64;                                   // [64]
    float* den = asum + 64;                                   // [G][km]
    int* ovf = reinterpret_cast<int*>(den + G * km);          // [NF][64]

    // ---- pass 1: fine phalf (per lane), area-weighted coarse delp and phalf ----
    const float area = active ? a.area[(int64_t)tile * plane + fine] : 0.0f;
    lar[lane] = nan0(area);  // read only as nan0(area): the block sums and the denominators
    __syncthreads();
    if (lane < G)  // weights.coarsen().sum(): float32 (area's dtype)
        asum[lane] = block_sum<float>(f, [&](int jj) { return lar[lane * ff + jj]; });
    const DT* dp = a.delp + (int64_t)tile * km * plane + fine;
    const DT ptop = (DT)a.ptop;
    DT run = ptop;  // fine phalf = cumsum([ptop, delp]) (vertically_dependent.py:62-63)
    DT crun = ptop;  // lanes < G: coarse phalf = cumsum([ptop, delp_c]), sequential like np.cumsum
    if (lane < G) pc[lane * (km + 1)] = ptop;
    // the chunk after the current one (FV3_COARSEN_P1_DEPTH 2: the one after that) is
    // loaded before the current one is reduced
    constexpr int kCH = 8;
    const MRsrc rdp = mrsrc(a.delp + (int64_t)tile * km * plane);
    const uint32_t vdp = (uint32_t)(fine * (int64_t)sizeof(DT)), lbdp = (uint32_t)(plane * (int64_t)sizeof(DT));
    auto load_chunk = [&](DT (&dst)[kCH], int k0) {
#pragma unroll
        for (int kk = 0; kk < kCH; ++kk) {
            if (kk < CH && k0 + kk < km) {
                if constexpr (coarsen_bufload<NF>())
                    dst[kk] = bload<DT>(rdp, vdp, (uint32_t)(k0 + kk) * lbdp);
                else
                    dst[kk] = dp[(int64_t)(k0 + kk) * plane];
            }
        }
    };
    auto chunk = [&](const DT (&dcur)[kCH], int k0) {
        const int nk = min(CH, km - k0);
#pragma unroll
        for (int kk = 0; kk < kCH; ++kk) {
            if (kk < nk) {
                const DT d = active ? dcur[kk] : (DT)0;
                run = run + d;
                buf[kk * kRingLd + lane] = nan0(d * (DT)area);  // (delp * area) in delp's dtype
            }
        }
        __syncthreads();
        cell_sums<DT, cells_batch(FF)>(
            lane, G, f, nk, rowd, [&](int gi, int kk, int jj) { return buf[kk * kRingLd + gi * ff + jj]; },
            [&](int gi, int kk, DT acc) {
                const int k = k0 + kk, Xg = X0 + gi;
                const DT dc = acc / (DT)asum[gi];  // weighted_block_average (coarsen.py:213-215)
                pc[gi * (km + 1) + k + 1] = dc;
                if (Xg < nxc) {
                    const int64_t o = ((int64_t)tile * km + k) * cplane + (int64_t)Y * nxc + Xg;
                    if (a.delp_out) a.delp_out[o] = (float)dc;
                    if (a.delp_out64) a.delp_out64[o] = (double)dc;
                }
            });
        if (lane < G) {
            DT* p = pc + lane * (km + 1) + k0 + 1;
            for (int kk = 0; kk < nk; ++kk) {
                crun = crun + p[kk];
                p[kk] = crun;
            }
        }
    };
#if FV3_COARSEN_P1_DEPTH == 2
    // three register chunks in rotating roles (the loop unrolled by three, so no chunk is
    // copied: a copy waits for its loads at the end of the chunk before)
    DT d0[kCH], d1[kCH], d2[kCH];
    load_chunk(d0, 0);
    if (CH < km) load_chunk(d1, CH);
    for (int k0 = 0; k0 < km; k0 += 3 * CH) {
        if (k0 + 2 * CH < km) load_chunk(d2, k0 + 2 * CH);
        chunk(d0, k0);
        if (k0 + CH >= km) break;
        if (k0 + 3 * CH < km) load_chunk(d0, k0 + 3 * CH);
        chunk(d1, k0 + CH);
        if (k0 + 2 * CH >= km) break;
        if (k0 + 4 * CH < km) load_chunk(d1, k0 + 4 * CH);
        chunk(d2, k0 + 2 * CH);
    }
#else
    DT dcur[kCH], dnxt[kCH];
    load_chunk(dcur, 0);
    for (int k0 = 0; k0 < km; k0 += CH) {
        if (k0 + CH < km) load_chunk(dnxt, k0 + CH);
        chunk(dcur, k0);
#pragma unroll
        for (int kk = 0; kk < kCH; ++kk) dcur[kk] = dnxt[kk];
    }
#endif
    const DT pbot = run;  // phalf_fine[-1] of this fine column
    lpb[lane] = pbot;
    __syncthreads();
    // masked-area denominators of every level (the same for every field)
    for (int k0 = 0; k0 < km; k0 += CH) {
        const int nk = min(CH, km - k0);
        cell_sums<float, cells_batch(FF)>(
            lane, G, f, nk, rowf,
            [&](int gi, int kk, int jj) {
                const int l = gi * ff + jj;
                return (pc[gi * (km + 1) + k0 + kk + 1] < lpb[l]) ? lar[l] : 0.0f;
            },
            [&](int gi, int kk, float s) { den[gi * km + k0 + kk] = s; });
    }

    // ---- per group of NF fields: stream the remap, sum finished levels per cell ----
    const int64_t off = (int64_t)tile * km * plane + fine;
    const int iv = K1 ? 1 : a.iv, kord = K1 ? 1 : a.kord;
    int v0 = 0;
    for (; v0 + NF <= a.n_fields; v0 += NF)
        cells_field_group<NF, DT, FF>(a, v0, lane, f, CH, tile, Y, X0, nxc, cplane, pc, pc + gg * (km + 1), den,
                                      ring, ovf, rowf, off, dp, plane, ptop, pbot, area, active, iv, kord);
    if constexpr (NF > 1) {
        for (; v0 < a.n_fields; ++v0)
            cells_field_group<1, DT, FF>(a, v0, lane, f, CH, tile, Y, X0, nxc, cplane, pc, pc + gg * (km + 1), den,
                                         ring, ovf, rowf, off, dp, plane, ptop, pbot, area, active, iv, kord);
    }
}

// ====================================================================================
// Edge-weighted (D-grid u / v) pressure-level coarse-graining
//   regrid_to_edge_weighted_pressure   regridz.py:58-112
//     delp_staggered = xgcm interp of delp to the edges (0.5 * (left + right), halo
//                      cells from the connected faces, cubedsphere/xgcm.py:7-34)
//     edge_weighted_block_average(delp_staggered, spacing)   coarsen.py:221-271
//     _regrid_given_delp (staggered block_upsample_like, mappm, _mask_weights)
//   edge_weighted_block_average(u_regrid, masked spacing)     coarsen_restarts.py:493-509
// Only every f-th outer line survives the final average, and the upsampled coarse
// delp at those fine points is that of the same coarse edge, so a coarse edge needs
// just its own f fine edge points: lane = one of them, f consecutive lanes = one
// coarse edge, 64 / f coarse edges per one-wave block.
//   edge x (u): fine points (Y*f, X*f + j) on (y outer, x center); window along x
//               (memory-contiguous: numpy pairwise order, the xor tree for f = 8)
//   edge y (v): fine points (Y*f + j, X*f) on (y center, x outer); window along y
//               (strided: sequential order)
// ====================================================================================

// cubedsphere/xgcm.py FV3_FACE_CONNECTIONS: [tile][axis x=0,y=1][side left=0,right=1]
// = neighbour tile * 2 + its connecting axis.  A line from a face whose connecting
// axis is the other one runs reversed along the tangential index (pinned by the
// reference's regression data, oracle/coarsen.py face_halo).
__constant__ int kFaceConn[6][2][2] = {
    {{4 * 2 + 1, 1 * 2 + 0}, {5 * 2 + 1, 2 * 2 + 0}},
    {{0 * 2 + 0, 3 * 2 + 1}, {5 * 2 + 0, 2 * 2 + 1}},
    {{0 * 2 + 1, 3 * 2 + 0}, {1 * 2 + 1, 4 * 2 + 0}},
    {{2 * 2 + 0, 5 * 2 + 1}, {1 * 2 + 0, 4 * 2 + 1}},
    {{2 * 2 + 1, 5 * 2 + 0}, {3 * 2 + 1, 0 * 2 + 0}},
    {{4 * 2 + 0, 1 * 2 + 1}, {3 * 2 + 0, 0 * 2 + 1}},
};

template <typename DT>
struct EdgeArgs {
    const DT* delp;        // (6, km, n, n) cell centers
    const float* spacing;  // (6, ny_e, nx_e) edge lengths
    const float* fields[kMaxFields];
    float* out[kMaxFields];  // (6, km, nyc_e, nxc_e)
    int n_fields, km, n, f, iv, kord, edge;  // edge 0: "x" (u), 1: "y" (v)
    double ptop;
    float* scratch;  // [km][gridDim * 64]: each lane's remapped column (input-driven path)
};

// element offset (level 0) of delp cell (tile t, row r, col c), r/c possibly one past
// an edge of the tile: then the halo cell of the connected face
__device__ __forceinline__ int64_t halo_cell(int t, int r, int c, int n, int64_t tstride)
{
    int axis = -1, side = 0, i = 0;
    if (r < 0) { axis = 1; side = 0; i = c; }
    else if (r >= n) { axis = 1; side = 1; i = c; }
    else if (c < 0) { axis = 0; side = 0; i = r; }
    else if (c >= n) { axis = 0; side = 1; i = r; }
    if (axis < 0) return (int64_t)t * tstride + (int64_t)r * n + c;
    const int code = kFaceConn[t][axis][side];
    const int nb = code >> 1, nax = code & 1;
    const int ti = (nax != axis) ? n - 1 - i : i;  // rotated face: reversed tangential order
    int rr, cc;
    if (nax == 1) { rr = side == 0 ? n - 1 : 0; cc = ti; }  // neighbour's last / first row
    else { cc = side == 0 ? n - 1 : 0; rr = ti; }           // neighbour's last / first column
    return (int64_t)nb * tstride + (int64_t)rr * n + cc;
}

// sum over the f lanes of this lane's coarse edge (first lane `base`); every lane of
// the edge gets the same value
template <typename T>
__device__ __forceinline__ T edge_sum(T v, int f, int base, bool pairwise)
{
    if (pairwise) return row_sum<T>(v, f, base);
    T s = __shfl(v, base, 64);
    for (int i = 1; i < f; ++i) s = s + __shfl(v, base + i, 64);
    return s;
}

// fine edge column: p_in streamed from the running cumsum of the staggered delp
template <typename DT>
struct EdgeCol {
    const float* q;
    const DT* da;  // the two delp cells either side of this edge point, level 0
    const DT* db;
    int64_t plane;   // delp level stride (cell grid)
    int64_t qplane;  // field level stride (edge grid)
    const DT* pc;
    DT ptop, pbot, run;
    int next, km, kn;
    __device__ __forceinline__ float q1(int k) const { return q[(int64_t)(k - 1) * qplane]; }
    __device__ __forceinline__ float pe1(int k)
    {
        if (k == 1) return (float)ptop;
        if (k == km + 1) return (float)pbot;
        while (next < k - 1) {
            run = run + (DT)0.5 * (da[(int64_t)next * plane] + db[(int64_t)next * plane]);
            ++next;
        }
        return (float)run;
    }
    __device__ __forceinline__ float pe2(int k) const { return (float)pc[k - 1]; }
    __device__ __forceinline__ void emit(int k, float v)
    {
        if (out) out[(int64_t)(k - 1) * ostride] = v;
    }
    __device__ __forceinline__ float next_edge(int k) const { return (k + 1 <= kn + 1) ? pe2(k + 1) : 0.0f; }
    float* out = nullptr;  // this lane's remapped column in the scratch (stride ostride), or NULL
    int64_t ostride = 0;
};

// SCR: input-driven remap through the per-lane scratch (default); !SCR: the cursor
template <typename DT, bool SCR>
__global__ __launch_bounds__(64) void regrid_coarsen_edge_kernel(EdgeArgs<DT> a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int f = a.f, km = a.km, n = a.n;
    const int C = 64 / f;
    const int lane = threadIdx.x;
    const int nc = n / f;
    // coarse edge grid: edge x (nc + 1) rows x nc columns, edge y nc rows x (nc + 1) columns
    const int ncx = a.edge == 0 ? nc : nc + 1;
    const int ncy = a.edge == 0 ? nc + 1 : nc;
    const int nseg = (ncx + C - 1) / C;
    int64_t bi = blockIdx.x;
    const int seg = (int)(bi % nseg);
    bi /= nseg;
    const int Y = (int)(bi % ncy);
    const int tile = (int)(bi / ncy);
    const int lc = lane / f;
    const int cell = min(lc, C - 1);
    const int j = lane - lc * f;
    const int X = seg * C + cell;
    const bool active = lc < C && X < ncx;
    const int Xa = min(X, ncx - 1);
    const int base = cell * f;
    // this lane's fine edge point and its two delp cells
    int fr, fcol, ar, ac, br, bc;
    const int nxe = a.edge == 0 ? n : n + 1;  // fine edge grid width
    if (a.edge == 0) {
        fr = Y * f;
        fcol = Xa * f + (active ? j : 0);
        ar = fr - 1; ac = fcol; br = fr; bc = fcol;
    } else {
        fr = Y * f + (active ? j : 0);
        fcol = Xa * f;
        ar = fr; ac = fcol - 1; br = fr; bc = fcol;
    }
    const int64_t plane = (int64_t)n * n;
    const int64_t tstride = (int64_t)km * plane;
    const DT* da = a.delp + halo_cell(tile, ar, ac, n, tstride);
    const DT* db = a.delp + halo_cell(tile, br, bc, n, tstride);
    const int nye = a.edge == 0 ? n + 1 : n;
    const int64_t eplane = (int64_t)nye * nxe;
    const int64_t fine = (int64_t)fr * nxe + fcol;
    const float sp = active ? a.spacing[(int64_t)tile * eplane + fine] : 0.0f;
    const bool pw = a.edge == 0;  // window along x: numpy's pairwise kernel

    DT* pc = reinterpret_cast<DT*>(smem);  // [C][km+1] coarse phalf of each coarse edge
    // ---- pass 1: staggered delp, fine phalf, edge-weighted coarse delp and phalf ----
    const float den0 = edge_sum<float>(nan0(sp), f, base, pw);  // spacing.coarsen().sum(): float32
    const DT ptop = (DT)a.ptop;
    DT run = ptop, crun = ptop;
    if (active && j == 0) pc[cell * (km + 1)] = ptop;
    for (int k = 0; k < km; ++k) {
        const DT ds = active ? (DT)0.5 * (da[(int64_t)k * plane] + db[(int64_t)k * plane]) : (DT)0;
        run = run + ds;
        const DT num = edge_sum<DT>(nan0((DT)sp * ds), f, base, pw);  // (spacing * delp) in delp's dtype
        crun = crun + num / (DT)den0;  // coarse phalf = cumsum([ptop, delp_c])
        if (active && j == 0) pc[cell * (km + 1) + k + 1] = crun;
    }
    const DT pbot = run;
    __syncthreads();

    // ---- per field: remap each fine edge column, masked edge-weighted mean ----
    const DT* pcc = pc + cell * (km + 1);
    const int ncol_out = ncx;
    const int64_t cplane = (int64_t)ncy * ncx;
    for (int v = 0; v < a.n_fields; ++v) {
        EdgeCol<DT> col;
        col.q = a.fields[v] + (int64_t)tile * km * eplane + fine;
        col.da = da;
        col.db = db;
        col.plane = plane;
        col.qplane = eplane;
        col.pc = pcc;
        col.ptop = ptop;
        col.pbot = pbot;
        col.run = ptop;
        col.next = 0;
        col.km = km;
        col.kn = km;
        float* o = a.out[v] + (int64_t)tile * km * cplane + (int64_t)Y * ncol_out + Xa;
        auto level_sum = [&](int k, float q2) {
            const float w = (pcc[k + 1] < pbot) ? sp : 0.0f;  // _mask_weights (compared in delp's dtype)
            const float num = edge_sum<float>(nan0(q2 * w), f, base, pw);
            const float den = edge_sum<float>(nan0(w), f, base, pw);
            if (active && j == 0) o[(int64_t)k * cplane] = num / den;
        };
        if constexpr (SCR) {  // as in regrid_coarsen_kernel: uniform over input layers
            const int64_t sstride = (int64_t)gridDim.x * 64;
            float* const mine = a.scratch + (int64_t)blockIdx.x * 64 + threadIdx.x;
            col.out = mine;
            col.ostride = sstride;
            mappm_ppm_column(col, km, km, a.iv, a.kord);
            for (int k = 0; k < km; ++k) level_sum(k, mine[(int64_t)k * sstride]);
        } else {
            PpmCursor<EdgeCol<DT>> cur(col, km, km, a.iv, a.kord);
            for (int k = 0; k < km; ++k) level_sum(k, cur.next());
        }
    }
}

}  // namespace



template <typename DT>
int regrid_coarsen_impl(const DT* delp, const float* area, const float* const* fields, float* const* out,
                        int n_fields, float* delp_out, double* delp_out64, int ntile, int km, int ny, int nx,
                        int factor, int iv, int kord, double ptop_toa, void* stream)
{
    using namespace fv3;
    clear_error();
    FV3_REQUIRE(ntile >= 1 && ny >= 1 && nx >= 1, "regrid_coarsen: bad grid (%d, %d, %d)", ntile, ny, nx);
    FV3_REQUIRE(km >= 4 && km <= kMaxLev, "regrid_coarsen: km must be in [4, %d] (got %d)", kMaxLev, km);
    FV3_REQUIRE(factor >= 1 && factor <= 8, "regrid_coarsen: coarsening factor must be in [1, 8]");
    FV3_REQUIRE(ny % factor == 0 && nx % factor == 0, "regrid_coarsen: %dx%d not divisible by factor %d", ny, nx,
                factor);
    FV3_REQUIRE(n_fields >= 0 && n_fields <= kMaxFields, "regrid_coarsen: n_fields must be in [0, %d]",
                kMaxFields);
    FV3_REQUIRE(delp && area, "regrid_coarsen: NULL delp/area");
    if (kord > 7) {
        set_error("regrid_coarsen: kord > 7 (cs_profile) is not fused in this build; use fv3_mappm_ex");
        return FV3_ERR_UNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    CoarsenArgs<DT> a{};
    if (n_fields > 0) FV3_REQUIRE(fields && out, "regrid_coarsen: NULL field tables");
    for (int v = 0; v < n_fields; ++v) {
        FV3_REQUIRE(fields[v] && out[v], "regrid_coarsen: NULL field/output %d", v);
        a.fields[v] = fields[v];
        a.out[v] = out[v];
    }
    a.delp = delp;
    a.area = area;
    a.delp_out = delp_out;
    a.delp_out64 = delp_out64;
    a.n_fields = n_fields;
    a.ntile = ntile;
    a.km = km;
    a.ny = ny;
    a.nx = nx;
    a.f = factor;
    a.iv = iv;
    a.kord = kord;
    a.ptop = ptop_toa;
    // one block per coarse row segment of C = 64 / f cells: f waves
    const int C = 64 / factor;
    const int nxc = nx / factor;
    const int64_t nseg = (nxc + C - 1) / C;
    const int64_t blocks = (int64_t)ntile * (ny / factor) * nseg;
    const size_t lds = sizeof(DT) * ((size_t)C * (km + 1) + (size_t)factor * 64) + sizeof(float) * (factor * 64 + 64) +
                       std::max(sizeof(float) * (size_t)km * 64, sizeof(DT) * kChunk * 64);
    FV3_REQUIRE(lds <= 160 * 1024, "regrid_coarsen: %zu B of LDS needed", lds);
    FV3_REQUIRE(blocks < (int64_t)0x7fffffff, "regrid_coarsen: grid too large");
    // per-lane remapped columns for the input-driven path: km x (blocks x 64 f) floats from
    // the stream-ordered pool (C384 79 levels: ~285 MB, reused by every field of the call;
    // FV3_COARSEN_CURSOR=1 selects the scratch-free output-driven path for A/B)
    // FV3_COARSEN_PATH = cells (default for f >= 2) | rows (the f-wave row-segment
    // blocks with a per-lane scratch column) | cursor (rows, scratch-free cursor remap)
    const char* path = fv3::variant_env("FV3_COARSEN_PATH");
    const bool cursor = (path && path[0] == 'c' && path[1] == 'u') || fv3::variant_env("FV3_COARSEN_CURSOR");
    const bool cells = !cursor && factor >= 2 && !(path && path[0] == 'r');
    void* scratch = nullptr;
    if (cells) {
        // fields remapped NF = 2 at a time (one streaming pass shares the pressure work;
        // FV3_COARSEN_NF=1 for A/B)
        const char* nfe = fv3::variant_env("FV3_COARSEN_NF");
        const int NF = (n_fields >= 2 && !(nfe && nfe[0] == '1')) ? 2 : 1;
        const int ff = factor * factor, G = 64 / ff;
        const int CH = std::min(8, 64 / (G * factor));
        const int64_t cblocks = (int64_t)ntile * (ny / factor) * ((nxc + G - 1) / G);
        const size_t lds_c = sizeof(DT) * ((size_t)G * (km + 1) + 64 + 64) +
                             std::max(sizeof(DT) * CH * kRingLd, sizeof(float) * NF * ring_levels(NF) * kRingLd) +
                             sizeof(float) * (64 * 3 + (size_t)G * km) + sizeof(int) * 64 * NF;
        FV3_REQUIRE(lds_c <= 64 * 1024, "regrid_coarsen: %zu B of LDS needed", lds_c);
        FV3_REQUIRE(cblocks < (int64_t)0x7fffffff, "regrid_coarsen: grid too large");
        // buffer loads: a tile's levels at 32-bit byte offsets (FV3_COARSEN_BUFLOAD)
        FV3_REQUIRE((int64_t)km * ny * nx * (int64_t)sizeof(DT) <= (int64_t)0xffffffff,
                    "regrid_coarsen: one tile of %d levels spans more than 4 GiB", km);
        // per-lane overflow columns: only written by lanes that run ring_levels(NF) levels ahead
        if (n_fields > 0)
            FV3_HIP(hipMallocAsync(&scratch, sizeof(float) * NF * (size_t)km * (size_t)cblocks * 64, s));
        a.scratch = (float*)scratch;
        const dim3 grid((unsigned)cblocks), block(64);
        // register targets: the two-field pass 4 waves per SIMD (118 VGPRs; at 6 it spills
        // its remap state, 3.4 ms for 4 fields), the one-field pass 6 on float32 delp
        // (0.756 -> 0.716 ms at C384, profiles/r05zzk_coarsen_wpe_ab.log) and 5 on float64
#ifndef FV3_COARSEN_W1F
#define FV3_COARSEN_W1F 6  // tools/ variant builds: the register targets under A/B
#endif
#ifndef FV3_COARSEN_W2
#ifdef FV3_FAST_ARITH  // 113 VGPRs at 4; 5 waves per SIMD measured 1.633-1.645 -> 1.595 ms for 4 fields
#define FV3_COARSEN_W2 5  // (profiles/r06l_coarsen_wpe_ab.log); the exact pass (119 VGPRs) stays at 4
#else
#define FV3_COARSEN_W2 4
#endif
#endif
        constexpr int W1 = std::is_same<DT, float>::value ? FV3_COARSEN_W1F : 5;
        constexpr int W2 = FV3_COARSEN_W2;
        const bool k1 = iv == 1 && kord == 1;
        if (factor == 8 && NF == 2)
            hipLaunchKernelGGL((k1 ? regrid_coarsen_cells_kernel<DT, 8, 2, W2, true>
                                  : regrid_coarsen_cells_kernel<DT, 8, 2, W2, false>), grid, block, lds_c, s, a);
        else if (factor == 8)
            hipLaunchKernelGGL((k1 ? regrid_coarsen_cells_kernel<DT, 8, 1, W1, true>
                                  : regrid_coarsen_cells_kernel<DT, 8, 1, W1, false>), grid, block, lds_c, s, a);
        else if (NF == 2)
            hipLaunchKernelGGL((regrid_coarsen_cells_kernel<DT, 0, 2, W2, false>), grid, block, lds_c, s, a);
        else
            hipLaunchKernelGGL((regrid_coarsen_cells_kernel<DT, 0, 1, W1, false>), grid, block, lds_c, s, a);
        FV3_LAUNCH_CHECK();
        if (scratch) FV3_HIP(hipFreeAsync(scratch, s));
        return FV3_OK;
    }
    if (n_fields > 0 && !cursor)
        FV3_HIP(hipMallocAsync(&scratch, sizeof(float) * (size_t)km * (size_t)blocks * 64 * factor, s));
    a.scratch = (float*)scratch;
    if (scratch)
        hipLaunchKernelGGL((regrid_coarsen_kernel<DT, true>), dim3((unsigned)blocks), dim3(64 * factor), lds, s, a);
    else
        hipLaunchKernelGGL((regrid_coarsen_kernel<DT, false>), dim3((unsigned)blocks), dim3(64 * factor), lds, s, a);
    FV3_LAUNCH_CHECK();
    if (scratch) FV3_HIP(hipFreeAsync(scratch, s));
    return FV3_OK;
}

template <typename DT>
int regrid_coarsen_edge_impl(const DT* delp, const float* spacing, const float* const* fields, float* const* out,
                             int n_fields, int ntile, int km, int ny, int nx, int factor, int edge, int iv, int kord,
                             double ptop_toa, void* stream)
{
    clear_error();
    FV3_REQUIRE(ntile == 6, "regrid_coarsen_edge: the face connections need all 6 tiles (got %d)", ntile);
    FV3_REQUIRE(ny == nx && nx >= 1, "regrid_coarsen_edge: tiles must be square (got %d x %d)", ny, nx);
    FV3_REQUIRE(edge == 0 || edge == 1, "regrid_coarsen_edge: edge must be 0 ('x') or 1 ('y')");
    FV3_REQUIRE(km >= 4 && km <= kMaxLev, "regrid_coarsen_edge: km must be in [4, %d] (got %d)", kMaxLev, km);
    FV3_REQUIRE(factor >= 1 && factor <= 8, "regrid_coarsen_edge: coarsening factor must be in [1, 8]");
    FV3_REQUIRE(nx % factor == 0, "regrid_coarsen_edge: %d not divisible by factor %d", nx, factor);
    // block_upsample_like (coarsen.py:928-933) infers staggering from the coarse size's
    // parity: only an even number of coarse cells per tile upsamples correctly there
    FV3_REQUIRE((nx / factor) % 2 == 0,
                "regrid_coarsen_edge: %d coarse cells per tile side is odd; the reference's "
                "block_upsample_like mistakes the center axis for a staggered one", nx / factor);
    FV3_REQUIRE(n_fields >= 0 && n_fields <= kMaxFields, "regrid_coarsen_edge: n_fields must be in [0, %d]",
                kMaxFields);
    FV3_REQUIRE(delp && spacing, "regrid_coarsen_edge: NULL delp/spacing");
    if (kord > 7) {
        set_error("regrid_coarsen_edge: kord > 7 (cs_profile) is not fused in this build; use fv3_mappm_ex");
        return FV3_ERR_UNSUPPORTED;
    }
    EdgeArgs<DT> a{};
    if (n_fields > 0) FV3_REQUIRE(fields && out, "regrid_coarsen_edge: NULL field tables");
    for (int v = 0; v < n_fields; ++v) {
        FV3_REQUIRE(fields[v] && out[v], "regrid_coarsen_edge: NULL field/output %d", v);
        a.fields[v] = fields[v];
        a.out[v] = out[v];
    }
    a.delp = delp;
    a.spacing = spacing;
    a.n_fields = n_fields;
    a.km = km;
    a.n = nx;
    a.f = factor;
    a.iv = iv;
    a.kord = kord;
    a.edge = edge;
    a.ptop = ptop_toa;
    const int C = 64 / factor;
    const int nc = nx / factor;
    const int ncx = edge == 0 ? nc : nc + 1, ncy = edge == 0 ? nc + 1 : nc;
    const int64_t blocks = (int64_t)6 * ncy * ((ncx + C - 1) / C);
    const size_t lds = sizeof(DT) * (size_t)C * (km + 1);
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;  // per-lane remapped columns (see regrid_coarsen_impl)
    if (n_fields > 0 && !fv3::variant_env("FV3_COARSEN_CURSOR"))
        FV3_HIP(hipMallocAsync(&scratch, sizeof(float) * (size_t)km * (size_t)blocks * 64, s));
    a.scratch = (float*)scratch;
    if (scratch)
        hipLaunchKernelGGL((regrid_coarsen_edge_kernel<DT, true>), dim3((unsigned)blocks), dim3(64), lds, s, a);
    else
        hipLaunchKernelGGL((regrid_coarsen_edge_kernel<DT, false>), dim3((unsigned)blocks), dim3(64), lds, s, a);
    FV3_LAUNCH_CHECK();
    if (scratch) FV3_HIP(hipFreeAsync(scratch, s));
    return FV3_OK;
}

// explicit instantiations: the C ABI below (exact unit) calls the fast unit's
template int regrid_coarsen_impl<float>(const float*, const float*, const float* const*, float* const*, int, float*,
                                        double*, int, int, int, int, int, int, int, double, void*);
template int regrid_coarsen_impl<double>(const double*, const float*, const float* const*, float* const*, int,
                                         float*, double*, int, int, int, int, int, int, int, double, void*);
template int regrid_coarsen_edge_impl<float>(const float*, const float*, const float* const*, float* const*, int,
                                             int, int, int, int, int, int, int, int, double, void*);
template int regrid_coarsen_edge_impl<double>(const double*, const float*, const float* const*, float* const*,
                                              int, int, int, int, int, int, int, int, int, double, void*);

}  // namespace FV3_ARITH_NS

#ifndef FV3_FAST_ARITH
namespace fast {  // coarsen_fast.hip
template <typename DT>
int regrid_coarsen_impl(const DT* delp, const float* area, const float* const* fields, float* const* out,
                        int n_fields, float* delp_out, double* delp_out64, int ntile, int km, int ny, int nx,
                        int factor, int iv, int kord, double ptop_toa, void* stream);
template <typename DT>
int regrid_coarsen_edge_impl(const DT* delp, const float* spacing, const float* const* fields, float* const* out,
                             int n_fields, int ntile, int km, int ny, int nx, int factor, int edge, int iv, int kord,
                             double ptop_toa, void* stream);
extern template int regrid_coarsen_impl<float>(const float*, const float*, const float* const*, float* const*, int,
                                               float*, double*, int, int, int, int, int, int, int, double, void*);
extern template int regrid_coarsen_impl<double>(const double*, const float*, const float* const*, float* const*,
                                                int, float*, double*, int, int, int, int, int, int, int, double,
                                                void*);
extern template int regrid_coarsen_edge_impl<float>(const float*, const float*, const float* const*,
                                                    float* const*, int, int, int, int, int, int, int, int, int,
                                                    double, void*);
extern template int regrid_coarsen_edge_impl<double>(const double*, const float*, const float* const*,
                                                     float* const*, int, int, int, int, int, int, int, int, int,
                                                     double, void*);
}  // namespace fast
#endif

}  // namespace fv3

#ifndef FV3_FAST_ARITH  // the C ABI: one definition, dispatching on the arithmetic
namespace {
template <typename DT>
int coarsen_arith(int arith, const DT* delp, const float* area, const float* const* fields, float* const* out,
                  int n_fields, float* delp_out, double* delp_out64, int ntile, int km, int ny, int nx, int factor,
                  int iv, int kord, double ptop_toa, void* stream)
{
    fv3::clear_error();
    FV3_REQUIRE(arith == FV3_ARITH_EXACT || arith == FV3_ARITH_FAST, "regrid_coarsen: unknown arithmetic %d", arith);
    auto f = arith == FV3_ARITH_FAST ? fv3::fast::regrid_coarsen_impl<DT> : fv3::exact::regrid_coarsen_impl<DT>;
    return f(delp, area, fields, out, n_fields, delp_out, delp_out64, ntile, km, ny, nx, factor, iv, kord, ptop_toa,
             stream);
}
template <typename DT>
int coarsen_edge_arith(int arith, const DT* delp, const float* spacing, const float* const* fields, float* const* out,
                       int n_fields, int ntile, int km, int ny, int nx, int factor, int edge, int iv, int kord,
                       double ptop_toa, void* stream)
{
    fv3::clear_error();
    FV3_REQUIRE(arith == FV3_ARITH_EXACT || arith == FV3_ARITH_FAST, "regrid_coarsen_edge: unknown arithmetic %d",
                arith);
    auto f = arith == FV3_ARITH_FAST ? fv3::fast::regrid_coarsen_edge_impl<DT>
                                     : fv3::exact::regrid_coarsen_edge_impl<DT>;
    return f(delp, spacing, fields, out, n_fields, ntile, km, ny, nx, factor, edge, iv, kord, ptop_toa, stream);
}
}  // namespace

extern "C" int fv3_regrid_coarsen_edge(const float* delp, const float* spacing, const float* const* fields,
                                       float* const* out, int n_fields, int ntile, int km, int ny, int nx,
                                       int factor, int edge, int iv, int kord, double ptop_toa, int arith,
                                       void* stream)
{
    return coarsen_edge_arith<float>(arith, delp, spacing, fields, out, n_fields, ntile, km, ny, nx, factor, edge,
                                     iv, kord, ptop_toa, stream);
}

extern "C" int fv3_regrid_coarsen_edge_f64(const double* delp, const float* spacing, const float* const* fields,
                                           float* const* out, int n_fields, int ntile, int km, int ny, int nx,
                                           int factor, int edge, int iv, int kord, double ptop_toa, int arith,
                                           void* stream)
{
    return coarsen_edge_arith<double>(arith, delp, spacing, fields, out, n_fields, ntile, km, ny, nx, factor, edge,
                                      iv, kord, ptop_toa, stream);
}

extern "C" int fv3_regrid_coarsen(const float* delp, const float* area, const float* const* fields,
                                  float* const* out, int n_fields, float* delp_out, int ntile, int km, int ny,
                                  int nx, int factor, int iv, int kord, double ptop_toa, int arith, void* stream)
{
    return coarsen_arith<float>(arith, delp, area, fields, out, n_fields, delp_out, nullptr, ntile, km, ny, nx,
                                factor, iv, kord, ptop_toa, stream);
}

extern "C" int fv3_regrid_coarsen_f64(const double* delp, const float* area, const float* const* fields,
                                      float* const* out, int n_fields, float* delp_out, int ntile, int km, int ny,
                                      int nx, int factor, int iv, int kord, double ptop_toa, int arith, void* stream)
{
    return coarsen_arith<double>(arith, delp, area, fields, out, n_fields, delp_out, nullptr, ntile, km, ny, nx,
                                 factor, iv, kord, ptop_toa, stream);
}

extern "C" int fv3_regrid_coarsen_f64d(const double* delp, const float* area, const float* const* fields,
                                       float* const* out, int n_fields, double* delp_out, int ntile, int km, int ny,
                                       int nx, int factor, int iv, int kord, double ptop_toa, int arith,
                                       void* stream)
{
    return coarsen_arith<double>(arith, delp, area, fields, out, n_fields, nullptr, delp_out, ntile, km, ny, nx,
                                 factor, iv, kord, ptop_toa, stream);
}
#endif  // FV3_FAST_ARITH
