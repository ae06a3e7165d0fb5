// fv3net_amd — the dense column model handle shared by the two forward kernels:
// dense.hip (exact f32 MFMA) and dense_b3.hip (bf16x3 split MFMA).
#pragma once

#include <vector>

#include "common.h"

namespace fv3 {

constexpr int kMaxVars = 16;
constexpr int kMaxOutTiles = 64;
constexpr int kMaxSlots = 96;   // input feature rows per tile / (256 / columns per tile)
constexpr int kRawSlots = 20;   // slots prefetched into registers across tiles at 8 rows per slot

struct DenseInVar {
    const float* ptr;
    int64_t ld, bs;
    int step0;    // first padded k-step of this variable
    int nsteps;   // padded k-steps (4 features each)
    int z0;       // first kept level (clip start)
    int nkeep;    // kept levels
};

struct DenseOutTile {
    int var;  // output variable or -1 (padding tile)
    int z0;   // level of the tile's first row
    int nrow; // valid rows in this tile (<= 16)
};

struct DenseArgs {
    const float* in_mean;   // [KP] padded feature order
    const float* in_denom;  // [KP] 1 / f32(sigma + eps) (StandardNormLayer's divisor, inverted)
    const float* w1;        // [KP/4][4 waves][64][T4]
    const float* b1;        // [HP]
    const float* wh;        // [n_hidden-1][HP/4][4 waves][64][T4]
    const float* bh;        // [n_hidden-1][HP]
    const float* wo;        // [n_otiles][HP/16][64][4]: 4 k-steps per lane
    const float* oep;       // [6][KOP]: bias, sigma, mean, lo, hi, mask
    const float* wbase;     // the model allocation: weights are fetched as buffer loads
    int w1_off, wh_off, wo_off;  // byte offsets of w1 / wh / wo in it
    int wbytes;             // its size (buffer range)
    // input slots (per launch): slot q covers feature rows [fdst, fdst + 256/NCOL) of one
    // variable; thread row fq reads base[blk * bs + ii + fq * ld] if fq < nk, writes
    // padded feature fdst + fq if fq < nf.  meta = var << 27 | fdst << 16 | nk << 8 | nf
    // (var: the slot's input variable).  Slots past nslots are all zero (no rows).
    // Every field is 4-byte: read with scalar loads (a byte array here would be a
    // vector load and a vmcnt(0) wait per slot)
    const float* slot_base[kMaxSlots];
    int slot_bs[kMaxSlots];
    int slot_ld[kMaxSlots];
    int slot_meta[kMaxSlots];
    float slot_leps[kMaxSlots];  // > 0: the slot's variable enters as log(max(x, eps)) (emulator LogTransform)
    float* out_ptr[kMaxVars];
    int64_t out_ld[kMaxVars];
    int64_t out_bs[kMaxVars];
    DenseOutTile otile[kMaxOutTiles];
    // residual outputs (emulator Difference.backward: after = before + to): the raw
    // input added to output variable o after de-normalisation, or NULL
    const float* res_ptr[kMaxVars];
    int res_ld[kMaxVars];
    int res_bs[kMaxVars];
    int64_t ncol, ncol_blk, ntiles;
    int n_in, n_hidden_extra, n_otiles, kp;
    int in_steps_total, nslots;
    int lds_x;              // f32x4 offset of the constants area (after activations and inputs)
    int lds_s;              // f32x4 offset of the staged inputs (after the activations)
    int has_log;            // any slot with a LogTransform (selects the staging variant)
    int fast_stage;         // every slot FPS-aligned: the short staging path
    long long* trace;       // profiling hook (fv3_dense_set_trace): [tiles][8] timestamps, or NULL
    int prio;               // wave issue priority (s_setprio 0..3) for the whole kernel (FV3_DENSE_PRIO)
};
static_assert(sizeof(DenseArgs) <= 4096, "kernel arguments are limited to 4 KiB");

struct B3Pack;  // dense_b3.hip: a bf16 split weight stream (bf16x3 / bf16x6) and its constants
struct B3Desc;  // dense_b3.hip: a host copy of the model description (the bf16x6 stream is packed from it on first use)

}  // namespace fv3

struct fv3_dense_model {
    int n_in = 0, n_out = 0, k_in = 0, k_out = 0, width = 0, ht = 0, hp = 0, n_hidden = 0;
    int kp = 0, n_otiles = 0, steps_total = 0;
    int w1_off8 = -1, wh_off8 = -1;  // layer-1 / hidden streams packed for 8-wave blocks (-1: none)
    std::vector<int> in_nz, out_nz, in_z0, in_nkeep, in_step0, in_nsteps, out_residual;
    std::vector<float> in_log_eps;
    std::vector<fv3::DenseOutTile> otiles;
    void* dbuf = nullptr;
    fv3::DenseArgs tmpl{};  // device pointers filled, per-call fields empty
    fv3::B3Pack* b3 = nullptr;  // bf16x3 weight stream (2 bf16 parts per weight)
    fv3::B3Pack* b6 = nullptr;  // bf16x6 weight stream (3 parts), packed on the first bf16x6 forward
    fv3::B3Desc* b6_src = nullptr;  // what b6 is packed from (released once packed)
};

namespace fv3 {
// dense_b3.hip: build / free the bf16x3 pack of a model (called by fv3_dense_create/destroy)
int b3_pack(fv3_dense_model* m, const fv3_dense_desc* d);
void b3_free(fv3_dense_model* m);
}  // namespace fv3
