// lnerf_internal.h -- shared declarations between the HIP kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lnerf.h"
#include "lnerf_marshal.h"

namespace lnerf {

constexpr int kWmaxParts = 32;   // blocks per layer of the max|W| pass before the fp16x3 packing
constexpr int kDefaultDwGrid = 512;   // dW workgroups per step unless LNERF_OPT_DW_GRID says otherwise

// ---- fp16x3 exponent shifts ------------------------------------------------------------------
// The shift e that puts a group's largest magnitude m in [2^13, 2^14) for the fp16 hi/lo split
// (0 for m = 0 or non-finite m). Clamped to 2^127 so the scale 2^e stays a finite float even for
// groups whose maximum is a tiny or subnormal value (m < 2^-113: underflowed transmittance, a
// ray behind an opaque one); the unscale 2^-(e_w + e_x) is then still exact.
__device__ __forceinline__ int fp16x3_shift(float m) {
    if (!(m > 0.0f) || !(m < __builtin_inff())) return 0;
    int e;
    (void)__builtin_frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
    const int sh = 14 - e;
    return sh > 127 ? 127 : sh;
}

// ---- ray sampling (train_nerf.py:289-306), float64 as numpy computes it -----------------------
// t_j = np.linspace(near, far, S)[j]: j * ((far - near) / (S - 1)) + near, the last one = far.
__host__ __device__ inline double ray_depth(int j, int S, float near_t, float far_t) {
    if (S <= 1) return (double)near_t;
    if (j == S - 1) return (double)far_t;
    return (double)j * (((double)far_t - (double)near_t) / (double)(S - 1)) + (double)near_t;
}
// dists_j = t_{j+1} - t_j, the last 1e8 (then float32 at the ABI)
__host__ __device__ inline float ray_delta(int j, int S, float near_t, float far_t) {
    if (j >= S - 1) return 1e8f;
    return (float)(ray_depth(j + 1, S, near_t, far_t) - ray_depth(j, S, near_t, far_t));
}
// coordinate c of sample j of a ray [o, d]: o + d * t (pts = o + d * t[None, :, None])
__host__ __device__ inline double ray_point(const float* ray6, int c, int j, int S, float near_t,
                                            float far_t) {
    return (double)ray6[c] + (double)ray6[3 + c] * ray_depth(j, S, near_t, far_t);
}

// ----------------------------------------------------------------------------------------------
// Generic ("loma-order") path: one loma call on flat device rectangles. Field meaning follows
// scripts/nerf.py:1-22; loop bounds are exactly the reference's.
// ----------------------------------------------------------------------------------------------

struct LgBuffers {
    // primal (device)
    const float* X;
    const float* W;
    const float* B;
    const float* T;
    float* IO;      // intermediate_outputs, mutated in place
    float* rgba;    // (th, S, 4)
    const float* dists;
    float* alpha;
    float* cp;
    float* wsamp;
    float* acc;     // (th, acc_cols)
    // snapshots for the reverse sweep (nullable in a forward-only call)
    float* zpre;    // io right after each layer's bias stage
    float* cpC;     // cumprod buffer after its init stage (c_j)
    float* cpP;     // after the inclusive product (P_j)
};

struct LgAdjoints {
    float* dX;      // nullable
    float* dW;
    float* dB;
    float* dT;
    float* dIO;
    float* drgba;
    float* ddists;
    float* dalpha;
    float* dcp;
    float* dwsamp;
    float* dacc;
};

// nerf_evaluate_and_march on device; writes the loss to *loss_dev.
void lg_nerf_forward(const LgDims& d, const LgBuffers& b, float* loss_dev, hipStream_t s);
// grad_nerf_evaluate_and_march: b must hold a *fresh copy* of the primal inputs (the forward is
// re-executed on it, snapshots filled); adjoints accumulate in `a`. `seed_dev` is a device
// scalar (so the seed may be a loss computed on the device).
void lg_nerf_grad(const LgDims& d, const LgBuffers& b, const LgAdjoints& a, const float* seed_dev,
                  hipStream_t s);
void lg_mlp_fit_forward(const LgDims& d, const LgBuffers& b, float* loss_dev, hipStream_t s);
void lg_mlp_fit_grad(const LgDims& d, const LgBuffers& b, const LgAdjoints& a,
                     const float* seed_dev, hipStream_t s);
void lg_mult_a_b(const float* a, int a_h, int a_w, const float* b, int b_w, float* c,
                 hipStream_t s);

// small helpers
void k_fill(float* p, float v, size_t n, hipStream_t s);
void k_scale_by_scalar(float* p, size_t n, const float* scale, hipStream_t s);
// RAYS mode producers for the generic path: the encoded sample rows (f64 points, f64 trig) and
// the per-sample dists.
void k_positional_encoding_rays(const float* rays, int nrays, int S, float near_t, float far_t,
                                int F, float* out, int out_cols, hipStream_t s);
void k_ray_dists(int nrays, int S, float near_t, float far_t, float* out, hipStream_t s);
void k_get_rays(int width, const double* K, const double* c2w, float* rays, hipStream_t s);
void k_positional_encoding(const float* pts, int n, int F, float* out, int out_cols,
                           hipStream_t s);
void k_adam(float* params, const float* grads, float* m, float* v, size_t n, int t, float lr,
            float beta1, float beta2, float eps, hipStream_t s);

// ----------------------------------------------------------------------------------------------
// Fused MFMA path (the throughput path). See DESIGN.md "Kernels".
// ----------------------------------------------------------------------------------------------
struct FusedPlan {
    int L;
    int k[kMaxLayers], n[kMaxLayers];   // real widths
    int kt[kMaxLayers], nt[kMaxLayers]; // 32-wide tiles
    int w_k, w_n;
    int rays, S, R;                     // R = rays*S
    int tile;                           // samples per fused workgroup: 128, or 64 for k16 with
                                        // 4-wave workgroups (two per CU; S <= 64, fp16x3 / bf16)
    int rays_per_wg;                    // whole rays per workgroup tile
    int num_wg;                         // fused-kernel grid
    int blocks;                         // 32-sample slabs = num_wg * 4
    int input_mode, F;
    // workspace carve (device pointers)
    float* wf;        // forward-packed weights, per layer offsets below
    float* wb;        // backward-packed weights
    float* bp;        // biases in fragment order
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    int ht;           // hidden output tiles (1/2/4/8): the fused kernel's instantiation
    int x6;           // planes per operand: 3 = bf16x6 split (fp32-accurate), 2 = fp16x3 split
                      // (fp16 hi + lo with exponent shifts, 22-bit products; k16 only),
                      // 1 = bf16, 0 = exact f32 MFMA
    int fo[kMaxLayers], bo[kMaxLayers];  // packed output tiles of each layer's fwd / bwd MMA
    unsigned short* w6;                  // bf16x6 packed planes (u16 offsets below)
    size_t w6f_off[kMaxLayers], w6b_off[kMaxLayers], w6f_n[kMaxLayers], w6b_n[kMaxLayers];
    float* act;       // activation slabs: layer l at act_off[l], the input X slab at x_off
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;      // gradient slabs G_l at grad_off[l]
    size_t grad_off[kMaxLayers];
    float* loss_part; // per-workgroup partial loss (num_wg)
    float* dw_part;   // dW split partials
    float* db_part;   // dB split partials
    int dw_splits[kMaxLayers];
    int dw_mode[kMaxLayers];       // dW kernel instantiation per layer (0 = blocked 4x4)
    int dw_phases[kMaxLayers];     // partials per split (4 for phased small layers)
    int dw_split_off[kMaxLayers];  // workgroup offset of layer l in the dW grid
    size_t dwp_off[kMaxLayers];    // float offset of layer l's partial slabs in dw_part
    size_t dbp_off[kMaxLayers];
    int dw_grid;
    float* loss_total; // device scalar
    // k16 kernel (lnerf_k16.hip): 512-thread workgroups, two waves per SIMD, 16x16x32 MFMA
    int k16;                             // 1: the fused step runs k16 (pack16 + k16 kernel)
    int head_fit;                        // 1: the mlp_fit head (LNERF_HEAD_FIT), k16 only
    int ht16;                            // 16-wide hidden output tiles (1/2/4/8/16)
    int ks16_f[kMaxLayers], ks16_b[kMaxLayers];   // k-steps (32 features) per pass
    int to16_f[kMaxLayers], to16_b[kMaxLayers];   // 16-wide output tiles per pass
    unsigned short* w16;                 // packed planes, u16 offsets below
    size_t w16f_off[kMaxLayers], w16b_off[kMaxLayers];
    float* b16;                          // [L][256] zero-padded biases
    unsigned long long* mask_g;          // [num_wg][L-1][8 waves][64 lanes] ReLU mask bits
    int dw16;                            // 1: dW by dw16_kernel (lnerf_dw16.hip), one partial per split
    // k32 kernel (lnerf_k32.hip): 256-thread workgroups, one wave per SIMD, 32x32x16 MFMA
    int k32;                             // 1: the fused step runs k32 (pack32 + k32 kernel)
    int ht32;                            // 32-wide hidden output tiles (1/2/4/8)
    int to32_f[kMaxLayers], to32_b[kMaxLayers];     // 32-wide output tiles per pass (input tiles: ks16_*)
    size_t w32f_off[kMaxLayers], w32b_off[kMaxLayers];   // u16 offsets into w16
    int* wexp16;                         // x6 = 2: per-layer max|W| bits (fp16 weight plane shifts)
    int* wmax_part;                      // x6 = 2: max|W| bits per layer and wmax block [L][kWmaxParts]
    int* dw_shift;                       // dw16: per-layer product shift E_l (k1_reduce_kernel)
    signed char* sexp;                   // dw16: k1's per-sample slab shifts [L][num_wg * 128][2]
    int* epart;                          // dw16: k1's per-wave min of exA + exG [L][num_wg * 8]
};

bool fused_supported(const lnerf_mlp& mlp, int rays, int S, int input_mode, const char** why,
                     bool head_fit = false);
// train = false sizes the forward-only (render) workspace: packed weights + loss partials.
// dw_grid: the dW kernel's workgroup budget (0 = kDefaultDwGrid; LNERF_OPT_DW_GRID).
size_t fused_workspace_bytes(const lnerf_mlp& mlp, int rays, int S, bool train = true, int dw_grid = 0);
// flags select the kernels and the MFMA precision (LNERF_MFMA_*, LNERF_ONE_WAVE; lnerf.h)
void fused_plan(FusedPlan& p, const lnerf_mlp& mlp, const lnerf_batch& b, void* ws_base, int flags,
                bool train = true, int dw_grid = 0);
// ev: nullable array of 7 events recorded between the step's kernels (LNERF_TIMING)
void fused_train_step(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                      float seed, int flags, const lnerf_outputs& out, hipStream_t s,
                      hipEvent_t* ev);
void fused_render(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                  const lnerf_outputs& out, hipStream_t s);
void dw16_launch(const FusedPlan& p, hipStream_t s);
// after a training k1: the batch loss (loss_total, out_loss) and, for dw16 with x6 = 2, the
// layer-wide slab maxima, in one launch (lnerf_dw16.hip)
void k1_reduce_launch(const FusedPlan& p, float* out_loss, hipStream_t s);
// k16 kernel entry points (lnerf_k16.hip)
bool k16_supported(const FusedPlan& p);
void k16_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s);
void k16_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                bool want_grad, hipStream_t s);
// the last training k1's ReLU decisions as (L-1, R, 32) bytes (lnerf_ctx_relu_masks)
void k16_masks_launch(const FusedPlan& p, unsigned char* out, hipStream_t s);
// k32 kernel entry points (lnerf_k32.hip)
bool k32_supported(const FusedPlan& p);
void k32_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s);
void k32_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                bool want_grad, hipStream_t s);
void k32_masks_launch(const FusedPlan& p, unsigned char* out, hipStream_t s);

}  // namespace lnerf
