// lnerf_internal.h -- shared declarations between the HIP kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lnerf.h"
#include "lnerf_marshal.h"

namespace lnerf {

constexpr int kWmaxParts = 32;   // blocks per layer of the max|W| pass before the fp16x3 packing
constexpr int kHeadCols = 16;    // head columns with their own fp16x3 weight shift (k16 head outputs)
constexpr int kDefaultDwGrid = 512;   // dW workgroups per step unless LNERF_OPT_DW_GRID says otherwise
// The default budget for a batch of `samples` sample rows: 512 at the bench size and above, down to
// 256 for smaller batches, where k2 is latency-bound and its time flat from 256 to 512 workgroups
// while the in-order reduce over the splits grows with them (config 2, 32 768 samples, round 5:
// 256 -> 0.073 ms per step, 512 -> 0.082; cfg3 keeps 512: 384 -> 0.88 ms of k2, 512 -> 0.73)
__host__ __device__ constexpr int default_dw_grid(long long samples) {
    return samples / 128 >= kDefaultDwGrid ? kDefaultDwGrid : samples / 128 <= 256 ? 256 : (int)(samples / 128);
}
// ---- exceptional rows of the fp16x3 dW split (round 6) ------------------------------------------
// k2 (lnerf_dw16.hip) multiplies a sample's A row and G row as fp16 hi + lo pieces at per-row
// exponent shifts balanced around the layer's product shift E_l (the smallest xa + xg over the
// batch, i.e. its largest products): A 2^ea, G 2^eg, ea + eg = E_l, each operand lowered by half of
// the row's deficit d = xa + xg - E_l (sample_shifts). A row far below the layer's scale (round 5's
// edge_finite_6x8: rows at d = 30..110, behind opaque samples and at delta = 1e8) was pushed into
// fp16's subnormals, and lost up to ~2 % of a column made only of such rows. Round 6 multiplies
// them exactly instead: an EXCEPTIONAL row -- d > kXrowD0 (each operand more than kXrowD0 / 2
// binades under its own shift) or d < 0 (products above the layer's scale: a ray's last sample, the
// delta = 1e8 row of train_nerf.py:306-311, whose sigma gradient can sit 2^45 above its rgb
// gradients, and which therefore never sets E_l; such a row is exceptional only this way) -- is
// dropped from the fp16x3
// products and multiplied on the bf16x6 split (three bf16 planes per operand, fp32's exponent
// range) into the same accumulators (xrow_pass). k1 writes each row's bound dmax (kXrowD0, or
// kXrowLast for a last sample) beside its shifts; k2 tests d against it. Within the other rows an
// element r binades below its row's maximum sits near 2^(13 - r - d / 2), so the balanced split
// keeps elements down to 2^-(27 - kXrowD0 / 2) of their row's maximum in fp16's normal range.
constexpr int kXrowD0 = 12;
constexpr int kXrowLast = 127;   // a ray's last sample: exceptional only above the scale (d < 0)
// k1's per-sample slab word [l][position], 4 bytes: byte 0 xa (the input row's shift), byte 2 xg (the
// G row's), byte 3 dmax; byte 1 unused
__host__ __device__ constexpr int sexp_xa(unsigned e) { return (int)(signed char)(e & 0xFFu); }
__host__ __device__ constexpr int sexp_xg(unsigned e) { return (int)(signed char)((e >> 16) & 0xFFu); }
__host__ __device__ constexpr int sexp_dmax(unsigned e) { return (int)(signed char)(e >> 24); }

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

// fp16x3 operand split of a pair (x0, x1), packed as two f16 per register: hi = round_f16(x sc),
// lo = round_f16(x sc - hi), fused multiply-adds with one rounding to f16 each (x sc is exact, sc
// a power of two; x sc - hi is exact), so |x sc - hi - lo| <= 2^-22 |x sc| in fp16's normal range.
// Plain C on purpose: the compiler pads the MFMA wait states around these writes, which it does
// not do inside an asm statement (a write into a register an in-flight MFMA still reads as C or
// will write as D; tests/test_isa.py). Built with -fno-slp-vectorize (Makefile) the compiler
// selects v_fma_mix{lo,hi}_f16 for it, 5 instructions per pair, not packed f32 math with widening
// converts.
__device__ __forceinline__ void split_h2(float x0, float x1, float sc, unsigned& hi, unsigned& lo) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const _Float16 h0 = (_Float16)__builtin_fmaf(x0, sc, 0.0f);
    const _Float16 h1 = (_Float16)__builtin_fmaf(x1, sc, 0.0f);
    const _Float16 l0 = (_Float16)__builtin_fmaf(x0, sc, -(float)h0);
    const _Float16 l1 = (_Float16)__builtin_fmaf(x1, sc, -(float)h1);
    hi = __builtin_bit_cast(unsigned, (h2){h0, h1});
    lo = __builtin_bit_cast(unsigned, (h2){l0, l1});
}

// ---- int24 activation slabs (fp16x3 training) --------------------------------------------------
// k1 stores each A_l value (X for l = 0) that k2 reads as q = rint(x 2^(xa + 8)), xa = the
// sample's row shift (fp16x3_shift of its max|x|, so |q| < 2^22), as the low 24 bits of the float
// 1.5 2^23 + q (whose mantissa field is 2^22 + q); 4 values in 12 B. 2^-22 of the row's max|x|,
// the precision fp16x3 keeps of it anyway; 25 % fewer bytes through HBM for the A half of the
// slabs. G_l slabs stay fp32 (their rows span more range: tests/test_gpu_edge.py). A tile-block
// (32 samples x 32 features) is then 3 KiB = 768 float slots instead of 1024.
#ifndef LNERF_A24
#define LNERF_A24 1
#endif
__host__ __device__ constexpr bool a24_slabs(int PL) { return PL == 2 && LNERF_A24 != 0; }
// k1's shift byte of an activation row holding a NaN or an infinity (its max is non-finite): the row
// is encoded at shift 0, and dw16 decodes its out-of-range codes (|q| >= 2^22: +-inf leaves 2^22,
// NaN 1.5 2^23) as NaN, so a non-finite activation still makes its dW terms non-finite
constexpr int kSexpNonFinite = -127;
__host__ __device__ constexpr int a_tile_floats(int PL) { return a24_slabs(PL) ? 768 : 1024; }

// ---- build fingerprint (lnerf_build_knobs): one bit per compile-time knob of the kernel objects
// set away from the product default. The shipped library reports 0; tests and bench.py record it.
enum : unsigned {
    kKnobK16FullDma = 1u << 0, kKnobK16KDist = 1u << 1, kKnobK16SplitAt = 1u << 2, kKnobK16Sched = 1u << 3,
    kKnobK16Prio = 1u << 4, kKnobK16Spread = 1u << 5, kKnobProf = 1u << 6, kKnobA24 = 1u << 7,
    kKnobK16Only = 1u << 8, kKnobDwSplitLate = 1u << 9, kKnobDwDepth = 1u << 10, kKnobDwSwz = 1u << 11,
    kKnobK16Pin = 1u << 12, kKnobK16FdSrc = 1u << 13, kKnobKrStagger = 1u << 15, kKnobDwXrow = 1u << 17,
    kKnobGuard = 1u << 25, kKnobK16G2 = 1u << 26, kKnobKrSched = 1u << 18, kKnobDwWaves = 1u << 14, kKnobKrDist = 1u << 19, kKnobPeDoubling = 1u << 20, kKnobK16OneChunk = 1u << 22, kKnobK16WaveComp = 1u << 23, kKnobK16EpiFma = 1u << 24,
};
unsigned k16_build_knobs();
unsigned dw16_build_knobs();
unsigned kr_build_knobs();

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
    int kt[kMaxLayers], nt[kMaxLayers]; // 32-wide slab tiles
    int w_k, w_n;
    int rays, S, R;                     // R = rays*S
    int tile;                           // samples per k16 workgroup: 128, or 64 with LNERF_K16_W4
                                        // (4-wave workgroups, two per CU; S <= 64, fp16x3 / bf16)
    int rays_per_wg;                    // whole rays per workgroup tile
    int num_wg;                         // k1 grid
    int blocks;                         // 32-sample slab blocks = num_wg * tile / 32
    int input_mode, F;
    int x6;                             // operand planes: 2 = fp16x3 split (default), 3 = bf16x6
                                        // split (both fp32-class), 1 = plain bf16 (inference)
    int head_fit;                       // 1: the mlp_fit head (LNERF_HEAD_FIT)
    // workspace carve (device pointers)
    float* act;       // activation slabs: layer l at act_off[l], the input X slab at x_off
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;      // gradient slabs G_l at grad_off[l]
    size_t grad_off[kMaxLayers];
    float* loss_part; // per-workgroup partial loss (num_wg)
    float* dw_part;   // dW split partials
    float* db_part;   // dB split partials
    int dw_splits[kMaxLayers];
    int dw_split_off[kMaxLayers];  // workgroup offset of layer l in the dW grid
    size_t dwp_off[kMaxLayers];    // float offset of layer l's partial slabs in dw_part
    size_t dbp_off[kMaxLayers];
    int dw_grid;
    float* loss_total; // device scalar
    float* loss_stage; // the render loss's stage-1 block sums (loss_stage1_kernel)
    // k16 weight stream (lnerf_k16.hip): 16x16x32 MFMA, two waves per SIMD
    int ht16;                            // 16-wide hidden output tiles (1/2/4/8/16)
    int ks16_f[kMaxLayers], ks16_b[kMaxLayers];   // k-steps (32 features) per pass
    int to16_f[kMaxLayers], to16_b[kMaxLayers];   // 16-wide output tiles per pass
    unsigned short* w16;                 // packed planes, u16 offsets below
    unsigned short* w16x;                // nullable: the bf16x6 planes of the floor guard's re-run, written by
                                         // the fp16x3 step's own pack (same offsets, three planes)
    size_t w16f_off[kMaxLayers], w16b_off[kMaxLayers];
    float* b16;                          // [L][256] zero-padded biases
    unsigned long long* mask_g;          // [num_wg][L-1][waves][64 lanes] ReLU mask bits
    int* wexp16;                         // x6 = 2: per-layer max|W| bits (fp16 weight plane shifts)
    int* wmax_part;                      // x6 = 2: max|W| bits per layer and wmax block [L][kWmaxParts],
                                         // then the head's per-column partials [kWmaxParts][kHeadCols]
    int* hexp16;                         // x6 = 2: the head's per-column max|W| bits [kHeadCols]
    int* dw_shift;                       // per-layer dW product shift E_l (k1_reduce_kernel)
    unsigned* sexp;                      // k1's per-sample slab words [L][num_wg * tile] (sexp_xa ...)
    int* xcount;                         // per dW workgroup: exceptional rows it multiplied, of them rays'
                                         // last samples (xrow_pass) [dw_grid][2]
    int* epart;                          // k1's per-wave min of exA + exG [L][num_wg * waves]
    // the fp16x3 floor guard (kGuardExp): the primary fp16x3 step's k1 sets *guard, its pack zeroes it
    // first; the bf16x6 re-run's kernels (gate = the same word) exit at once unless it is set
    int* guard;                          // nullable: no floor test
    const int* gate;                     // nullable: run unconditionally
};

// ---- the fp16x3 floor guard (round 6) ----------------------------------------------------------
// k1's reverse chain splits each G row at the row's own shift (max in [2^13, 2^14)), so an element
// of a G row that sits below 2^kGuardExp after that shift -- about 2^-37.5 of its row's maximum --
// has nothing left in either fp16 piece (fp16's smallest subnormal is 2^-24) and is lost from every
// product and every G row the chain derives from it, which no later exact arithmetic can restore
// (edge_finite_6x8: rgb adjoints 2^40 below their sample's sigma adjoint, carried by the fixture's
// permutation weights into a dW column of their own, came out ~0.5 % wrong). k1 tests the head row
// as its pass splits it (column-scaled) and every hidden G row it produces (G_{L-2} .. G_0) against
// that floor; a step where any element fails is re-run on the bf16x6 split (fp32's exponent range per
// element) before the dW/db reduction, on the device, without a host round trip (fused_train_step).
// The default precision only (an explicit LNERF_MFMA_F16X3 asks for fp16x3 exactly). On the cfg3
// bench batch the smallest G element sits at 2^-16.1 after its row's shift (hidden rows) and 2^-4.7
// (head rows; scripts/xcheck_study.py), eight binades and more above the floor.
constexpr int kGuardExp = -24;
// GUARD: A/B knob (0: no floor test in k1 and no gated re-run; the round-5 behaviour)
#ifndef LNERF_GUARD
#define LNERF_GUARD 1
#endif

bool fused_supported(const lnerf_mlp& mlp, int rays, int S, int input_mode, const char** why,
                     bool head_fit = false);
// train = false sizes the forward-only (render) workspace: packed weights + loss partials.
// dw_grid: the dW kernel's workgroup budget (0 = default_dw_grid; LNERF_OPT_DW_GRID).
size_t fused_workspace_bytes(const lnerf_mlp& mlp, int rays, int S, bool train = true, int dw_grid = 0);
// flags select the MFMA precision and the workgroup shape (LNERF_MFMA_*, LNERF_K16_W4; lnerf.h)
void fused_plan(FusedPlan& p, const lnerf_mlp& mlp, const lnerf_batch& b, void* ws_base, int flags,
                bool train = true, int dw_grid = 0);
// ev: nullable array of 7 events recorded between the step's kernels (LNERF_TIMING)
// px (nullable): the bf16x6 plan of the same batch on the same workspace, run gated on p.guard (the
// fp16x3 floor guard, kGuardExp)
void fused_train_step(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                      float seed, int flags, const lnerf_outputs& out, hipStream_t s,
                      hipEvent_t* ev, const FusedPlan* px = nullptr);
// ev: nullable array of events as fused_train_step's ([1]-[2] bracket the forward kernel)
void fused_render(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                  const lnerf_outputs& out, hipStream_t s, int flags, hipEvent_t* ev);
bool fused_render_uses_kr(const FusedPlan& p, int flags);
void dw16_launch(const FusedPlan& p, hipStream_t s);
// after a training k1: the batch loss (loss_total, out_loss) and the per-layer dW product shifts,
// in one launch (lnerf_dw16.hip)
void k1_reduce_launch(const FusedPlan& p, float* out_loss, hipStream_t s);
// k16 kernel entry points (lnerf_k16.hip)
void k16_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s);
void k16_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                bool want_grad, hipStream_t s);
// the last training k1's ReLU decisions as (L-1, R, 32) bytes (lnerf_ctx_relu_masks)
void k16_masks_launch(const FusedPlan& p, unsigned char* out, hipStream_t s);
// kr, the forward-only bf16 render kernel (lnerf_render.hip): two 16-sample groups per wave
bool kr_supported(const FusedPlan& p);
int kr_num_wg(const FusedPlan& p);
void kr_launch(const FusedPlan& p, const lnerf_batch& b, const lnerf_outputs& out, hipStream_t s);

}  // namespace lnerf
