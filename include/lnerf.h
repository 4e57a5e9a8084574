/*
 * lnerf.h -- C ABI of libloma_nerf.so, the MI355X-native NeRF ray-marching engine.
 *
 * Two levels, both exported by the same library (see INTEGRATION.md for the bindings):
 *
 *  (1) loma-compat entry points with the exact signatures loma's C target generates for
 *      scripts/nerf.py and scripts/mlp_fit.py (codegen_c.py:8-30,47-57; reverse_diff.py:504-517).
 *      Arrays are nested host pointer tables (mlp_utils.py:33-118), exactly what ctypes passes.
 *      They gather into pinned memory, run the HIP kernels on the calling thread's stream and
 *      scatter the results back, with loma's semantics.
 *
 *  (2) the native batched API on device-resident, contiguous buffers (the throughput path).
 *
 * No torch or HIP types appear here: streams are passed as `void*` (a hipStream_t; NULL = the
 * device's default (null) stream, which is torch's default stream). Every entry point returns 0
 * on success / a negative error code, or (loma-compat float returns) NaN on failure; lnerf_last_error() describes it.
 */
#ifndef LNERF_H
#define LNERF_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LNERF_MAX_LAYERS 16

/* ------------------------------------------------------------------------------------------ */
/* (1) loma-compat ABI                                                                          */
/* ------------------------------------------------------------------------------------------ */

/* Replaces the loma-generated `nerf_evaluate_and_march` (scripts/nerf.py:1-304, bound at
 * train_nerf.py:212 and called at :325 and :616). Returns the sum-of-squares loss. */
float nerf_evaluate_and_march(float** layer_input, int layer_input_h, int layer_input_w,
                              float*** ws, float** bs, float** target_image, int target_image_h,
                              int target_image_w, int num_weights, int** weight_shapes,
                              int** bias_shapes, int** intermediate_output_shapes,
                              float*** intermediate_outputs, float*** img_sample_rgba_arr,
                              int num_samples, float** dists, float** alpha,
                              float** cumprod_alpha, float** weights_samples,
                              float** accumulated_color);

/* Replaces `grad_nerf_evaluate_and_march = rev_diff(nerf_evaluate_and_march)`
 * (scripts/nerf.py:306, bound at train_nerf.py:213, called at :395-478). Every In array is
 * followed by its adjoint buffer, every In int by an int* adjoint (never written), and the last
 * argument is the seed `_dreturn` (reverse_diff.py:504-517). Adjoint buffers are accumulated
 * into; primal buffers are left unchanged. */
void grad_nerf_evaluate_and_march(
    float** layer_input, float** d_layer_input, int layer_input_h, int* d_layer_input_h,
    int layer_input_w, int* d_layer_input_w, float*** ws, float*** d_ws, float** bs,
    float** d_bs, float** target_image, float** d_target_image, int target_image_h,
    int* d_target_image_h, int target_image_w, int* d_target_image_w, int num_weights,
    int* d_num_weights, int** weight_shapes, int** d_weight_shapes, int** bias_shapes,
    int** d_bias_shapes, int** intermediate_output_shapes, int** d_intermediate_output_shapes,
    float*** intermediate_outputs, float*** d_intermediate_outputs,
    float*** img_sample_rgba_arr, float*** d_img_sample_rgba_arr, int num_samples,
    int* d_num_samples, float** dists, float** d_dists, float** alpha, float** d_alpha,
    float** cumprod_alpha, float** d_cumprod_alpha, float** weights_samples,
    float** d_weights_samples, float** accumulated_color, float** d_accumulated_color,
    float _dreturn);

/* Replaces loma's `mlp_fit` (scripts/mlp_fit.py:1-147; fit_img.py:359,515-530). `layer_output`
 * is unused, as in the reference. */
float mlp_fit(float** layer_input, int layer_input_h, int layer_input_w, float** layer_output,
              float*** ws, float** bs, float** target_image, int target_image_h,
              int target_image_w, int num_weights, int** weight_shapes, int** bias_shapes,
              int** intermediate_output_shapes, float*** intermediate_outputs);

/* Replaces `grad_mlp_fit = rev_diff(mlp_fit)` (scripts/mlp_fit.py:174; fit_img.py:361,468-498). */
void grad_mlp_fit(float** layer_input, float** d_layer_input, int layer_input_h,
                  int* d_layer_input_h, int layer_input_w, int* d_layer_input_w,
                  float** layer_output, float** d_layer_output, float*** ws, float*** d_ws,
                  float** bs, float** d_bs, float** target_image, float** d_target_image,
                  int target_image_h, int* d_target_image_h, int target_image_w,
                  int* d_target_image_w, int num_weights, int* d_num_weights,
                  int** weight_shapes, int** d_weight_shapes, int** bias_shapes,
                  int** d_bias_shapes, int** intermediate_output_shapes,
                  int** d_intermediate_output_shapes, float*** intermediate_outputs,
                  float*** d_intermediate_outputs, float _dreturn);

/* Replaces loma's `mult_a_b` (scripts/mlp_fit.py:150-172; fit_img.py:360,370). */
void mult_a_b(float** a, int a_h, int a_w, float** b, int b_h, int b_w, float** c);

/* ------------------------------------------------------------------------------------------ */
/* (2) native batched API (device pointers)                                                    */
/* ------------------------------------------------------------------------------------------ */

typedef struct lnerf_ctx lnerf_ctx;

/* MLP shape. Weights use the reference's padded layout (mlp_utils.py:272-313): ws[l][k][j] at
 * ws[(l*w_k + k)*w_n + j], bs[l][j] at bs[l*w_n + j]; layer l maps k[l] -> n[l] features,
 * ReLU on hidden layers, head = sigmoid(rgb) + ReLU(sigma) (scripts/nerf.py:134-167). */
typedef struct {
    int num_layers;
    int k[LNERF_MAX_LAYERS];
    int n[LNERF_MAX_LAYERS];
    int w_k, w_n;
} lnerf_mlp;

enum {
    LNERF_INPUT_ENCODED = 0, /* x = layer_input, (rays*S, k[0]) float32 row-major          */
    LNERF_INPUT_POINTS = 1,  /* x = sample positions, (rays*S, 3) float32; the engine      */
                             /*     applies positional_encoding_3d (pos_encoding.py:38-69)  */
    LNERF_INPUT_RAYS = 2     /* x = rays, (rays, 6) float32 [origin xyz, direction xyz]; the */
                             /*     engine samples t = linspace(near, far, S), the points   */
                             /*     o + d t and dists = [diff(t), 1e8] in float64           */
                             /*     (train_nerf.py:289-306), then applies the encoding      */
};

/* One batch of rays; all pointers are device pointers. Sample r of ray i is row i*S + r
 * (train_nerf.py:327). */
typedef struct {
    int rays;
    int samples;         /* S */
    int input_mode;      /* LNERF_INPUT_* */
    int num_freqs;       /* F (POINTS mode; k[0] must equal 3 + 6F) */
    const float* x;
    const float* dists;  /* (rays, S) delta t, last = 1e8 in the reference (train_nerf.py:306); */
                         /* ignored (may be NULL) in RAYS mode                               */
    const float* target; /* (rays, 3) */
    float near_t, far_t; /* RAYS mode: sampling range (train_nerf.py: near 2, far 6)          */
} lnerf_batch;

enum {
    LNERF_SEED_CONST = 0,     /* gradients seeded with `seed`                                 */
    LNERF_SEED_LOSS = 1,      /* seeded with the batch loss itself (train_nerf.py:477)        */
    LNERF_ACCUMULATE = 2,     /* add into d_ws/d_bs (loma semantics) instead of overwriting   */
    LNERF_WANT_DX = 4,        /* also produce d_x (d_layer_input), ENCODED mode only          */
    LNERF_GENERIC = 8,        /* force the stage-by-stage loma-order kernels (no MFMA fusion) */
    LNERF_FAST = 16,          /* require the fused MFMA path (error if the shape is unsupported) */
    LNERF_TIMING = 32,        /* record per-kernel HIP events (read with lnerf_ctx_timings)   */
    LNERF_MFMA_F32 = 64,      /* removed in round 4 (the one-wave exact-f32 MFMA kernel): an
                                 error; exact fp32 arithmetic is LNERF_GENERIC                 */
    LNERF_MFMA_BF16 = 128,    /* fused path: plain bf16 operands, fp32 accumulate (one MFMA per
                                 product; reduced precision -- inference / config 5 render)   */
    LNERF_MFMA_F16X3 = 256,   /* fused path: the fp16x3 split, the fused path's default:
                                 x 2^e = hi + lo in fp16 with per-sample (k1) or per-sample
                                 balanced (k2) and per-layer weight exponent shifts, three fp16
                                 MFMAs per product, fp32 accumulate. Each product drops
                                 <= ~3 2^-22 of its operands' shifted magnitudes, i.e. relative to
                                 max|w| max|x| of the shift group (one sample's row of one layer),
                                 not to |w x| itself: an operand x scaled by 2^e keeps
                                 |x 2^e - hi - lo| <= 2^-22 |x 2^e| + 2^-25, so a value more than
                                 ~2^17 below its row's maximum loses bits to fp16's subnormals
                                 (e.g. a dW column whose G values sit 1e-9 below the row's other
                                 columns keeps ~2 % -- tests/test_gpu_edge.py fp16x3_dw_bound;
                                 LNERF_MFMA_BF16X6 has fp32's exponent range and no such limit).
                                 The head's weights carry a shift per output column and, in
                                 training, its dW runs on the bf16x6 split, so rgb and sigma
                                 adjoints far apart (delta = 1e8 rays) keep their own ranges.
                                 Training in fp16x3 keeps the activations it hands from the
                                 forward to the dW pass as int24 (x rounded to a multiple of
                                 2^-23 of its row's max|x|), inside the same row-relative bound;
                                 a row holding NaN/inf is marked and reaches dW as NaN.        */
    LNERF_MFMA_BF16X6 = 512,  /* fused path: the bf16x6 split (x = hi+mid+lo in bf16, six bf16
                                 MFMAs per product, dropped terms <= 2^-24 |w x|)              */
    LNERF_K32 = 2048,         /* removed in round 4 (it lost to k16): an error                 */
    LNERF_HEAD_FIT = 8192,    /* the mlp_fit head instead of the NeRF one (scripts/mlp_fit.py:
                                 120-145, fit_img.py:423-532): sigmoid on every output channel,
                                 loss = sum over rows x outputs of (sigmoid(z) - target)^2, no
                                 compositing. samples must be 1 (a "ray" is one row of the
                                 image), input ENCODED (rows, k[0]), target (rows, n_out) with
                                 1 <= n_out <= 4, dists unused; acc_color receives the sigmoid
                                 outputs (rows, n_out) and d_target (rows, n_out). Runs on k16
                                 in fp16x3 or bf16 only (LNERF_GENERIC / LNERF_MFMA_BF16X6 are
                                 errors).                                                      */
    LNERF_K16_W4 = 4096,      /* fused path: k16 on 4-wave, 64-sample workgroups (two per CU)
                                 instead of 8-wave, 128-sample ones (samples <= 64, fp16x3 or
                                 plain bf16, else an error; A/B -- measured slower at cfg3)     */
    LNERF_RENDER_K16 = 16384, /* lnerf_render in plain bf16: k16's forward (one 16-sample group
                                 per wave) instead of kr (lnerf_render.hip: two groups per wave,
                                 each weight fragment read from LDS feeds both; A/B)           */
    LNERF_ONE_WAVE = 1024     /* removed in round 4 (the one-wave-per-SIMD kernel pair): an error.
                                 At most one LNERF_MFMA_* precision flag may be set; any fused-
                                 path flag (LNERF_MFMA_*, LNERF_K16_W4) on a shape the fused path
                                 cannot run (a head over 16 outputs, samples over 128) is an
                                 error, as is LNERF_GENERIC together with one.                  */
};

/* Engine options (lnerf_ctx_set_option). */
enum {
    LNERF_OPT_DW_GRID = 1     /* dW kernel workgroups per step (16..4096; 0 = the default: 512 from
                                 65 536 sample rows up, samples / 128 below, at least 256)       */
};

/* Optional outputs (device pointers; any may be NULL). */
typedef struct {
    float* loss;         /* 1 float                                     */
    float* acc_color;    /* (rays, 3)                                   */
    float* d_ws;         /* (L, w_k, w_n) padded                        */
    float* d_bs;         /* (L, w_n)                                    */
    float* d_x;          /* (rays*S, k[0]) with LNERF_WANT_DX           */
    float* d_dists;      /* (rays, S)                                   */
    float* d_target;     /* (rays, 3)                                   */
} lnerf_outputs;

const char* lnerf_last_error(void);
const char* lnerf_version(void);
/* Build fingerprint: a bitmask of the kernel objects' compile-time knobs (k1 / k2 scheduling, the
   int24 slab format, the phase-profiling build) that differ from the product build. 0 for the
   shipped library; A/B variants (Makefile defvariant / dwdefvariant) report what they moved.
   No reference counterpart (engine-only). */
unsigned lnerf_build_knobs(void);

int lnerf_ctx_create(lnerf_ctx** out, int device);
void lnerf_ctx_destroy(lnerf_ctx* ctx);
/* Bytes of device workspace a train step needs (activation slabs, partials). */
size_t lnerf_workspace_bytes(const lnerf_mlp* mlp, int rays, int samples);

/* Forward (PE + MLP + compositing + loss) and reverse pass over the MLP weights: the work of one
 * nerf_evaluate_and_march + grad_nerf_evaluate_and_march pair on the whole batch. */
int lnerf_train_step(lnerf_ctx* ctx, const lnerf_mlp* mlp, const float* ws, const float* bs,
                     const lnerf_batch* batch, float seed, int flags, const lnerf_outputs* out,
                     void* stream);

/* get_rays (train_nerf.py:23-62) on the device: the width x width pixel grid of
 * linspace(0, 1, width) (the reference uses `width` for both axes), directions
 * [(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -1] rotated by c2w[:3,:3], origins
 * c2w[:3,3], computed in float64 and stored as float32 rays (width*width, 6) = [o, d], ready for
 * LNERF_INPUT_RAYS. K (3x3) and c2w (3x4 or the top of a 4x4, row-major) are host arrays. */
int lnerf_get_rays(int width, const double* K, const double* c2w, float* rays, void* stream);

/* Forward only (eval render, train_nerf.py:616-661): acc_color and, if target != NULL, loss. */
int lnerf_render(lnerf_ctx* ctx, const lnerf_mlp* mlp, const float* ws, const float* bs,
                 const lnerf_batch* batch, int flags, const lnerf_outputs* out, void* stream);

/* Per-kernel times (ms) of the last LNERF_TIMING step or render on `ctx`, measured with HIP events
 * on its stream: [0] weight pack, [1] fused fwd+reverse-chain kernel (a render: the forward
 * kernel), [2] loss reduce, [3] dW kernel, [4] dW/db reduce, [5] whole step (0 for the kernels a
 * render does not run). Synchronises on the step. Returns the number
 * of values written (0 if no timed step ran on the fused path). */
int lnerf_ctx_timings(lnerf_ctx* ctx, float* ms_out, int n);

/* Which kernels the last lnerf_train_step / lnerf_render on `ctx` ran (for tests and benches):
 * a mask of LNERF_PATH_* bits, the operand planes of the fused MFMAs in bits 8-9 (3 = bf16x6
 * split, 2 = fp16x3 split, 1 = plain bf16, 0 = the generic path), or a negative
 * error code. 0 if no step has run. */
enum {
    LNERF_PATH_GENERIC = 1,   /* the loma-order stage-by-stage kernels                        */
    LNERF_PATH_FUSED = 2,     /* the fused MFMA step (k16, + dw16 when training)              */
    LNERF_PATH_K16 = 4,       /* fused kernel on wave pairs (k16_fwd_bwd_kernel)              */
    LNERF_PATH_DW16 = 8,      /* dW kernel on wave pairs (dw16_kernel)                        */
    LNERF_PATH_K32 = 16,      /* reserved (k32, removed in round 4)                           */
    LNERF_PATH_K16_W4 = 32,   /* k16 on 4-wave, 64-sample workgroups (two per CU)             */
    LNERF_PATH_KR = 64,       /* the render ran kr (lnerf_render.hip), not k16's forward      */
    LNERF_PATH_A24 = 128      /* training kept the activation slabs as int24 (fp16x3)         */
};
int lnerf_ctx_last_path(lnerf_ctx* ctx);

/* The hidden-layer ReLU decisions of the last training step on `ctx` (k16 path only, for parity
 * tests: scripts/nerf.py:141-144 takes z > 0): `out` (device) receives (L-1) x R x 32 bytes, bit
 * f % 8 of byte [(l R + r) 32 + f / 8] set when feature f of hidden layer l at sample row r was
 * positive. Valid until the next call on `ctx`; an error after any other kind of call. */
int lnerf_ctx_relu_masks(lnerf_ctx* ctx, unsigned char* out, size_t out_bytes, void* stream);

/* The exceptional rows of the last training step on `ctx` (k16 + dw16 with the fp16x3 split): the
 * sample rows, summed over the layers, that dw16 multiplied on the bf16x6 split instead of the
 * fp16x3 one because fp16's range at their balanced shift could not keep every nonzero element to
 * 2^-17 (every ray's last sample always is one; lnerf_internal.h kXrowT); *last_samples (nullable)
 * receives how many of them were rays' last samples. 0 for the other precisions. Synchronises the
 * device. An extension (no loma counterpart). */
int lnerf_ctx_exceptional_rows(lnerf_ctx* ctx, long long* rows, long long* last_samples);

/* The fp16x3 floor guard of the last training step on `ctx`: *fired = 1 if k1 met a hidden-layer
 * gradient element below what the fp16x3 split can carry (more than ~2^37 below its row's maximum,
 * lnerf_internal.h kGuardExp) and the step was therefore re-run on the device on the bf16x6 split
 * (every output of the step comes from that re-run), 0 if not, -1 if the last call on `ctx` had no
 * guard (a training step with an explicit precision flag, the generic path, LNERF_HEAD_FIT or
 * LNERF_K16_W4; a render). Synchronises the device. An extension (no loma counterpart). */
int lnerf_ctx_guard_fired(lnerf_ctx* ctx, int* fired);

/* Sets an engine option (LNERF_OPT_*) for later steps on `ctx`. Returns 0, or a negative code for
 * an unknown option or an out-of-range value. */
int lnerf_ctx_set_option(lnerf_ctx* ctx, int option, int value);

/* buf[i] *= *scale for i < n (device pointers): applies a loss seed after an all-reduce of
 * unit-seeded gradients (the data-parallel path). */
int lnerf_scale_by_device_scalar(float* buf, size_t n, const float* scale, void* stream);

/* The reference's Adam (train_nerf.py:133-161) on device: params -= lr_t m_hat/(sqrt(v_hat)+eps).
 * `t` is the 1-based step count after the increment. */
int lnerf_adam_update(float* params, const float* grads, float* m, float* v, size_t n, int t,
                      float lr, float beta1, float beta2, float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LNERF_H */
