/*
 * nerf_oracle.h -- TEST INFRASTRUCTURE ONLY (the CPU oracle / checker).
 *
 * Plain-C restatement of the reference's NeRF hot path:
 *   forward  = scripts/nerf.py:1-304  (nerf_evaluate_and_march)
 *   backward = scripts/nerf.py:306    (grad_nerf_evaluate_and_march = rev_diff(...)),
 *              i.e. the reverse sweep that loma_public/reverse_diff.py:492-1016 emits.
 * and of scripts/mlp_fit.py:1-147,150-172 (mlp_fit, mult_a_b) + grad_mlp_fit (:174).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (loma-nerf_amd/) never links or calls it.
 *
 * PARITY STATUS: the reference ships no golden vectors for this path and building/running the
 * loma compiler (or code it generates) was denied in SURVEY.md §8c, so this restatement is
 * "parity unpinned" against the reference binary. It is cross-validated independently by a
 * numpy float64 restatement, torch autograd and finite differences (tests/test_oracle.py), and
 * pinned by the one known-answer test the reference holds (fit_img.py:363-374, mult_a_b).
 *
 * Buffers are flat row-major with explicit extents (the nested pointer tables of the loma ABI
 * gathered into rectangles). Loop bounds are exactly the reference's.
 */
#ifndef LNERF_ORACLE_H
#define LNERF_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_LAYERS 16

typedef struct {
    int num_weights;              /* L                                  nerf.py:10 */
    int layer_input_h;            /* rows of layer_input                nerf.py:3  */
    int layer_input_w;            /* cols of layer_input                nerf.py:4  */
    int target_image_h;           /* rays (img_size)                    nerf.py:7  */
    int target_image_w;           /* colour channels in the loss        nerf.py:8  */
    int num_samples;              /* S                                  nerf.py:16 */
    int weight_shapes[ORACLE_MAX_LAYERS][2];              /* nerf.py:11 */
    int bias_shapes[ORACLE_MAX_LAYERS][2];                /* nerf.py:12 (never read) */
    int intermediate_output_shapes[ORACLE_MAX_LAYERS][2]; /* nerf.py:13 */
    /* extents (strides) of the flat buffers */
    int x_cols;                   /* layer_input[i][k] = X[i*x_cols + k]            */
    int w_k, w_n;                 /* ws[l][k][j] = W[(l*w_k + k)*w_n + j]            */
    int b_n;                      /* bs[l][j]    = B[l*b_n + j]                      */
    int io_rows, io_cols;         /* io[l][i][j] = IO[(l*io_rows + i)*io_cols + j]   */
    int t_cols;                   /* target[i][c] = T[i*t_cols + c]                  */
    int acc_cols;                 /* accumulated_color[i][c] = C[i*acc_cols + c]     */
} oracle_dims;

/* nerf_evaluate_and_march (scripts/nerf.py:1-304). Mutates io/rgba/alpha/cumprod/wsamp/acc in
 * place exactly like the loma C target and returns the loss. rgba is (h, S, 4); dists/alpha/
 * cumprod/wsamp are (h, S). */
float oracle_nerf_forward(const oracle_dims* d, const float* X, const float* W, const float* B,
                          const float* T, float* IO, float* rgba, const float* dists,
                          float* alpha, float* cumprod, float* wsamp, float* acc);

/* grad_nerf_evaluate_and_march: the exact reverse sweep of the forward above, seeded with
 * `dreturn`. Every d* buffer is accumulated into (its incoming value acts as the cotangent of the
 * array's final state, as in loma's reverse mode); primal buffers are left unchanged (loma restores
 * them from its tape, reverse_diff.py:597-603). */
void oracle_nerf_grad(const oracle_dims* d,
                      const float* X, float* dX, const float* W, float* dW, const float* B,
                      float* dB, const float* T, float* dT, const float* IO, float* dIO,
                      const float* rgba, float* drgba, const float* dists, float* ddists,
                      const float* alpha, float* dalpha, const float* cumprod, float* dcumprod,
                      const float* wsamp, float* dwsamp, const float* acc, float* dacc,
                      float dreturn);

/* mlp_fit (scripts/mlp_fit.py:1-147): same MLP, sigmoid on every output channel of the last
 * layer, sum-of-squares against target over (target_image_h, target_image_w) of io[L-1]. Uses
 * the same oracle_dims (num_samples, acc_cols unused). */
float oracle_mlp_fit_forward(const oracle_dims* d, const float* X, const float* W, const float* B,
                             const float* T, float* IO);
void oracle_mlp_fit_grad(const oracle_dims* d, const float* X, float* dX, const float* W,
                         float* dW, const float* B, float* dB, const float* T, float* dT,
                         const float* IO, float* dIO, float dreturn);

/* mult_a_b (scripts/mlp_fit.py:150-172): c[i][j] += a[i][k] * b[k][j]. */
void oracle_mult_a_b(const float* a, int a_h, int a_w, int a_cols, const float* b, int b_h,
                     int b_w, int b_cols, float* c, int c_cols);

/* positional_encoding_3d (pos_encoding.py:38-69): pts (n, 3) float64 -> out (n, 3 + 6F) float32,
 * block-major [x, sin(2^0 x), cos(2^0 x), ..., sin(2^{F-1} x), cos(2^{F-1} x)], computed in
 * float64 and rounded to float32 once. */
void oracle_positional_encoding_3d(const double* pts, long n, int num_functions, float* out);

/* CPU baseline: the standard-semantics training step (zero-initialised buffers, seed = the loss
 * itself as train_nerf.py:477 passes it) over `rays` rays, i.e. forward + grad of every chunk,
 * using `threads` OpenMP threads over rays (1 = the scalar loma-order path). dW/dB accumulate. */
float oracle_train_step(int L, const int* k_dims, const int* n_dims, int w_k, int w_n,
                        const float* X, int rays, int S, const float* dists, const float* T,
                        const float* W, const float* B, float* dW, float* dB, int threads);

/* The two loma entry points above behind the reference's own nested-pointer ABI (SURVEY.md §8b;
 * nerf_oracle_abi.c): gather the touched rows, run the flat oracle, scatter back. For timing the
 * reference's per-chunk call pair on the CPU through the same tables the GPU library gets. */
float oracle_abi_nerf_evaluate_and_march(float** layer_input, int layer_input_h, int layer_input_w,
                                         float*** ws, float** bs, float** target_image, int target_image_h,
                                         int target_image_w, int num_weights, int** weight_shapes,
                                         int** bias_shapes, int** intermediate_output_shapes,
                                         float*** intermediate_outputs, float*** img_sample_rgba_arr,
                                         int num_samples, float** dists, float** alpha, float** cumprod_alpha,
                                         float** weights_samples, float** accumulated_color);
void oracle_abi_grad_nerf_evaluate_and_march(
    float** layer_input, float** d_layer_input, int layer_input_h, int* d_h, int layer_input_w, int* d_w,
    float*** ws, float*** d_ws, float** bs, float** d_bs, float** target_image, float** d_target,
    int target_image_h, int* d_th, int target_image_w, int* d_tw, int num_weights, int* d_nw,
    int** weight_shapes, int** d_wsh, int** bias_shapes, int** d_bsh, int** intermediate_output_shapes,
    int** d_ios, float*** intermediate_outputs, float*** d_io, float*** img_sample_rgba_arr, float*** d_rgba,
    int num_samples, int* d_ns, float** dists, float** d_dists, float** alpha, float** d_alpha,
    float** cumprod_alpha, float** d_cumprod, float** weights_samples, float** d_wsamp,
    float** accumulated_color, float** d_acc, float dreturn);

#ifdef __cplusplus
}
#endif
#endif
