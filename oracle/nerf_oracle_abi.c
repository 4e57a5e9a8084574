/*
 * nerf_oracle_abi.c -- TEST INFRASTRUCTURE ONLY (the CPU oracle / checker).
 *
 * The C oracle behind the reference's own nested-pointer loma ABI (codegen_c.py:8-30,47-57;
 * reverse_diff.py:504-517), so that a benchmark can time the reference's per-chunk
 * call pair (train_nerf.py:325-478) on the CPU through exactly the pointer tables it hands the GPU
 * library: gather the touched rows into flat buffers, run oracle_nerf_forward / oracle_nerf_grad,
 * scatter the mutated buffers back. The extents are the reference's loop bounds (SURVEY.md §8a row
 * a4); this is an independent restatement of them, not the product's gather code.
 *
 * Only tests/ and scripts/bench_compat.py's CPU leg call this; the product never links it.
 */
#include <stdlib.h>
#include <string.h>

#include "nerf_oracle.h"

typedef struct {
    oracle_dims d;
    int K[ORACLE_MAX_LAYERS];     /* contraction length of layer l */
    int rows[ORACLE_MAX_LAYERS];  /* touched rows of io[l] */
    int cols[ORACLE_MAX_LAYERS];  /* touched cols of io[l] */
    int ncols[ORACLE_MAX_LAYERS]; /* weight_shapes[l][1] */
} abi_shape;

static int imax(int a, int b) { return a > b ? a : b; }

/* nerf.py:67-170 loop bounds: layer 0 reads layer_input (rows in_h, K in_w), layer l >= 1 reads
 * io[l-1] (rows ios[l-1][0], K ios[l-1][1]); bias/activation touch ios[l]; the reshape copy reads
 * io[L-1] rows th*S x 4 (nerf.py:176-191). */
static int make_shape(abi_shape* c, int in_h, int in_w, int th, int tw, int L, int** ws_shape,
                      int** bs_shape, int** ios, int S) {
    if (L < 1 || L > ORACLE_MAX_LAYERS) return -1;
    memset(c, 0, sizeof(*c));
    oracle_dims* d = &c->d;
    d->num_weights = L;
    d->layer_input_h = in_h;
    d->layer_input_w = in_w;
    d->target_image_h = th;
    d->target_image_w = tw;
    d->num_samples = S;
    int w_k = 1, w_n = 1, io_r = 1, io_c = 4;
    for (int l = 0; l < L; ++l) {
        d->weight_shapes[l][0] = ws_shape[l][0];
        d->weight_shapes[l][1] = ws_shape[l][1];
        d->bias_shapes[l][0] = bs_shape[l][0];
        d->bias_shapes[l][1] = bs_shape[l][1];
        d->intermediate_output_shapes[l][0] = ios[l][0];
        d->intermediate_output_shapes[l][1] = ios[l][1];
        c->ncols[l] = ws_shape[l][1];
        c->K[l] = l == 0 ? in_w : ios[l - 1][1];
        int r = imax(l == 0 ? in_h : ios[l - 1][0], ios[l][0]);
        int cc = imax(ws_shape[l][1], ios[l][1]);
        if (l == L - 1) {
            r = imax(r, th * S);
            cc = imax(cc, 4);
        }
        c->rows[l] = r;
        c->cols[l] = cc;
        w_k = imax(w_k, c->K[l]);
        w_n = imax(w_n, imax(ws_shape[l][1], ios[l][1]));
        io_r = imax(io_r, r);
        io_c = imax(io_c, cc);
    }
    d->x_cols = imax(in_w, 1);
    d->w_k = w_k;
    d->w_n = w_n;
    d->b_n = w_n;
    d->io_rows = io_r;
    d->io_cols = io_c;
    d->t_cols = imax(tw, 1);
    d->acc_cols = imax(tw, 3);
    return 0;
}

static void g2(float* dst, float** src, int rows, int cols, int ld) {
    for (int i = 0; i < rows; ++i) memcpy(dst + (size_t)i * ld, src[i], sizeof(float) * (size_t)cols);
}
static void s2(float** dst, const float* src, int rows, int cols, int ld) {
    for (int i = 0; i < rows; ++i) memcpy(dst[i], src + (size_t)i * ld, sizeof(float) * (size_t)cols);
}
static void g3(float* dst, float*** src, int d0, int d1, int d2) {
    for (int i = 0; i < d0; ++i)
        for (int j = 0; j < d1; ++j) memcpy(dst + ((size_t)i * d1 + j) * d2, src[i][j], sizeof(float) * (size_t)d2);
}
static void s3(float*** dst, const float* src, int d0, int d1, int d2) {
    for (int i = 0; i < d0; ++i)
        for (int j = 0; j < d1; ++j) memcpy(dst[i][j], src + ((size_t)i * d1 + j) * d2, sizeof(float) * (size_t)d2);
}
static void gw(float* dst, float*** ws, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        for (int k = 0; k < c->K[l]; ++k)
            memcpy(dst + ((size_t)l * c->d.w_k + k) * c->d.w_n, ws[l][k], sizeof(float) * (size_t)c->ncols[l]);
}
static void sw(float*** ws, const float* src, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        for (int k = 0; k < c->K[l]; ++k)
            memcpy(ws[l][k], src + ((size_t)l * c->d.w_k + k) * c->d.w_n, sizeof(float) * (size_t)c->ncols[l]);
}
static void gb(float* dst, float** bs, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        memcpy(dst + (size_t)l * c->d.b_n, bs[l], sizeof(float) * (size_t)c->d.intermediate_output_shapes[l][1]);
}
static void sb(float** bs, const float* src, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        memcpy(bs[l], src + (size_t)l * c->d.b_n, sizeof(float) * (size_t)c->d.intermediate_output_shapes[l][1]);
}
static void gio(float* dst, float*** io, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        for (int i = 0; i < c->rows[l]; ++i)
            memcpy(dst + ((size_t)l * c->d.io_rows + i) * c->d.io_cols, io[l][i], sizeof(float) * (size_t)c->cols[l]);
}
static void sio(float*** io, const float* src, const abi_shape* c) {
    for (int l = 0; l < c->d.num_weights; ++l)
        for (int i = 0; i < c->rows[l]; ++i)
            memcpy(io[l][i], src + ((size_t)l * c->d.io_rows + i) * c->d.io_cols, sizeof(float) * (size_t)c->cols[l]);
}

typedef struct {
    float *X, *W, *B, *T, *IO, *rgba, *dists, *alpha, *cp, *wsamp, *acc;
} flat;

static float* zalloc(size_t n) { return (float*)calloc(n ? n : 1, sizeof(float)); }

static void flat_alloc(flat* f, const abi_shape* c) {
    const oracle_dims* d = &c->d;
    const size_t nS = (size_t)d->target_image_h * d->num_samples;
    f->X = zalloc((size_t)d->layer_input_h * d->x_cols);
    f->W = zalloc((size_t)d->num_weights * d->w_k * d->w_n);
    f->B = zalloc((size_t)d->num_weights * d->b_n);
    f->T = zalloc((size_t)d->target_image_h * d->t_cols);
    f->IO = zalloc((size_t)d->num_weights * d->io_rows * d->io_cols);
    f->rgba = zalloc(nS * 4);
    f->dists = zalloc(nS);
    f->alpha = zalloc(nS);
    f->cp = zalloc(nS);
    f->wsamp = zalloc(nS);
    f->acc = zalloc((size_t)d->target_image_h * d->acc_cols);
}
static void flat_free(flat* f) {
    free(f->X), free(f->W), free(f->B), free(f->T), free(f->IO), free(f->rgba), free(f->dists);
    free(f->alpha), free(f->cp), free(f->wsamp), free(f->acc);
}

/* gather every array of one call (primals, or with the adjoint tables the adjoints) */
static void gather_primal(flat* f, const abi_shape* c, float** X, float*** ws, float** bs, float** T,
                          float*** io, float*** rgba, float** dists, float** alpha, float** cp,
                          float** wsamp, float** acc) {
    const oracle_dims* d = &c->d;
    const int th = d->target_image_h, S = d->num_samples;
    if (X) g2(f->X, X, d->layer_input_h, d->layer_input_w, d->x_cols);
    gw(f->W, ws, c);
    gb(f->B, bs, c);
    g2(f->T, T, th, d->target_image_w, d->t_cols);
    gio(f->IO, io, c);
    g3(f->rgba, rgba, th, S, 4);
    g2(f->dists, dists, th, S, S);
    g2(f->alpha, alpha, th, S, S);
    g2(f->cp, cp, th, S, S);
    g2(f->wsamp, wsamp, th, S, S);
    g2(f->acc, acc, th, 3, d->acc_cols);
}

float oracle_abi_nerf_evaluate_and_march(float** layer_input, int layer_input_h, int layer_input_w,
                                         float*** ws, float** bs, float** target_image, int target_image_h,
                                         int target_image_w, int num_weights, int** weight_shapes,
                                         int** bias_shapes, int** intermediate_output_shapes,
                                         float*** intermediate_outputs, float*** img_sample_rgba_arr,
                                         int num_samples, float** dists, float** alpha, float** cumprod_alpha,
                                         float** weights_samples, float** accumulated_color) {
    abi_shape c;
    if (make_shape(&c, layer_input_h, layer_input_w, target_image_h, target_image_w, num_weights,
                   weight_shapes, bias_shapes, intermediate_output_shapes, num_samples))
        return 0.0f / 0.0f;
    flat f;
    flat_alloc(&f, &c);
    gather_primal(&f, &c, layer_input, ws, bs, target_image, intermediate_outputs, img_sample_rgba_arr, dists,
                  alpha, cumprod_alpha, weights_samples, accumulated_color);
    const float loss = oracle_nerf_forward(&c.d, f.X, f.W, f.B, f.T, f.IO, f.rgba, f.dists, f.alpha, f.cp,
                                           f.wsamp, f.acc);
    const int th = target_image_h, S = num_samples;
    sio(intermediate_outputs, f.IO, &c);
    s3(img_sample_rgba_arr, f.rgba, th, S, 4);
    s2(alpha, f.alpha, th, S, S);
    s2(cumprod_alpha, f.cp, th, S, S);
    s2(weights_samples, f.wsamp, th, S, S);
    s2(accumulated_color, f.acc, th, 3, c.d.acc_cols);
    flat_free(&f);
    return loss;
}

void oracle_abi_grad_nerf_evaluate_and_march(
    float** layer_input, float** d_layer_input, int layer_input_h, int* d_h, int layer_input_w, int* d_w,
    float*** ws, float*** d_ws, float** bs, float** d_bs, float** target_image, float** d_target,
    int target_image_h, int* d_th, int target_image_w, int* d_tw, int num_weights, int* d_nw,
    int** weight_shapes, int** d_wsh, int** bias_shapes, int** d_bsh, int** intermediate_output_shapes,
    int** d_ios, float*** intermediate_outputs, float*** d_io, float*** img_sample_rgba_arr, float*** d_rgba,
    int num_samples, int* d_ns, float** dists, float** d_dists, float** alpha, float** d_alpha,
    float** cumprod_alpha, float** d_cumprod, float** weights_samples, float** d_wsamp,
    float** accumulated_color, float** d_acc, float dreturn) {
    (void)d_h, (void)d_w, (void)d_th, (void)d_tw, (void)d_nw, (void)d_wsh, (void)d_bsh, (void)d_ios, (void)d_ns;
    abi_shape c;
    if (make_shape(&c, layer_input_h, layer_input_w, target_image_h, target_image_w, num_weights,
                   weight_shapes, bias_shapes, intermediate_output_shapes, num_samples))
        return;
    flat p, a;
    flat_alloc(&p, &c);
    flat_alloc(&a, &c);
    gather_primal(&p, &c, layer_input, ws, bs, target_image, intermediate_outputs, img_sample_rgba_arr, dists,
                  alpha, cumprod_alpha, weights_samples, accumulated_color);
    gather_primal(&a, &c, d_layer_input, d_ws, d_bs, d_target, d_io, d_rgba, d_dists, d_alpha, d_cumprod,
                  d_wsamp, d_acc);
    oracle_nerf_grad(&c.d, p.X, d_layer_input ? a.X : NULL, p.W, a.W, p.B, a.B, p.T, a.T, p.IO, a.IO, p.rgba, a.rgba, p.dists, a.dists,
                     p.alpha, a.alpha, p.cp, a.cp, p.wsamp, a.wsamp, p.acc, a.acc, dreturn);
    const oracle_dims* d = &c.d;
    const int th = target_image_h, S = num_samples;
    if (d_layer_input) s2(d_layer_input, a.X, d->layer_input_h, d->layer_input_w, d->x_cols);
    sw(d_ws, a.W, &c);
    sb(d_bs, a.B, &c);
    s2(d_target, a.T, th, target_image_w, d->t_cols);
    sio(d_io, a.IO, &c);
    s3(d_rgba, a.rgba, th, S, 4);
    s2(d_dists, a.dists, th, S, S);
    s2(d_alpha, a.alpha, th, S, S);
    s2(d_cumprod, a.cp, th, S, S);
    s2(d_wsamp, a.wsamp, th, S, S);
    s2(d_acc, a.acc, th, 3, d->acc_cols);
    flat_free(&p);
    flat_free(&a);
}
