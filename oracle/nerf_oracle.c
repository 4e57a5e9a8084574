/*
 * nerf_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference NeRF hot path.
 * See nerf_oracle.h for scope and parity status ("parity unpinned" vs the loma .so; pinned by
 * independent restatements + the mult_a_b known answer).
 *
 * Float semantics follow loma's C target (loma_public/codegen_c.py): every local is fp32,
 * literals are (float)(lit) (codegen_c.py:165-166), exp -> expf (:212-213), unary minus is
 * 0 - x (parser.py:257-259), int literals in float context are int2float casts
 * (type_inference.py:143-145). Built with -O2 -ffp-contract=off, which is what gcc -O2 on
 * x86-64 (compiler.py:154) produces for this code (no FMA in the baseline ISA).
 *
 * The reverse sweep restates, statement by statement, what reverse_diff.py emits:
 *   assignment  x = f(...)  ->  adj_i = df/dargs * d_x ; d_x = 0 ; d_args += adj_i
 *                               (mutate_assign :576-616, with primal restored first :597-603)
 *   loops run backwards (mutate_while :673-696), if/else re-evaluates its condition on the
 *   current (not yet restored) primal (mutate_ifelse :618-625).
 * Loop orders below are therefore all "descending" as in the generated code.
 */
#include "nerf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IO_AT(d, A, l, i, j) (A)[((size_t)(l) * (d)->io_rows + (i)) * (d)->io_cols + (j)]
#define W_AT(d, A, l, k, j) (A)[((size_t)(l) * (d)->w_k + (k)) * (d)->w_n + (j)]
#define B_AT(d, A, l, j) (A)[(size_t)(l) * (d)->b_n + (j)]
#define X_AT(d, A, i, k) (A)[(size_t)(i) * (d)->x_cols + (k)]

static size_t io_elems(const oracle_dims* d) {
    return (size_t)d->num_weights * d->io_rows * d->io_cols;
}

/* ---- MLP forward: scripts/nerf.py:67-170 (and mlp_fit.py:39-135 with all-sigmoid head) ---- */
static void mlp_forward(const oracle_dims* d, const float* X, const float* W, const float* B,
                        float* IO, float* zpre /* nullable: IO snapshot after bias */,
                        int nerf_head) {
    const int L = d->num_weights;
    const int (*ios)[2] = d->intermediate_output_shapes;
    for (int l = 0; l < L; ++l) {
        if (l == 0) {
            /* nerf.py:81-89 */
            for (int i = 0; i < d->layer_input_h; ++i)
                for (int j = 0; j < d->weight_shapes[0][1]; ++j)
                    for (int k = 0; k < d->layer_input_w; ++k)
                        IO_AT(d, IO, 0, i, j) = IO_AT(d, IO, 0, i, j) + X_AT(d, X, i, k) * W_AT(d, W, 0, k, j);
        } else {
            /* nerf.py:108-116 */
            for (int i = 0; i < ios[l - 1][0]; ++i)
                for (int j = 0; j < d->weight_shapes[l][1]; ++j)
                    for (int k = 0; k < ios[l - 1][1]; ++k)
                        IO_AT(d, IO, l, i, j) = IO_AT(d, IO, l, i, j) + IO_AT(d, IO, l - 1, i, k) * W_AT(d, W, l, k, j);
        }
        /* bias: nerf.py:95-100 / :122-127 */
        for (int i = 0; i < ios[l][0]; ++i)
            for (int j = 0; j < ios[l][1]; ++j)
                IO_AT(d, IO, l, i, j) = IO_AT(d, IO, l, i, j) + B_AT(d, B, l, j);
        if (zpre) {
            for (int i = 0; i < d->io_rows; ++i)
                for (int j = 0; j < d->io_cols; ++j)
                    IO_AT(d, zpre, l, i, j) = IO_AT(d, IO, l, i, j);
        }
        if (l < L - 1) {
            /* ReLU nerf.py:138-146 */
            for (int i = 0; i < ios[l][0]; ++i)
                for (int j = 0; j < ios[l][1]; ++j) {
                    float v = IO_AT(d, IO, l, i, j);
                    IO_AT(d, IO, l, i, j) = (v > (float)0) ? v : (float)0;
                }
        } else {
            /* head nerf.py:153-167 (channel 3 ReLU, others sigmoid); mlp_fit.py:127-132 (all sigmoid) */
            for (int i = 0; i < ios[l][0]; ++i)
                for (int j = 0; j < ios[l][1]; ++j) {
                    float v = IO_AT(d, IO, l, i, j);
                    if (nerf_head && j == 3) {
                        IO_AT(d, IO, l, i, j) = (v > (float)0) ? v : (float)0;
                    } else {
                        IO_AT(d, IO, l, i, j) = (float)1 / ((float)1 + expf((float)0 - v));
                    }
                }
        }
    }
}

/* ---- MLP reverse: reverse of nerf.py:67-170 ----
 * IOf = final (post-activation) io state, zpre = io right after the bias stage. dIO holds the
 * adjoints accumulated by the stages that consumed io[L-1] (compositing or mlp_fit loss). */
static void mlp_reverse(const oracle_dims* d, const float* X, float* dX, const float* W,
                        float* dW, float* dB, const float* IOf, const float* zpre, float* dIO,
                        int nerf_head) {
    const int L = d->num_weights;
    const int (*ios)[2] = d->intermediate_output_shapes;
    for (int l = L - 1; l >= 0; --l) {
        /* activation reverse (the forward's last statement of the layer) */
        for (int i = ios[l][0] - 1; i >= 0; --i)
            for (int j = ios[l][1] - 1; j >= 0; --j) {
                float post = IO_AT(d, IOf, l, i, j);
                int relu = (l < L - 1) || (nerf_head && j == 3);
                if (relu) {
                    /* if (io > 0) io = io else io = 0; condition on the current (post) value */
                    if (post > (float)0) {
                        float adj = IO_AT(d, dIO, l, i, j);
                        IO_AT(d, dIO, l, i, j) = (float)0.0;
                        IO_AT(d, dIO, l, i, j) += adj;
                    } else {
                        IO_AT(d, dIO, l, i, j) = (float)0.0;
                    }
                } else {
                    /* io = 1 / (1 + exp(0 - io)) with io restored to its pre value:
                     * Div rule (reverse_diff.py:774-793), exp rule (:903-917), Sub rule (:751-758) */
                    float x = IO_AT(d, zpre, l, i, j);
                    float dz = IO_AT(d, dIO, l, i, j);
                    float adj_div = (((float)0.0 - dz) * (float)1) /
                                    (((float)1 + expf((float)0 - x)) * ((float)1 + expf((float)0 - x)));
                    float adj_exp = adj_div * expf((float)0 - x);
                    float adj_x = (float)0.0 - adj_exp;
                    IO_AT(d, dIO, l, i, j) = (float)0.0;
                    IO_AT(d, dIO, l, i, j) += adj_x;
                }
            }
        /* bias reverse: io = io + b -> d_io passes, d_b += d_io */
        for (int i = ios[l][0] - 1; i >= 0; --i)
            for (int j = ios[l][1] - 1; j >= 0; --j) {
                float a_io = IO_AT(d, dIO, l, i, j);
                float a_b = IO_AT(d, dIO, l, i, j);
                IO_AT(d, dIO, l, i, j) = (float)0.0;
                IO_AT(d, dIO, l, i, j) += a_io;
                B_AT(d, dB, l, j) += a_b;
            }
        /* matmul reverse: io[l][i][j] = io[l][i][j] + A[i][k] * W[l][k][j] */
        int rows = (l == 0) ? d->layer_input_h : ios[l - 1][0];
        int cols = d->weight_shapes[l][1];
        int kk = (l == 0) ? d->layer_input_w : ios[l - 1][1];
        for (int i = rows - 1; i >= 0; --i)
            for (int j = cols - 1; j >= 0; --j)
                for (int k = kk - 1; k >= 0; --k) {
                    float dz = IO_AT(d, dIO, l, i, j);
                    float a_val = (l == 0) ? X_AT(d, X, i, k) : IO_AT(d, IOf, l - 1, i, k);
                    float a_io = dz;
                    float a_A = W_AT(d, W, l, k, j) * dz;
                    float a_W = a_val * dz;
                    IO_AT(d, dIO, l, i, j) = (float)0.0;
                    IO_AT(d, dIO, l, i, j) += a_io;
                    if (l == 0) {
                        if (dX) X_AT(d, dX, i, k) += a_A;
                    } else {
                        IO_AT(d, dIO, l - 1, i, k) += a_A;
                    }
                    W_AT(d, dW, l, k, j) += a_W;
                }
    }
}

/* ---- compositing forward: scripts/nerf.py:176-302 ---- */
static float composite_forward(const oracle_dims* d, const float* IO, const float* T,
                               float* rgba, const float* dists, float* alpha, float* cp,
                               float* wsamp, float* acc, float* cpC /* nullable snapshot c_j */,
                               float* cpP /* nullable snapshot P_j */) {
    const int L = d->num_weights, S = d->num_samples, H = d->target_image_h;
    const int img_size = H; /* nerf.py:176 */
    /* copy nerf.py:182-191 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            for (int k = 0; k < 4; ++k)
                rgba[((size_t)i * S + j) * 4 + k] = IO_AT(d, IO, L - 1, i * S + j, k);
    /* alpha nerf.py:200-205 ; -x is 0 - x (parser.py:259) */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            alpha[(size_t)i * S + j] =
                (float)(1.0) - expf(((float)0 - rgba[((size_t)i * S + j) * 4 + 3]) * dists[(size_t)i * S + j]);
    /* cumprod init nerf.py:215-220 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            cp[(size_t)i * S + j] = ((float)(1.0) - alpha[(size_t)i * S + j]) + (float)(1e-10);
    if (cpC) memcpy(cpC, cp, sizeof(float) * (size_t)img_size * S);
    /* inclusive cumprod nerf.py:226-232 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            if (j > 0) cp[(size_t)i * S + j] = cp[(size_t)i * S + j - 1] * cp[(size_t)i * S + j];
    if (cpP) memcpy(cpP, cp, sizeof(float) * (size_t)img_size * S);
    /* shift nerf.py:238-246 (overwritten below) */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            wsamp[(size_t)i * S + j] = (j == 0) ? alpha[(size_t)i * S + j] : cp[(size_t)i * S + j - 1];
    /* T_0 = 1 nerf.py:252-258 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            if (j == 0) cp[(size_t)i * S + j] = (float)((int)1);
    /* weights nerf.py:267-272 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            wsamp[(size_t)i * S + j] = alpha[(size_t)i * S + j] * cp[(size_t)i * S + j];
    /* colour nerf.py:281-288 */
    for (int i = 0; i < img_size; ++i)
        for (int j = 0; j < S; ++j)
            for (int c = 0; c < 3; ++c)
                acc[(size_t)i * d->acc_cols + c] = acc[(size_t)i * d->acc_cols + c] +
                    wsamp[(size_t)i * S + j] * rgba[((size_t)i * S + j) * 4 + c];
    /* loss nerf.py:297-302 */
    float loss = (float)((int)0);
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < d->target_image_w; ++j) {
            float a = acc[(size_t)i * d->acc_cols + j], t = T[(size_t)i * d->t_cols + j];
            loss = loss + (a - t) * (a - t);
        }
    return loss;
}

float oracle_nerf_forward(const oracle_dims* d, const float* X, const float* W, const float* B,
                          const float* T, float* IO, float* rgba, const float* dists,
                          float* alpha, float* cumprod, float* wsamp, float* acc) {
    mlp_forward(d, X, W, B, IO, NULL, 1);
    return composite_forward(d, IO, T, rgba, dists, alpha, cumprod, wsamp, acc, NULL, NULL);
}

void oracle_nerf_grad(const oracle_dims* d,
                      const float* X, float* dX, const float* W, float* dW, const float* B,
                      float* dB, const float* T, float* dT, const float* IO, float* dIO,
                      const float* rgba, float* drgba, const float* dists, float* ddists,
                      const float* alpha, float* dalpha, const float* cumprod, float* dcumprod,
                      const float* wsamp, float* dwsamp, const float* acc, float* dacc,
                      float dreturn) {
    const int L = d->num_weights, S = d->num_samples, H = d->target_image_h;
    const size_t nS = (size_t)H * S;
    /* Re-run the forward on private copies (the caller's primal buffers are restored by loma). */
    float* IOf = (float*)malloc(sizeof(float) * io_elems(d));
    float* zpre = (float*)malloc(sizeof(float) * io_elems(d));
    float* rg = (float*)malloc(sizeof(float) * nS * 4 + 4);
    float* al = (float*)malloc(sizeof(float) * nS + 4);
    float* cp = (float*)malloc(sizeof(float) * nS + 4);
    float* cpC = (float*)malloc(sizeof(float) * nS + 4);
    float* cpP = (float*)malloc(sizeof(float) * nS + 4);
    float* ws = (float*)malloc(sizeof(float) * nS + 4);
    float* ac = (float*)malloc(sizeof(float) * (size_t)H * d->acc_cols + 4);
    memcpy(IOf, IO, sizeof(float) * io_elems(d));
    memcpy(rg, rgba, sizeof(float) * nS * 4);
    memcpy(al, alpha, sizeof(float) * nS);
    memcpy(cp, cumprod, sizeof(float) * nS);
    memcpy(ws, wsamp, sizeof(float) * nS);
    memcpy(ac, acc, sizeof(float) * (size_t)H * d->acc_cols);
    mlp_forward(d, X, W, B, IOf, zpre, 1);
    (void)composite_forward(d, IOf, T, rg, dists, al, cp, ws, ac, cpC, cpP);

    /* return loss -> d_loss += _dreturn */
    float dloss = (float)0;
    dloss += dreturn;
    /* loss reverse (nerf.py:297-302) */
    for (int i = H - 1; i >= 0; --i)
        for (int j = d->target_image_w - 1; j >= 0; --j) {
            float a = ac[(size_t)i * d->acc_cols + j], t = T[(size_t)i * d->t_cols + j];
            float a0 = dloss;
            float a1 = (a - t) * dloss;
            float a2 = (float)0.0 - ((a - t) * dloss);
            float a3 = (a - t) * dloss;
            float a4 = (float)0.0 - ((a - t) * dloss);
            dloss = (float)0.0;
            dloss += a0;
            dacc[(size_t)i * d->acc_cols + j] += a1;
            dT[(size_t)i * d->t_cols + j] += a2;
            dacc[(size_t)i * d->acc_cols + j] += a3;
            dT[(size_t)i * d->t_cols + j] += a4;
        }
    /* colour reverse (nerf.py:281-288), statements c = 2, 1, 0 */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j)
            for (int c = 2; c >= 0; --c) {
                float adj = dacc[(size_t)i * d->acc_cols + c];
                float a_acc = adj;
                float a_w = rg[((size_t)i * S + j) * 4 + c] * adj;
                float a_rgb = ws[(size_t)i * S + j] * adj;
                dacc[(size_t)i * d->acc_cols + c] = (float)0.0;
                dacc[(size_t)i * d->acc_cols + c] += a_acc;
                dwsamp[(size_t)i * S + j] += a_w;
                drgba[((size_t)i * S + j) * 4 + c] += a_rgb;
            }
    /* weights reverse (nerf.py:267-272): w = alpha * cp (cp = T here) */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j) {
            size_t o = (size_t)i * S + j;
            float adj = dwsamp[o];
            float a_al = cp[o] * adj;
            float a_cp = al[o] * adj;
            dwsamp[o] = (float)0.0;
            dalpha[o] += a_al;
            dcumprod[o] += a_cp;
        }
    /* T_0 = 1 reverse (nerf.py:252-258): d_cp[i][0] = 0 */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j)
            if (j == 0) dcumprod[(size_t)i * S] = (float)0.0;
    /* shift reverse (nerf.py:238-246) */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j) {
            size_t o = (size_t)i * S + j;
            float adj = dwsamp[o];
            dwsamp[o] = (float)0.0;
            if (j == 0) dalpha[o] += adj;
            else dcumprod[o - 1] += adj;
        }
    /* cumprod reverse (nerf.py:226-232): cp[j] = cp[j-1] * cp[j], cp[j] restored to c_j */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j)
            if (j > 0) {
                size_t o = (size_t)i * S + j;
                float adj = dcumprod[o];
                float a_left = cpC[o] * adj;       /* d/d cp[j-1] = cp[j] (restored c_j) */
                float a_right = cpP[o - 1] * adj;  /* d/d cp[j]   = cp[j-1] = P_{j-1}     */
                dcumprod[o] = (float)0.0;
                dcumprod[o - 1] += a_left;
                dcumprod[o] += a_right;
            }
    /* cumprod init reverse (nerf.py:215-220): cp = (1 - alpha) + 1e-10 */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j) {
            size_t o = (size_t)i * S + j;
            float adj = dcumprod[o];
            float a_al = (float)0.0 - adj;
            dcumprod[o] = (float)0.0;
            dalpha[o] += a_al;
        }
    /* alpha reverse (nerf.py:200-205): alpha = 1 - exp((0 - sigma) * delta) */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j) {
            size_t o = (size_t)i * S + j;
            float sigma = rg[o * 4 + 3], delta = dists[o];
            float adj = dalpha[o];
            float adj1 = (float)0.0 - adj;
            float adj2 = adj1 * expf(((float)0 - sigma) * delta);
            float a_sigma = (float)0.0 - (delta * adj2);
            float a_delta = ((float)0 - sigma) * adj2;
            dalpha[o] = (float)0.0;
            drgba[o * 4 + 3] += a_sigma;
            ddists[o] += a_delta;
        }
    /* copy reverse (nerf.py:182-191) */
    for (int i = H - 1; i >= 0; --i)
        for (int j = S - 1; j >= 0; --j)
            for (int k = 3; k >= 0; --k) {
                size_t o = ((size_t)i * S + j) * 4 + k;
                float adj = drgba[o];
                drgba[o] = (float)0.0;
                IO_AT(d, dIO, L - 1, i * S + j, k) += adj;
            }
    mlp_reverse(d, X, dX, W, dW, dB, IOf, zpre, dIO, 1);

    free(IOf); free(zpre); free(rg); free(al); free(cp); free(cpC); free(cpP); free(ws); free(ac);
}

/* ---------------------------------------------------------------------------------------- */
/* mlp_fit (scripts/mlp_fit.py:1-147). Loss over io[L-1] (mlp_fit.py:140-145).              */
float oracle_mlp_fit_forward(const oracle_dims* d, const float* X, const float* W, const float* B,
                             const float* T, float* IO) {
    const int L = d->num_weights;
    mlp_forward(d, X, W, B, IO, NULL, 0);
    float loss = (float)((int)0);
    for (int i = 0; i < d->target_image_h; ++i)
        for (int j = 0; j < d->target_image_w; ++j) {
            float a = IO_AT(d, IO, L - 1, i, j), t = T[(size_t)i * d->t_cols + j];
            loss = loss + (a - t) * (a - t);
        }
    return loss;
}

void oracle_mlp_fit_grad(const oracle_dims* d, const float* X, float* dX, const float* W,
                         float* dW, const float* B, float* dB, const float* T, float* dT,
                         const float* IO, float* dIO, float dreturn) {
    const int L = d->num_weights;
    float* IOf = (float*)malloc(sizeof(float) * io_elems(d));
    float* zpre = (float*)malloc(sizeof(float) * io_elems(d));
    memcpy(IOf, IO, sizeof(float) * io_elems(d));
    mlp_forward(d, X, W, B, IOf, zpre, 0);
    float dloss = (float)0;
    dloss += dreturn;
    for (int i = d->target_image_h - 1; i >= 0; --i)
        for (int j = d->target_image_w - 1; j >= 0; --j) {
            float a = IO_AT(d, IOf, L - 1, i, j), t = T[(size_t)i * d->t_cols + j];
            float a0 = dloss;
            float a1 = (a - t) * dloss;
            float a2 = (float)0.0 - ((a - t) * dloss);
            float a3 = (a - t) * dloss;
            float a4 = (float)0.0 - ((a - t) * dloss);
            dloss = (float)0.0;
            dloss += a0;
            IO_AT(d, dIO, L - 1, i, j) += a1;
            dT[(size_t)i * d->t_cols + j] += a2;
            IO_AT(d, dIO, L - 1, i, j) += a3;
            dT[(size_t)i * d->t_cols + j] += a4;
        }
    mlp_reverse(d, X, dX, W, dW, dB, IOf, zpre, dIO, 0);
    free(IOf); free(zpre);
}

void oracle_mult_a_b(const float* a, int a_h, int a_w, int a_cols, const float* b, int b_h,
                     int b_w, int b_cols, float* c, int c_cols) {
    (void)b_h;
    for (int i = 0; i < a_h; ++i)
        for (int j = 0; j < b_w; ++j)
            for (int k = 0; k < a_w; ++k)
                c[(size_t)i * c_cols + j] = c[(size_t)i * c_cols + j] + a[(size_t)i * a_cols + k] * b[(size_t)k * b_cols + j];
}

void oracle_positional_encoding_3d(const double* pts, long n, int F, float* out) {
    const int C = 3 + 6 * F;
    for (long s = 0; s < n; ++s) {
        const double* p = pts + 3 * s;
        float* o = out + (size_t)s * C;
        for (int c = 0; c < 3; ++c) o[c] = (float)p[c];
        for (int f = 0; f < F; ++f) {
            double sc = ldexp(1.0, f); /* 2.0 ** f, exact */
            for (int c = 0; c < 3; ++c) {
                o[3 + 6 * f + c] = (float)sin(sc * p[c]);
                o[3 + 6 * f + 3 + c] = (float)cos(sc * p[c]);
            }
        }
    }
}

/* ---------------------------------------------------------------------------------------- */
/* CPU baseline step. Standard semantics: one loma call per ray block with io rows = block rows,
 * zero-initialised buffers, unit seed; the grads are then scaled by the total loss (the
 * reference seeds its gradient with the loss, train_nerf.py:477). threads > 1 splits the rays
 * into contiguous blocks, one private dW/dB per thread, summed at the end.                   */
static float step_block(int L, const int* kd, const int* nd, int w_k, int w_n, const float* X,
                        int rays, int S, const float* dists, const float* T, const float* W,
                        const float* B, float* dW, float* dB) {
    oracle_dims d;
    memset(&d, 0, sizeof(d));
    const int R = rays * S;
    int maxc = 4;
    for (int l = 0; l < L; ++l) maxc = nd[l] > maxc ? nd[l] : maxc;
    d.num_weights = L;
    d.layer_input_h = R;
    d.layer_input_w = kd[0];
    d.target_image_h = rays;
    d.target_image_w = 3;
    d.num_samples = S;
    for (int l = 0; l < L; ++l) {
        d.weight_shapes[l][0] = kd[l];
        d.weight_shapes[l][1] = nd[l];
        d.bias_shapes[l][0] = nd[l];
        d.bias_shapes[l][1] = 1;
        d.intermediate_output_shapes[l][0] = R;
        d.intermediate_output_shapes[l][1] = nd[l];
    }
    d.x_cols = kd[0];
    d.w_k = w_k;
    d.w_n = w_n;
    d.b_n = w_n;
    d.io_rows = R;
    d.io_cols = maxc;
    d.t_cols = 3;
    d.acc_cols = 3;
    size_t nio = (size_t)L * R * maxc, nS = (size_t)rays * S;
    float* IO = (float*)calloc(nio, sizeof(float));
    float* dIO = (float*)calloc(nio, sizeof(float));
    float* rgba = (float*)calloc(nS * 4, sizeof(float));
    float* drgba = (float*)calloc(nS * 4, sizeof(float));
    float* al = (float*)calloc(nS, sizeof(float));
    float* dal = (float*)calloc(nS, sizeof(float));
    float* cp = (float*)calloc(nS, sizeof(float));
    float* dcp = (float*)calloc(nS, sizeof(float));
    float* ws = (float*)calloc(nS, sizeof(float));
    float* dws = (float*)calloc(nS, sizeof(float));
    float* ddist = (float*)calloc(nS, sizeof(float));
    float* acc = (float*)calloc((size_t)rays * 3, sizeof(float));
    float* dacc = (float*)calloc((size_t)rays * 3, sizeof(float));
    float* dT = (float*)calloc((size_t)rays * 3, sizeof(float));
    float* IO0 = (float*)calloc(nio, sizeof(float));
    float* rg0 = (float*)calloc(nS * 4, sizeof(float));
    float* acc0 = (float*)calloc((size_t)rays * 3, sizeof(float));
    float loss = oracle_nerf_forward(&d, X, W, B, T, IO, rgba, dists, al, cp, ws, acc);
    /* grad call receives fresh zero primal buffers, as train_nerf.py:395-478 builds them */
    memset(al, 0, nS * sizeof(float));
    memset(cp, 0, nS * sizeof(float));
    memset(ws, 0, nS * sizeof(float));
    oracle_nerf_grad(&d, X, NULL, W, dW, B, dB, T, dT, IO0, dIO, rg0, drgba, dists, ddist, al, dal,
                     cp, dcp, ws, dws, acc0, dacc, 1.0f);
    free(IO); free(dIO); free(rgba); free(drgba); free(al); free(dal); free(cp); free(dcp);
    free(ws); free(dws); free(ddist); free(acc); free(dacc); free(dT); free(IO0); free(rg0);
    free(acc0);
    return loss;
}

float oracle_train_step(int L, const int* kd, const int* nd, int w_k, int w_n, const float* X,
                        int rays, int S, const float* dists, const float* T, const float* W,
                        const float* B, float* dW, float* dB, int threads) {
    if (threads < 1) threads = 1;
    if (threads > rays) threads = rays;
    const size_t nW = (size_t)L * w_k * w_n, nB = (size_t)L * w_n;
    float* pw = (float*)calloc(nW * threads, sizeof(float));
    float* pb = (float*)calloc(nB * threads, sizeof(float));
    float* pl = (float*)calloc((size_t)threads, sizeof(float));
    const int x_cols = kd[0];
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
    for (int t = 0; t < threads; ++t) {
        int r0 = (int)((long)rays * t / threads), r1 = (int)((long)rays * (t + 1) / threads);
        if (r1 > r0)
            pl[t] = step_block(L, kd, nd, w_k, w_n, X + (size_t)r0 * S * x_cols, r1 - r0, S,
                               dists + (size_t)r0 * S, T + (size_t)r0 * 3, W, B, pw + nW * t,
                               pb + nB * t);
    }
    float loss = 0.0f;
    for (int t = 0; t < threads; ++t) loss += pl[t];
    for (size_t e = 0; e < nW; ++e) {
        float s = 0.0f;
        for (int t = 0; t < threads; ++t) s += pw[nW * t + e];
        dW[e] += s * loss;
    }
    for (size_t e = 0; e < nB; ++e) {
        float s = 0.0f;
        for (int t = 0; t < threads; ++t) s += pb[nB * t + e];
        dB[e] += s * loss;
    }
    free(pw); free(pb); free(pl);
    return loss;
}
