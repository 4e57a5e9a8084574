// lnerf_generic.hip -- the loma-order path on the GPU.
//
// A stage-by-stage restatement of scripts/nerf.py (forward, :1-304) and of the reverse sweep its
// rev_diff generates (:306 -> loma_public/reverse_diff.py:492-1016), with the reference's exact
// loop bounds (including the intermediate_output_shapes row quirk) and the
// reference's per-element accumulation order. It backs the loma-compat C ABI (small chunks,
// arbitrary shapes) and is the cross-check for the fused MFMA path.
//
// Compiled with -ffp-contract=off: loma's C target is built by `gcc -O2` (compiler.py:154), which
// on x86-64 evaluates `a + b * c` as a rounded multiply then a rounded add.
#include "lnerf_internal.h"

#include <math.h>

namespace lnerf {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float& io_at(const LgDims& d, float* IO, int l, int i, int j) {
    return IO[((size_t)l * d.io_rows + i) * d.io_cols + j];
}
__device__ __forceinline__ float io_get(const LgDims& d, const float* IO, int l, int i, int j) {
    return IO[((size_t)l * d.io_rows + i) * d.io_cols + j];
}
__device__ __forceinline__ float w_get(const LgDims& d, const float* W, int l, int k, int j) {
    return W[((size_t)l * d.w_k + k) * d.w_n + j];
}

inline unsigned grid_for(size_t n) {
    size_t g = (n + kThreads - 1) / kThreads;
    if (g < 1) g = 1;
    if (g > 65535u * 8u) g = 65535u * 8u;
    return (unsigned)g;
}

// ---- forward --------------------------------------------------------------------------------

// nerf.py:81-89 (l == 0) and :108-116 (l > 0): io[l][i][j] = io[l][i][j] + A[i][k] * W[l][k][j]
__global__ void lg_matmul_kernel(LgDims d, int l, const float* __restrict__ X,
                                 const float* __restrict__ W, float* IO) {
    const int rows = (l == 0) ? d.in_h : d.ios0[l - 1];
    const int cols = d.wsh1[l];
    const int K = (l == 0) ? d.in_w : d.ios1[l - 1];
    const size_t n = (size_t)rows * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / cols), j = (int)(e % cols);
        float z = io_get(d, IO, l, i, j);
        if (l == 0) {
            for (int k = 0; k < K; ++k) z = z + X[(size_t)i * d.x_cols + k] * w_get(d, W, 0, k, j);
        } else {
            for (int k = 0; k < K; ++k) z = z + io_get(d, IO, l - 1, i, k) * w_get(d, W, l, k, j);
        }
        io_at(d, IO, l, i, j) = z;
    }
}

// bias (nerf.py:95-100 / :122-127) then activation (:138-167; mlp_fit.py:108-132). Both loops
// run over the same rectangle and are elementwise, so fusing them keeps loma's results.
__global__ void lg_bias_act_kernel(LgDims d, int l, const float* __restrict__ B, float* IO,
                                   float* zpre) {
    const int rows = d.ios0[l], cols = d.ios1[l];
    const size_t n = (size_t)rows * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / cols), j = (int)(e % cols);
        float v = io_get(d, IO, l, i, j) + B[(size_t)l * d.b_n + j];
        if (zpre) io_at(d, zpre, l, i, j) = v;
        const bool relu = (l < d.L - 1) || (d.nerf_head && j == 3);
        if (relu) {
            v = (v > 0.0f) ? v : 0.0f;
        } else {
            v = 1.0f / (1.0f + expf(0.0f - v));
        }
        io_at(d, IO, l, i, j) = v;
    }
}

// Rendering, nerf.py:176-288, one thread per ray (every stage only touches its own ray's row).
__global__ void lg_composite_fwd_kernel(LgDims d, const float* __restrict__ IO, float* rgba,
                                        const float* __restrict__ dists, float* alpha, float* cp,
                                        float* wsamp, float* acc, float* cpC, float* cpP) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.th) return;
    const int S = d.S, L = d.L;
    const size_t o = (size_t)i * S;
    for (int j = 0; j < S; ++j)                                           // copy :182-191
        for (int k = 0; k < 4; ++k) rgba[(o + j) * 4 + k] = io_get(d, IO, L - 1, i * S + j, k);
    for (int j = 0; j < S; ++j)                                           // alpha :200-205
        alpha[o + j] = 1.0f - expf((0.0f - rgba[(o + j) * 4 + 3]) * dists[o + j]);
    for (int j = 0; j < S; ++j) cp[o + j] = (1.0f - alpha[o + j]) + (float)(1e-10);  // :215-220
    if (cpC)
        for (int j = 0; j < S; ++j) cpC[o + j] = cp[o + j];
    for (int j = 1; j < S; ++j) cp[o + j] = cp[o + j - 1] * cp[o + j];   // inclusive :226-232
    if (cpP)
        for (int j = 0; j < S; ++j) cpP[o + j] = cp[o + j];
    for (int j = 0; j < S; ++j) wsamp[o + j] = (j == 0) ? alpha[o] : cp[o + j - 1];  // :238-246
    if (S > 0) cp[o] = 1.0f;                                              // :252-258
    for (int j = 0; j < S; ++j) wsamp[o + j] = alpha[o + j] * cp[o + j];  // :267-272
    float* a = acc + (size_t)i * d.acc_cols;
    for (int j = 0; j < S; ++j) {                                         // :281-288
        a[0] = a[0] + wsamp[o + j] * rgba[(o + j) * 4 + 0];
        a[1] = a[1] + wsamp[o + j] * rgba[(o + j) * 4 + 1];
        a[2] = a[2] + wsamp[o + j] * rgba[(o + j) * 4 + 2];
    }
}

// Loss, nerf.py:297-302: one thread, the reference's sequential summation order.
__global__ void lg_loss_kernel(LgDims d, const float* __restrict__ acc, int acc_cols,
                               const float* __restrict__ T, float* loss_out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    float loss = 0.0f;
    for (int i = 0; i < d.th; ++i)
        for (int j = 0; j < d.tw; ++j) {
            const float a = acc[(size_t)i * acc_cols + j], t = T[(size_t)i * d.t_cols + j];
            loss = loss + (a - t) * (a - t);
        }
    *loss_out = loss;
}

// ---- reverse --------------------------------------------------------------------------------

// Reverse of the loss + rendering stages for one ray (reverse_diff.py mutate_assign :576-616
// applied to nerf.py:182-302, stages in reverse order, loops descending).
__global__ void lg_composite_bwd_kernel(LgDims d, const float* __restrict__ T,
                                        const float* __restrict__ acc,
                                        const float* __restrict__ rgba,
                                        const float* __restrict__ dists,
                                        const float* __restrict__ alpha,
                                        const float* __restrict__ cpT,   // final cp (T values)
                                        const float* __restrict__ cpC,
                                        const float* __restrict__ cpP,
                                        const float* __restrict__ wsamp, LgAdjoints a,
                                        const float* __restrict__ seed_dev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.th) return;
    const int S = d.S, L = d.L;
    const size_t o = (size_t)i * S;
    float dloss = 0.0f;
    dloss += *seed_dev;  // return loss -> d_loss += _dreturn
    float* dacc = a.dacc + (size_t)i * d.acc_cols;
    // loss reverse (:297-302)
    for (int j = d.tw - 1; j >= 0; --j) {
        const float av = acc[(size_t)i * d.acc_cols + j], t = T[(size_t)i * d.t_cols + j];
        const float a0 = dloss;
        const float a1 = (av - t) * dloss;
        const float a2 = 0.0f - ((av - t) * dloss);
        const float a3 = (av - t) * dloss;
        const float a4 = 0.0f - ((av - t) * dloss);
        dloss = 0.0f;
        dloss += a0;
        dacc[j] += a1;
        a.dT[(size_t)i * d.t_cols + j] += a2;
        dacc[j] += a3;
        a.dT[(size_t)i * d.t_cols + j] += a4;
    }
    // colour reverse (:281-288), statements c = 2, 1, 0
    for (int j = S - 1; j >= 0; --j)
        for (int c = 2; c >= 0; --c) {
            const float adj = dacc[c];
            const float a_w = rgba[(o + j) * 4 + c] * adj;
            const float a_rgb = wsamp[o + j] * adj;
            dacc[c] = 0.0f;
            dacc[c] += adj;
            a.dwsamp[o + j] += a_w;
            a.drgba[(o + j) * 4 + c] += a_rgb;
        }
    // weights reverse (:267-272)
    for (int j = S - 1; j >= 0; --j) {
        const float adj = a.dwsamp[o + j];
        const float a_al = cpT[o + j] * adj;
        const float a_cp = alpha[o + j] * adj;
        a.dwsamp[o + j] = 0.0f;
        a.dalpha[o + j] += a_al;
        a.dcp[o + j] += a_cp;
    }
    // T_0 = 1 reverse (:252-258)
    if (S > 0) a.dcp[o] = 0.0f;
    // shift reverse (:238-246)
    for (int j = S - 1; j >= 0; --j) {
        const float adj = a.dwsamp[o + j];
        a.dwsamp[o + j] = 0.0f;
        if (j == 0) a.dalpha[o] += adj;
        else a.dcp[o + j - 1] += adj;
    }
    // cumprod reverse (:226-232)
    for (int j = S - 1; j >= 1; --j) {
        const float adj = a.dcp[o + j];
        const float a_left = cpC[o + j] * adj;
        const float a_right = cpP[o + j - 1] * adj;
        a.dcp[o + j] = 0.0f;
        a.dcp[o + j - 1] += a_left;
        a.dcp[o + j] += a_right;
    }
    // cumprod init reverse (:215-220)
    for (int j = S - 1; j >= 0; --j) {
        const float adj = a.dcp[o + j];
        a.dcp[o + j] = 0.0f;
        a.dalpha[o + j] += 0.0f - adj;
    }
    // alpha reverse (:200-205): alpha = 1 - exp((0 - sigma) * delta)
    for (int j = S - 1; j >= 0; --j) {
        const float sigma = rgba[(o + j) * 4 + 3], delta = dists[o + j];
        const float adj = a.dalpha[o + j];
        const float adj1 = 0.0f - adj;
        const float adj2 = adj1 * expf((0.0f - sigma) * delta);
        const float a_sigma = 0.0f - (delta * adj2);
        const float a_delta = (0.0f - sigma) * adj2;
        a.dalpha[o + j] = 0.0f;
        a.drgba[(o + j) * 4 + 3] += a_sigma;
        a.ddists[o + j] += a_delta;
    }
    // copy reverse (:182-191)
    for (int j = S - 1; j >= 0; --j)
        for (int k = 3; k >= 0; --k) {
            const float adj = a.drgba[(o + j) * 4 + k];
            a.drgba[(o + j) * 4 + k] = 0.0f;
            io_at(d, a.dIO, L - 1, i * S + j, k) += adj;
        }
}

// mlp_fit.py:140-145 loss reverse (loss over io[L-1]); single thread, order irrelevant since
// every (i, j) touches its own elements.
__global__ void lg_fit_loss_bwd_kernel(LgDims d, const float* __restrict__ IOf,
                                       const float* __restrict__ T, LgAdjoints a,
                                       const float* __restrict__ seed_dev) {
    const size_t n = (size_t)d.th * d.tw;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / d.tw), j = (int)(e % d.tw);
        float dloss = 0.0f;
        dloss += *seed_dev;
        const float av = io_get(d, IOf, d.L - 1, i, j), t = T[(size_t)i * d.t_cols + j];
        const float a1 = (av - t) * dloss;
        const float a2 = 0.0f - ((av - t) * dloss);
        io_at(d, a.dIO, d.L - 1, i, j) += a1;
        a.dT[(size_t)i * d.t_cols + j] += a2;
        io_at(d, a.dIO, d.L - 1, i, j) += a1;
        a.dT[(size_t)i * d.t_cols + j] += a2;
    }
}

// Activation reverse: ReLU keeps d where the post value > 0 (mutate_ifelse re-evaluates the
// condition on the un-restored primal), sigmoid uses loma's Div/exp/Sub adjoint expression on the
// restored pre value (reverse_diff.py:751-793, :903-917).
__global__ void lg_act_bwd_kernel(LgDims d, int l, const float* __restrict__ IOf,
                                  const float* __restrict__ zpre, float* dIO) {
    const int rows = d.ios0[l], cols = d.ios1[l];
    const size_t n = (size_t)rows * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / cols), j = (int)(e % cols);
        const bool relu = (l < d.L - 1) || (d.nerf_head && j == 3);
        float& g = io_at(d, dIO, l, i, j);
        if (relu) {
            if (!(io_get(d, IOf, l, i, j) > 0.0f)) g = 0.0f;
        } else {
            const float x = io_get(d, zpre, l, i, j);
            const float dz = g;
            const float u = 1.0f + expf(0.0f - x);
            const float adj_div = ((0.0f - dz) * 1.0f) / (u * u);
            const float adj_exp = adj_div * expf(0.0f - x);
            g = 0.0f;
            g += 0.0f - adj_exp;
        }
    }
}

// Bias reverse: d_b[l][j] += d_io[l][i][j] over rows descending (d_io passes through unchanged).
__global__ void lg_bias_bwd_kernel(LgDims d, int l, const float* __restrict__ dIO, float* dB) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.ios1[l]) return;
    float acc = dB[(size_t)l * d.b_n + j];
    for (int i = d.ios0[l] - 1; i >= 0; --i) acc += io_get(d, dIO, l, i, j);
    dB[(size_t)l * d.b_n + j] = acc;
}

// Matmul reverse, d_W part: d_W[l][k][j] += A[i][k] * d_io[l][i][j] over i descending.
__global__ void lg_matmul_bwd_w_kernel(LgDims d, int l, const float* __restrict__ X,
                                       const float* __restrict__ IOf,
                                       const float* __restrict__ dIO, float* dW) {
    const int rows = (l == 0) ? d.in_h : d.ios0[l - 1];
    const int cols = d.wsh1[l];
    const int K = (l == 0) ? d.in_w : d.ios1[l - 1];
    const size_t n = (size_t)K * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / cols), j = (int)(e % cols);
        float acc = dW[((size_t)l * d.w_k + k) * d.w_n + j];
        for (int i = rows - 1; i >= 0; --i) {
            const float av = (l == 0) ? X[(size_t)i * d.x_cols + k] : io_get(d, IOf, l - 1, i, k);
            acc += av * io_get(d, dIO, l, i, j);
        }
        dW[((size_t)l * d.w_k + k) * d.w_n + j] = acc;
    }
}

// Matmul reverse, d_A part: d_A[i][k] += W[l][k][j] * d_io[l][i][j] over j descending, where
// d_A is d_io[l-1] (post-activation adjoint of the previous layer) or d_layer_input.
__global__ void lg_matmul_bwd_a_kernel(LgDims d, int l, const float* __restrict__ W,
                                       float* dIO, float* dX) {
    const int rows = (l == 0) ? d.in_h : d.ios0[l - 1];
    const int cols = d.wsh1[l];
    const int K = (l == 0) ? d.in_w : d.ios1[l - 1];
    const size_t n = (size_t)rows * K;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / K), k = (int)(e % K);
        float* tgt = (l == 0) ? (dX + (size_t)i * d.x_cols + k) : &io_at(d, dIO, l - 1, i, k);
        float acc = *tgt;
        for (int j = cols - 1; j >= 0; --j) acc += w_get(d, W, l, k, j) * io_get(d, dIO, l, i, j);
        *tgt = acc;
    }
}

__global__ void lg_mult_a_b_kernel(const float* __restrict__ A, int a_h, int a_w,
                                   const float* __restrict__ Bm, int b_w, float* C) {
    const size_t n = (size_t)a_h * b_w;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / b_w), j = (int)(e % b_w);
        float c = C[e];
        for (int k = 0; k < a_w; ++k) c = c + A[(size_t)i * a_w + k] * Bm[(size_t)k * b_w + j];
        C[e] = c;
    }
}

// ---- small helpers --------------------------------------------------------------------------
__global__ void fill_kernel(float* p, float v, size_t n) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x)
        p[e] = v;
}
__global__ void scale_kernel(float* p, size_t n, const float* __restrict__ s) {
    const float v = *s;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x)
        p[e] = p[e] * v;
}
// positional_encoding_3d (pos_encoding.py:38-69): float64 trig, one rounding to float32.
__global__ void pe_kernel(const float* __restrict__ pts, int n, int F, float* out, int out_cols) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    float* o = out + (size_t)s * out_cols;
    for (int c = 0; c < 3; ++c) o[c] = pts[(size_t)s * 3 + c];
    for (int f = 0; f < F; ++f)
        for (int c = 0; c < 3; ++c) {
            const double x = ldexp((double)pts[(size_t)s * 3 + c], f);
            o[3 + 6 * f + c] = (float)sin(x);
            o[3 + 6 * f + 3 + c] = (float)cos(x);
        }
}
// RAYS mode: sample points o + d t in float64 (train_nerf.py:295-299), encoded like pe_kernel.
__global__ void pe_rays_kernel(const float* __restrict__ rays, int nrays, int S, float near_t,
                               float far_t, int F, float* out, int out_cols) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nrays * S) return;
    const int ray = s / S, j = s - ray * S;
    float* o = out + (size_t)s * out_cols;
    for (int c = 0; c < 3; ++c) {
        const double p = ray_point(rays + (size_t)ray * 6, c, j, S, near_t, far_t);
        o[c] = (float)p;
        for (int f = 0; f < F; ++f) {
            const double x = ldexp(p, f);
            o[3 + 6 * f + c] = (float)sin(x);
            o[3 + 6 * f + 3 + c] = (float)cos(x);
        }
    }
}
__global__ void ray_dists_kernel(int n, int S, float near_t, float far_t, float* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) out[s] = ray_delta(s % S, S, near_t, far_t);
}
// get_rays, train_nerf.py:23-62 (float64 math, float32 [o, d] rows)
struct RayCam {
    double K[9];
    double c2w[12];
};
__global__ void get_rays_kernel(int width, RayCam cam, float* rays) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= width * width) return;
    const int row = p / width, col = p - row * width;
    // np.linspace(0, 1, width): k * step, the last exactly 1
    const double step = width > 1 ? 1.0 / (double)(width - 1) : 0.0;
    const double i = (col == width - 1 && width > 1) ? 1.0 : (double)col * step;
    const double j = (row == width - 1 && width > 1) ? 1.0 : (double)row * step;
    const double dir[3] = {(i - cam.K[2]) / cam.K[0], -(j - cam.K[5]) / cam.K[4], -1.0};
    float* r = rays + (size_t)p * 6;
    for (int a = 0; a < 3; ++a) {
        r[a] = (float)cam.c2w[a * 4 + 3];
        double d = 0.0;
        for (int b = 0; b < 3; ++b) d += dir[b] * cam.c2w[a * 4 + b];   // directions @ R.T
        r[3 + a] = (float)d;
    }
}

// Adam, train_nerf.py:143-161 (lr_t folds sqrt(1-b2^t)/(1-b1^t); m_hat/v_hat as written there).
__global__ void adam_kernel(float* p, const float* __restrict__ g, float* m, float* v, size_t n,
                            float lr_t, float b1, float b2, float eps, float bc1, float bc2) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x) {
        const float ge = g[e];
        const float me = b1 * m[e] + (1.0f - b1) * ge;
        const float ve = b2 * v[e] + (1.0f - b2) * (ge * ge);
        m[e] = me;
        v[e] = ve;
        const float mh = me / bc1, vh = ve / bc2;
        p[e] -= lr_t * mh / (sqrtf(vh) + eps);
    }
}

}  // namespace

// ---- host launchers -------------------------------------------------------------------------

static void mlp_forward(const LgDims& d, const LgBuffers& b, hipStream_t s) {
    for (int l = 0; l < d.L; ++l) {
        const size_t mm = (size_t)((l == 0) ? d.in_h : d.ios0[l - 1]) * d.wsh1[l];
        if (mm) lg_matmul_kernel<<<grid_for(mm), kThreads, 0, s>>>(d, l, b.X, b.W, b.IO);
        const size_t ba = (size_t)d.ios0[l] * d.ios1[l];
        if (ba) lg_bias_act_kernel<<<grid_for(ba), kThreads, 0, s>>>(d, l, b.B, b.IO, b.zpre);
    }
}

static void mlp_reverse(const LgDims& d, const LgBuffers& b, const LgAdjoints& a,
                        hipStream_t s) {
    for (int l = d.L - 1; l >= 0; --l) {
        const size_t ba = (size_t)d.ios0[l] * d.ios1[l];
        if (ba) {
            lg_act_bwd_kernel<<<grid_for(ba), kThreads, 0, s>>>(d, l, b.IO, b.zpre, a.dIO);
            lg_bias_bwd_kernel<<<(d.ios1[l] + kThreads - 1) / kThreads, kThreads, 0, s>>>(
                d, l, a.dIO, a.dB);
        }
        const int rows = (l == 0) ? d.in_h : d.ios0[l - 1];
        const int K = (l == 0) ? d.in_w : d.ios1[l - 1];
        const size_t nw = (size_t)K * d.wsh1[l];
        if (nw && rows)
            lg_matmul_bwd_w_kernel<<<grid_for(nw), kThreads, 0, s>>>(d, l, b.X, b.IO, a.dIO, a.dW);
        const size_t na = (size_t)rows * K;
        if (na && d.wsh1[l] && (l > 0 || a.dX))
            lg_matmul_bwd_a_kernel<<<grid_for(na), kThreads, 0, s>>>(d, l, b.W, a.dIO, a.dX);
    }
}

void lg_nerf_forward(const LgDims& d, const LgBuffers& b, float* loss_dev, hipStream_t s) {
    mlp_forward(d, b, s);
    if (d.th > 0)
        lg_composite_fwd_kernel<<<(d.th + 127) / 128, 128, 0, s>>>(
            d, b.IO, b.rgba, b.dists, b.alpha, b.cp, b.wsamp, b.acc, b.cpC, b.cpP);
    lg_loss_kernel<<<1, 64, 0, s>>>(d, b.acc, d.acc_cols, b.T, loss_dev);
}

void lg_nerf_grad(const LgDims& d, const LgBuffers& b, const LgAdjoints& a, const float* seed_dev,
                  hipStream_t s) {
    // re-execute the forward on the private primal copy, with snapshots
    mlp_forward(d, b, s);
    if (d.th > 0) {
        lg_composite_fwd_kernel<<<(d.th + 127) / 128, 128, 0, s>>>(
            d, b.IO, b.rgba, b.dists, b.alpha, b.cp, b.wsamp, b.acc, b.cpC, b.cpP);
        lg_composite_bwd_kernel<<<(d.th + 127) / 128, 128, 0, s>>>(
            d, b.T, b.acc, b.rgba, b.dists, b.alpha, b.cp, b.cpC, b.cpP, b.wsamp, a, seed_dev);
    }
    mlp_reverse(d, b, a, s);
}

void lg_mlp_fit_forward(const LgDims& d, const LgBuffers& b, float* loss_dev, hipStream_t s) {
    mlp_forward(d, b, s);
    // loss over io[L-1] (mlp_fit.py:140-145): acc = io[L-1] with row stride io_cols
    lg_loss_kernel<<<1, 64, 0, s>>>(d, b.IO + (size_t)(d.L - 1) * d.io_rows * d.io_cols,
                                    d.io_cols, b.T, loss_dev);
}

void lg_mlp_fit_grad(const LgDims& d, const LgBuffers& b, const LgAdjoints& a,
                     const float* seed_dev, hipStream_t s) {
    mlp_forward(d, b, s);
    const size_t n = (size_t)d.th * d.tw;
    if (n) lg_fit_loss_bwd_kernel<<<grid_for(n), kThreads, 0, s>>>(d, b.IO, b.T, a, seed_dev);
    mlp_reverse(d, b, a, s);
}

void lg_mult_a_b(const float* A, int a_h, int a_w, const float* B, int b_w, float* C,
                 hipStream_t s) {
    const size_t n = (size_t)a_h * b_w;
    if (n) lg_mult_a_b_kernel<<<grid_for(n), kThreads, 0, s>>>(A, a_h, a_w, B, b_w, C);
}

void k_fill(float* p, float v, size_t n, hipStream_t s) {
    if (n) fill_kernel<<<grid_for(n), kThreads, 0, s>>>(p, v, n);
}
void k_scale_by_scalar(float* p, size_t n, const float* scale, hipStream_t s) {
    if (n) scale_kernel<<<grid_for(n), kThreads, 0, s>>>(p, n, scale);
}
void k_positional_encoding(const float* pts, int n, int F, float* out, int out_cols,
                           hipStream_t s) {
    if (n > 0) pe_kernel<<<(n + 255) / 256, 256, 0, s>>>(pts, n, F, out, out_cols);
}
void k_positional_encoding_rays(const float* rays, int nrays, int S, float near_t, float far_t,
                                int F, float* out, int out_cols, hipStream_t s) {
    const int n = nrays * S;
    if (n > 0) pe_rays_kernel<<<(n + 255) / 256, 256, 0, s>>>(rays, nrays, S, near_t, far_t, F, out, out_cols);
}
void k_ray_dists(int nrays, int S, float near_t, float far_t, float* out, hipStream_t s) {
    const int n = nrays * S;
    if (n > 0) ray_dists_kernel<<<(n + 255) / 256, 256, 0, s>>>(n, S, near_t, far_t, out);
}
void k_get_rays(int width, const double* K, const double* c2w, float* rays, hipStream_t s) {
    RayCam cam;
    for (int i = 0; i < 9; ++i) cam.K[i] = K[i];
    for (int i = 0; i < 12; ++i) cam.c2w[i] = c2w[i];
    const int n = width * width;
    if (n > 0) get_rays_kernel<<<(n + 255) / 256, 256, 0, s>>>(width, cam, rays);
}
void k_adam(float* params, const float* grads, float* m, float* v, size_t n, int t, float lr,
            float beta1, float beta2, float eps, hipStream_t s) {
    // train_nerf.py:149-159: lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t) AND bias-corrected m/v
    // (the reference applies both corrections); host math in double like numpy's scalars.
    const double bc1 = 1.0 - pow((double)beta1, t), bc2 = 1.0 - pow((double)beta2, t);
    const float lr_t = (float)((double)lr * sqrt(bc2) / bc1);
    if (n)
        adam_kernel<<<grid_for(n), kThreads, 0, s>>>(params, grads, m, v, n, lr_t, beta1, beta2,
                                                     eps, (float)bc1, (float)bc2);
}

}  // namespace lnerf
