// lnerf_composite.h -- per-sample input features and the per-tile compositing (forward,
// loss, reverse) shared by the fused kernels (lnerf_fused.hip, lnerf_k16.hip). Templates over the
// kernel's argument struct (fields: input_mode, x, S, k0, near_t, far_t, rays, rpw, dists,
// target, acc_color, seed, d_target, d_dists). A tile is TS samples of whole rays (128 for k16,
// 256 for the render kernel); threads 0..TS-1 own one sample each, every other thread of the
// workgroup only joins the barriers.
#pragma once
#include "lnerf_internal.h"

namespace lnerf {
namespace comp {

constexpr int kTileSamples = 128;
constexpr int kCompFloats = 21;            // per-sample compositing scratch floats in LDS (21 TS)

// Coordinate c of sample row gs: the given point (POINTS) or o + d t in float64 (RAYS).
template <class A>
__device__ __forceinline__ double sample_coord(const A& a, int gs, int c) {
    if (a.input_mode == LNERF_INPUT_RAYS) {
        const int ray = gs / a.S, j = gs - ray * a.S;
        return ray_point(a.x + (size_t)ray * 6, c, j, a.S, a.near_t, a.far_t);
    }
    return (double)a.x[(size_t)gs * 3 + c];
}

// positional_encoding_3d (pos_encoding.py:54-66) of coordinate c of one sample into its scratch
// row (block-major: x, then sin and cos of 2^q x for q < F). LNERF_PE_DOUBLING: one float64 sincos
// per coordinate, the higher frequencies by the double-angle identities in float64
// (sin 2y = 2 sin y cos y, cos 2y = (cos y - sin y)(cos y + sin y)); after q doublings the error
// is ABSOLUTE, <= ~2^(q+1) float64 ulps of 1 (2^-43 at F = 10; the cos step cancels where cos 2y ~ 0,
// so a value near a zero of sin / cos can be many float32 ulps of itself off, never more than that
// absolute bound, ~2^-19 of float32's resolution of the unit-scale features; on random coordinates
// the rounded float32 values differ from per-frequency sin/cos in <= 7 of 5e6, by one ulp:
// tests/test_pe_doubling.py).
// Otherwise one sincos per frequency, as numpy evaluates it.
#ifndef LNERF_PE_DOUBLING
#define LNERF_PE_DOUBLING 1
#endif
__device__ __forceinline__ void encode_coord(double xc, int F, float* row, int c) {
    row[c] = (float)xc;
    double sn, cs;
    if (LNERF_PE_DOUBLING) sincos(xc, &sn, &cs);
    for (int q = 0; q < F; ++q) {
        if (!LNERF_PE_DOUBLING) sincos(ldexp(xc, q), &sn, &cs);
        row[3 + 6 * q + c] = (float)sn;
        row[6 + 6 * q + c] = (float)cs;
        if (LNERF_PE_DOUBLING) {
            const double s2 = 2.0 * sn * cs;
            cs = (cs - sn) * (cs + sn);
            sn = s2;
        }
    }
}

template <class A>
__device__ __forceinline__ float input_feature(const A& a, int gs, bool valid, int f) {
    if (!valid || f >= a.k0) return 0.0f;
    if (a.input_mode == LNERF_INPUT_ENCODED) return a.x[(size_t)gs * a.k0 + f];
    // positional_encoding_3d (pos_encoding.py:54-66): block-major, float64 trig, rounded once
    const int c = f % 3, blk = f / 3;
    const double xc = sample_coord(a, gs, c);
    if (blk == 0) return (float)xc;
    const int fb = blk - 1, freq = fb >> 1;
    const double arg = ldexp(xc, freq);
    return (fb & 1) ? (float)cos(arg) : (float)sin(arg);
}

// ---- rendering (nerf.py:176-302), loss and its reverse for one TS-sample tile -----------------
// One thread per sample (threads 0..TS-1; a ray = S consecutive samples = one scan segment), the
// along-ray dependencies as segmented Hillis-Steele scans in LDS (log2 S rounds):
//   forward  P_j = prod_{i<=j} c_i (inclusive, T_0 = 1, T_j = P_j: nerf.py:226-272),
//            C = sum_j w_j rgb_j (segmented sum, read at the ray's last sample);
//   reverse  G_j = a_j + c_{j+1} G_{j+1} (the reverse of the inclusive cumprod,
//            a_j = alpha_j dL/dw_j for j >= 1), dc_j = P_{j-1} G_j, dc_0 = G_0.
// Every per-sample expression is loma's (composite rules of lnerf_generic.hip); only the
// association of the along-ray products and sums differs from loma's sequential loops, at fp32
// rounding level (the parity tolerance covers it; the generic path keeps the exact order).
// LDS (floats): z [TS][4] at 0 (in), gz [TS][4] at 4 TS (out), two [4][TS] ping-pong scan
// buffers at 8 TS / 12 TS, P at 16 TS, per-ray dacc [TS][4] at 17 TS (kCompFloats = 21 per sample).
template <int TS = kTileSamples>
__device__ __forceinline__ void seg_scan_fwd(float* buf0, float* buf1, int ls, int j, int S, int nv,
                                             float (&v)[4], bool prod_first) {
    // inclusive segmented scan of nv values (v[0] by product if prod_first, the rest by sum)
    float* cur = buf0;
    float* nxt = buf1;
    for (int d = 1; d < S; d <<= 1) {
        if (ls < TS)
            for (int q = 0; q < nv; ++q) cur[q * TS + ls] = v[q];
        __syncthreads();
        if (ls < TS && j >= d) {
            for (int q = 0; q < nv; ++q) {
                const float o = cur[q * TS + ls - d];
                v[q] = (q == 0 && prod_first) ? o * v[q] : o + v[q];
            }
        }
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    __syncthreads();   // the next scan may write the buffer this one read last
}

template <int TS = kTileSamples, class A>
__device__ __forceinline__ float composite_tile(const A& a, int wg, float* comp, float* rayloss,
                                                bool grad) {
    const int tid = threadIdx.x, S = a.S;
    float* c_z = comp;
    float* c_gz = comp + 4 * TS;
    float* sb0 = comp + 8 * TS;
    float* sb1 = comp + 12 * TS;
    float* c_P = comp + 16 * TS;
    float* c_ray = comp + 17 * TS;            // [TS rays][4]: dacc0..2 of each ray
    const int ntile = a.rpw * S;              // samples of whole rays in this tile
    const int ls = tid < TS ? tid : TS;       // threads >= TS only sync
    const int rl = ls / S, j = ls - rl * S;   // ray within the tile, sample within the ray
    const int ray = wg * a.rpw + rl;
    const bool valid = ls < ntile && ray < a.rays;
    const size_t gs = (size_t)ray * S + j;
    float z[4] = {0, 0, 0, 0}, rgb[3] = {0, 0, 0}, sigma = 0, delta = 0, al = 0, cc = 1;
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = c_z[ls * 4 + k];
        // head activation (nerf.py:153-167): channel 3 ReLU, 0..2 sigmoid
#pragma unroll
        for (int k = 0; k < 3; ++k) rgb[k] = 1.0f / (1.0f + expf(0.0f - z[k]));
        sigma = (z[3] > 0.0f) ? z[3] : 0.0f;
        delta = a.dists ? a.dists[gs] : ray_delta(j, S, a.near_t, a.far_t);
        al = 1.0f - expf((0.0f - sigma) * delta);
        cc = (1.0f - al) + (float)(1e-10);
    }
    // P_j (inclusive product), T_j, w_j
    float v[4] = {cc, 0, 0, 0};
    seg_scan_fwd<TS>(sb0, sb1, ls, j, S, 1, v, true);
    const float P = v[0];
    const float T = (j == 0) ? 1.0f : P;
    const float w = al * T;
    if (ls < TS) c_P[ls] = P;
    // colour: segmented sum of w * rgb (read at the ray's last sample)
    float cv[4] = {w * rgb[0], w * rgb[1], w * rgb[2], 0};
    seg_scan_fwd<TS>(sb0, sb1, ls, j, S, 3, cv, false);
    float loss = 0.0f;
    const bool last = valid && j == S - 1;
    if (last) {
        const float* t = a.target + (size_t)ray * 3;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            loss = loss + (cv[k] - t[k]) * (cv[k] - t[k]);
            if (a.acc_color) a.acc_color[(size_t)ray * 3 + k] = cv[k];
        }
        if (grad) {
            // reverse of the loss (lg_composite_bwd_kernel): dacc = 2 seed (C - t)
            for (int k = 2; k >= 0; --k) {
                const float a1 = (cv[k] - t[k]) * a.seed;
                const float a2 = 0.0f - ((cv[k] - t[k]) * a.seed);
                c_ray[rl * 4 + k] = 0.0f + a1 + a1;
                if (a.d_target) a.d_target[(size_t)ray * 3 + k] = (0.0f + a2) + a2;
            }
        }
    }
    if (tid < a.rpw) rayloss[tid] = 0.0f;
    __syncthreads();
    if (last) rayloss[rl] = loss;
    if (!grad) return 0.0f;

    // ---- reverse, per sample ----
    float dacc[3] = {0, 0, 0}, dw = 0.0f, drgb[4] = {0, 0, 0, 0};
    if (valid) {
#pragma unroll
        for (int k = 0; k < 3; ++k) dacc[k] = c_ray[rl * 4 + k];
        for (int k = 2; k >= 0; --k) {
            dw += rgb[k] * dacc[k];
            drgb[k] += w * dacc[k];
        }
    }
    float dal = T * dw;
    // G_j = a_j + c_{j+1} G_{j+1}: segmented suffix scan of (a, b) pairs
    float ga = (j >= 1) ? al * dw : 0.0f;
    float gb = 0.0f;
    if (ls < TS) sb0[ls] = cc;
    __syncthreads();
    if (valid && j + 1 < S) gb = sb0[ls + 1];
    __syncthreads();
    {
        float* cur = sb0;
        float* nxt = sb1;
        for (int d = 1; d < S; d <<= 1) {
            if (ls < TS) {
                cur[ls] = ga;
                cur[TS + ls] = gb;
            }
            __syncthreads();
            if (ls < TS && j + d < S) {
                const float oa = cur[ls + d], ob = cur[TS + ls + d];
                ga = ga + gb * oa;
                gb = gb * ob;
            }
            float* t = cur;
            cur = nxt;
            nxt = t;
        }
    }
    if (valid) {
        const float dc = (j >= 1) ? c_P[ls - 1] * ga : ga;
        dal += 0.0f - dc;                                       // cC = (1 - al) + 1e-10
        const float adj2 = (0.0f - dal) * expf((0.0f - sigma) * delta);   // alpha reverse
        drgb[3] += 0.0f - (delta * adj2);
        if (a.d_dists) a.d_dists[gs] = 0.0f + (0.0f - sigma) * adj2;
        // head activation reverse (reverse_diff.py Div/exp/Sub rules; ReLU on the post value)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float dz = drgb[k];
            float g;
            if (k == 3) {
                g = (sigma > 0.0f) ? dz : 0.0f;
            } else {
                const float x = z[k];
                const float u = 1.0f + expf(0.0f - x);
                const float adj_div = ((0.0f - dz) * 1.0f) / (u * u);
                g = 0.0f + (0.0f - adj_div * expf(0.0f - x));
            }
            c_gz[ls * 4 + k] = g;
        }
    } else if (ls < TS) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c_gz[ls * 4 + k] = 0.0f;
    }
    return 0.0f;
}

// ---- forward-only compositing for the render (kr): composite_tile's per-sample expressions and
// results, with each along-ray scan done inside the wave (shuffles, log2 64 steps) plus one carry
// across the waves a ray spans (its earlier waves' partials through LDS): two workgroup barriers
// instead of composite_tile's 2 (log2 S + 1). The products and sums associate differently from
// composite_tile's LDS rounds (and from loma's sequential loops), at fp32 rounding level. Threads
// 0..TS-1 own one sample each; z [TS][4] at comp[0], the wave partials [TS / 64][4] at comp[4 TS].
template <int TS, class A>
__device__ __forceinline__ void composite_fwd_wave(const A& a, int wg, float* comp, float* rayloss) {
    static_assert(TS % 64 == 0, "whole waves of samples");
    const int tid = threadIdx.x, S = a.S, lane = tid & 63, wv = tid >> 6;
    float* c_z = comp;
    float* pub = comp + 4 * TS;
    const bool act = tid < TS;
    const int ls = act ? tid : 0;
    const int rl = ls / S, j = ls - rl * S;   // ray within the tile, sample within the ray
    const int ray = wg * a.rpw + rl;
    const int ntile = a.rpw * S;
    const bool valid = act && ls < ntile && ray < a.rays;
    const size_t gs = (size_t)ray * S + j;
    float rgb[3] = {0, 0, 0}, al = 0, cc = 1;
    if (valid) {
        float z[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = c_z[ls * 4 + k];
        // head activation (nerf.py:153-167): channel 3 ReLU, 0..2 sigmoid
#pragma unroll
        for (int k = 0; k < 3; ++k) rgb[k] = 1.0f / (1.0f + expf(0.0f - z[k]));
        const float sigma = (z[3] > 0.0f) ? z[3] : 0.0f;
        const float delta = a.dists ? a.dists[gs] : ray_delta(j, S, a.near_t, a.far_t);
        al = 1.0f - expf((0.0f - sigma) * delta);
        cc = (1.0f - al) + (float)(1e-10);
    }
    const int jw = j < lane ? j : lane;        // this ray's samples before this one in this wave
    const int ws = (ls - j) >> 6;              // the wave holding the ray's first sample
    // P_j, the inclusive product (nerf.py:226-272): in-wave, then the earlier waves' partials
    float P = cc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(P, d, 64);
        if (jw >= d) P = o * P;
    }
    if (act && lane == 63) pub[wv * 4] = P;
    __syncthreads();
    if (act)
        for (int w = wv - 1; w >= ws; --w) P = pub[w * 4] * P;
    const float T = (j == 0) ? 1.0f : P;
    const float wgt = al * T;
    // colour: the segmented sum of w rgb, read at the ray's last sample
    float cv[3] = {wgt * rgb[0], wgt * rgb[1], wgt * rgb[2]};
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float o = __shfl_up(cv[k], d, 64);
            if (jw >= d) cv[k] = o + cv[k];
        }
    }
    if (act && lane == 63)
#pragma unroll
        for (int k = 0; k < 3; ++k) pub[wv * 4 + 1 + k] = cv[k];
    __syncthreads();
    if (act && j == S - 1 && ls < ntile) {
        for (int w = wv - 1; w >= ws; --w)
#pragma unroll
            for (int k = 0; k < 3; ++k) cv[k] = pub[w * 4 + 1 + k] + cv[k];
        float loss = 0.0f;
        if (valid) {
            const float* t = a.target + (size_t)ray * 3;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                loss = loss + (cv[k] - t[k]) * (cv[k] - t[k]);
                if (a.acc_color) a.acc_color[(size_t)ray * 3 + k] = cv[k];
            }
        }
        rayloss[rl] = loss;
    }
}

// ---- composite_tile with the along-ray scans inside the wave (training, k1): the same per-sample
// expressions and outputs (z in at comp[0], gz out at comp[4 TS], rayloss, acc_color, d_target,
// d_dists), the forward scans as in composite_fwd_wave and the reverse suffix scan of
// G_j = a_j + c_{j+1} G_{j+1} by shuffles down plus the later waves' partials: four workgroup
// barriers instead of composite_tile's 3 log2(S) + 4. LDS: wave partials [TS / 64][8] at 8 TS,
// c_j at 9 TS, P_j at 10 TS, per-ray dacc [rays][4] at 11 TS (within kCompFloats = 21 per sample).
template <int TS, class A>
__device__ __forceinline__ void composite_tile_wave(const A& a, int wg, float* comp, float* rayloss, bool grad) {
    static_assert(TS % 64 == 0, "whole waves of samples");
    static_assert((TS / 64) * 8 <= TS, "the wave partials [TS / 64][8] fit their TS-float region at 8 TS");
    const int tid = threadIdx.x, S = a.S, lane = tid & 63, wv = tid >> 6;
    float* c_z = comp;
    float* c_gz = comp + 4 * TS;
    float* pub = comp + 8 * TS;
    float* c_cc = comp + 9 * TS;
    float* c_P = comp + 10 * TS;
    float* c_ray = comp + 11 * TS;
    const bool act = tid < TS;
    const int ls = act ? tid : 0;
    const int rl = ls / S, j = ls - rl * S;   // ray within the tile, sample within the ray
    const int ray = wg * a.rpw + rl;
    const int ntile = a.rpw * S;
    const bool valid = act && ls < ntile && ray < a.rays;
    const size_t gs = (size_t)ray * S + j;
    float z[4] = {0, 0, 0, 0}, rgb[3] = {0, 0, 0}, sigma = 0, delta = 0, al = 0, cc = 1;
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = c_z[ls * 4 + k];
        // head activation (nerf.py:153-167): channel 3 ReLU, 0..2 sigmoid
#pragma unroll
        for (int k = 0; k < 3; ++k) rgb[k] = 1.0f / (1.0f + expf(0.0f - z[k]));
        sigma = (z[3] > 0.0f) ? z[3] : 0.0f;
        delta = a.dists ? a.dists[gs] : ray_delta(j, S, a.near_t, a.far_t);
        al = 1.0f - expf((0.0f - sigma) * delta);
        cc = (1.0f - al) + (float)(1e-10);
    }
    const int jw = j < lane ? j : lane;        // this ray's samples before this one in this wave
    const int ws = (ls - j) >> 6;              // the wave holding the ray's first sample
    // P_j, the inclusive product (nerf.py:226-272)
    float P = cc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(P, d, 64);
        if (jw >= d) P = o * P;
    }
    if (act) {
        if (lane == 63) pub[wv * 8] = P;
        c_cc[ls] = cc;
    }
    __syncthreads();
    if (act) {
        for (int w = wv - 1; w >= ws; --w) P = pub[w * 8] * P;
        c_P[ls] = P;
    }
    const float T = (j == 0) ? 1.0f : P;
    const float wgt = al * T;
    // colour: the segmented sum of w rgb, read at the ray's last sample
    float cv[3] = {wgt * rgb[0], wgt * rgb[1], wgt * rgb[2]};
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float o = __shfl_up(cv[k], d, 64);
            if (jw >= d) cv[k] = o + cv[k];
        }
    }
    if (act && lane == 63)
#pragma unroll
        for (int k = 0; k < 3; ++k) pub[wv * 8 + 1 + k] = cv[k];
    __syncthreads();
    if (act && j == S - 1 && ls < ntile) {
        for (int w = wv - 1; w >= ws; --w)
#pragma unroll
            for (int k = 0; k < 3; ++k) cv[k] = pub[w * 8 + 1 + k] + cv[k];
        float loss = 0.0f;
        if (valid) {
            const float* t = a.target + (size_t)ray * 3;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                loss = loss + (cv[k] - t[k]) * (cv[k] - t[k]);
                if (a.acc_color) a.acc_color[(size_t)ray * 3 + k] = cv[k];
            }
            if (grad) {
                // reverse of the loss (lg_composite_bwd_kernel): dacc = 2 seed (C - t)
                for (int k = 2; k >= 0; --k) {
                    const float a1 = (cv[k] - t[k]) * a.seed;
                    const float a2 = 0.0f - ((cv[k] - t[k]) * a.seed);
                    c_ray[rl * 4 + k] = 0.0f + a1 + a1;
                    if (a.d_target) a.d_target[(size_t)ray * 3 + k] = (0.0f + a2) + a2;
                }
            }
        }
        rayloss[rl] = loss;
    }
    if (!grad) return;
    __syncthreads();

    // ---- reverse, per sample ----
    float dacc[3] = {0, 0, 0}, dw = 0.0f, drgb[4] = {0, 0, 0, 0};
    if (valid) {
#pragma unroll
        for (int k = 0; k < 3; ++k) dacc[k] = c_ray[rl * 4 + k];
        for (int k = 2; k >= 0; --k) {
            dw += rgb[k] * dacc[k];
            drgb[k] += wgt * dacc[k];
        }
    }
    float dal = T * dw;
    // G_j = a_j + c_{j+1} G_{j+1}: the suffix composition of (a, b) pairs, in-wave, then the later
    // waves' partials (their lane 0's composition; the ray's last sample has b = 0)
    float ga = (j >= 1) ? al * dw : 0.0f;
    float gb = (valid && j + 1 < S) ? c_cc[ls + 1] : 0.0f;
    const int rest = S - 1 - j, lrest = 63 - lane;
    const int je = rest < lrest ? rest : lrest;   // this ray's samples after this one in this wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const float oa = __shfl_down(ga, d, 64), ob = __shfl_down(gb, d, 64);
        if (je >= d) {
            ga = ga + gb * oa;
            gb = gb * ob;
        }
    }
    if (act && lane == 0) {
        pub[wv * 8 + 4] = ga;
        pub[wv * 8 + 5] = gb;
    }
    __syncthreads();
    // the wave holding the ray's last sample; a pseudo-ray past the tile's last whole ray (ls >=
    // ntile, never valid) may end past the last wave: clamped, so the carry never reads past pub's
    // [TS / 64][8] partials
    const int we = min((ls - j + S - 1) >> 6, TS / 64 - 1);
    if (act && we > wv) {
        float gn = 0.0f;
        for (int w = we; w > wv; --w) gn = pub[w * 8 + 4] + pub[w * 8 + 5] * gn;
        ga = ga + gb * gn;
    }
    if (valid) {
        const float dc = (j >= 1) ? c_P[ls - 1] * ga : ga;
        dal += 0.0f - dc;                                       // cC = (1 - al) + 1e-10
        const float adj2 = (0.0f - dal) * expf((0.0f - sigma) * delta);   // alpha reverse
        drgb[3] += 0.0f - (delta * adj2);
        if (a.d_dists) a.d_dists[gs] = 0.0f + (0.0f - sigma) * adj2;
        // head activation reverse (reverse_diff.py Div/exp/Sub rules; ReLU on the post value)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float dz = drgb[k];
            float g;
            if (k == 3) {
                g = (sigma > 0.0f) ? dz : 0.0f;
            } else {
                const float x = z[k];
                const float u = 1.0f + expf(0.0f - x);
                const float adj_div = ((0.0f - dz) * 1.0f) / (u * u);
                g = 0.0f + (0.0f - adj_div * expf(0.0f - x));
            }
            c_gz[ls * 4 + k] = g;
        }
    } else if (act) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c_gz[ls * 4 + k] = 0.0f;
    }
}

// ---- the mlp_fit head (scripts/mlp_fit.py:120-145, fit_img.py:423-532) for one tile ----------
// One thread per row (S = 1, so a "ray" is a row): sigmoid on each of the nout <= 4 head outputs
// (mlp_fit.py:127-132: 1 / (1 + exp(0 - x))), loss = sum_c (o_c - t_c)^2 (mlp_fit.py:140-145;
// the rows' partial sums are added in a tree by the caller instead of loma's sequential loop),
// and its reverse with loma's adjoint expressions: d_o = 0 + a1 + a1 with a1 = (o - t) seed
// (the two reads of the squared difference), d_target = (0 + a2) + a2, a2 = 0 - (o - t) seed,
// then the sigmoid's Div/exp/Sub reverse on the pre-activation (lg_act_bwd_kernel's form).
// LDS as composite_tile: comp[0..512) z [128][4] in, [512..1024) gz [128][4] out. `nout` is the
// head width; a.target / a.acc_color / a.d_target are (rows, nout).
template <class A>
__device__ __forceinline__ float fit_tile(const A& a, int wg, float* comp, float* rayloss, bool grad, int nout) {
    const int tid = threadIdx.x;
    float* c_z = comp;
    float* c_gz = comp + 512;
    const int ls = tid < kTileSamples ? tid : kTileSamples;
    const int row = wg * a.rpw + ls;
    const bool valid = ls < a.rpw && row < a.rays;
    float loss = 0.0f;
    if (valid) {
        const float* t = a.target + (size_t)row * nout;
        for (int k = 0; k < nout; ++k) {
            const float x = c_z[ls * 4 + k];
            const float o = 1.0f / (1.0f + expf(0.0f - x));
            loss = loss + (o - t[k]) * (o - t[k]);
            if (a.acc_color) a.acc_color[(size_t)row * nout + k] = o;
            if (grad) {
                const float a1 = (o - t[k]) * a.seed;
                const float a2 = 0.0f - ((o - t[k]) * a.seed);
                const float dz = 0.0f + a1 + a1;
                if (a.d_target) a.d_target[(size_t)row * nout + k] = (0.0f + a2) + a2;
                const float u = 1.0f + expf(0.0f - x);
                const float adj_div = ((0.0f - dz) * 1.0f) / (u * u);
                c_gz[ls * 4 + k] = 0.0f + (0.0f - adj_div * expf(0.0f - x));
            }
        }
        if (grad)
            for (int k = nout; k < 4; ++k) c_gz[ls * 4 + k] = 0.0f;
    } else if (grad && ls < kTileSamples) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c_gz[ls * 4 + k] = 0.0f;
    }
    if (ls < a.rpw) rayloss[ls] = loss;
    __syncthreads();
    return 0.0f;
}

}  // namespace comp
}  // namespace lnerf
