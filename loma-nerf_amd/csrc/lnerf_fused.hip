// lnerf_fused.hip -- the throughput path's plan and orchestration: the workspace layout, the
// reductions, and the kernel sequence of one fused training step or render.
//
// Hot path of the reference: scripts/nerf.py:1-304 (forward) and its rev_diff (:306), called per
// chunk from train_nerf.py:325/395. Here one step handles the whole batch:
//
//  k0  wmax16 + pack16       the fp16x3 / bf16 weight planes in fragment order (lnerf_k16.hip)
//  k1  k16_fwd_bwd_kernel    sampling + PE + MLP forward + compositing + loss + reverse chain on
//                            v_mfma_f32_16x16x32_{f16,bf16}, writing the A_l / G_l slabs
//                            (lnerf_k16.hip)
//  k1r k1_reduce_kernel      the batch loss and the per-layer dW product shifts (lnerf_dw16.hip)
//  k2  dw16_kernel           dW_l = sum_s A_{l-1}^T G_l, db_l = sum_s G_l from the slabs
//                            (lnerf_dw16.hip)
//  k3  grad_reduce_kernel    in-order split sums into the reference's padded (L, Kmax, Nmax) layout,
//                            scaled by the loss seed (deterministic, no atomics)
//
// Round 4 removed the round-1 one-wave-per-SIMD kernel pair (exact-f32 MFMA and an older bf16x6
// schedule; LNERF_ONE_WAVE / LNERF_MFMA_F32) and k32 (LNERF_K32): both lost to k16 on time and both
// read LDS through inline asm whose destination registers the compiler could reuse before the data
// landed. Exact fp32 arithmetic stays available on the loma-order path
// (LNERF_GENERIC).
#include "lnerf_internal.h"

#include <stdio.h>

namespace lnerf {

namespace {

constexpr int kTileSamples = 128;   // samples per k16 workgroup (8 waves x 16); 64 with K16_W4

// ---------------------------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------------------------
// Deterministic two-level sum of the per-workgroup partial losses (render): 256 strided
// sequential sums, then a fixed-order tree in LDS (the same order as k1_reduce_kernel's).
__global__ void __launch_bounds__(256) loss_reduce_kernel(const float* __restrict__ part, int n,
                                                          float* total, float* out_loss) {
    __shared__ float red[256];
    const int t = threadIdx.x;
    float s = 0.0f;
    for (int i = t; i < n; i += 256) s += part[i];
    red[t] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) red[t] = red[t] + red[t + w];
        __syncthreads();
    }
    if (t == 0) {
        *total = red[0];
        if (out_loss) *out_loss = red[0];
    }
}

// Stage 1 of the render's loss reduction (one 256-thread block summing the
// 320 000 partials of a config-5 frame serially took 0.285 ms): block b sums the contiguous range
// [b per, (b + 1) per) of the partials by the same strided-then-tree order, into stage[b];
// loss_reduce_kernel then sums the kLossStage1 block sums. Fixed grid, fixed order: deterministic.
constexpr int kLossStage1 = 256;
__global__ void __launch_bounds__(256) loss_stage1_kernel(const float* __restrict__ part, int n, int per,
                                                          float* __restrict__ stage) {
    __shared__ float red[256];
    const int t = threadIdx.x, b0 = blockIdx.x * per, b1 = min(n, b0 + per);
    float s = 0.0f;
    for (int i = b0 + t; i < b1; i += 256) s += part[i];
    red[t] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) red[t] = red[t] + red[t + w];
        __syncthreads();
    }
    if (t == 0) stage[blockIdx.x] = red[0];
}

struct ReduceArgs {
    int L;
    int k[kMaxLayers], n[kMaxLayers], kt[kMaxLayers], nt[kMaxLayers];
    int w_k, w_n;
    int splits[kMaxLayers];      // dW / dB partials per layer
    const float* dw_part;
    size_t dwp_off[kMaxLayers];
    const float* db_part;
    size_t dbp_off[kMaxLayers];
    float* d_ws;
    float* d_bs;
    const float* scale;          // nullable device scalar (seed = loss)
    int accumulate;
};

// In-order sum of n strided partials (deterministic); loads are issued 8 at a time so the
// reduction streams at HBM rate instead of waiting on one load per add.
__device__ __forceinline__ float sum_parts(const float* __restrict__ p, size_t stride, int n) {
    float s = 0.0f;
    int q = 0;
    for (; q + 8 <= n; q += 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = __builtin_nontemporal_load(p + (size_t)(q + u) * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; q < n; ++q) s += p[(size_t)q * stride];
    return s;
}

__global__ void grad_reduce_kernel(ReduceArgs a) {
    const size_t nW = (size_t)a.L * a.w_k * a.w_n, nB = (size_t)a.L * a.w_n;
    const float sc = a.scale ? *a.scale : 1.0f;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nW + nB;
         e += (size_t)gridDim.x * blockDim.x) {
        if (e < nW) {
            if (!a.d_ws) continue;
            const int l = (int)(e / ((size_t)a.w_k * a.w_n));
            const int k = (int)((e / a.w_n) % a.w_k), j = (int)(e % a.w_n);
            float v = 0.0f;
            if (k < a.k[l] && j < a.n[l]) {
                const int ncol = a.nt[l] * 32;
                const size_t slab = (size_t)a.kt[l] * 32 * ncol;
                const float* p = a.dw_part + a.dwp_off[l] + (size_t)k * ncol + j;
                v = sum_parts(p, slab, a.splits[l]);
                if (a.scale) v *= sc;
            }
            a.d_ws[e] = a.accumulate ? a.d_ws[e] + v : v;
        } else {
            if (!a.d_bs) continue;
            const size_t eb = e - nW;
            const int l = (int)(eb / a.w_n), j = (int)(eb % a.w_n);
            float v = 0.0f;
            if (j < a.n[l]) {
                const int ncol = a.nt[l] * 32;
                const float* p = a.db_part + a.dbp_off[l] + j;
                v = sum_parts(p, (size_t)ncol, a.splits[l]);
                if (a.scale) v *= sc;
            }
            a.d_bs[eb] = a.accumulate ? a.d_bs[eb] + v : v;
        }
    }
}

constexpr size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
inline int pow2_16(int t) { return t <= 1 ? 1 : t <= 2 ? 2 : t <= 4 ? 4 : t <= 8 ? 8 : 16; }

// Sizes and offsets of one step's workspace (floats unless noted).
struct Layout {
    int ht16, ks16_f[kMaxLayers], ks16_b[kMaxLayers], to16_f[kMaxLayers], to16_b[kMaxLayers];
    size_t w16f_off[kMaxLayers], w16b_off[kMaxLayers], w16_total;   // u16
    size_t b16_total;
    size_t mask_total;                                               // u64
    size_t act_off[kMaxLayers], x_off, act_total;
    size_t grad_off[kMaxLayers], grad_total;
    int splits[kMaxLayers], wg_off[kMaxLayers], dw_grid;
    size_t dwp_off[kMaxLayers], dwp_total, dbp_off[kMaxLayers], dbp_total;
    int num_wg, blocks, rpw;
};

// train = false (render): no slabs, masks or dW partials (the forward-only kernel writes none).
// a_tile: float slots per 32 x 32 tile-block of an activation slab (a_tile_floats: 768 for int24 A
// slabs, 1024 for fp32; the workspace is sized with 1024)
void make_layout(Layout& y, const lnerf_mlp& m, int rays, int S, bool train, int dw_grid, int tile,
                 int a_tile = 1024) {
    const int L = m.num_layers;
    int kt[kMaxLayers], nt[kMaxLayers];
    for (int l = 0; l < L; ++l) {
        kt[l] = (m.k[l] + 31) / 32;
        nt[l] = (m.n[l] + 31) / 32;
    }
    // k16 packing: every hidden layer's forward and every l >= 1 backward with ht16 16-wide output
    // tiles, the head forward with 1 and the dX pass with pow2(k0 / 16); per layer and pass, 3
    // planes of [k-step][output tile][1 KiB] (sized for bf16x6; fp16x3 / bf16 use 2 / 1)
    int mx16 = 1;
    for (int l = 0; l + 1 < L; ++l) mx16 = (m.n[l] + 15) / 16 > mx16 ? (m.n[l] + 15) / 16 : mx16;
    y.ht16 = pow2_16(mx16);
    size_t off = 0;
    for (int l = 0; l < L; ++l) {
        y.ks16_f[l] = kt[l];
        y.ks16_b[l] = nt[l];
        y.to16_f[l] = (l < L - 1) ? y.ht16 : 1;
        y.to16_b[l] = (l >= 1) ? y.ht16 : pow2_16((m.k[0] + 15) / 16);
        y.w16f_off[l] = off; off += align_up((size_t)y.ks16_f[l] * y.to16_f[l] * 3 * 512, 512);
        y.w16b_off[l] = off; off += align_up((size_t)y.ks16_b[l] * y.to16_b[l] * 3 * 512, 512);
    }
    y.w16_total = off;
    y.b16_total = (size_t)L * 256;
    y.rpw = S >= tile ? 1 : tile / S;
    y.num_wg = (rays + y.rpw - 1) / y.rpw;
    y.mask_total = train ? (size_t)y.num_wg * (L > 1 ? L - 1 : 0) * (tile / 16) * 64 : 0;
    y.blocks = y.num_wg * (tile / 32);
    off = 0;
    y.x_off = off; off += (size_t)y.blocks * kt[0] * a_tile;
    for (int l = 0; l < L - 1; ++l) { y.act_off[l] = off; off += (size_t)y.blocks * nt[l] * a_tile; }
    y.act_total = train ? off : 0;
    off = 0;
    for (int l = 0; l < L; ++l) { y.grad_off[l] = off; off += (size_t)y.blocks * nt[l] * 1024; }
    y.grad_total = train ? off : 0;
    // dW: one launch over every layer, ~dw_grid workgroups (lnerf_ctx_set_option
    // LNERF_OPT_DW_GRID; 512 by default) split between the layers in proportion to the slab bytes
    // each one streams (kt + nt tiles per 32-sample block): the kernel is bandwidth-bound, so
    // equal bytes per workgroup balance it. One partial per split.
    const int grid = dw_grid > 0 ? (dw_grid < 16 ? 16 : dw_grid > 4096 ? 4096 : dw_grid)
                                 : default_dw_grid((long long)rays * S);
    auto weight = [&](int l) { return kt[l] + nt[l]; };
    int tiles_sum = 0;
    for (int l = 0; l < L; ++l) tiles_sum += weight(l);
    size_t dwp = 0, dbp = 0;
    int wg = 0;
    for (int l = 0; l < L; ++l) {
        int sp = (int)((long long)grid * weight(l) / tiles_sum);
        sp = sp < 1 ? 1 : sp;
        sp = sp > y.blocks ? y.blocks : sp;
        y.splits[l] = sp;
        y.wg_off[l] = wg;
        wg += sp;
        y.dwp_off[l] = dwp;
        dwp += (size_t)sp * kt[l] * 32 * nt[l] * 32;
        y.dbp_off[l] = dbp;
        dbp += (size_t)sp * nt[l] * 32;
    }
    y.dw_grid = wg;
    y.dwp_total = train ? dwp : 0;
    y.dbp_total = train ? dbp : 0;
}

}  // namespace

bool fused_supported(const lnerf_mlp& m, int rays, int S, int input_mode, const char** why, bool head_fit) {
    const char* w = nullptr;
    if (m.num_layers < 1 || m.num_layers > kMaxLayers) w = "num_layers out of range";
    else if (S < 1 || S > kTileSamples) w = "fused path needs 1 <= samples <= 128";
    else if (rays < 1) w = "no rays";
    else if (head_fit && (S != 1 || m.n[m.num_layers - 1] > 4 || input_mode != LNERF_INPUT_ENCODED))
        w = "the mlp_fit head needs samples == 1, 1..4 outputs and ENCODED input";
    else if (!head_fit && m.n[m.num_layers - 1] < 4) w = "head must have >= 4 outputs (rgb + sigma)";
    else if (m.n[m.num_layers - 1] > 16) w = "fused path needs a head with <= 16 outputs (one 16-wide tile)";
    else {
        for (int l = 0; l < m.num_layers && !w; ++l) {
            if (m.k[l] < 1 || m.k[l] > 256 || m.n[l] < 1 || m.n[l] > 256) w = "layer widths must be in 1..256";
            else if (l > 0 && m.k[l] != m.n[l - 1]) w = "k[l] must equal n[l-1]";
            else if (m.k[l] > m.w_k || m.n[l] > m.w_n) w = "padded weight layout too small";
        }
    }
    if (why) *why = w;
    return w == nullptr;
}

static size_t workspace_floats(const lnerf_mlp& m, int rays, int S, bool train, int dw_grid, int tile) {
    Layout y;
    make_layout(y, m, rays, S, train, dw_grid, tile);
    return 64 + align_up(y.act_total, 64) + align_up(y.grad_total, 64) + align_up((size_t)y.num_wg, 64) +
           align_up(y.dwp_total, 64) + align_up(y.dbp_total, 64) + 64 + align_up((size_t)kLossStage1, 64) +
           2 * align_up((y.w16_total + 1) / 2, 64) +   // + the guard's bf16x6 planes
           align_up(y.b16_total, 64) + align_up(y.mask_total * 2, 64) + 64 +   // + the fp16x3 shifts
           align_up((size_t)kMaxLayers * kWmaxParts + kWmaxParts * kHeadCols, 64) +   // per-block max|W|
           align_up((size_t)kHeadCols, 64) +                                     // head column max|W|
           (train ? align_up((size_t)m.num_layers * y.num_wg * tile, 64) +      // per-sample words
                        align_up((size_t)m.num_layers * y.num_wg * 8, 64) +         // per-wave minima
                        align_up((size_t)2 * y.dw_grid, 64) : 0);                   // exceptional rows
}

// Either tile size (fused_plan runs 64 under LNERF_K16_W4, 128 otherwise).
size_t fused_workspace_bytes(const lnerf_mlp& m, int rays, int S, bool train, int dw_grid) {
    size_t f = workspace_floats(m, rays, S, train, dw_grid, kTileSamples);
    if (S <= 64) {
        const size_t f64 = workspace_floats(m, rays, S, train, dw_grid, 64);
        f = f64 > f ? f64 : f;
    }
    return f * sizeof(float);
}

static void fused_plan_tile(FusedPlan& p, const lnerf_mlp& m, const lnerf_batch& b, void* ws_base, int flags,
                            bool train, int dw_grid, int tile) {
    const int x6 = (flags & LNERF_MFMA_BF16) ? 1 : (flags & LNERF_MFMA_BF16X6) ? 3 : 2;   // fp16x3 default
    Layout y;
    make_layout(y, m, b.rays, b.samples, train, dw_grid, tile, a_tile_floats(x6));
    p = FusedPlan{};
    p.tile = tile;
    p.L = m.num_layers;
    p.x6 = x6;
    for (int l = 0; l < p.L; ++l) {
        p.k[l] = m.k[l];
        p.n[l] = m.n[l];
        p.kt[l] = (m.k[l] + 31) / 32;
        p.nt[l] = (m.n[l] + 31) / 32;
        p.act_off[l] = (l < p.L - 1) ? y.act_off[l] : 0;
        p.grad_off[l] = y.grad_off[l];
        p.dw_splits[l] = y.splits[l];
        p.dw_split_off[l] = y.wg_off[l];
        p.dwp_off[l] = y.dwp_off[l];
        p.dbp_off[l] = y.dbp_off[l];
        p.ks16_f[l] = y.ks16_f[l];
        p.ks16_b[l] = y.ks16_b[l];
        p.to16_f[l] = y.to16_f[l];
        p.to16_b[l] = y.to16_b[l];
        p.w16f_off[l] = y.w16f_off[l];
        p.w16b_off[l] = y.w16b_off[l];
    }
    p.ht16 = y.ht16;
    p.w_k = m.w_k;
    p.w_n = m.w_n;
    p.rays = b.rays;
    p.S = b.samples;
    p.R = b.rays * b.samples;
    p.rays_per_wg = y.rpw;
    p.num_wg = y.num_wg;
    p.blocks = y.blocks;
    p.input_mode = b.input_mode;
    p.F = b.num_freqs;
    p.dw_grid = y.dw_grid;
    p.x_off = y.x_off;
    float* base = (float*)ws_base;
    size_t off = 0;
    auto take = [&](size_t floats) {
        float* q = base + off;
        off += align_up(floats, 64);
        return q;
    };
    // every region but the activation slabs (whose size follows the split: a_tile_floats) first, so
    // that the fp16x3 plan and its bf16x6 re-run (the floor guard) share all other pointers
    p.guard = (int*)take(64);
    p.grad = take(y.grad_total);
    p.loss_part = take((size_t)y.num_wg);
    p.dw_part = take(y.dwp_total);
    p.db_part = take(y.dbp_total);
    p.loss_total = take(1);
    p.loss_stage = take(kLossStage1);
    p.w16 = (unsigned short*)take((y.w16_total + 1) / 2);
    p.w16x = (unsigned short*)take((y.w16_total + 1) / 2);
    p.b16 = take(y.b16_total);
    p.mask_g = (unsigned long long*)take(y.mask_total * 2);
    p.wexp16 = (int*)take(2 * kMaxLayers);
    p.dw_shift = p.wexp16 + kMaxLayers;
    p.wmax_part = (int*)take((size_t)kMaxLayers * kWmaxParts + kWmaxParts * kHeadCols);
    p.hexp16 = (int*)take((size_t)kHeadCols);
    p.sexp = (unsigned*)(base + off);                                // L x num_wg x tile words
    if (train) off += align_up((size_t)p.L * y.num_wg * tile, 64);
    p.epart = (int*)(base + off);
    if (train) off += align_up((size_t)p.L * y.num_wg * 8, 64);
    p.xcount = (int*)(base + off);
    if (train) off += align_up((size_t)2 * y.dw_grid, 64);
    p.act = take(y.act_total);
}

void fused_plan(FusedPlan& p, const lnerf_mlp& m, const lnerf_batch& b, void* ws_base, int flags, bool train,
                int dw_grid) {
    if (flags & LNERF_K16_W4) {
        // k16 on 4-wave, 64-sample workgroups (two per CU): whole rays must fit 64 samples and the
        // ring 80 KiB (fp16x3 / plain bf16). Measured slower than the 8-wave workgroup at cfg3
        // (the second workgroup doubles the weight stream's LDS-DMA). An explicit
        // request that cannot run is an error, never a silent fall-back.
        if (flags & LNERF_MFMA_BF16X6) marshal::fail("LNERF_K16_W4 does not run the bf16x6 split (its ring needs 96 KiB)");
        if (b.samples > 64) marshal::fail("LNERF_K16_W4 needs samples <= 64 (whole rays in a 64-sample tile)");
        fused_plan_tile(p, m, b, ws_base, flags, train, dw_grid, 64);
    } else {
        fused_plan_tile(p, m, b, ws_base, flags, train, dw_grid, kTileSamples);
    }
    p.head_fit = (flags & LNERF_HEAD_FIT) ? 1 : 0;
}

static ReduceArgs reduce_args(const FusedPlan& p, const lnerf_outputs& out, int flags) {
    ReduceArgs ra{};
    ra.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        ra.k[l] = p.k[l];
        ra.n[l] = p.n[l];
        ra.kt[l] = p.kt[l];
        ra.nt[l] = p.nt[l];
        ra.splits[l] = p.dw_splits[l];
        ra.dwp_off[l] = p.dwp_off[l];
        ra.dbp_off[l] = p.dbp_off[l];
    }
    ra.w_k = p.w_k;
    ra.w_n = p.w_n;
    ra.dw_part = p.dw_part;
    ra.db_part = p.db_part;
    ra.d_ws = out.d_ws;
    ra.d_bs = out.d_bs;
    ra.scale = (flags & LNERF_SEED_LOSS) ? p.loss_total : nullptr;
    ra.accumulate = (flags & LNERF_ACCUMULATE) ? 1 : 0;
    return ra;
}

void fused_train_step(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b, float seed,
                      int flags, const lnerf_outputs& out, hipStream_t s, hipEvent_t* ev, const FusedPlan* px) {
    const bool seed_loss = (flags & LNERF_SEED_LOSS) != 0;
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ev[i], s);
    };
    const size_t nred = (size_t)p.L * p.w_k * p.w_n + (size_t)p.L * p.w_n;
    const unsigned rgrid = (unsigned)((nred + 255) / 256);
    mark(0);
    k16_pack(p, ws, bs, s);
    mark(1);
    k16_launch(p, b, seed_loss ? 1.0f : seed, out, true, s);
    mark(2);
    k1_reduce_launch(p, out.loss, s);
    mark(3);
    dw16_launch(p, s);
    mark(4);
    if (px && p.guard) {
        // the floor guard (lnerf_internal.h kGuardExp): the same step again on the bf16x6 split (px:
        // the same workspace, every pointer but the activation slabs shared, the dW/db partials
        // included), each kernel exiting at once while k1 left the guard clear; the one reduction
        // below then sums whichever partials the last dW kernel wrote
        // (px's bf16x6 planes came out of p's pack: k16_pack wrote both formats)
        k16_launch(*px, b, seed_loss ? 1.0f : seed, out, true, s);
        k1_reduce_launch(*px, out.loss, s);
        dw16_launch(*px, s);
    }
    const ReduceArgs ra = reduce_args(p, out, flags);
    grad_reduce_kernel<<<rgrid, 256, 0, s>>>(ra);
    if (seed_loss) {
        if (out.d_dists) k_scale_by_scalar(out.d_dists, (size_t)p.R, p.loss_total, s);
        if (out.d_target)
            k_scale_by_scalar(out.d_target, (size_t)p.rays * (p.head_fit ? p.n[p.L - 1] : 3), p.loss_total, s);
        if (out.d_x) k_scale_by_scalar(out.d_x, (size_t)p.R * p.k[0], p.loss_total, s);
    }
    mark(5);
}

// Plain bf16 (config 5's inference precision) runs kr (lnerf_render.hip: every weight fragment
// feeds two 16-sample groups) unless LNERF_RENDER_K16 asks for k16's forward; the split
// precisions run k16's forward. Both read k16_pack's planes.
bool fused_render_uses_kr(const FusedPlan& p, int flags) { return !(flags & LNERF_RENDER_K16) && kr_supported(p); }

void fused_render(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                  const lnerf_outputs& out, hipStream_t s, int flags, hipEvent_t* ev) {
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ev[i], s);
    };
    mark(0);
    k16_pack(p, ws, bs, s);
    mark(1);
    int parts = p.num_wg;
    if (fused_render_uses_kr(p, flags)) {
        kr_launch(p, b, out, s);
        parts = kr_num_wg(p);
    } else {
        k16_launch(p, b, 1.0f, out, false, s);
    }
    mark(2);
    if (parts > 4 * 256) {
        const int per = (parts + kLossStage1 - 1) / kLossStage1;
        loss_stage1_kernel<<<kLossStage1, 256, 0, s>>>(p.loss_part, parts, per, p.loss_stage);
        loss_reduce_kernel<<<1, 256, 0, s>>>(p.loss_stage, kLossStage1, p.loss_total, out.loss);
    } else {
        loss_reduce_kernel<<<1, 256, 0, s>>>(p.loss_part, parts, p.loss_total, out.loss);
    }
    mark(3);
    mark(4);
    mark(5);
}

}  // namespace lnerf
