// lnerf_fused.hip -- the throughput path: fused PE + MLP + compositing + reverse chain on MFMA.
//
// Hot path of the reference: scripts/nerf.py:1-304 (forward) and its rev_diff (:306), called per
// chunk from train_nerf.py:325/395. Here one launch handles the whole batch:
//
//  k1  fused_fwd_bwd_kernel  one 256-thread workgroup per 128-sample tile (whole rays). Each wave
//      owns 32 samples. Activations live in registers in the *transposed* MFMA accumulator layout
//      (lane = sample, the 16 accumulator registers x 8 tiles = 256 features), so layer l+1 consumes
//      layer l's accumulator directly as its B operand (v_mfma_f32_32x32x2_f32, exact fp32).
//      Weights stream through LDS in pre-packed fragment order (one 16-B LDS read feeds 4 MFMAs).
//      After the forward, one thread per ray composites (alpha, inclusive cumprod, weights, colour,
//      loss) and runs the compositing reverse; then the reverse chain G_{l-1} = (W_l G_l) * relu'
//      runs back through the layers with the same register layout, ReLU masks kept as wave ballots
//      in LDS. Post-ReLU activations A_l and gradients G_l are written to HBM as 32-sample slabs.
//  k2  dw_kernel             dW_l = sum_s A_{l-1}[s]^T G_l[s] (+ db) over sample splits, from the
//      slabs via LDS, fp32 MFMA; deterministic per-split partials.
//  k3  reduce kernels        partials -> dW/db in the reference's padded layout, loss, seed scaling.
#include "lnerf_internal.h"

#include <math.h>

namespace lnerf {

typedef float fx16 __attribute__((ext_vector_type(16)));
typedef float fx4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kWgThreads = 256;
constexpr int kWaves = 4;
constexpr int kTileSamples = 128;          // samples per fused workgroup
constexpr int kNT = 8;                     // max 32-wide feature tiles (256 features)
constexpr int kChunkMax = 16 * 2 * 256;    // floats per staged weight chunk (r x nt4 x 64 lanes x 4)
constexpr int kMaxMaskLayers = kMaxLayers - 1;
constexpr int kCompFloats = 24;            // per-sample compositing scratch floats in LDS

// Feature held by accumulator register r of tile t in lane half h (32x32 C/D layout:
// row = (r&3) + 8(r>>2) + 4h). Using an accumulator as the next MFMA's B operand makes this the
// contraction order of that MFMA.
__host__ __device__ __forceinline__ int frag_feature(int t, int r, int h) {
    return 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
}

struct FusedArgs {
    int L;
    int kt[kMaxLayers], nt[kMaxLayers];
    int k0;
    const float* wf;
    const float* wb;
    const float* bp;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    float* act;
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;
    size_t grad_off[kMaxLayers];
    int rays, S, rpw, R, input_mode, F;
    const float* x;
    const float* dists;
    const float* target;
    float* loss_part;
    float* acc_color;
    float* d_dists;
    float* d_target;
    float* d_x;
    float seed;
    int want_grad;
};

// ---- LDS carve (one __shared__ array; see cdna_hip_programming.md §5 item 4(a)) --------------
constexpr int kLdsW = 2 * kChunkMax;                                    // floats
constexpr int kLdsMaskU64 = kWaves * kMaxMaskLayers * kNT * 16;         // 64-bit words
constexpr int kLdsComp = kTileSamples * kCompFloats;                    // floats
constexpr int kLdsRay = kTileSamples;                                   // per-ray loss partials
constexpr size_t kLdsBytes = (size_t)kLdsW * 4 + (size_t)kLdsMaskU64 * 8 + (size_t)kLdsComp * 4 +
                             (size_t)kLdsRay * 4;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

// Stage `cf` floats of packed weights into LDS with LDS-DMA (global_load_lds_dwordx4): lane-linear
// destination, 1 KiB per wave instruction.
__device__ __forceinline__ void stage_chunk(const float* __restrict__ src, float* dst, int cf) {
    const int tid = threadIdx.x, wave = tid >> 6;
    for (int base = 0; base < cf; base += kWgThreads * 4) {
        const float* g = src + base + tid * 4;
        float* l = dst + base + wave * 256;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 16, 0, 0);
    }
}

// out[o] += sum_{c < nchunks, r} Wpack[c][r][o] (x) in[c][r], the packed weights of one layer
// streamed chunk by chunk (chunk c = contraction tile c) through a 2-deep LDS ring.
__device__ __forceinline__ void mma_stream(const float* __restrict__ src, int nchunks, int nto,
                                           const fx16 (&in)[kNT], fx16 (&out)[kNT], float* ldsw) {
    const int lane = threadIdx.x & 63;
    const int nt4 = (nto + 3) >> 2;
    const int cf = 16 * nt4 * 256;
    stage_chunk(src, ldsw, cf);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kNT; ++c) {
        if (c < nchunks) {
            const float* cur = ldsw + (c & 1) * kChunkMax;
            if (c + 1 < nchunks) stage_chunk(src + (size_t)(c + 1) * cf, ldsw + ((c + 1) & 1) * kChunkMax, cf);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                fx4 w0 = *(const fx4*)(cur + (r * nt4 + 0) * 256 + lane * 4);
                fx4 w1 = {0.f, 0.f, 0.f, 0.f};
                if (nt4 > 1) w1 = *(const fx4*)(cur + (r * nt4 + 1) * 256 + lane * 4);
                const float b = in[c][r];
#pragma unroll
                for (int o = 0; o < kNT; ++o) {
                    if (o < nto) {
                        const float a = (o < 4) ? w0[o & 3] : w1[o & 3];
                        out[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, out[o], 0, 0, 0);
                    }
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ float input_feature(const FusedArgs& a, int gs, bool valid, int f) {
    if (!valid || f >= a.k0) return 0.0f;
    if (a.input_mode == LNERF_INPUT_ENCODED) return a.x[(size_t)gs * a.k0 + f];
    // positional_encoding_3d (pos_encoding.py:54-66): block-major, float64 trig, rounded once
    const int c = f % 3, blk = f / 3;
    const float xc = a.x[(size_t)gs * 3 + c];
    if (blk == 0) return xc;
    const int fb = blk - 1, freq = fb >> 1;
    const double arg = ldexp((double)xc, freq);
    return (fb & 1) ? (float)cos(arg) : (float)sin(arg);
}

// One ray: rendering (nerf.py:176-302) and its reverse with loma's statement order (see
// lnerf_generic.hip, lg_composite_fwd/bwd), on LDS scratch. z = head pre-activations [S][4].
struct RayScratch {
    float* z;      // [S][4] head pre-activation
    float* rgba;   // [S][4]
    float* al;     // [S]
    float* cC;     // [S]
    float* cP;     // [S]
    float* cT;     // [S]
    float* w;      // [S]
    float* dw;     // [S]
    float* dal;    // [S]
    float* dcp;    // [S]
    float* drgba;  // [S][4]
    float* gz;     // [S][4] output: dL/dz head
};

__device__ float composite_ray(const FusedArgs& a, int ray, const RayScratch& s, bool grad) {
    const int S = a.S;
    const float* dists = a.dists + (size_t)ray * S;
    // head activation (nerf.py:153-167): channel 3 ReLU, 0..2 sigmoid
    for (int j = 0; j < S; ++j)
        for (int k = 0; k < 4; ++k) {
            const float v = s.z[j * 4 + k];
            s.rgba[j * 4 + k] = (k == 3) ? ((v > 0.0f) ? v : 0.0f) : 1.0f / (1.0f + expf(0.0f - v));
        }
    for (int j = 0; j < S; ++j) s.al[j] = 1.0f - expf((0.0f - s.rgba[j * 4 + 3]) * dists[j]);
    for (int j = 0; j < S; ++j) s.cC[j] = (1.0f - s.al[j]) + (float)(1e-10);
    float p = 0.0f;
    for (int j = 0; j < S; ++j) {
        p = (j == 0) ? s.cC[0] : p * s.cC[j];
        s.cP[j] = p;
        s.cT[j] = (j == 0) ? 1.0f : p;
    }
    for (int j = 0; j < S; ++j) s.w[j] = s.al[j] * s.cT[j];
    float acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f;
    for (int j = 0; j < S; ++j) {
        acc0 = acc0 + s.w[j] * s.rgba[j * 4 + 0];
        acc1 = acc1 + s.w[j] * s.rgba[j * 4 + 1];
        acc2 = acc2 + s.w[j] * s.rgba[j * 4 + 2];
    }
    const float* t = a.target + (size_t)ray * 3;
    float loss = 0.0f;
    loss = loss + (acc0 - t[0]) * (acc0 - t[0]);
    loss = loss + (acc1 - t[1]) * (acc1 - t[1]);
    loss = loss + (acc2 - t[2]) * (acc2 - t[2]);
    if (a.acc_color) {
        a.acc_color[(size_t)ray * 3 + 0] = acc0;
        a.acc_color[(size_t)ray * 3 + 1] = acc1;
        a.acc_color[(size_t)ray * 3 + 2] = acc2;
    }
    if (!grad) return loss;

    // ---- reverse (lg_composite_bwd_kernel with zero incoming adjoints) ----
    const float seed = a.seed;
    float dacc[3] = {0.0f, 0.0f, 0.0f};
    const float accv[3] = {acc0, acc1, acc2};
    for (int c = 2; c >= 0; --c) {
        const float a1 = (accv[c] - t[c]) * seed;
        const float a2 = 0.0f - ((accv[c] - t[c]) * seed);
        dacc[c] += a1;
        dacc[c] += a1;
        if (a.d_target) a.d_target[(size_t)ray * 3 + c] = (0.0f + a2) + a2;
    }
    for (int j = 0; j < S; ++j) {
        s.dw[j] = 0.0f;
        s.dal[j] = 0.0f;
        s.dcp[j] = 0.0f;
        for (int k = 0; k < 4; ++k) s.drgba[j * 4 + k] = 0.0f;
    }
    for (int j = S - 1; j >= 0; --j)
        for (int c = 2; c >= 0; --c) {
            s.dw[j] += s.rgba[j * 4 + c] * dacc[c];
            s.drgba[j * 4 + c] += s.w[j] * dacc[c];
        }
    for (int j = S - 1; j >= 0; --j) {
        const float adj = s.dw[j];
        s.dal[j] += s.cT[j] * adj;
        s.dcp[j] += s.al[j] * adj;
    }
    s.dcp[0] = 0.0f;                                   // T_0 = 1
    for (int j = S - 1; j >= 1; --j) {                 // inclusive cumprod reverse
        const float adj = s.dcp[j];
        const float a_left = s.cC[j] * adj;
        const float a_right = s.cP[j - 1] * adj;
        s.dcp[j] = 0.0f;
        s.dcp[j - 1] += a_left;
        s.dcp[j] += a_right;
    }
    for (int j = S - 1; j >= 0; --j) s.dal[j] += 0.0f - s.dcp[j];   // cumprod init reverse
    for (int j = S - 1; j >= 0; --j) {                               // alpha reverse
        const float sigma = s.rgba[j * 4 + 3], delta = dists[j];
        const float adj2 = (0.0f - s.dal[j]) * expf((0.0f - sigma) * delta);
        s.drgba[j * 4 + 3] += 0.0f - (delta * adj2);
        if (a.d_dists) a.d_dists[(size_t)ray * S + j] = 0.0f + (0.0f - sigma) * adj2;
    }
    // head activation reverse (reverse_diff.py Div/exp/Sub rules; ReLU on the post value)
    for (int j = 0; j < S; ++j)
        for (int k = 0; k < 4; ++k) {
            const float dz = s.drgba[j * 4 + k];
            float g;
            if (k == 3) {
                g = (s.rgba[j * 4 + 3] > 0.0f) ? dz : 0.0f;
            } else {
                const float x = s.z[j * 4 + k];
                const float u = 1.0f + expf(0.0f - x);
                const float adj_div = ((0.0f - dz) * 1.0f) / (u * u);
                g = 0.0f + (0.0f - adj_div * expf(0.0f - x));
            }
            s.gz[j * 4 + k] = g;
        }
    return loss;
}

__global__ void __launch_bounds__(kWgThreads, 1) fused_fwd_bwd_kernel(FusedArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kLdsBytes];
    float* ldsw = (float*)lds_raw;
    unsigned long long* masks = (unsigned long long*)(lds_raw + (size_t)kLdsW * 4);
    float* comp = (float*)(lds_raw + (size_t)kLdsW * 4 + (size_t)kLdsMaskU64 * 8);
    float* rayloss = comp + kLdsComp;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const int wg = blockIdx.x;
    const int ls = wave * 32 + (lane & 31);           // local sample 0..127
    const int tile_samples = a.rpw * a.S;
    const int gs = wg * tile_samples + ls;            // global sample row (ray*S + j)
    const bool valid = (ls < tile_samples) && (gs < a.R);
    const size_t blk = (size_t)wg * kWaves + wave;    // 32-sample slab index
    unsigned long long* wmask = masks + (size_t)wave * kMaxMaskLayers * kNT * 16;

    fx16 act[kNT], out[kNT];
    // ---- layer-0 input: features in accumulator order, X slab for dW_0 ----
#pragma unroll
    for (int t = 0; t < kNT; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) act[t][r] = 0.0f;
        if (t < a.kt[0]) {
            float* xs = a.act + a.x_off + blk * (size_t)(a.kt[0] * 1024);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = frag_feature(t, r, h);
                const float v = input_feature(a, gs, valid, f);
                act[t][r] = v;
                if (a.want_grad) xs[f * 32 + (lane & 31)] = v;
            }
        }
    }

    // ---- forward through the layers ----
    for (int l = 0; l < a.L; ++l) {
        const int nto = a.nt[l];
#pragma unroll
        for (int o = 0; o < kNT; ++o) out[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        mma_stream(a.wf + a.wf_off[l], a.kt[l], nto, act, out, ldsw);
        const float* bpl = a.bp + a.bp_off[l];
        if (l < a.L - 1) {
            float* as = a.act + a.act_off[l] + blk * (size_t)(nto * 1024);
#pragma unroll
            for (int o = 0; o < kNT; ++o) {
                if (o < nto) {
                    const float* bo = bpl + (o * 2 + h) * 16;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        float v = out[o][r] + bo[r];
                        v = (v > 0.0f) ? v : 0.0f;               // ReLU nerf.py:141-144
                        out[o][r] = v;
                        const unsigned long long m = __ballot(v > 0.0f);
                        if (lane == 0) wmask[((size_t)l * kNT + o) * 16 + r] = m;
                        if (a.want_grad) as[frag_feature(o, r, h) * 32 + (lane & 31)] = v;
                    }
                }
            }
#pragma unroll
            for (int o = 0; o < kNT; ++o) act[o] = out[o];
        } else {
            // head pre-activations (features 0..3 live in regs 0..3 of lane half 0)
            const float* bo = bpl;  // tile 0, h = 0
            if (h == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) comp[ls * 4 + r] = out[0][r] + bo[r];  // c_z[ls][r]
            }
        }
    }
    __syncthreads();


    // ---- rendering + loss + rendering reverse: one thread per ray ----
    // comp (struct of arrays over the tile's 128 local samples; ray-major like the samples)
    float* c_z = comp;                          // [128][4]  (written by the head epilogue)
    float* c_rgba = comp + kTileSamples * 4;    // [128][4]
    float* c_drgba = comp + kTileSamples * 8;   // [128][4]
    float* c_gz = comp + kTileSamples * 12;     // [128][4]
    float* c_vec = comp + kTileSamples * 16;    // 8 x [128]
    if (tid < a.rpw) {
        const int ray = wg * a.rpw + tid;
        float loss = 0.0f;
        if (ray < a.rays) {
            const int o = tid * a.S;
            RayScratch s;
            s.z = c_z + o * 4;
            s.rgba = c_rgba + o * 4;
            s.drgba = c_drgba + o * 4;
            s.gz = c_gz + o * 4;
            s.al = c_vec + 0 * kTileSamples + o;
            s.cC = c_vec + 1 * kTileSamples + o;
            s.cP = c_vec + 2 * kTileSamples + o;
            s.cT = c_vec + 3 * kTileSamples + o;
            s.w = c_vec + 4 * kTileSamples + o;
            s.dw = c_vec + 5 * kTileSamples + o;
            s.dal = c_vec + 6 * kTileSamples + o;
            s.dcp = c_vec + 7 * kTileSamples + o;
            loss = composite_ray(a, ray, s, a.want_grad != 0);
        }
        rayloss[tid] = loss;
    }
    __syncthreads();
    if (tid == 0) {
        float l = 0.0f;
        for (int r = 0; r < a.rpw; ++r) l = l + rayloss[r];
        a.loss_part[wg] = l;
    }
    if (!a.want_grad) return;

    // ---- reverse chain: G_{L-1} from the head, then G_{l-1} = (W_l G_l) * 1[A_{l-1} > 0] ----
    fx16 g[kNT], go[kNT];
#pragma unroll
    for (int t = 0; t < kNT; ++t) g[t] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (h == 0 && valid) {
#pragma unroll
        for (int r = 0; r < 4; ++r) g[0][r] = c_gz[ls * 4 + r];
    }
    {
        const int ntl = a.nt[a.L - 1];
        float* gsl = a.grad + a.grad_off[a.L - 1] + blk * (size_t)(ntl * 1024);
#pragma unroll
        for (int o = 0; o < kNT; ++o)
            if (o < ntl) {
#pragma unroll
                for (int r = 0; r < 16; ++r) gsl[frag_feature(o, r, h) * 32 + (lane & 31)] = g[o][r];
            }
    }
    for (int l = a.L - 1; l >= 1; --l) {
        const int kto = a.kt[l];  // outputs: input features of layer l (= nt[l-1])
#pragma unroll
        for (int o = 0; o < kNT; ++o) go[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        mma_stream(a.wb + a.wb_off[l], a.nt[l], kto, g, go, ldsw);
        float* gsl = a.grad + a.grad_off[l - 1] + blk * (size_t)(kto * 1024);
#pragma unroll
        for (int o = 0; o < kNT; ++o) {
            if (o < kto) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const unsigned long long m = wmask[((size_t)(l - 1) * kNT + o) * 16 + r];
                    const float v = ((m >> lane) & 1ull) ? go[o][r] : 0.0f;
                    go[o][r] = v;
                    gsl[frag_feature(o, r, h) * 32 + (lane & 31)] = v;
                }
            }
        }
#pragma unroll
        for (int o = 0; o < kNT; ++o) g[o] = go[o];
    }
    if (a.d_x) {
        // d_layer_input = G_0 W_0^T (ENCODED mode), written row-major (rows = samples)
        const int kto = a.kt[0];
#pragma unroll
        for (int o = 0; o < kNT; ++o) go[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        mma_stream(a.wb + a.wb_off[0], a.nt[0], kto, g, go, ldsw);
        if (valid) {
#pragma unroll
            for (int o = 0; o < kNT; ++o)
                if (o < kto) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int f = frag_feature(o, r, h);
                        if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = go[o][r];
                    }
                }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// dW_l = sum_s A_{l-1}[:, s] G_l[:, s]^T over a split of the 32-sample slabs, fp32 MFMA.
// Each workgroup stages one slab pair (A: KT*32 rows, G: NTo*32 rows, 32 samples each) into LDS
// with a 33-float row pitch (conflict-free column reads), double-buffered through registers.
// Waves own 4x4 blocks of 32x32 output tiles; when the layer has fewer than 4 blocks, waves split
// the 16 sample pairs of a slab by phase and write separate partials.
// ---------------------------------------------------------------------------------------------
constexpr int kPitch = 33;
constexpr int kDwStageFloats = 2 * kNT * 32 * kPitch;  // A + G rows of one slab pair

struct DwArgs {
    int L;
    int kt[kMaxLayers], nt[kMaxLayers];
    const float* act;
    size_t a_off[kMaxLayers];   // A_{l-1} slab base per layer (X slab for l = 0)
    const float* grad;
    size_t g_off[kMaxLayers];
    int blocks;
    int splits[kMaxLayers];
    int wg_off[kMaxLayers];     // first workgroup of layer l
    float* dw_part;
    size_t dwp_off[kMaxLayers];
    float* db_part;
    size_t dbp_off[kMaxLayers];
};

__device__ __forceinline__ void dw_load_regs(fx4 (&regs)[16], const float* a_src, const float* g_src,
                                             int a_floats, int g_floats) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int e = (q * kWgThreads + tid) * 4;
        if (e < a_floats) regs[q] = *(const fx4*)(a_src + e);
        else if (e - a_floats < g_floats) regs[q] = *(const fx4*)(g_src + (e - a_floats));
    }
}

__device__ __forceinline__ void dw_store_lds(const fx4 (&regs)[16], float* lds, int a_floats,
                                             int g_floats) {
    const int tid = threadIdx.x;
    float* ga = lds + kNT * 32 * kPitch;  // G rows start after the A rows
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int e = (q * kWgThreads + tid) * 4;
        if (e < a_floats + g_floats) {
            const bool isA = e < a_floats;
            const int ee = isA ? e : e - a_floats;
            const int row = ee >> 5, col = ee & 31;
            float* d = (isA ? lds : ga) + row * kPitch + col;
            d[0] = regs[q][0];
            d[1] = regs[q][1];
            d[2] = regs[q][2];
            d[3] = regs[q][3];
        }
    }
}

__global__ void __launch_bounds__(kWgThreads, 1) dw_kernel(DwArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[2 * kDwStageFloats];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    // which layer / split
    int l = 0;
    while (l + 1 < a.L && (int)blockIdx.x >= a.wg_off[l + 1]) ++l;
    const int sp = blockIdx.x - a.wg_off[l];
    const int KT = a.kt[l], NTo = a.nt[l];
    const int nbk = (KT + 3) >> 2, nbj = (NTo + 3) >> 2, nblk = nbk * nbj;
    const int P = (nblk >= kWaves) ? 1 : (kWaves / nblk);
    const int myblk = wave % nblk, phase = wave / nblk;
    const bool active = phase < P;
    const int kb = (myblk / nbj) * 4, jb = (myblk % nbj) * 4;
    const int splits = a.splits[l];
    const int per = (a.blocks + splits - 1) / splits;
    const int b0 = sp * per, b1 = min(a.blocks, b0 + per);
    const int a_floats = KT * 1024, g_floats = NTo * 1024;
    const float* A = a.act + a.a_off[l];
    const float* G = a.grad + a.g_off[l];

    fx16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float dbsum = 0.0f;

    fx4 regs[16];
    if (b0 < b1) {
        dw_load_regs(regs, A + (size_t)b0 * a_floats, G + (size_t)b0 * g_floats, a_floats, g_floats);
        dw_store_lds(regs, lds, a_floats, g_floats);
    }
    __syncthreads();
    for (int b = b0; b < b1; ++b) {
        const float* cur = lds + ((b - b0) & 1) * kDwStageFloats;
        if (b + 1 < b1)
            dw_load_regs(regs, A + (size_t)(b + 1) * a_floats, G + (size_t)(b + 1) * g_floats,
                         a_floats, g_floats);
        const float* ca = cur;
        const float* cg = cur + kNT * 32 * kPitch;
        if (active) {
#pragma unroll 4
            for (int q = phase; q < 16; q += P) {
                const int s = 2 * q + h;
                float af[4], bf[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    af[i] = (kb + i < KT) ? ca[((kb + i) * 32 + (lane & 31)) * kPitch + s] : 0.0f;
                    bf[i] = (jb + i < NTo) ? cg[((jb + i) * 32 + (lane & 31)) * kPitch + s] : 0.0f;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (kb + i < KT && jb + j < NTo)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
            }
        }
        if (tid < NTo * 32) {
#pragma unroll 8
            for (int s = 0; s < 32; ++s) dbsum += cg[tid * kPitch + s];
        }
        if (b + 1 < b1) dw_store_lds(regs, lds + ((b + 1 - b0) & 1) * kDwStageFloats, a_floats, g_floats);
        __syncthreads();
    }
    // partial slab: [split*P + phase][k][j], k < KT*32, j < NTo*32
    if (active) {
        const int ncol = NTo * 32;
        float* part = a.dw_part + a.dwp_off[l] + (size_t)(sp * P + phase) * (KT * 32) * ncol;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (kb + i < KT && jb + j < NTo) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = (kb + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const int jj = (jb + j) * 32 + (lane & 31);
                        part[(size_t)k * ncol + jj] = acc[i][j][r];
                    }
                }
    }
    if (tid < NTo * 32) a.db_part[a.dbp_off[l] + (size_t)sp * (NTo * 32) + tid] = dbsum;
}

// ---------------------------------------------------------------------------------------------
// weight packing (once per step; weights change every optimizer step)
// ---------------------------------------------------------------------------------------------
struct PackArgs {
    int L;
    int k[kMaxLayers], n[kMaxLayers], kt[kMaxLayers], nt[kMaxLayers];
    int w_k, w_n;
    const float* W;
    const float* B;
    float* wf;
    float* wb;
    float* bp;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    size_t wf_n[kMaxLayers], wb_n[kMaxLayers], bp_n[kMaxLayers];
};

__global__ void pack_kernel(PackArgs a, int l) {
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const size_t nf = a.wf_n[l], nb = a.wb_n[l], np = a.bp_n[l];
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nf + nb + np;
         e += (size_t)gridDim.x * blockDim.x) {
        if (e < nf) {
            // WF[t][r][jt4][lane][e4] = W[f(t,r,h)][32 jt + lane&31]
            const int nt4 = (a.nt[l] + 3) >> 2;
            size_t x = e;
            const int e4 = x & 3; x >>= 2;
            const int ln = x & 63; x >>= 6;
            const int jt4 = x % nt4; x /= nt4;
            const int r = x & 15; x >>= 4;
            const int t = (int)x;
            const int kk = frag_feature(t, r, ln >> 5), jj = 32 * (4 * jt4 + e4) + (ln & 31);
            a.wf[a.wf_off[l] + e] = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        } else if (e < nf + nb) {
            // WB[jt][r][kt4][lane][e4] = W[32 kt + lane&31][f(jt,r,h)]
            const size_t eb = e - nf;
            const int kt4n = (a.kt[l] + 3) >> 2;
            size_t x = eb;
            const int e4 = x & 3; x >>= 2;
            const int ln = x & 63; x >>= 6;
            const int kt4 = x % kt4n; x /= kt4n;
            const int r = x & 15; x >>= 4;
            const int jt = (int)x;
            const int kk = 32 * (4 * kt4 + e4) + (ln & 31), jj = frag_feature(jt, r, ln >> 5);
            a.wb[a.wb_off[l] + eb] = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        } else {
            // BP[o][h][r] = b[f(o,r,h)]
            const size_t ep = e - nf - nb;
            const int r = ep & 15, hh = (ep >> 4) & 1, o = (int)(ep >> 5);
            const int jj = frag_feature(o, r, hh);
            a.bp[a.bp_off[l] + ep] = (jj < N) ? a.B[(size_t)l * a.w_n + jj] : 0.0f;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------------------------
__global__ void loss_reduce_kernel(const float* __restrict__ part, int n, float* total,
                                   float* out_loss) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float s = 0.0f;
    for (int i = 0; i < n; ++i) s = s + part[i];
    *total = s;
    if (out_loss) *out_loss = s;
}

struct ReduceArgs {
    int L;
    int k[kMaxLayers], n[kMaxLayers], kt[kMaxLayers], nt[kMaxLayers];
    int w_k, w_n;
    int nparts[kMaxLayers];      // splits * phases (dW)
    int splits[kMaxLayers];      // (dB)
    const float* dw_part;
    size_t dwp_off[kMaxLayers];
    const float* db_part;
    size_t dbp_off[kMaxLayers];
    float* d_ws;
    float* d_bs;
    const float* scale;          // nullable device scalar (seed = loss)
    int accumulate;
};

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
                float s = 0.0f;
                for (int q = 0; q < a.nparts[l]; ++q) s += p[(size_t)q * slab];
                v = a.scale ? s * sc : s;
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
                float s = 0.0f;
                for (int q = 0; q < a.splits[l]; ++q) s += p[(size_t)q * ncol];
                v = a.scale ? s * sc : s;
            }
            a.d_bs[eb] = a.accumulate ? a.d_bs[eb] + v : v;
        }
    }
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct Layout {
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    size_t wf_n[kMaxLayers], wb_n[kMaxLayers], bp_n[kMaxLayers];
    size_t pack_total;
    size_t act_off[kMaxLayers], x_off, act_total;
    size_t grad_off[kMaxLayers], grad_total;
    int splits[kMaxLayers], phases[kMaxLayers], wg_off[kMaxLayers], dw_grid;
    size_t dwp_off[kMaxLayers], dwp_total, dbp_off[kMaxLayers], dbp_total;
    int num_wg, blocks, rpw;
};

void make_layout(Layout& y, const lnerf_mlp& m, int rays, int S) {
    const int L = m.num_layers;
    int kt[kMaxLayers], nt[kMaxLayers];
    for (int l = 0; l < L; ++l) {
        kt[l] = (m.k[l] + 31) / 32;
        nt[l] = (m.n[l] + 31) / 32;
    }
    size_t off = 0;
    for (int l = 0; l < L; ++l) {
        y.wf_n[l] = (size_t)kt[l] * 16 * ((nt[l] + 3) / 4) * 256;
        y.wb_n[l] = (size_t)nt[l] * 16 * ((kt[l] + 3) / 4) * 256;
        y.bp_n[l] = (size_t)nt[l] * 32;
        y.wf_off[l] = off; off += align_up(y.wf_n[l], 64);
        y.wb_off[l] = off; off += align_up(y.wb_n[l], 64);
        y.bp_off[l] = off; off += align_up(y.bp_n[l], 64);
    }
    y.pack_total = off;
    y.rpw = S >= kTileSamples ? 1 : kTileSamples / S;
    y.num_wg = (rays + y.rpw - 1) / y.rpw;
    y.blocks = y.num_wg * kWaves;
    off = 0;
    y.x_off = off; off += (size_t)y.blocks * kt[0] * 1024;
    for (int l = 0; l < L - 1; ++l) { y.act_off[l] = off; off += (size_t)y.blocks * nt[l] * 1024; }
    y.act_total = off;
    off = 0;
    for (int l = 0; l < L; ++l) { y.grad_off[l] = off; off += (size_t)y.blocks * nt[l] * 1024; }
    y.grad_total = off;
    // dW grid: ~32 splits for a full 8x8-tile layer, proportionally fewer for small layers
    int wg = 0;
    size_t dwp = 0, dbp = 0;
    for (int l = 0; l < L; ++l) {
        const int tiles = kt[l] * nt[l];
        int sp = (32 * tiles + 63) / 64;
        sp = sp < 1 ? 1 : sp;
        sp = sp > y.blocks ? y.blocks : sp;
        const int nblk = ((kt[l] + 3) / 4) * ((nt[l] + 3) / 4);
        y.splits[l] = sp;
        y.phases[l] = nblk >= kWaves ? 1 : kWaves / nblk;
        y.wg_off[l] = wg;
        wg += sp;
        y.dwp_off[l] = dwp;
        dwp += (size_t)sp * y.phases[l] * kt[l] * 32 * nt[l] * 32;
        y.dbp_off[l] = dbp;
        dbp += (size_t)sp * nt[l] * 32;
    }
    y.dw_grid = wg;
    y.dwp_total = dwp;
    y.dbp_total = dbp;
}

}  // namespace

bool fused_supported(const lnerf_mlp& m, int rays, int S, int input_mode, const char** why) {
    const char* w = nullptr;
    if (m.num_layers < 1 || m.num_layers > kMaxLayers) w = "num_layers out of range";
    else if (S < 1 || S > kTileSamples) w = "fused path needs 1 <= samples <= 128";
    else if (rays < 1) w = "no rays";
    else if (m.n[m.num_layers - 1] < 4) w = "head must have >= 4 outputs (rgb + sigma)";
    else {
        for (int l = 0; l < m.num_layers && !w; ++l) {
            if (m.k[l] < 1 || m.k[l] > kNT * 32 || m.n[l] < 1 || m.n[l] > kNT * 32)
                w = "layer widths must be in 1..256";
            else if (l > 0 && m.k[l] != m.n[l - 1]) w = "k[l] must equal n[l-1]";
            else if (m.k[l] > m.w_k || m.n[l] > m.w_n) w = "padded weight layout too small";
        }
    }
    (void)input_mode;
    if (why) *why = w;
    return w == nullptr;
}

size_t fused_workspace_bytes(const lnerf_mlp& m, int rays, int S) {
    Layout y;
    make_layout(y, m, rays, S);
    size_t f = align_up(y.pack_total, 64) + align_up(y.act_total, 64) + align_up(y.grad_total, 64) +
               align_up((size_t)y.num_wg, 64) + align_up(y.dwp_total, 64) + align_up(y.dbp_total, 64) +
               64;
    return f * sizeof(float);
}

void fused_plan(FusedPlan& p, const lnerf_mlp& m, const lnerf_batch& b, void* ws_base) {
    Layout y;
    make_layout(y, m, b.rays, b.samples);
    p.L = m.num_layers;
    for (int l = 0; l < p.L; ++l) {
        p.k[l] = m.k[l];
        p.n[l] = m.n[l];
        p.kt[l] = (m.k[l] + 31) / 32;
        p.nt[l] = (m.n[l] + 31) / 32;
        p.wf_off[l] = y.wf_off[l];
        p.wb_off[l] = y.wb_off[l];
        p.bp_off[l] = y.bp_off[l];
        p.act_off[l] = (l < p.L - 1) ? y.act_off[l] : 0;
        p.grad_off[l] = y.grad_off[l];
        p.dw_splits[l] = y.splits[l];
        p.dw_split_off[l] = y.wg_off[l];
        p.dwp_off[l] = y.dwp_off[l];
        p.dbp_off[l] = y.dbp_off[l];
    }
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
    float* base = (float*)ws_base;
    size_t off = 0;
    p.wf = base + off;            // wf/wb/bp share one packed region (offsets above)
    p.wb = base + off;
    p.bp = base + off;
    off += align_up(y.pack_total, 64);
    p.act = base + off;
    off += align_up(y.act_total, 64);
    p.grad = base + off;
    off += align_up(y.grad_total, 64);
    p.loss_part = base + off;
    off += align_up((size_t)y.num_wg, 64);
    p.dw_part = base + off;
    off += align_up(y.dwp_total, 64);
    p.db_part = base + off;
    off += align_up(y.dbp_total, 64);
    p.loss_total = base + off;
    // remember x slab offset in act_off[kMaxLayers-1] slot is not possible; keep it in a static
    p.act_off[kMaxLayers - 1] = y.x_off;
}

static void launch_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s) {
    PackArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.k[l] = p.k[l];
        a.n[l] = p.n[l];
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = p.wf_off[l];
        a.wb_off[l] = p.wb_off[l];
        a.bp_off[l] = p.bp_off[l];
        a.wf_n[l] = (size_t)p.kt[l] * 16 * ((p.nt[l] + 3) / 4) * 256;
        a.wb_n[l] = (size_t)p.nt[l] * 16 * ((p.kt[l] + 3) / 4) * 256;
        a.bp_n[l] = (size_t)p.nt[l] * 32;
    }
    a.w_k = p.w_k;
    a.w_n = p.w_n;
    a.W = ws;
    a.B = bs;
    a.wf = p.wf;
    a.wb = p.wb;
    a.bp = p.bp;
    for (int l = 0; l < p.L; ++l) {
        const size_t n = a.wf_n[l] + a.wb_n[l] + a.bp_n[l];
        unsigned g = (unsigned)((n + 255) / 256);
        pack_kernel<<<g, 256, 0, s>>>(a, l);
    }
}

static FusedArgs make_fused_args(const FusedPlan& p, const lnerf_batch& b, float seed,
                                 const lnerf_outputs& out, bool want_grad) {
    FusedArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = p.wf_off[l];
        a.wb_off[l] = p.wb_off[l];
        a.bp_off[l] = p.bp_off[l];
        a.act_off[l] = p.act_off[l];
        a.grad_off[l] = p.grad_off[l];
    }
    a.k0 = p.k[0];
    a.wf = p.wf;
    a.wb = p.wb;
    a.bp = p.bp;
    a.act = p.act;
    a.x_off = p.act_off[kMaxLayers - 1];
    a.grad = p.grad;
    a.rays = p.rays;
    a.S = p.S;
    a.rpw = p.rays_per_wg;
    a.R = p.R;
    a.input_mode = b.input_mode;
    a.F = b.num_freqs;
    a.x = b.x;
    a.dists = b.dists;
    a.target = b.target;
    a.loss_part = p.loss_part;
    a.acc_color = out.acc_color;
    a.d_dists = want_grad ? out.d_dists : nullptr;
    a.d_target = want_grad ? out.d_target : nullptr;
    a.d_x = want_grad ? out.d_x : nullptr;
    a.seed = seed;
    a.want_grad = want_grad ? 1 : 0;
    return a;
}

void fused_train_step(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                      float seed, int flags, const lnerf_outputs& out, hipStream_t s,
                      hipEvent_t* ev) {
    const bool seed_loss = (flags & LNERF_SEED_LOSS) != 0;
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ev[i], s);
    };
    mark(0);
    launch_pack(p, ws, bs, s);
    mark(1);
    FusedArgs fa = make_fused_args(p, b, seed_loss ? 1.0f : seed, out, true);
    fused_fwd_bwd_kernel<<<p.num_wg, kWgThreads, 0, s>>>(fa);
    mark(2);
    loss_reduce_kernel<<<1, 64, 0, s>>>(p.loss_part, p.num_wg, p.loss_total, out.loss);
    mark(3);
    DwArgs da{};
    da.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        da.kt[l] = p.kt[l];
        da.nt[l] = p.nt[l];
        da.a_off[l] = (l == 0) ? p.act_off[kMaxLayers - 1] : p.act_off[l - 1];
        da.g_off[l] = p.grad_off[l];
        da.splits[l] = p.dw_splits[l];
        da.wg_off[l] = p.dw_split_off[l];
        da.dwp_off[l] = p.dwp_off[l];
        da.dbp_off[l] = p.dbp_off[l];
    }
    da.act = p.act;
    da.grad = p.grad;
    da.blocks = p.blocks;
    da.dw_part = p.dw_part;
    da.db_part = p.db_part;
    dw_kernel<<<p.dw_grid, kWgThreads, 0, s>>>(da);
    mark(4);
    ReduceArgs ra{};
    ra.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        ra.k[l] = p.k[l];
        ra.n[l] = p.n[l];
        ra.kt[l] = p.kt[l];
        ra.nt[l] = p.nt[l];
        const int nblk = ((p.kt[l] + 3) / 4) * ((p.nt[l] + 3) / 4);
        const int P = nblk >= kWaves ? 1 : kWaves / nblk;
        ra.nparts[l] = p.dw_splits[l] * P;
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
    ra.scale = seed_loss ? p.loss_total : nullptr;
    ra.accumulate = (flags & LNERF_ACCUMULATE) ? 1 : 0;
    const size_t nred = (size_t)p.L * p.w_k * p.w_n + (size_t)p.L * p.w_n;
    grad_reduce_kernel<<<(unsigned)((nred + 255) / 256), 256, 0, s>>>(ra);
    if (seed_loss) {
        if (out.d_dists) k_scale_by_scalar(out.d_dists, (size_t)p.R, p.loss_total, s);
        if (out.d_target) k_scale_by_scalar(out.d_target, (size_t)p.rays * 3, p.loss_total, s);
        if (out.d_x) k_scale_by_scalar(out.d_x, (size_t)p.R * p.k[0], p.loss_total, s);
    }
    mark(5);
}

void fused_render(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                  const lnerf_outputs& out, hipStream_t s) {
    launch_pack(p, ws, bs, s);
    FusedArgs fa = make_fused_args(p, b, 1.0f, out, false);
    fused_fwd_bwd_kernel<<<p.num_wg, kWgThreads, 0, s>>>(fa);
    loss_reduce_kernel<<<1, 64, 0, s>>>(p.loss_part, p.num_wg, p.loss_total, out.loss);
}

}  // namespace lnerf
