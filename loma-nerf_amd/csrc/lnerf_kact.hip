// lnerf_kact.hip -- k1 with the activations resident in LDS: the fused PE + MLP + compositing +
// reverse chain for the fp16x3 split, the default fused kernel wherever it applies.
//
// Same work and outputs as k16 (lnerf_k16.hip; reference scripts/nerf.py:1-304 and its rev_diff,
// train_nerf.py:325/395), with the operand roles of the 128-sample workgroup tile swapped:
//  * the layer input of all 128 samples lives in LDS, already split into its fp16 hi / lo planes
//    in the MFMA B-operand layout, act[k-step 8][sample group 8][plane 2][lane 64][16 B]
//    (128 KiB); it is written once per layer by the wave that produced those features;
//  * wave w owns the 32 output features 32w .. 32w + 31 (16-wide tiles 2w, 2w + 1) of every
//    layer for all 128 samples: 8 groups x 2 tiles of v_mfma_f32_16x16x32_f16 accumulators
//    (64 registers), and streams exactly its weight fragments straight from L2 into registers
//    (4 x 16 B per lane and k-step, three k-steps in flight): no LDS-DMA, no weight ring and no
//    barrier inside a layer's MMA;
//  * a weight fragment feeds 8 sample groups and an activation fragment feeds two tiles, so the
//    LDS reads per MFMA are a quarter of k16's and none of it is written by DMA;
//  * the producing wave's accumulator register j of lane (n, g) is exactly element j of the next
//    layer's B fragment for k-step w (the phi permutation of the packed weights, k16_pack), so a
//    layer epilogue splits its own registers and writes two lane-linear ds_write_b128 per group;
//  * per-sample exponent shifts (fp16x3): a sample's 256 features are spread over 8 waves, so
//    the epilogue exchanges per-wave maxima through LDS (three barriers per layer).
// The slabs (A_l, G_l), ReLU masks and per-wave slab maxima are written in exactly k16's layouts,
// so dw16 and the reduce kernels are shared.
#include "lnerf_composite.h"
#include "lnerf_internal.h"

#include <stddef.h>
#include <stdio.h>

#include <utility>

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kGroups = 8;                       // 16-sample groups per 128-sample tile
constexpr int kTile = comp::kTileSamples;        // 128
constexpr int kActBytes = 8 * kGroups * 2 * 1024;  // 8 k-steps x 8 groups x 2 planes x 1 KiB
constexpr int kOffComp = kActBytes;
constexpr int kCompBytes = 2688 * 4;             // composite_tile's scratch
constexpr int kOffRay = kOffComp + kCompBytes;
constexpr int kOffPm = kOffRay + kTile * 4;      // per-wave per-sample maxima [8][128] f32
constexpr int kOffSx = kOffPm + kWaves * kTile * 4;   // per-sample exponent shifts [2][128] i32
constexpr int kOffBias = kOffSx + 2 * kTile * 4;  // biases [L][256] f32 (copied once)
constexpr int kLdsBytes = kOffBias + kMaxLayers * 256 * 4;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct KaArgs {
    int L;
    int ks_f[kMaxLayers], ks_b[kMaxLayers];   // k-steps (32 input features) per pass
    int to_f[kMaxLayers], to_b[kMaxLayers];   // 16-wide output tiles per pass (packed)
    int nt[kMaxLayers];                       // 32-wide slab tiles of each layer's output
    int k0;
    const unsigned short* w16;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];   // u16 offsets (k16_pack layout, 2 planes)
    const float* b16;                                // [L][256] zero-padded biases
    const int* wexp;                                 // per-layer max|W| bits
    unsigned long long* mask_g;                      // [wg][L-1][wave][lane]
    float* act;
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;
    size_t grad_off[kMaxLayers];
    float* smax;                                     // [2L][num_wg * 8] per-wave slab maxima
    int rays, S, rpw, R, input_mode, F;
    float near_t, far_t;
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

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---- optional in-kernel phase timing (-DLNERF_KACT_PROF=1, never in the product build): per-wave
// s_memtime deltas summed into g_kact_prof (atomics at the end; diagnostic build only)
#ifndef LNERF_KACT_PROF
#define LNERF_KACT_PROF 0
#endif
enum { kQpPe, kQpMma, kQpEpi, kQpBar, kQpComp, kQpTotal, kQpN };
#if LNERF_KACT_PROF
__device__ unsigned long long g_kact_prof[8];
#define QP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define QP_ADD(cat, t0) do { qp[cat] += __builtin_amdgcn_s_memtime() - (t0); } while (0)
#else
#define QP_T(v)
#define QP_ADD(cat, t0)
#endif

__device__ __forceinline__ fx4 mfma_h(const u4& a, const u4& b, fx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
                                                  0);
}

// (x0, x1) -> packed f16 hi = round(x sc), lo = round(x sc - hi) (v_fma_mix: one rounding each;
// x sc and x sc - hi are exact)
__device__ __forceinline__ void split_h2(float x0, float x1, float sc, unsigned& hi, unsigned& lo) {
    asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=&v"(hi) : "v"(x0), "v"(sc));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(hi) : "v"(x1), "v"(sc));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(x0), "v"(sc), "v"(hi));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "+v"(lo) : "v"(x1), "v"(sc), "v"(hi));
}

// exponent shift e with m 2^e in [2^13, 2^14); 0 for m = 0 or non-finite; clamped to +-60 so that
// 2^e and an epilogue's 2^-(e + ew) stay normal floats (the unscale is then one exact multiply)
__device__ __forceinline__ int shift_of(float m) {
    if (!(m > 0.0f) || !(m < __builtin_inff())) return 0;
    int e;
    (void)__builtin_frexpf(m, &e);
    const int s = 14 - e;
    return s < -60 ? -60 : s > 60 ? 60 : s;
}

// ReLU with its mask bit: r = v > 0 ? v : 0 (NaN -> 0, nerf.py:141-144), m = 2 m + (v > 0): three
// VALU ops, the comparison shared (the bits enter MSB-first: value j of 32 ends at bit 31 - j)
__device__ __forceinline__ float relu_bit(float v, unsigned& m) {
    float r;
    asm("v_cmp_lt_f32 vcc, 0, %2\n\t"
        "v_cndmask_b32 %0, 0, %2, vcc\n\t"
        "v_addc_co_u32 %1, vcc, %1, %1, vcc"
        : "=&v"(r), "+v"(m) : "v"(v) : "vcc");
    return r;
}

// bit 31 - j of m set ? x : +0 (the backward's mask, relu_bit's order)
__device__ __forceinline__ float keep_if(unsigned m, int j, float x) {
    const int t = __builtin_amdgcn_sbfe((int)m, 31 - j, 1);
    return __int_as_float(t & __float_as_int(x));
}

// act fragment address (bytes): k-step s, group q, plane p, this lane
__device__ __forceinline__ unsigned char* act_frag(unsigned char* act, int s, int q, int p) {
    return act + ((s * kGroups + q) * 2 + p) * 1024 + (threadIdx.x & 63) * 16;
}

// Split a group's 8 B-operand values (element j = tile j >> 2, register j & 3) with 2^ex and write
// them as k-step s's fragments of group q.
__device__ __forceinline__ void put_group(unsigned char* act, int s, int q, const fx4& t0, const fx4& t1, int ex) {
    const float sc = __builtin_ldexpf(1.0f, ex);
    unsigned h[4], l[4];
    split_h2(t0[0], t0[1], sc, h[0], l[0]);
    split_h2(t0[2], t0[3], sc, h[1], l[1]);
    split_h2(t1[0], t1[1], sc, h[2], l[2]);
    split_h2(t1[2], t1[3], sc, h[3], l[3]);
    *(u4*)act_frag(act, s, q, 0) = u4{h[0], h[1], h[2], h[3]};
    *(u4*)act_frag(act, s, q, 1) = u4{l[0], l[1], l[2], l[3]};
}

// Slab store of one 16-sample group's two 16-wide tiles (the wave's 32-feature slab tile): rows
// 16 tl + 4 g + i of [32 rows][16 samples] of the group's half-block; 4 runs of 64 B per register.
__device__ __forceinline__ void store_slab(float* __restrict__ half, const fx4& t0, const fx4& t1) {
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        __builtin_nontemporal_store(t0[i], half + (4 * g + i) * 16 + n);
        __builtin_nontemporal_store(t1[i], half + (16 + 4 * g + i) * 16 + n);
    }
}

// Element I (group I >> 3, tile (I >> 2) & 1, register I & 3) of a deferred slab store: the
// previous epilogue's 64 values per lane are stored one per MMA step of the next pass, so the
// slab writes stream under the MFMAs instead of bunching in the epilogue.
template <int I>
__device__ __forceinline__ void store_one(float* pend, int nt, const fx4 (&pv)[kGroups][2]) {
    constexpr int q = I >> 3, tl = (I >> 2) & 1, i = I & 3;
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
    float* half = pend + (size_t)(q >> 1) * nt * 1024 + (q & 1) * 512;
    __builtin_nontemporal_store(pv[q][tl][i], half + (16 * tl + 4 * g + i) * 16 + n);
}
#ifndef LNERF_KACT_DEFER
#define LNERF_KACT_DEFER 0
#endif
constexpr bool kDefer = LNERF_KACT_DEFER != 0;   // slab stores under the next pass (else in the epilogue)

template <int... I>
__device__ __forceinline__ void store_range(std::integer_sequence<int, I...>, float* pend, int nt,
                                            const fx4 (&pv)[kGroups][2]) {
    (store_one<I>(pend, nt, pv), ...);
}

template <int B, int... J>
__device__ __forceinline__ void store_from(std::integer_sequence<int, J...>, float* pend, int nt,
                                           const fx4 (&pv)[kGroups][2]) {
    (store_one<B + J>(pend, nt, pv), ...);
}

// max over the lanes of a sample (n, n + 16, n + 32, n + 48)
__device__ __forceinline__ float sample_reduce(float m) {
    m = __builtin_fmaxf(m, __shfl_xor(m, 16));
    return __builtin_fmaxf(m, __shfl_xor(m, 32));
}

// Workgroup barrier for LDS hand-offs only: every LDS access of the wave done (lgkmcnt(0)), then
// s_barrier -- no vmcnt(0): __syncthreads' fence would also wait for the slab stores in flight,
// which no other wave reads in this kernel.
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ---- one layer pass: acc[q][t] += W (tiles 2w, 2w + 1) x act (k-steps 0 .. ks-1), all groups ----
// weight-fragment register sets in flight (k-steps s % kWRing; a k-step is ~1.5k SIMD cycles)
#ifndef LNERF_KACT_WRING
#define LNERF_KACT_WRING 2
#endif
constexpr int kWRing = LNERF_KACT_WRING;
static_assert(kWRing == 2 || kWRing == 3, "weight ring depth");
struct WFrag {
    u4 v[4];   // tile 0 planes 0, 1; tile 1 planes 0, 1
};

__device__ __forceinline__ void load_w(const unsigned short* base, int s, int to, int t0, bool two, WFrag& f) {
    const int lane = threadIdx.x & 63;
    const unsigned short* p0 = base + ((size_t)(s * to + t0) * 2) * 512 + lane * 8;
    f.v[0] = *(const u4*)p0;
    f.v[1] = *(const u4*)(p0 + 512);
    if (two) {
        f.v[2] = *(const u4*)(p0 + 1024);
        f.v[3] = *(const u4*)(p0 + 1536);
    }
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 at an immediate offset, outside the compiler's waitcnt bookkeeping (the matching
// lgkm_wait below is the only wait, so the next group's reads stay in flight under the MFMAs)
template <int OFF>
__device__ __forceinline__ u4 ds_read_at(unsigned addr) {
    u4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
template <int N>
__device__ __forceinline__ void lgkm_wait(u4& a, u4& b) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}

// the hi / lo B fragments of step I = 8 s + q (act k-step s, group q); offsets past 64 KiB from
// the second base address
template <int I>
__device__ __forceinline__ void read_b(unsigned b0, unsigned b1, u4& h, u4& l) {
    constexpr int off = I * 2048;
    if constexpr (off < 65536 - 1024) {
        h = ds_read_at<off>(b0);
        l = ds_read_at<off + 1024>(b0);
    } else {
        h = ds_read_at<off - 65536>(b1);
        l = ds_read_at<off + 1024 - 65536>(b1);
    }
}

// step I of the unrolled pass: prefetch the weights of k-step s + 2 (at a k-step's first group),
// read the next step's B fragments, wait for this step's, 6 (3) MFMAs (small terms first)
template <int KS, bool TWO, int I>
__device__ __forceinline__ void pass_step(unsigned b0, unsigned b1, const unsigned short* wb, int to, int t0,
                                          WFrag (&w)[kWRing], u4 (&bh)[2], u4 (&bl)[2], fx4 (&acc)[kGroups][2],
                                          const fx4 (&pv)[kGroups][2], float* pend, int pnt) {
    constexpr int s = I / kGroups, q = I % kGroups, N = KS * kGroups;
    if (pend) store_one<I>(pend, pnt, pv);
    if constexpr (q == 0 && s + kWRing - 1 < KS)
        load_w(wb, s + kWRing - 1, to, t0, TWO, w[(s + kWRing - 1) % kWRing]);
    if constexpr (I + 1 < N) read_b<I + 1>(b0, b1, bh[(I + 1) & 1], bl[(I + 1) & 1]);
    if constexpr (I + 1 < N) lgkm_wait<2>(bh[I & 1], bl[I & 1]);
    else lgkm_wait<0>(bh[I & 1], bl[I & 1]);
    const WFrag& f = w[s % kWRing];
    fx4 c = acc[q][0];
    c = mfma_h(f.v[0], bl[I & 1], c);
    c = mfma_h(f.v[1], bh[I & 1], c);
    c = mfma_h(f.v[0], bh[I & 1], c);
    acc[q][0] = c;
    if constexpr (TWO) {
        fx4 d = acc[q][1];
        d = mfma_h(f.v[2], bl[I & 1], d);
        d = mfma_h(f.v[3], bh[I & 1], d);
        d = mfma_h(f.v[2], bh[I & 1], d);
        acc[q][1] = d;
    }
}

template <int KS, bool TWO, int... I>
__device__ __forceinline__ void pass_steps(std::integer_sequence<int, I...>, unsigned b0, unsigned b1,
                                           const unsigned short* wb, int to, int t0, WFrag (&w)[kWRing], u4 (&bh)[2],
                                           u4 (&bl)[2], fx4 (&acc)[kGroups][2], const fx4 (&pv)[kGroups][2],
                                           float* pend, int pnt) {
    (pass_step<KS, TWO, I>(b0, b1, wb, to, t0, w, bh, bl, acc, pv, pend, pnt), ...);
}

// the deferred stores a pass of KS k-steps (8 KS steps) did not take
template <int KS>
__device__ __forceinline__ void store_rest(float* pend, int pnt, const fx4 (&pv)[kGroups][2]) {
    if constexpr (KS * kGroups < 64) {
        if (pend) store_from<KS * kGroups>(std::make_integer_sequence<int, 64 - KS * kGroups>{}, pend, pnt, pv);
    }
}

// One pass over KS k-steps, fully unrolled (weights three k-steps ahead in a register ring, B
// fragments one group ahead). w[0], w[1] hold k-steps 0 and 1, requested by the caller (pass_pre)
// before the previous pass's epilogue so their L2 latency hides behind it.
template <int KS, bool TWO>
__device__ __forceinline__ void mma_pass_t(unsigned char* act, const unsigned short* wb, int to, int t0,
                                           WFrag (&w)[kWRing], fx4 (&acc)[kGroups][2], const fx4 (&pv)[kGroups][2],
                                           float* pend, int pnt) {
    const unsigned b0 = lds_addr(act) + (threadIdx.x & 63) * 16, b1 = b0 + 65536;
    u4 bh[2], bl[2];
    read_b<0>(b0, b1, bh[0], bl[0]);
    pass_steps<KS, TWO>(std::make_integer_sequence<int, KS * kGroups>{}, b0, b1, wb, to, t0, w, bh, bl, acc, pv,
                        pend, pnt);
    store_rest<KS>(pend, pnt, pv);
}

// A pass (or, for a wave without output tiles, just the deferred stores). `pend` (nullable):
// the slab half-block base of the previous epilogue's values `pv`, stored during this pass.
__device__ __forceinline__ void mma_pass(unsigned char* act, const unsigned short* wb, int ks, int to, int t0,
                                         WFrag (&w)[kWRing], fx4 (&acc)[kGroups][2], const fx4 (&pv)[kGroups][2],
                                         float* pend, int pnt) {
    if (t0 >= to) {
        if (pend) store_range(std::make_integer_sequence<int, 64>{}, pend, pnt, pv);
        return;
    }
#define LNERF_KACT_PASS(TWO)                                                              \
    switch (ks) {                                                                         \
        case 1: mma_pass_t<1, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 2: mma_pass_t<2, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 3: mma_pass_t<3, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 4: mma_pass_t<4, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 5: mma_pass_t<5, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 6: mma_pass_t<6, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        case 7: mma_pass_t<7, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;        \
        default: mma_pass_t<8, TWO>(act, wb, to, t0, w, acc, pv, pend, pnt); break;       \
    }
    if (t0 + 1 < to) {
        LNERF_KACT_PASS(true)
    } else {
        LNERF_KACT_PASS(false)
    }
#undef LNERF_KACT_PASS
}

// request k-steps 0 and 1 of a pass (this wave's tiles t0, t0 + 1 if they exist)
__device__ __forceinline__ void pass_pre(const unsigned short* wb, int ks, int to, int t0, WFrag (&w)[kWRing]) {
    if (t0 >= to) return;
    const bool two = t0 + 1 < to;
    load_w(wb, 0, to, t0, two, w[0]);
    if (kWRing == 3 && ks > 1) load_w(wb, 1, to, t0, two, w[1]);
}

__device__ __forceinline__ void zero_acc(fx4 (&acc)[kGroups][2]) {
#pragma unroll
    for (int q = 0; q < kGroups; ++q) acc[q][0] = acc[q][1] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
}

// Epilogue part 2 and 3 of a layer whose outputs (unscaled fp32, in v[q][t]) become the next
// pass's input: exchange the per-sample maxima, then split + write k-step w of every group. The
// caller has written its partial maxima pm[w][*] before calling (bar 1 here).
__device__ __forceinline__ void publish(unsigned char* lds, const fx4 (&v)[kGroups][2], int sxi, bool act_out) {
    float* pm = (float*)(lds + kOffPm);
    int* sx = (int*)(lds + kOffSx) + sxi * kTile;
    const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15;
    bar();   // every wave's MMA over act is done; the partial maxima are in pm
    if (lane < 16) {
        float m = 0.0f;
#pragma unroll
        for (int w2 = 0; w2 < kWaves; ++w2) m = __builtin_fmaxf(m, pm[w2 * kTile + 16 * wave + n]);
        sx[16 * wave + n] = shift_of(m);
    }
    bar();
    if (act_out) {
#pragma unroll
        for (int q = 0; q < kGroups; ++q) put_group(lds, wave, q, v[q][0], v[q][1], sx[16 * q + n]);
    }
    bar();
}

// partial maxima of the wave's 32 features per sample -> pm[w][*]; returns the wave's overall max
__device__ __forceinline__ float partial_max(unsigned char* lds, const fx4 (&v)[kGroups][2]) {
    float* pm = (float*)(lds + kOffPm);
    const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15;
    float all = 0.0f;
#pragma unroll
    for (int q = 0; q < kGroups; ++q) {
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fabsf(v[q][0][i]), __builtin_fabsf(v[q][1][i])));   // v_max3
        m = sample_reduce(m);
        if (lane < 16) pm[wave * kTile + 16 * q + n] = m;
        all = __builtin_fmaxf(all, m);
    }
    return all;
}

// the wave's max of a slab -> smax[slab][global wave] (dw16's layer-wide exponent shifts)
__device__ __forceinline__ void slab_max(float* part, int slab, float m) {
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) m = __builtin_fmaxf(m, __shfl_xor(m, d));
    if ((threadIdx.x & 63) == 0)
        part[(size_t)slab * gridDim.x * kWaves + blockIdx.x * kWaves + (threadIdx.x >> 6)] = m;
}

__global__ void __launch_bounds__(kThreads, 1) kact_fwd_bwd_kernel(KaArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kLdsBytes];
#if LNERF_KACT_PROF
    unsigned long long qp[kQpN] = {};
    QP_T(q_start);
#endif
    float* comp = (float*)(lds + kOffComp);
    float* rayloss = (float*)(lds + kOffRay);
    int* sx0 = (int*)(lds + kOffSx);

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), g = lane >> 4, n = lane & 15;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
    const bool st = a.want_grad != 0;
    const int t0 = 2 * wave;
    // per-layer weight exponent shifts in lane l
    int wexp_lane = 0;
    if (lane < a.L) {
        const float mx = __int_as_float(a.wexp[lane]);
        wexp_lane = shift_of(mx);
    }
    // the biases into LDS (read by every epilogue; visible after the PE stage's barrier)
    float* lbias = (float*)(lds + kOffBias);
    for (int i = tid; i < a.L * 64; i += kThreads) ((fx4*)lbias)[i] = ((const fx4*)a.b16)[i];
    int sxi = 0;   // sx buffer holding the current pass input's per-sample shifts
    fx4 acc[kGroups][2];
    fx4 vout[kGroups][2];

    // ---- layer-0 input: wave w encodes group q = w (pos_encoding.py:54-66), X slab, act k-steps
    QP_T(q_pe);
    {
        const int ks0 = a.ks_f[0];
        const int ls = 16 * wave + n, gs = wg * tile_samples + ls;
        const bool valid = ls < tile_samples && gs < a.R;
        float m = 0.0f;
        float xv[8][8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (s < ks0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int f = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
                    xv[s][j] = comp::input_feature(a, gs, valid, f);
                    m = __builtin_fmaxf(m, __builtin_fabsf(xv[s][j]));
                }
            }
        }
        m = sample_reduce(m);
        const int ex = shift_of(m);
        if (lane < 16) sx0[ls] = ex;
        float* xs = a.act + a.x_off + ((size_t)wg * 4 + (wave >> 1)) * (size_t)(ks0 * 1024) + (wave & 1) * 512;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (s < ks0) {
                const fx4 t0v = {xv[s][0], xv[s][1], xv[s][2], xv[s][3]};
                const fx4 t1v = {xv[s][4], xv[s][5], xv[s][6], xv[s][7]};
                put_group(lds, s, wave, t0v, t1v, ex);
                if (st) store_slab(xs + s * 1024, t0v, t1v);
            }
        }
        if (st) slab_max(a.smax, 0, m);   // (m is per sample; slab_max folds the 16 samples)
        bar();
    }

    unsigned long long* mask_w = a.mask_g + ((size_t)wg * (a.L - 1) * kWaves + wave) * 64 + lane;
    QP_ADD(kQpPe, q_pe);
    WFrag wf[kWRing];   // the weight-fragment ring (k-steps s % kWRing)
    float* pend = nullptr;   // deferred slab stores of vout (store_one)
    int pnt = 1;
    pass_pre(a.w16 + a.wf_off[0], a.ks_f[0], a.to_f[0], t0, wf);

    // ---- forward hidden layers ----
    for (int l = 0; l + 1 < a.L; ++l) {
        const int to = a.to_f[l], ks = a.ks_f[l];
        const unsigned short* wb = a.w16 + a.wf_off[l];
        const bool on = t0 < to;
        zero_acc(acc);
        QP_T(q_m);
        mma_pass(lds, wb, ks, to, t0, wf, acc, vout, pend, pnt);
        QP_ADD(kQpMma, q_m);
        QP_T(q_e);
        if (l + 2 < a.L) pass_pre(a.w16 + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], t0, wf);
        // epilogue: 2^-(ex + ew) (exact), bias after the sum (nerf.py:98,125), ReLU
        // (nerf.py:141-144) and its mask bits, A_l slab, partial maxima
        const int* sx = sx0 + sxi * kTile;
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        const float* bl = lbias + l * 256 + 16 * t0 + 4 * g;
        const fx4 b0 = *(const fx4*)bl, b1 = *(const fx4*)(bl + 16);
        unsigned mb[2] = {0u, 0u};
        // acc 2^-(ex + ew) is exact (shifts clamped), so the fma rounds exactly like the sum
        // ldexp(acc) + b
#pragma unroll
        for (int q = 0; q < kGroups; ++q) {
            const float sc = __builtin_ldexpf(1.0f, -(sx[16 * q + n] + ew));
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    vout[q][t][i] = relu_bit(__builtin_fmaf(acc[q][t][i], sc, t ? b1[i] : b0[i]), mb[q >> 2]);
        }
        if (st && on) mask_w[(size_t)l * kWaves * 64] = (unsigned long long)mb[0] | ((unsigned long long)mb[1] << 32);
        // the A_l slab (the wave's 32-feature slab tile, if it exists), stored during the next pass
        pend = st && wave < a.nt[l] ? a.act + a.act_off[l] + (size_t)wg * 4 * a.nt[l] * 1024 + (size_t)wave * 1024
                                    : nullptr;
        pnt = a.nt[l];
        if (!kDefer && pend) {
            store_range(std::make_integer_sequence<int, 64>{}, pend, pnt, vout);
            pend = nullptr;
        }
        const float wm = partial_max(lds, vout);
        if (st) slab_max(a.smax, l + 1, wm);   // every wave writes its entry (0 past the layer)
        sxi ^= 1;
        QP_ADD(kQpEpi, q_e);
        QP_T(q_b);
        publish(lds, vout, sxi, on);
        QP_ADD(kQpBar, q_b);
    }

    // ---- head (nerf.py:150-167 pre-activations): wave w computes group q = w, all k-steps ----
    {
        const int l = a.L - 1, ks = a.ks_f[l], to = a.to_f[l];
        const unsigned short* wb = a.w16 + a.wf_off[l];
        const int* sx = sx0 + sxi * kTile;
        fx4 c = {0.0f, 0.0f, 0.0f, 0.0f};
        if (pend) store_range(std::make_integer_sequence<int, 64>{}, pend, pnt, vout);   // A_{L-2}
        pend = nullptr;
        for (int s = 0; s < ks; ++s) {
            const unsigned short* p0 = wb + ((size_t)(s * to) * 2) * 512 + lane * 8;
            const u4 wh = *(const u4*)p0, wl = *(const u4*)(p0 + 512);
            const u4 bh = *(const u4*)act_frag(lds, s, wave, 0);
            const u4 blo = *(const u4*)act_frag(lds, s, wave, 1);
            c = mfma_h(wh, blo, c);
            c = mfma_h(wl, bh, c);
            c = mfma_h(wh, bh, c);
        }
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        const int sh = -(sx[16 * wave + n] + ew);
        if (g == 0) {
            const fx4 bv = *(const fx4*)(lbias + l * 256);
#pragma unroll
            for (int i = 0; i < 4; ++i) comp[(16 * wave + n) * 4 + i] = __builtin_ldexpf(c[i], sh) + bv[i];
        }
    }
    QP_T(q_c);
    bar();
    // ---- rendering + loss + rendering reverse (one thread per sample, scans along rays) ----
    comp::composite_tile(a, wg, comp, rayloss, st);
    bar();
    QP_ADD(kQpComp, q_c);
    if (tid == 0) {
        float lsum = 0.0f;
        for (int r = 0; r < a.rpw; ++r) lsum = lsum + rayloss[r];
        a.loss_part[wg] = lsum;
    }
    if (!st) return;

    // ---- G_{L-1} (head gradients, features 0..3 = elements 0..3 of lane group 0): slab, act ----
    pass_pre(a.w16 + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], t0, wf);
    {
        const int l = a.L - 1;
        const float* c_gz = comp + 512;
        fx4 gh = {0.0f, 0.0f, 0.0f, 0.0f};
        const fx4 z = {0.0f, 0.0f, 0.0f, 0.0f};
        const int ls = 16 * wave + n;
        if (g == 0 && ls < tile_samples) gh = *(const fx4*)(c_gz + ls * 4);
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) m = __builtin_fmaxf(m, __builtin_fabsf(gh[i]));
        m = sample_reduce(m);
        const int ex = shift_of(m);
        sxi ^= 1;
        if (lane < 16) sx0[sxi * kTile + ls] = ex;
        put_group(lds, 0, wave, gh, z, ex);
        float* sl = a.grad + a.grad_off[l] + ((size_t)wg * 4 + (wave >> 1)) * (size_t)(a.nt[l] * 1024) + (wave & 1) * 512;
        store_slab(sl, gh, z);
        for (int s = 1; s < a.nt[l]; ++s) store_slab(sl + s * 1024, z, z);
        slab_max(a.smax, a.L + l, m);
        bar();
    }

    // ---- reverse chain: G_{l-1} = (W_l^T G_l) * 1[A_{l-1} > 0], l = L-1 .. 1 ----
    for (int l = a.L - 1; l >= 1; --l) {
        const int to = a.to_b[l], ks = a.ks_b[l];
        const unsigned short* wb = a.w16 + a.wb_off[l];
        const bool on = t0 < to;
        zero_acc(acc);
        const unsigned long long mb64 = on ? mask_w[(size_t)(l - 1) * kWaves * 64] : 0ull;
        QP_T(q_m);
        mma_pass(lds, wb, ks, to, t0, wf, acc, vout, pend, pnt);
        QP_ADD(kQpMma, q_m);
        QP_T(q_e);
        if (l > 1) pass_pre(a.w16 + a.wb_off[l - 1], a.ks_b[l - 1], a.to_b[l - 1], t0, wf);
        else if (a.d_x) pass_pre(a.w16 + a.wb_off[0], a.ks_b[0], a.to_b[0], t0, wf);
        const int* sx = sx0 + sxi * kTile;
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        const unsigned mw[2] = {(unsigned)mb64, (unsigned)(mb64 >> 32)};
#pragma unroll
        for (int q = 0; q < kGroups; ++q) {
            const float sc = __builtin_ldexpf(1.0f, -(sx[16 * q + n] + ew));
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    vout[q][t][i] = keep_if(mw[q >> 2], 8 * (q & 3) + 4 * t + i, acc[q][t][i] * sc);
        }
        // the G_{l-1} slab, stored during the next pass (or after the chain)
        pend = wave < a.nt[l - 1]
                   ? a.grad + a.grad_off[l - 1] + (size_t)wg * 4 * a.nt[l - 1] * 1024 + (size_t)wave * 1024
                   : nullptr;
        pnt = a.nt[l - 1];
        if (!kDefer && pend) {
            store_range(std::make_integer_sequence<int, 64>{}, pend, pnt, vout);
            pend = nullptr;
        }
        const float wm = partial_max(lds, vout);
        slab_max(a.smax, a.L + l - 1, wm);
        sxi ^= 1;
        // G_0 is the last slab; its act copy is only needed by the d_x pass
        QP_ADD(kQpEpi, q_e);
        QP_T(q_b);
        publish(lds, vout, sxi, on && (l > 1 || a.d_x));
        QP_ADD(kQpBar, q_b);
    }

    // ---- d_layer_input = G_0 W_0^T (ENCODED mode) ----
    if (a.d_x) {
        const int to = a.to_b[0], ks = a.ks_b[0];
        const unsigned short* wb = a.w16 + a.wb_off[0];
        const bool on = t0 < to;
        zero_acc(acc);
        mma_pass(lds, wb, ks, to, t0, wf, acc, vout, pend, pnt);   // also stores G_0
        pend = nullptr;
        if (on) {
            const int* sx = sx0 + sxi * kTile;
            const int ew = __builtin_amdgcn_readlane(wexp_lane, 0);
#pragma unroll
            for (int q = 0; q < kGroups; ++q) {
                const int ls = 16 * q + n, gs = wg * tile_samples + ls;
                if (ls < tile_samples && gs < a.R) {
                    const int sh = -(sx[ls] + ew);
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int f = 16 * (t0 + t) + 4 * g + i;
                            if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = __builtin_ldexpf(acc[q][t][i], sh);
                        }
                }
            }
        }
    }
    if (pend) store_range(std::make_integer_sequence<int, 64>{}, pend, pnt, vout);   // G_0
#if LNERF_KACT_PROF
    QP_ADD(kQpTotal, q_start);
    if (lane == 0)
        for (int i = 0; i < kQpN; ++i) atomicAdd(&g_kact_prof[i], qp[i]);
#endif
}

}  // namespace

bool kact_supported(const FusedPlan& p) {
    if (p.x6 != 2) return false;                 // the fp16x3 planes only
    if (p.n[p.L - 1] > 16) return false;         // head: one 16-wide output tile
    if (p.L < 2) return false;
    return true;
}

void kact_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                 bool want_grad, hipStream_t s) {
    KaArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.ks_f[l] = p.ks16_f[l];
        a.ks_b[l] = p.ks16_b[l];
        a.to_f[l] = p.to16_f[l];
        a.to_b[l] = p.to16_b[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = p.w16f_off[l];
        a.wb_off[l] = p.w16b_off[l];
        a.act_off[l] = p.act_off[l];
        a.grad_off[l] = p.grad_off[l];
    }
    a.k0 = p.k[0];
    a.w16 = p.w16;
    a.b16 = p.b16;
    a.wexp = p.wexp16;
    a.mask_g = p.mask_g;
    a.act = p.act;
    a.x_off = p.x_off;
    a.grad = p.grad;
    a.smax = p.smax_part;
    a.rays = p.rays;
    a.S = p.S;
    a.rpw = p.rays_per_wg;
    a.R = p.R;
    a.input_mode = b.input_mode;
    a.F = b.num_freqs;
    a.near_t = b.near_t;
    a.far_t = b.far_t;
    a.x = b.x;
    a.dists = b.input_mode == LNERF_INPUT_RAYS ? nullptr : b.dists;
    a.target = b.target;
    a.loss_part = p.loss_part;
    a.acc_color = out.acc_color;
    a.d_dists = want_grad ? out.d_dists : nullptr;
    a.d_target = want_grad ? out.d_target : nullptr;
    a.d_x = want_grad ? out.d_x : nullptr;
    a.seed = seed;
    a.want_grad = want_grad ? 1 : 0;
    static_assert(sizeof(KaArgs) <= 4096, "kernel arguments");
    kact_fwd_bwd_kernel<<<p.num_wg, kThreads, 0, s>>>(a);
#if LNERF_KACT_PROF
    if (want_grad) {
        unsigned long long h[8] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_kact_prof), sizeof(h));
        const char* names[] = {"pe", "mma", "epilogue", "publish", "composite", "total"};
        fprintf(stderr, "LNERF_PROF kact per-wave cycles:");
        for (int i = 0; i < kQpN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / ((double)p.num_wg * kWaves));
        fprintf(stderr, "\n");
        unsigned long long z[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kact_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
