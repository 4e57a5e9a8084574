// lnerf_kact.hip -- k1 with the activations resident in LDS: the fused PE + MLP + compositing +
// reverse chain for the fp16x3 split, the default fused kernel wherever it applies.
//
// Same work and outputs as k16 (lnerf_k16.hip; reference scripts/nerf.py:1-304 and its rev_diff,
// train_nerf.py:325/395), with the operand roles of the 128-sample workgroup tile swapped:
//  * the layer input of all 128 samples lives in LDS, already split into its fp16 hi / lo planes
//    in the MFMA B-operand layout, act[k-step 8][sample group 8][plane 2][lane 64][16 B]
//    (128 KiB); it is written once per layer by the wave that produced those features;
//  * wave w owns the 32 output features 32w .. 32w + 31 (16-wide tiles 2w, 2w + 1) of every
//    layer and streams exactly its weight fragments straight from L2 into registers (a ring of
//    kWRing k-steps): no LDS-DMA, no weight ring in LDS;
//  * a weight fragment feeds 4 sample groups and an activation fragment feeds two tiles;
//  * the producing wave's accumulator register j of lane (n, g) is exactly element j of the next
//    layer's B fragment for k-step w (the phi permutation of the packed weights, k16_pack), so a
//    layer epilogue splits its own registers and writes two lane-linear ds_write_b128 per group;
//  * the 128 samples run as two halves half a layer apart: while the MFMAs of one half stream,
//    the other half's epilogue (unscale, bias, ReLU + mask bits, slab stores, the per-sample
//    exponent exchange through LDS, the split into the next act) is woven between them, so the
//    epilogue VALU issues in the MFMA shadow (two barriers per half-layer slot).
// The slabs (A_l, G_l), ReLU masks and per-wave slab maxima go to k16's HBM layouts, so dw16 and
// the reduce kernels are shared (the mask bit order is kact's own: epi_unit1 / keep_if).
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
constexpr int kOffPm = kOffRay + kTile * 4;      // per-sample per-wave maxima [128][8] f32
constexpr int kOffSx = kOffPm + kWaves * kTile * 4;   // per-sample exponent shifts [128] i32 (+ spare)
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
enum { kQpPe, kQpMma, kQpComp, kQpTotal, kQpN };
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

// bit 31 - j of m set ? x : +0 (the backward's mask, in epi_unit1's order)
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

// Workgroup barrier for LDS hand-offs only: every LDS access of the wave done (lgkmcnt(0)), then
// s_barrier -- no vmcnt(0): __syncthreads' fence would also wait for the slab stores in flight,
// which no other wave reads in this kernel.
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ---- weight fragments: wave w's tiles t0 = 2w, t0 + 1 of a pass, k-step s, both fp16 planes ----
// (a k-step feeds 4 sample groups x 2 tiles x 3 MFMAs ~ 400 SIMD cycles; kWRing k-steps in flight)
// timing experiments only (wrong results; never in the product build): no slab stores, every
// weight load from k-step 0, no epilogue arithmetic (barriers kept)
#ifndef LNERF_KACT_NOSTORE
#define LNERF_KACT_NOSTORE 0
#endif
#ifndef LNERF_KACT_WFIX
#define LNERF_KACT_WFIX 0
#endif
#ifndef LNERF_KACT_NOEPI
#define LNERF_KACT_NOEPI 0   // 1: no epilogue arithmetic; 2: part 1 only; 3: part 2 only
#endif
#ifndef LNERF_KACT_ILV_KS
#define LNERF_KACT_ILV_KS 8  // shortest pass (k-steps) the epilogue is woven into
#endif
#ifndef LNERF_KACT_WRING
#define LNERF_KACT_WRING 2
#endif
constexpr int kWRing = LNERF_KACT_WRING;
static_assert(kWRing == 2 || kWRing == 3 || kWRing == 4, "weight ring depth");
struct WFrag {
    u4 v[4];   // tile 0 planes 0, 1; tile 1 planes 0, 1
};

// A pass's weights as a buffer: fragment (k-step s, tile t, plane p) of lane l at byte
// (s to + t) 2048 + p 1024 + 16 l (k16_pack), so every load shares one lane offset VGPR and the
// rest is scalar. Without a second tile (odd tile count) tile 0's fragments are loaded twice; the
// caller zeroes that accumulator (clear_second), so no branch enters the unrolled pass.
struct WSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    int kstride;   // to 2048 (bytes per k-step)
    int t0off;     // t0 2048
    int t1off;     // 2048 with a second tile, else 0
};
__device__ __forceinline__ WSrc wsrc(const unsigned short* wb, int ks, int to, int t0) {
    WSrc w;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(wb), 0, ks * to * 2048, 0x00020000);
    w.kstride = to * 2048;
    w.t0off = t0 * 2048;
    w.t1off = t0 + 1 < to ? 2048 : 0;
    return w;
}
__device__ __forceinline__ u4 wload(const WSrc& w, int off, int soff) {
    return __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, (int)(threadIdx.x & 63) * 16 + off, soff, 0));
}
__device__ __forceinline__ void load_w(const WSrc& w, int s, WFrag& f) {
    const int so = (LNERF_KACT_WFIX ? 0 : s) * w.kstride + w.t0off;
    f.v[0] = wload(w, 0, so);
    f.v[1] = wload(w, 1024, so);
    f.v[2] = wload(w, 0, so + w.t1off);
    f.v[3] = wload(w, 1024, so + w.t1off);
}

// request the first kWRing - 1 k-steps of a pass (issued before the previous slot's barrier, so
// their L2 latency hides behind it)
__device__ __forceinline__ void pass_pre(const unsigned short* wb, int ks, int to, int t0, WFrag (&w)[kWRing]) {
    if (t0 >= to) return;
    const WSrc src = wsrc(wb, ks, to, t0);
#pragma unroll
    for (int s = 0; s + 1 < kWRing; ++s)
        if (s < ks) load_w(src, s, w[s]);
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 at an immediate offset, outside the compiler's waitcnt bookkeeping (the matching
// lgkm_wait below is the only wait, so the next group's reads stay in flight under the MFMAs;
// any LDS operation the compiler adds in between only makes that wait longer, never too short)
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

// the hi / lo B fragments of act k-step s, group q (J = 8 s + q); offsets past 64 KiB from the
// second base address
template <int J>
__device__ __forceinline__ void read_b(unsigned b0, unsigned b1, u4& h, u4& l) {
    constexpr int off = J * 2048;
    if constexpr (off < 65536 - 1024) {
        h = ds_read_at<off>(b0);
        l = ds_read_at<off + 1024>(b0);
    } else {
        h = ds_read_at<off - 65536>(b1);
        l = ds_read_at<off + 1024 - 65536>(b1);
    }
}

// ---------------------------------------------------------------------------------------------
// Epilogues. A layer's outputs are finished per sample half (groups 4h .. 4h + 3) while the MMA
// of the other half runs: part 1 (unscale, bias, ReLU + mask bits or the backward's mask, slab
// stores, per-sample partial maxima -> pm), one barrier, part 2 (the per-sample shift from the
// eight waves' maxima, split, write k-step `wave` of the next pass's act). Each slice is placed
// between MFMA steps of the pass at compile time, so its VALU work issues in the MFMA shadow.
// ---------------------------------------------------------------------------------------------
enum { kEpiNone = 0, kEpiFwd = 1, kEpiBwd = 2 };
constexpr int kInterleaveKs = LNERF_KACT_ILV_KS;

struct Ctx {
    unsigned char* lds;
    int sxr[kGroups];   // input shift of sample 16 q + n of the pass being finished / next
    float wmax;         // the wave's max over the layer being finished (dw16 slab shifts)
    unsigned mb[2];     // forward: ReLU mask bits per half; backward: the mask words in use
    fx4 pmv[2];         // part 2's pm read, one group ahead
};

// slab stores of one half's epilogue: hardware-dropped when disabled (num_records 0), so no
// branch splits the unrolled pass
struct Epi {
    fx4 b[2];   // forward: biases of tiles t0, t0 + 1
    int ew;     // the layer's weight shift
    __amdgpu_buffer_rsrc_t rsrc;
    int voff;   // lane part of a slab address (bytes)
    int so[2];  // half-block pair offsets (bytes) of groups 4h + {0, 1} and 4h + {2, 3}
};

__device__ __forceinline__ Epi make_epi(const float* lbias, int l, int ew, float* slab, int nt, int h, bool fwd) {
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
    const int t0 = 2 * (threadIdx.x >> 6);
    Epi e;
    if (fwd) {
        const float* bl = lbias + l * 256 + 16 * t0 + 4 * g;
        e.b[0] = *(const fx4*)bl;
        e.b[1] = *(const fx4*)(bl + 16);
    } else {
        e.b[0] = e.b[1] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    e.ew = ew;
    e.rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, slab && !LNERF_KACT_NOSTORE ? nt * 16384 : 0, 0x00020000);
    e.voff = 256 * g + 4 * n;
    e.so[0] = 2 * h * nt * 4096;
    e.so[1] = (2 * h + 1) * nt * 4096;
    return e;
}

// max3 without the compiler's NaN canonicalisation of loaded operands (the values are finite or
// the shift falls back to 0 either way)
__device__ __forceinline__ float max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float amax3(float a, float b, float c) {   // max(a, |b|, |c|)
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// max over the 4 lanes of a sample (n, n + 16, n + 32, n + 48): two permlane swaps
__device__ __forceinline__ float sample_max4(float m) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    m = __builtin_fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return __builtin_fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

// part 1, unit K = 2 ql + t of half H: the 4 values of tile t, group 4 H + ql
template <int KIND, int H, int K>
__device__ __forceinline__ void epi_unit1(Ctx& c, fx4 (&v)[4][2], const Epi& e) {
    if constexpr (LNERF_KACT_NOEPI == 1 || LNERF_KACT_NOEPI == 3) return;
    constexpr int ql = K >> 1, t = K & 1, q = 4 * H + ql;
    const float sc = __builtin_ldexpf(1.0f, -(c.sxr[q] + e.ew));
    if constexpr (KIND == kEpiFwd) {
        // 2^-(ex + ew) is exact (shifts clamped), so the fma rounds like ldexp(acc) + b; bias
        // after the sum (nerf.py:98,125), ReLU (nerf.py:141-144); the mask bits of value
        // j = 4 K + i at bit 31 - j (keep_if's order), four independent compare/selects
        unsigned nib = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x = __builtin_fmaf(v[ql][t][i], sc, e.b[t][i]);
            const bool p = x > 0.0f;
            v[ql][t][i] = p ? x : 0.0f;
            nib |= (p ? 1u : 0u) << (3 - i);
        }
        if constexpr (K == 0) c.mb[H] = nib << 28;
        else c.mb[H] |= nib << (28 - 4 * K);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[ql][t][i] = keep_if(c.mb[H], 8 * ql + 4 * t + i, v[ql][t][i] * sc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[ql][t][i]), e.rsrc, e.voff,
                                              e.so[ql >> 1] + (ql & 1) * 2048 + (16 * t + i) * 64, 2);
    if constexpr (t == 1) {
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            m = amax3(m, v[ql][0][i], v[ql][1][i]);
        m = sample_max4(m);
        float* pm = (float*)(c.lds + kOffPm);
        const int lane = threadIdx.x & 63, n = lane & 15;
        pm[(16 * q + n) * kWaves + wave_id()] = m;   // the 4 lanes of a sample write the same value
        c.wmax = __builtin_fmaxf(c.wmax, m);
    }
}

template <int H, int QL>
__device__ __forceinline__ void pm_read(Ctx& c) {
    const int n = threadIdx.x & 15;
    const fx4* p = (const fx4*)(c.lds + kOffPm) + (16 * (4 * H + QL) + n) * 2;
    c.pmv[0] = p[0];
    c.pmv[1] = p[1];
}

// part 2, group ql of half H: shift from the 8 waves' maxima, split, write act k-step `wave`
template <int H, int QL>
__device__ __forceinline__ void epi_unit2(Ctx& c, fx4 (&v)[4][2]) {
    if constexpr (LNERF_KACT_NOEPI == 1 || LNERF_KACT_NOEPI == 2) return;
    constexpr int q = 4 * H + QL;
    const fx4 a = c.pmv[0], b = c.pmv[1];
    if constexpr (QL + 1 < 4) pm_read<H, QL + 1>(c);
    const float m = max3(max3(a[0], a[1], a[2]), max3(a[3], b[0], b[1]), max3(b[2], b[3], 0.0f));
    const int ex = shift_of(m);
    c.sxr[q] = ex;
    const int n = threadIdx.x & 15;
    ((int*)(c.lds + kOffSx))[16 * q + n] = ex;   // (the head reads it; same value from every lane)
    put_group(c.lds, wave_id(), q, v[QL][0], v[QL][1], ex);
}

// the slice of half H's epilogue that goes with step I of an N-step pass: part 1 units at steps
// (K h) / 8, the barrier at h = N / 2, part 2 units from h + 1 on
template <int KIND, int H, int I, int N, int... K>
__device__ __forceinline__ void epi_part1_at(std::integer_sequence<int, K...>, Ctx& c, fx4 (&v)[4][2], const Epi& e) {
    constexpr int h = N / 2;
    ((((K * h) / 8 == I) ? (epi_unit1<KIND, H, K>(c, v, e), 0) : 0), ...);
}
template <int H, int I, int N, int... U>
__device__ __forceinline__ void epi_part2_at(std::integer_sequence<int, U...>, Ctx& c, fx4 (&v)[4][2]) {
    constexpr int h = N / 2;
    (((h + 1 + (U * (h - 1)) / 4 == I) ? (epi_unit2<H, U>(c, v), 0) : 0), ...);
}

template <int KIND, int H, int I, int N>
__device__ __forceinline__ void epi_slice(Ctx& c, fx4 (&v)[4][2], const Epi& e) {
    if constexpr (KIND != kEpiNone) {
        constexpr int h = N / 2;
        if constexpr (I < h) epi_part1_at<KIND, H, I, N>(std::make_integer_sequence<int, 8>{}, c, v, e);
        if constexpr (I == h) {
            bar();   // every wave's partial maxima of half H are in pm
            pm_read<H, 0>(c);
        }
        if constexpr (I > h) epi_part2_at<H, I, N>(std::make_integer_sequence<int, 4>{}, c, v);
    }
}

// a whole epilogue of half H without an MMA beside it (same barrier count as a slot)
template <int KIND, int H>
__device__ __forceinline__ void epi_alone(Ctx& c, fx4 (&v)[4][2], const Epi& e) {
    epi_part1_at<KIND, H, 0, 2>(std::make_integer_sequence<int, 8>{}, c, v, e);
    bar();
    pm_read<H, 0>(c);
    epi_unit2<H, 0>(c, v);
    epi_unit2<H, 1>(c, v);
    epi_unit2<H, 2>(c, v);
    epi_unit2<H, 3>(c, v);
}

// ---- one slot: the MMA of half HM over KS k-steps (acc am) with half HE's epilogue (acc ae)
// woven in. Step I = 4 s + ql: prefetch the weights of k-step s + kWRing - 1 (at ql = 0), the
// epilogue slice, the next step's B fragments, wait for this step's, 6 MFMAs (small terms first).
template <int KS, int HM, int KIND, int HE, int I>
__device__ __forceinline__ void slot_step(Ctx& c, unsigned b0, unsigned b1, const WSrc& ws,
                                          WFrag (&w)[kWRing], u4 (&bh)[2], u4 (&bl)[2], fx4 (&am)[4][2],
                                          fx4 (&ae)[4][2], const Epi& e) {
    constexpr int N = KS * 4, s = I / 4, ql = I % 4;
    constexpr int J = 8 * s + 4 * HM + ql, Jn = 8 * ((I + 1) / 4) + 4 * HM + (I + 1) % 4;
    if constexpr (ql == 0 && s + kWRing - 1 < KS) load_w(ws, s + kWRing - 1, w[(s + kWRing - 1) % kWRing]);
    epi_slice<KIND, HE, I, N>(c, ae, e);
    if constexpr (I + 1 < N) {
        read_b<Jn>(b0, b1, bh[(I + 1) & 1], bl[(I + 1) & 1]);
        lgkm_wait<2>(bh[I & 1], bl[I & 1]);
    } else {
        lgkm_wait<0>(bh[I & 1], bl[I & 1]);
    }
    (void)J;
    const WFrag& f = w[s % kWRing];
    fx4 x = am[ql][0];
    x = mfma_h(f.v[0], bl[I & 1], x);
    x = mfma_h(f.v[1], bh[I & 1], x);
    x = mfma_h(f.v[0], bh[I & 1], x);
    am[ql][0] = x;
    fx4 y = am[ql][1];
    y = mfma_h(f.v[2], bl[I & 1], y);
    y = mfma_h(f.v[3], bh[I & 1], y);
    y = mfma_h(f.v[2], bh[I & 1], y);
    am[ql][1] = y;
}

template <int KS, int HM, int KIND, int HE, int... I>
__device__ __forceinline__ void slot_steps(std::integer_sequence<int, I...>, Ctx& c, unsigned b0, unsigned b1,
                                           const WSrc& ws, WFrag (&w)[kWRing],
                                           u4 (&bh)[2], u4 (&bl)[2], fx4 (&am)[4][2], fx4 (&ae)[4][2],
                                           const Epi& e) {
    (slot_step<KS, HM, KIND, HE, I>(c, b0, b1, ws, w, bh, bl, am, ae, e), ...);
}

template <int KS, int HM, int KIND, int HE>
__device__ __forceinline__ void slot_t(Ctx& c, const WSrc& ws, WFrag (&w)[kWRing],
                                       fx4 (&am)[4][2], fx4 (&ae)[4][2], const Epi& e) {
    const unsigned b0 = lds_addr(c.lds) + (threadIdx.x & 63) * 16, b1 = b0 + 65536;
    u4 bh[2], bl[2];
    read_b<4 * HM>(b0, b1, bh[0], bl[0]);
    slot_steps<KS, HM, KIND, HE>(std::make_integer_sequence<int, KS * 4>{}, c, b0, b1, ws, w, bh, bl, am, ae, e);
}

__device__ __forceinline__ void zero4(fx4 (&a)[4][2]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q][0] = a[q][1] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
}

// a pass with one tile leaves tile 0's duplicate in the second accumulator: clear it
__device__ __forceinline__ void clear_second(fx4 (&a)[4][2], int to, int t0) {
    if (t0 + 1 >= to) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q][1] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
    }
}

// One slot: MMA of half HM (layer pass wb / ks / to) beside half HE's epilogue of kind KIND.
// A wave without output tiles in the pass runs the epilogue alone (same single barrier).
template <int HM, int KIND, int HE>
__device__ __forceinline__ void slot(Ctx& c, const unsigned short* wb, int ks, int to, int t0, WFrag (&w)[kWRing],
                                     fx4 (&am)[4][2], fx4 (&ae)[4][2], const Epi& e) {
    zero4(am);
    if (t0 >= to) {
        if constexpr (KIND != kEpiNone) epi_alone<KIND, HE>(c, ae, e);
        return;
    }
    const WSrc ws = wsrc(wb, ks, to, t0);
    // the epilogue is woven into full-depth passes only (kInterleaveKs k-steps and more); shorter
    // passes run it first, whole, then the bare MMA (a short pass has too few MFMA gaps to hide
    // it, and its crammed slices would raise the kernel's register peak)
    if constexpr (KIND != kEpiNone) {
        if (ks >= kInterleaveKs) {
            slot_t<8, HM, KIND, HE>(c, ws, w, am, ae, e);
            clear_second(am, to, t0);
            return;
        }
        epi_alone<KIND, HE>(c, ae, e);
    }
#define LNERF_KACT_SLOT(K) \
    case K: slot_t<K, HM, kEpiNone, HE>(c, ws, w, am, ae, e); break;
    switch (ks) {
        LNERF_KACT_SLOT(1)
        LNERF_KACT_SLOT(2)
        LNERF_KACT_SLOT(3)
        LNERF_KACT_SLOT(4)
        LNERF_KACT_SLOT(5)
        LNERF_KACT_SLOT(6)
        LNERF_KACT_SLOT(7)
        default: slot_t<8, HM, kEpiNone, HE>(c, ws, w, am, ae, e); break;
    }
#undef LNERF_KACT_SLOT
    clear_second(am, to, t0);
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
    int* sxl = (int*)(lds + kOffSx);

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
    Ctx c;
    c.lds = lds;
    c.wmax = 0.0f;
    c.mb[0] = c.mb[1] = 0u;
    fx4 acc0[4][2], acc1[4][2];   // sample halves: groups 0..3, 4..7
    WFrag wf[kWRing];             // the weight-fragment ring (k-steps s % kWRing)
    const Epi none{};
    // slab base of the wave's 32-feature tile in layer l's slab at `base` (nullptr: no slab)
    auto slab_of = [&](float* base, size_t off, int nt) -> float* {
        return st && wave < nt ? base + off + (size_t)wg * 4 * nt * 1024 + (size_t)wave * 1024 : nullptr;
    };

    // ---- layer-0 input: wave w encodes group q = w (pos_encoding.py:54-66), X slab, act k-steps
    pass_pre(a.w16 + a.wf_off[0], a.ks_f[0], a.to_f[0], t0, wf);
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
        m = sample_max4(m);
        const int ex = shift_of(m);
        sxl[ls] = ex;
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
#pragma unroll
        for (int q = 0; q < kGroups; ++q) c.sxr[q] = sxl[16 * q + n];
    }
    QP_ADD(kQpPe, q_pe);

    unsigned long long* mask_w = a.mask_g + ((size_t)wg * (a.L - 1) * kWaves + wave) * 64 + lane;

    // ---- forward hidden layers, the two sample halves half a layer apart:
    //   F0: MMA(0, H0); then per layer l: A(l): MMA(l, H1) | epilogue(l, H0),
    //   B(l): MMA(l + 1, H0) | epilogue(l, H1)  (the last layer's B: the epilogue alone)
    QP_T(q_m);
    slot<0, kEpiNone, 1>(c, a.w16 + a.wf_off[0], a.ks_f[0], a.to_f[0], t0, wf, acc0, acc1, none);
    pass_pre(a.w16 + a.wf_off[0], a.ks_f[0], a.to_f[0], t0, wf);
    for (int l = 0; l + 1 < a.L; ++l) {
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        float* slab = slab_of(a.act, a.act_off[l], a.nt[l]);
        const bool more = l + 2 < a.L;   // another hidden pass follows
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l], 0, true);
            slot<1, kEpiFwd, 0>(c, a.w16 + a.wf_off[l], a.ks_f[l], a.to_f[l], t0, wf, acc1, acc0, e);
            if (more) pass_pre(a.w16 + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], t0, wf);
            bar();
        }
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l], 1, true);
            if (more) {
                slot<0, kEpiFwd, 1>(c, a.w16 + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], t0, wf, acc0, acc1, e);
                pass_pre(a.w16 + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], t0, wf);
            } else {
                epi_alone<kEpiFwd, 1>(c, acc1, e);
            }
            if (st && t0 < a.to_f[l])
                mask_w[(size_t)l * kWaves * 64] = (unsigned long long)c.mb[0] | ((unsigned long long)c.mb[1] << 32);
            if (st) slab_max(a.smax, l + 1, c.wmax);   // every wave writes its entry (0 past the layer)
            c.wmax = 0.0f;
            bar();
        }
    }
    QP_ADD(kQpMma, q_m);

    // ---- head (nerf.py:150-167 pre-activations): wave w computes group q = w, all k-steps ----
    {
        const int l = a.L - 1, ks = a.ks_f[l], to = a.to_f[l];
        const unsigned short* wb = a.w16 + a.wf_off[l];
        fx4 hc = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int s = 0; s < ks; ++s) {
            const unsigned short* p0 = wb + ((size_t)(s * to) * 2) * 512 + lane * 8;
            const u4 wh = *(const u4*)p0, wl = *(const u4*)(p0 + 512);
            const u4 bh = *(const u4*)act_frag(lds, s, wave, 0);
            const u4 blo = *(const u4*)act_frag(lds, s, wave, 1);
            hc = mfma_h(wh, blo, hc);
            hc = mfma_h(wl, bh, hc);
            hc = mfma_h(wh, bh, hc);
        }
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        const int sh = -(sxl[16 * wave + n] + ew);
        if (g == 0) {
            const fx4 bv = *(const fx4*)(lbias + l * 256);
#pragma unroll
            for (int i = 0; i < 4; ++i) comp[(16 * wave + n) * 4 + i] = __builtin_ldexpf(hc[i], sh) + bv[i];
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
    QP_T(q_g);
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
        m = sample_max4(m);
        const int ex = shift_of(m);
        sxl[ls] = ex;
        put_group(lds, 0, wave, gh, z, ex);
        float* sl = a.grad + a.grad_off[l] + ((size_t)wg * 4 + (wave >> 1)) * (size_t)(a.nt[l] * 1024) + (wave & 1) * 512;
        store_slab(sl, gh, z);
        for (int s = 1; s < a.nt[l]; ++s) store_slab(sl + s * 1024, z, z);
        slab_max(a.smax, a.L + l, m);
        bar();
#pragma unroll
        for (int q = 0; q < kGroups; ++q) c.sxr[q] = sxl[16 * q + n];
    }
    QP_ADD(kQpPe, q_g);

    // ---- reverse chain: G_{l-1} = (W_l^T G_l) * 1[A_{l-1} > 0], l = L-1 .. 1, halves as above:
    //   G0: MMA(L-1, H0); per l: A(l): MMA(l, H1) | epilogue(l, H0),
    //   B(l): MMA(next, H0) | epilogue(l, H1), next = l - 1 (or the d_x pass after l = 1)
    QP_T(q_r);
    unsigned long long mw = t0 < a.to_b[a.L - 1] ? mask_w[(size_t)(a.L - 2) * kWaves * 64] : 0ull;
    slot<0, kEpiNone, 1>(c, a.w16 + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], t0, wf, acc0, acc1, none);
    pass_pre(a.w16 + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], t0, wf);
    for (int l = a.L - 1; l >= 1; --l) {
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        float* slab = slab_of(a.grad, a.grad_off[l - 1], a.nt[l - 1]);
        const int nx = l - 1;                         // the next pass: W_{l-1}^T, or W_0^T for d_x
        const bool more = nx >= 1 || a.d_x != nullptr;
        c.mb[0] = (unsigned)mw;
        c.mb[1] = (unsigned)(mw >> 32);
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l - 1], 0, false);
            slot<1, kEpiBwd, 0>(c, a.w16 + a.wb_off[l], a.ks_b[l], a.to_b[l], t0, wf, acc1, acc0, e);
            if (more) pass_pre(a.w16 + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], t0, wf);
            bar();
        }
        {
            // the next layer's mask words, requested before this slot's slab stores
            if (nx >= 1) mw = t0 < a.to_b[nx] ? mask_w[(size_t)(nx - 1) * kWaves * 64] : 0ull;
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l - 1], 1, false);
            if (more) {
                slot<0, kEpiBwd, 1>(c, a.w16 + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], t0, wf, acc0, acc1, e);
                if (nx >= 1) pass_pre(a.w16 + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], t0, wf);
                else pass_pre(a.w16 + a.wb_off[0], a.ks_b[0], a.to_b[0], t0, wf);
            } else {
                epi_alone<kEpiBwd, 1>(c, acc1, e);
            }
            slab_max(a.smax, a.L + l - 1, c.wmax);
            c.wmax = 0.0f;
            bar();
        }
    }
    QP_ADD(kQpMma, q_r);

    // ---- d_layer_input = G_0 W_0^T (ENCODED mode): half 0's MMA ran beside the last epilogue ----
    if (a.d_x) {
        const int to = a.to_b[0];
        slot<1, kEpiNone, 0>(c, a.w16 + a.wb_off[0], a.ks_b[0], to, t0, wf, acc1, acc0, none);
        if (t0 < to) {
            const int ew = __builtin_amdgcn_readlane(wexp_lane, 0);
#pragma unroll
            for (int q = 0; q < kGroups; ++q) {
                const int ls = 16 * q + n, gs = wg * tile_samples + ls;
                if (ls < tile_samples && gs < a.R) {
                    const int sh = -(c.sxr[q] + ew);
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int f = 16 * (t0 + t) + 4 * g + i;
                            const float v = q < 4 ? acc0[q & 3][t][i] : acc1[q & 3][t][i];
                            if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = __builtin_ldexpf(v, sh);
                        }
                }
            }
        }
    }
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
        const char* names[] = {"pe+g", "chains", "composite", "total"};
        fprintf(stderr, "LNERF_PROF kact per-wave cycles:");
        for (int i = 0; i < kQpN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / ((double)p.num_wg * kWaves));
        fprintf(stderr, "\n");
        unsigned long long z[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kact_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
