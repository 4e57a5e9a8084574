// lnerf_kact.hip -- k1 with the activations resident in LDS: the fused PE + MLP + compositing +
// reverse chain for the fp16x3 split, opt-in with LNERF_KACT=1 (k16 stays the default: measured
// 1.49-1.54 vs 1.47-1.50 ms at cfg3; DESIGN.md §3 has where kact's time goes).
//
// Same work and outputs as k16 (lnerf_k16.hip; reference scripts/nerf.py:1-304 and its rev_diff,
// train_nerf.py:325/395), organised around v_mfma_f32_32x32x16_f16 in the transposed form
// Z^T = W^T X^T (M = 32 output features, N = 32 samples, K = 16 input features):
//  * the layer input of all 128 samples (4 groups of 32 = the 4 slab blocks) lives in LDS,
//    already split into its fp16 hi / lo planes in the B-operand layout,
//    act[K16-step 16][group 4][plane 2][lane 64][16 B] (128 KiB), written once per layer by the
//    wave that produced those features;
//  * wave w owns the 32 output features 32w .. 32w + 31 (tile w) of every layer and streams its
//    weight fragments straight from L2 into a register ring (kact_pack's layout);
//  * the accumulator of lane (n, h) holds rows 8 (r >> 2) + 4 h + (r & 3) of sample n; the
//    packing permutes every 16-feature K block by psi (below), so registers 8v .. 8v + 7 are
//    exactly the B fragment of K16-step 2w + v of the next layer: an epilogue splits its own
//    registers and writes lane-linear ds_write_b128;
//  * the 128 samples run as two halves half a layer apart: while the MFMAs of one half stream,
//    the other half's epilogue (unscale, bias, ReLU + mask bits, slab stores, the per-sample
//    exponent exchange through LDS, the split into the next act) is woven between them. A
//    32x32x16 MFMA blocks vector issue for 8 of its 32 cycles (16x16x32: 8 of 16), which leaves
//    the issue slots that epilogue needs.
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
typedef float fx16 __attribute__((ext_vector_type(16)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kGroups = 4;                       // 32-sample groups (slab blocks) per 128-sample tile
constexpr int kTile = comp::kTileSamples;        // 128
constexpr int kActBytes = 16 * kGroups * 2 * 1024;  // 16 K16-steps x 4 groups x 2 planes x 1 KiB
constexpr int kOffComp = kActBytes;
constexpr int kCompBytes = 2688 * 4;             // composite_tile's scratch
constexpr int kOffRay = kOffComp + kCompBytes;
constexpr int kOffPm = kOffRay + kTile * 4;      // per-sample per-wave maxima [128][8] f32
constexpr int kOffSx = kOffPm + kWaves * kTile * 4;   // per-sample exponent shifts [128] i32 (+ spare)
constexpr int kOffBias = kOffSx + 2 * kTile * 4;  // biases [L][256] f32 (copied once)
constexpr int kLdsBytes = kOffBias + kMaxLayers * 256 * 4;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

// Packed K order: element e of lane half h of K16-step u is input feature psi(u, 8 h + e), the
// row the 32x32 accumulator of the producing wave holds in register 8 (u & 1) + e.
__host__ __device__ __forceinline__ int psi(int u, int p) {
    const int h = p >> 3, e = p & 7;
    return 16 * u + 8 * (e >> 2) + 4 * h + (e & 3);
}

struct KaArgs {
    int L;
    int ks_f[kMaxLayers], ks_b[kMaxLayers];   // K16-steps (16 input features) per pass
    int to_f[kMaxLayers], to_b[kMaxLayers];   // 32-wide output tiles per pass
    int nt[kMaxLayers];                       // 32-wide slab tiles of each layer's output
    int kt0;                                  // slab tiles of the layer-0 input X
    int k0;
    const unsigned short* w;                  // kact_pack planes
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];   // u16 offsets
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

// timing experiments only (wrong results; never in the product build): no slab stores, every
// weight load from K16-step 0, no epilogue arithmetic (barriers kept)
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
#define LNERF_KACT_ILV_KS 16  // shortest pass (K16-steps) the epilogue is woven into
#endif
// weight-fragment register ring depth in K16-steps (a K16-step is 6 MFMAs = 192 cycles a wave)
#ifndef LNERF_KACT_WRING
#define LNERF_KACT_WRING 4
#endif
constexpr int kWRing = LNERF_KACT_WRING;
#ifndef LNERF_KACT_PRIO
#define LNERF_KACT_PRIO 0
#endif
static_assert(kWRing >= 2 && kWRing <= 8, "weight ring depth");

__device__ __forceinline__ fx16 mfma32(const u4& a, const u4& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
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
__host__ __device__ __forceinline__ int shift_of(float m) {
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

// max over the two lanes of a sample (n, n + 32): one permlane swap
__device__ __forceinline__ float sample_max2(float m) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return __builtin_fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// act fragment address (bytes): K16-step u, group q, plane p, this lane
__device__ __forceinline__ unsigned char* act_frag(unsigned char* act, int u, int q, int p) {
    return act + ((u * kGroups + q) * 2 + p) * 1024 + (threadIdx.x & 63) * 16;
}

// Split 8 B-operand values with 2^ex and write them as K16-step u's fragments of group q.
__device__ __forceinline__ void put8(unsigned char* act, int u, int q, const float (&x)[8], int ex) {
    const float sc = __builtin_ldexpf(1.0f, ex);
    unsigned h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) split_h2(x[2 * i], x[2 * i + 1], sc, h[i], l[i]);
    *(u4*)act_frag(act, u, q, 0) = u4{h[0], h[1], h[2], h[3]};
    *(u4*)act_frag(act, u, q, 1) = u4{l[0], l[1], l[2], l[3]};
}

// Workgroup barrier for LDS hand-offs only: every LDS access of the wave done (lgkmcnt(0)), then
// s_barrier -- no vmcnt(0): __syncthreads' fence would also wait for the slab stores in flight,
// which no other wave reads in this kernel.
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// the wave's max of a slab -> smax[slab][global wave] (dw16's layer-wide exponent shifts)
__device__ __forceinline__ void slab_max(float* part, int slab, float m) {
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) m = __builtin_fmaxf(m, __shfl_xor(m, d));   // (lanes n, n + 32 agree)
    if ((threadIdx.x & 63) == 0)
        part[(size_t)slab * gridDim.x * kWaves + blockIdx.x * kWaves + (threadIdx.x >> 6)] = m;
}

// ---- weight fragments: wave w's tile of a pass, K16-step u, both fp16 planes, as a buffer:
// fragment (u, t, p) of lane l at byte (u to + t) 2048 + p 1024 + 16 l, so every load shares one
// lane-offset VGPR and the rest is scalar.
struct WFrag {
    u4 hi, lo;
};
struct WSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    int ustride;   // to 2048 (bytes per K16-step)
    int toff;      // w 2048
};
__device__ __forceinline__ WSrc wsrc(const unsigned short* wb, int ks, int to, int t) {
    WSrc w;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(wb), 0, ks * to * 2048, 0x00020000);
    w.ustride = to * 2048;
    w.toff = t * 2048;
    return w;
}
__device__ __forceinline__ void load_w(const WSrc& w, int u, WFrag& f) {
    const int so = (LNERF_KACT_WFIX ? 0 : u) * w.ustride + w.toff;
    const int vo = (int)(threadIdx.x & 63) * 16;
    f.hi = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, vo, so, 0));
    f.lo = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, vo + 1024, so, 0));
}

// The next pass's first kWRing - 1 K16-steps, requested inside the current pass as its ring slots
// free up (the ring continues across the slot boundary when KS % kWRing == 0): the K16-step
// offset goes into voffset, so the buffer bounds check returns zeros instead of reading past the
// pass (or anything, for a wave without a tile in it: num_records 0).
struct WNext {
    __amdgpu_buffer_rsrc_t rsrc;
    int ustride, toff;
};
__device__ __forceinline__ WNext wnext(const unsigned short* wb, int ks, int to) {
    const int t = wave_id();
    WNext w;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(wb), 0, wb && t < to ? ks * to * 2048 : 0,
                                               0x00020000);
    w.ustride = to * 2048;
    w.toff = t * 2048;
    return w;
}
__device__ __forceinline__ void load_next(const WNext& w, int u, WFrag& f) {
    const int vo = (int)(threadIdx.x & 63) * 16 + u * w.ustride + w.toff;
    f.hi = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, vo, 0, 0));
    f.lo = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, vo + 1024, 0, 0));
}

// request the first kWRing - 1 K16-steps of a pass (issued before the previous slot's barrier, so
// their L2 latency hides behind it)
__device__ __forceinline__ void pass_pre(const unsigned short* wb, int ks, int to, WFrag (&w)[kWRing]) {
    const int t = wave_id();
    if (t >= to) return;
    const WSrc src = wsrc(wb, ks, to, t);
#pragma unroll
    for (int u = 0; u + 1 < kWRing; ++u)
        if (u < ks) load_w(src, u, w[u]);
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 at an immediate offset, outside the compiler's waitcnt bookkeeping (the matching
// lgkm_wait below is the only wait, so the next step's reads stay in flight under the MFMAs;
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

// the hi / lo B fragments of K16-step u, group q (J = 4 u + q); offsets past 64 KiB from the
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
// Epilogues. A layer's outputs are finished per sample half (groups 2h, 2h + 1) while the MMA of
// the other half runs: part 1 (unscale, bias, ReLU + mask bits or the backward's mask, slab
// stores, per-sample partial maxima -> pm), one barrier, part 2 (the per-sample shift from the
// eight waves' maxima, split, write K16-steps 2 wave, 2 wave + 1 of the next pass's act). Each
// slice sits between MFMA steps of the pass at compile time.
// ---------------------------------------------------------------------------------------------
enum { kEpiNone = 0, kEpiFwd = 1, kEpiBwd = 2 };
constexpr int kInterleaveKs = LNERF_KACT_ILV_KS;

struct Ctx {
    unsigned char* lds;
    int sxr[kGroups];   // input shift of sample 32 q + n of the pass being finished / next
    float wmax;         // the wave's max over the layer being finished (dw16 slab shifts)
    float gmax;         // running max of the group being finished (part 1)
    unsigned mb[2];     // forward: ReLU mask bits per half; backward: the mask words in use
    fx4 pmv[2];         // part 2's pm read, one group ahead
};

// per-slot epilogue constants: the layer, its weight shift, the slab (hardware-dropped stores
// when disabled: num_records 0, so no branch splits the unrolled pass)
struct Epi {
    const float* bias;   // LDS biases of the wave's tile rows 8 j + 4 h (+ 8 j per unit)
    int ew;
    __amdgpu_buffer_rsrc_t rsrc;
    int voff;            // lane part of a slab address (bytes)
    int so[2];           // block offsets (bytes) of groups 2h, 2h + 1
};

__device__ __forceinline__ Epi make_epi(const float* lbias, int l, int ew, float* slab, int nt, int h) {
    const int lane = threadIdx.x & 63, n = lane & 31, hh = lane >> 5;
    Epi e;
    e.bias = lbias + l * 256 + 32 * wave_id() + 4 * hh;
    e.ew = ew;
    e.rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, slab && !LNERF_KACT_NOSTORE ? 4 * nt * 4096 : 0,
                                               0x00020000);
    e.voff = ((n >> 4) * 512 + 4 * hh * 16 + (n & 15)) * 4;
    e.so[0] = 2 * h * nt * 4096;
    e.so[1] = (2 * h + 1) * nt * 4096;
    return e;
}

// part 1, unit K = 4 ql + j of half H: registers 4 j .. 4 j + 3 (rows 8 j + 4 h + i) of group
// 2 H + ql
template <int KIND, int H, int K>
__device__ __forceinline__ void epi_unit1(Ctx& c, fx16 (&v)[2], const Epi& e) {
    if constexpr (LNERF_KACT_NOEPI == 1 || LNERF_KACT_NOEPI == 3) return;
    constexpr int ql = K >> 2, j = K & 3, q = 2 * H + ql;
    const float sc = __builtin_ldexpf(1.0f, -(c.sxr[q] + e.ew));
    if constexpr (KIND == kEpiFwd) {
        // 2^-(ex + ew) is exact (shifts clamped), so the fma rounds like ldexp(acc) + b; bias
        // after the sum (nerf.py:98,125), ReLU (nerf.py:141-144); the mask bit of value
        // jj = 16 ql + 4 j + i at bit 31 - jj (keep_if's order)
        const fx4 b = *(const fx4*)(e.bias + 8 * j);
        unsigned nib = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x = __builtin_fmaf(v[ql][4 * j + i], sc, b[i]);
            const bool p = x > 0.0f;
            v[ql][4 * j + i] = p ? x : 0.0f;
            nib |= (p ? 1u : 0u) << (3 - i);
        }
        if constexpr (K == 0) c.mb[H] = nib << 28;
        else c.mb[H] |= nib << (28 - 4 * K);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            v[ql][4 * j + i] = keep_if(c.mb[H], 16 * ql + 4 * j + i, v[ql][4 * j + i] * sc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[ql][4 * j + i]), e.rsrc, e.voff,
                                              e.so[ql] + (8 * j + i) * 64, 2);
    float m = j == 0 ? 0.0f : c.gmax;
    m = amax3(m, v[ql][4 * j], v[ql][4 * j + 1]);
    m = amax3(m, v[ql][4 * j + 2], v[ql][4 * j + 3]);
    c.gmax = m;
    if constexpr (j == 3) {
        m = sample_max2(m);
        float* pm = (float*)(c.lds + kOffPm);
        const int n = threadIdx.x & 31;
        pm[(32 * q + n) * kWaves + wave_id()] = m;   // the 2 lanes of a sample write the same value
        c.wmax = __builtin_fmaxf(c.wmax, m);
    }
}

template <int H, int QL>
__device__ __forceinline__ void pm_read(Ctx& c) {
    const int n = threadIdx.x & 31;
    const fx4* p = (const fx4*)(c.lds + kOffPm) + (32 * (2 * H + QL) + n) * 2;
    c.pmv[0] = p[0];
    c.pmv[1] = p[1];
}

// part 2, unit U = 2 ql + v of half H: (v = 0) the shift of group 2 H + ql from the 8 waves'
// maxima, then split registers 8 v .. 8 v + 7 into K16-step 2 wave + v of the next pass
template <int H, int U>
__device__ __forceinline__ void epi_unit2(Ctx& c, fx16 (&v)[2]) {
    if constexpr (LNERF_KACT_NOEPI == 1 || LNERF_KACT_NOEPI == 2) return;
    constexpr int ql = U >> 1, vv = U & 1, q = 2 * H + ql;
    if constexpr (vv == 0) {
        const fx4 a = c.pmv[0], b = c.pmv[1];
        if constexpr (ql == 0) pm_read<H, 1>(c);
        const float m = max3(max3(a[0], a[1], a[2]), max3(a[3], b[0], b[1]), max3(b[2], b[3], 0.0f));
        const int ex = shift_of(m);
        c.sxr[q] = ex;
        const int n = threadIdx.x & 31;
        ((int*)(c.lds + kOffSx))[32 * q + n] = ex;   // (the head reads it; same value from every lane)
    }
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = v[ql][8 * vv + i];
    put8(c.lds, 2 * wave_id() + vv, q, x, c.sxr[q]);
}

// the slice of half H's epilogue that goes with step I of an N-step pass: part 1 units at steps
// (K h) / 8, the barrier at h = N / 2, part 2 units from h + 1 on
template <int KIND, int H, int I, int N, int... K>
__device__ __forceinline__ void epi_part1_at(std::integer_sequence<int, K...>, Ctx& c, fx16 (&v)[2], const Epi& e) {
    constexpr int h = N / 2;
    ((((K * h) / 8 == I) ? (epi_unit1<KIND, H, K>(c, v, e), 0) : 0), ...);
}
template <int H, int I, int N, int... U>
__device__ __forceinline__ void epi_part2_at(std::integer_sequence<int, U...>, Ctx& c, fx16 (&v)[2]) {
    constexpr int h = N / 2;
    (((h + 1 + (U * (h - 1)) / 4 == I) ? (epi_unit2<H, U>(c, v), 0) : 0), ...);
}

template <int KIND, int H, int I, int N>
__device__ __forceinline__ void epi_slice(Ctx& c, fx16 (&v)[2], const Epi& e) {
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
__device__ __forceinline__ void epi_alone(Ctx& c, fx16 (&v)[2], const Epi& e) {
    epi_part1_at<KIND, H, 0, 2>(std::make_integer_sequence<int, 8>{}, c, v, e);
    bar();
    pm_read<H, 0>(c);
    epi_unit2<H, 0>(c, v);
    epi_unit2<H, 1>(c, v);
    epi_unit2<H, 2>(c, v);
    epi_unit2<H, 3>(c, v);
}

// ---- one slot: the MMA of half HM over KS K16-steps (acc am) with half HE's epilogue (acc ae)
// woven in. Step I = 2 u + ql: prefetch the weights of K16-step u + kWRing - 1 (at ql = 0), the
// epilogue slice, the next step's B fragments, wait for this step's, 3 MFMAs (small terms first).
template <int KS, int HM, int KIND, int HE, int I>
__device__ __forceinline__ void slot_step(Ctx& c, unsigned b0, unsigned b1, const WSrc& ws, const WNext& wn,
                                          WFrag (&w)[kWRing], u4 (&bh)[2], u4 (&bl)[2], fx16 (&am)[2], fx16 (&ae)[2],
                                          const Epi& e) {
    constexpr int N = KS * 2, u = I / 2, ql = I % 2;
    constexpr int Jn = 4 * ((I + 1) / 2) + 2 * HM + (I + 1) % 2;
    if constexpr (ql == 0 && u + kWRing - 1 < KS) load_w(ws, u + kWRing - 1, w[(u + kWRing - 1) % kWRing]);
    if constexpr (ql == 0 && u + kWRing - 1 >= KS && KS % kWRing == 0)
        load_next(wn, u + kWRing - 1 - KS, w[(u + kWRing - 1) % kWRing]);
    epi_slice<KIND, HE, I, N>(c, ae, e);
    if constexpr (I + 1 < N) {
        read_b<Jn>(b0, b1, bh[(I + 1) & 1], bl[(I + 1) & 1]);
        lgkm_wait<2>(bh[I & 1], bl[I & 1]);
    } else {
        lgkm_wait<0>(bh[I & 1], bl[I & 1]);
    }
    const WFrag& f = w[u % kWRing];
    fx16 x = am[ql];
    x = mfma32(f.hi, bl[I & 1], x);
    x = mfma32(f.lo, bh[I & 1], x);
    x = mfma32(f.hi, bh[I & 1], x);
    am[ql] = x;
}

template <int KS, int HM, int KIND, int HE, int... I>
__device__ __forceinline__ void slot_steps(std::integer_sequence<int, I...>, Ctx& c, unsigned b0, unsigned b1,
                                           const WSrc& ws, const WNext& wn, WFrag (&w)[kWRing], u4 (&bh)[2],
                                           u4 (&bl)[2], fx16 (&am)[2], fx16 (&ae)[2], const Epi& e) {
    (slot_step<KS, HM, KIND, HE, I>(c, b0, b1, ws, wn, w, bh, bl, am, ae, e), ...);
}

template <int KS, int HM, int KIND, int HE>
__device__ __forceinline__ bool slot_t(Ctx& c, const WSrc& ws, const WNext& wn, WFrag (&w)[kWRing], fx16 (&am)[2],
                                       fx16 (&ae)[2], const Epi& e) {
    const unsigned b0 = lds_addr(c.lds) + (threadIdx.x & 63) * 16, b1 = b0 + 65536;
    u4 bh[2], bl[2];
    read_b<2 * HM>(b0, b1, bh[0], bl[0]);
    slot_steps<KS, HM, KIND, HE>(std::make_integer_sequence<int, KS * 2>{}, c, b0, b1, ws, wn, w, bh, bl, am, ae, e);
    return KS % kWRing == 0;   // the next pass's ring head is in flight
}

__device__ __forceinline__ void zero2(fx16 (&a)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) a[q][r] = 0.0f;
}

// One slot: MMA of half HM (layer pass wb / ks / to) beside half HE's epilogue of kind KIND,
// requesting the head of the next pass (nwb / nks / nto; nwb null: none) through the ring; the
// caller issues pass_pre itself when this returns false. A wave without an output tile in the
// pass runs the epilogue alone (same single barrier).
template <int HM, int KIND, int HE>
__device__ __forceinline__ bool slot(Ctx& c, const unsigned short* wb, int ks, int to, const unsigned short* nwb,
                                     int nks, int nto, WFrag (&w)[kWRing], fx16 (&am)[2], fx16 (&ae)[2],
                                     const Epi& e) {
    zero2(am);
    const int t = wave_id();
    if (t >= to) {
        if constexpr (KIND != kEpiNone) epi_alone<KIND, HE>(c, ae, e);
        return false;
    }
    const WSrc ws = wsrc(wb, ks, to, t);
    const WNext wn = wnext(nwb, nks, nto);
    // the epilogue is woven into full-depth passes only; shorter passes run it first, whole, then
    // the bare MMA (too few MFMA gaps to hide it, and crammed slices raise the register peak)
    if constexpr (KIND != kEpiNone) {
        if (ks >= kInterleaveKs) return slot_t<16, HM, KIND, HE>(c, ws, wn, w, am, ae, e);
        epi_alone<KIND, HE>(c, ae, e);
    }
#define LNERF_KACT_SLOT(K) \
    case K: return slot_t<K, HM, kEpiNone, HE>(c, ws, wn, w, am, ae, e);
    switch (ks) {
        LNERF_KACT_SLOT(1)
        LNERF_KACT_SLOT(2)
        LNERF_KACT_SLOT(3)
        LNERF_KACT_SLOT(4)
        LNERF_KACT_SLOT(5)
        LNERF_KACT_SLOT(6)
        LNERF_KACT_SLOT(7)
        LNERF_KACT_SLOT(8)
        LNERF_KACT_SLOT(9)
        LNERF_KACT_SLOT(10)
        LNERF_KACT_SLOT(11)
        LNERF_KACT_SLOT(12)
        LNERF_KACT_SLOT(13)
        LNERF_KACT_SLOT(14)
        LNERF_KACT_SLOT(15)
        default: return slot_t<16, HM, kEpiNone, HE>(c, ws, wn, w, am, ae, e);
    }
#undef LNERF_KACT_SLOT
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
    float* pm = (float*)(lds + kOffPm);

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), n = lane & 31, hh = lane >> 5;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
    const bool st = a.want_grad != 0;
    // per-layer weight exponent shifts in lane l
    int wexp_lane = 0;
    if (lane < a.L) wexp_lane = shift_of(__int_as_float(a.wexp[lane]));
    // the biases into LDS (read by every epilogue; visible after the PE stage's barrier)
    float* lbias = (float*)(lds + kOffBias);
    for (int i = tid; i < a.L * 64; i += kThreads) ((fx4*)lbias)[i] = ((const fx4*)a.b16)[i];
#if LNERF_KACT_PRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);   // the later-dispatched half wins arbitration
#endif
    Ctx c;
    c.lds = lds;
    c.wmax = 0.0f;
    c.gmax = 0.0f;
    c.mb[0] = c.mb[1] = 0u;
    fx16 acc0[2], acc1[2];   // sample halves: groups 0, 1 and 2, 3
    WFrag wf[kWRing];        // the weight-fragment ring (K16-steps u % kWRing)
    const Epi none{};
    // slab base of the wave's 32-feature tile in layer l's slab at `base` (nullptr: no slab)
    auto slab_of = [&](float* base, size_t off, int nt) -> float* {
        return st && wave < nt ? base + off + (size_t)wg * 4 * nt * 1024 + (size_t)wave * 1024 : nullptr;
    };

    // ---- layer-0 input (pos_encoding.py:54-66): wave w encodes group q = w >> 1, the K16-steps
    // of parity w & 1 (all slab rows of X, the padding included), X slab, act
    pass_pre(a.w + a.wf_off[0], a.ks_f[0], a.to_f[0], wf);
    QP_T(q_pe);
    {
        const int q = wave >> 1, ls = 32 * q + n, gs = wg * tile_samples + ls;
        const bool valid = ls < tile_samples && gs < a.R;
        const int nu = 2 * a.kt0;   // K16-steps covering the X slab tiles
        float xv[4][8];
        float m = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = 2 * k + (wave & 1);
            if (u < nu) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    xv[k][e] = comp::input_feature(a, gs, valid, psi(u, 8 * hh + e));
                    m = __builtin_fmaxf(m, __builtin_fabsf(xv[k][e]));
                }
            }
        }
        m = sample_max2(m);
        pm[ls * kWaves + (wave & 1)] = m;
        if (st) {
            float* xs = a.act + a.x_off + ((size_t)wg * 4 + q) * (size_t)(a.kt0 * 1024) + (n >> 4) * 512 + (n & 15);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int u = 2 * k + (wave & 1);
                if (u < nu) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int f = psi(u, 8 * hh + e);
                        __builtin_nontemporal_store(xv[k][e], xs + (f >> 5) * 1024 + (f & 31) * 16);
                    }
                }
            }
            slab_max(a.smax, 0, m);
        }
        bar();
        const int ex = shift_of(__builtin_fmaxf(pm[ls * kWaves], pm[ls * kWaves + 1]));
        sxl[ls] = ex;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = 2 * k + (wave & 1);
            if (u < nu) put8(lds, u, q, xv[k], ex);
        }
        bar();
#pragma unroll
        for (int g = 0; g < kGroups; ++g) c.sxr[g] = sxl[32 * g + n];
    }
    QP_ADD(kQpPe, q_pe);

    unsigned long long* mask_w = a.mask_g + ((size_t)wg * (a.L - 1) * kWaves + wave) * 64 + lane;

    // ---- forward hidden layers, the two sample halves half a layer apart:
    //   F0: MMA(0, H0); then per layer l: A(l): MMA(l, H1) | epilogue(l, H0),
    //   B(l): MMA(l + 1, H0) | epilogue(l, H1)  (the last layer's B: the epilogue alone)
    QP_T(q_m);
    if (!slot<0, kEpiNone, 1>(c, a.w + a.wf_off[0], a.ks_f[0], a.to_f[0], a.w + a.wf_off[0], a.ks_f[0], a.to_f[0], wf,
                              acc0, acc1, none))
        pass_pre(a.w + a.wf_off[0], a.ks_f[0], a.to_f[0], wf);
    for (int l = 0; l + 1 < a.L; ++l) {
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        float* slab = slab_of(a.act, a.act_off[l], a.nt[l]);
        const bool more = l + 2 < a.L;   // another hidden pass follows
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l], 0);
            const unsigned short* nwb = more ? a.w + a.wf_off[l + 1] : nullptr;
            if (!slot<1, kEpiFwd, 0>(c, a.w + a.wf_off[l], a.ks_f[l], a.to_f[l], nwb, a.ks_f[l + 1], a.to_f[l + 1], wf,
                                     acc1, acc0, e) && more)
                pass_pre(a.w + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], wf);
            bar();
        }
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l], 1);
            if (more) {
                if (!slot<0, kEpiFwd, 1>(c, a.w + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], a.w + a.wf_off[l + 1],
                                         a.ks_f[l + 1], a.to_f[l + 1], wf, acc0, acc1, e))
                    pass_pre(a.w + a.wf_off[l + 1], a.ks_f[l + 1], a.to_f[l + 1], wf);
            } else {
                epi_alone<kEpiFwd, 1>(c, acc1, e);
            }
            if (st && wave < a.to_f[l])
                mask_w[(size_t)l * kWaves * 64] = (unsigned long long)c.mb[0] | ((unsigned long long)c.mb[1] << 32);
            if (st) slab_max(a.smax, l + 1, c.wmax);   // every wave writes its entry (0 past the layer)
            c.wmax = 0.0f;
            bar();
        }
    }
    QP_ADD(kQpMma, q_m);

    // ---- head (nerf.py:150-167 pre-activations): wave w < 4 computes group q = w, all K16-steps;
    // rows 0..3 (the outputs) are registers 0..3 of lanes 0..31
    if (wave < kGroups) {
        const int l = a.L - 1, ks = a.ks_f[l];
        const WSrc ws = wsrc(a.w + a.wf_off[l], ks, 1, 0);
        fx16 hc;
#pragma unroll
        for (int r = 0; r < 16; ++r) hc[r] = 0.0f;
        for (int u = 0; u < ks; ++u) {
            WFrag f;
            load_w(ws, u, f);
            const u4 bh = *(const u4*)act_frag(lds, u, wave, 0);
            const u4 blo = *(const u4*)act_frag(lds, u, wave, 1);
            hc = mfma32(f.hi, blo, hc);
            hc = mfma32(f.lo, bh, hc);
            hc = mfma32(f.hi, bh, hc);
        }
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        const int ls = 32 * wave + n;
        const int sh = -(sxl[ls] + ew);
        if (hh == 0) {
            const fx4 bv = *(const fx4*)(lbias + l * 256);
#pragma unroll
            for (int i = 0; i < 4; ++i) comp[ls * 4 + i] = __builtin_ldexpf(hc[i], sh) + bv[i];
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

    // ---- G_{L-1} (head gradients: features 0..3 = elements 0..3 of lane half 0, K16-step 0):
    // the even wave of each group writes act and the slab tile (rows 4.. zero)
    pass_pre(a.w + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], wf);
    QP_T(q_g);
    {
        const int l = a.L - 1, q = wave >> 1, ls = 32 * q + n;
        float gv[8];
        float m = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int f = psi(0, 8 * hh + e);
            gv[e] = (f < 4 && ls < tile_samples) ? comp[512 + ls * 4 + f] : 0.0f;
            m = __builtin_fmaxf(m, __builtin_fabsf(gv[e]));
        }
        m = sample_max2(m);
        if ((wave & 1) == 0) {
            const int ex = shift_of(m);
            sxl[ls] = ex;
            put8(lds, 0, q, gv, ex);
            float* sl = a.grad + a.grad_off[l] + ((size_t)wg * 4 + q) * (size_t)(a.nt[l] * 1024) + (n >> 4) * 512 + (n & 15);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 16 * hh + r;
                const float g = (row < 4 && ls < tile_samples) ? comp[512 + ls * 4 + (row & 3)] : 0.0f;
                __builtin_nontemporal_store(g, sl + row * 16);
            }
            for (int t = 1; t < a.nt[l]; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) __builtin_nontemporal_store(0.0f, sl + t * 1024 + (16 * hh + r) * 16);
        }
        slab_max(a.smax, a.L + l, (wave & 1) == 0 ? m : 0.0f);
        bar();
#pragma unroll
        for (int g = 0; g < kGroups; ++g) c.sxr[g] = sxl[32 * g + n];
    }
    QP_ADD(kQpPe, q_g);

    // ---- reverse chain: G_{l-1} = (W_l^T G_l) * 1[A_{l-1} > 0], l = L-1 .. 1, halves as above:
    //   G0: MMA(L-1, H0); per l: A(l): MMA(l, H1) | epilogue(l, H0),
    //   B(l): MMA(next, H0) | epilogue(l, H1), next = l - 1 (or the d_x pass after l = 1)
    QP_T(q_r);
    unsigned long long mw = wave < a.to_b[a.L - 1] ? mask_w[(size_t)(a.L - 2) * kWaves * 64] : 0ull;
    if (!slot<0, kEpiNone, 1>(c, a.w + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], a.w + a.wb_off[a.L - 1],
                              a.ks_b[a.L - 1], a.to_b[a.L - 1], wf, acc0, acc1, none))
        pass_pre(a.w + a.wb_off[a.L - 1], a.ks_b[a.L - 1], a.to_b[a.L - 1], wf);
    for (int l = a.L - 1; l >= 1; --l) {
        const int ew = __builtin_amdgcn_readlane(wexp_lane, l);
        float* slab = slab_of(a.grad, a.grad_off[l - 1], a.nt[l - 1]);
        const int nx = l - 1;                         // the next pass: W_{l-1}^T, or W_0^T for d_x
        const bool more = nx >= 1 || a.d_x != nullptr;
        c.mb[0] = (unsigned)mw;
        c.mb[1] = (unsigned)(mw >> 32);
        {
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l - 1], 0);
            const unsigned short* nwb = more ? a.w + a.wb_off[nx] : nullptr;
            if (!slot<1, kEpiBwd, 0>(c, a.w + a.wb_off[l], a.ks_b[l], a.to_b[l], nwb, a.ks_b[nx], a.to_b[nx], wf, acc1,
                                     acc0, e) && more)
                pass_pre(a.w + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], wf);
            bar();
        }
        {
            // the next layer's mask words, requested before this slot's slab stores
            if (nx >= 1) mw = wave < a.to_b[nx] ? mask_w[(size_t)(nx - 1) * kWaves * 64] : 0ull;
            const Epi e = make_epi(lbias, l, ew, slab, a.nt[l - 1], 1);
            if (more) {
                if (!slot<0, kEpiBwd, 1>(c, a.w + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], a.w + a.wb_off[nx], a.ks_b[nx],
                                         a.to_b[nx], wf, acc0, acc1, e))
                    pass_pre(a.w + a.wb_off[nx], a.ks_b[nx], a.to_b[nx], wf);
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
        (void)slot<1, kEpiNone, 0>(c, a.w + a.wb_off[0], a.ks_b[0], to, nullptr, 0, 0, wf, acc1, acc0, none);
        if (wave < to) {
            const int ew = __builtin_amdgcn_readlane(wexp_lane, 0);
#pragma unroll
            for (int g = 0; g < kGroups; ++g) {
                const int ls = 32 * g + n, gs = wg * tile_samples + ls;
                if (ls < tile_samples && gs < a.R) {
                    const int sh = -(c.sxr[g] + ew);
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int f = 32 * wave + 8 * (r >> 2) + 4 * hh + (r & 3);
                        const float v = g < 2 ? acc0[g & 1][r] : acc1[g & 1][r];
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

// ---- packing (kact_pack): per-layer max|W| bits, then the fp16 hi / lo planes in the fragment
// layout above, both passes, and the zero-padded biases
struct PackArgs {
    int L;
    int k[kMaxLayers], n[kMaxLayers];
    int ks_f[kMaxLayers], ks_b[kMaxLayers], to_f[kMaxLayers], to_b[kMaxLayers];
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];
    int w_k, w_n;
    const float* W;
    const float* B;
    unsigned short* w;
    float* b16;
    int* wexp;
    int* wpart;  // [L][kWmaxParts] partial max|W| bits
};

// planes = 2: max|W_l| as the bits of a non-negative float (integer order = float order), one
// partial per block, grid (kWmaxParts, L): plain stores, no zeroing launch and no atomics; the
// packing kernel folds the layer's kWmaxParts partials itself.
__global__ void __launch_bounds__(256) kact_wmax_kernel(PackArgs a) {
    const int l = blockIdx.y;
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    float m = 0.0f;
    for (int k = blockIdx.x; k < K; k += gridDim.x)
        for (int j = threadIdx.x; j < N; j += blockDim.x) m = fmaxf(m, fabsf(W[(size_t)k * a.w_n + j]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)   // fmaxf drops NaNs: the max is finite, +inf or 0
        a.wpart[l * kWmaxParts + blockIdx.x] =
            __float_as_int(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// the layer's max|W| bits from its kWmaxParts partials (uniform per block); block (0, l) also
// publishes them in wexp[l] for k1
__device__ __forceinline__ int layer_wmax(PackArgs& a, int l) {
    int mb = 0;
    for (int i = 0; i < kWmaxParts; ++i) mb = max(mb, a.wpart[l * kWmaxParts + i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.wexp[l] = mb;
    return mb;
}

// fragment (u, t, plane) lane ln element e: row o = 32 t + (ln & 31), K index psi(u, 8 (ln >> 5) + e);
// forward W[k = psi][o], backward W[o][psi]
// every layer in one launch: grid (blocks of the largest layer, L)
__global__ void kact_pack_kernel(PackArgs a) {
    const int l = blockIdx.y;
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const int ws = shift_of(__int_as_float(layer_wmax(a, l)));
    const size_t nf = (size_t)a.ks_f[l] * a.to_f[l] * 512, nb = (size_t)a.ks_b[l] * a.to_b[l] * 512;
    for (size_t x0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x0 < nf + nb + 256;
         x0 += (size_t)gridDim.x * blockDim.x) {
        if (x0 >= nf + nb) {
            const int f = (int)(x0 - nf - nb);
            a.b16[(size_t)l * 256 + f] = f < N ? a.B[(size_t)l * a.w_n + f] : 0.0f;
            continue;
        }
        const bool fwd = x0 < nf;
        size_t x = fwd ? x0 : x0 - nf;
        const int to = fwd ? a.to_f[l] : a.to_b[l];
        const int e = x & 7;
        x >>= 3;
        const int ln = x & 63;
        x >>= 6;
        const int t = (int)(x % to);
        const int u = (int)(x / to);
        const int o = 32 * t + (ln & 31), f = psi(u, 8 * (ln >> 5) + e);
        const int kk = fwd ? f : o, jj = fwd ? o : f;
        const float w = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        const float xs = __builtin_ldexpf(w, ws);
        const _Float16 h = (_Float16)xs;
        const _Float16 lo = (_Float16)(xs - (float)h);
        unsigned short* dst = a.w + (fwd ? a.wf_off[l] : a.wb_off[l]) + ((size_t)(u * to + t) * 2) * 512 + ln * 8 + e;
        dst[0] = __builtin_bit_cast(unsigned short, h);
        dst[512] = __builtin_bit_cast(unsigned short, lo);
    }
}

// the pass shapes and packed offsets (u16) of every layer; returns the packed size (u16)
struct KactLayout {
    int ks_f[kMaxLayers], ks_b[kMaxLayers], to_f[kMaxLayers], to_b[kMaxLayers];
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];
    size_t total;
};
KactLayout kact_layout(const FusedPlan& p) {
    KactLayout y{};
    size_t off = 0;
    for (int l = 0; l < p.L; ++l) {
        y.ks_f[l] = (p.k[l] + 15) / 16;
        y.ks_b[l] = (p.n[l] + 15) / 16;
        y.to_f[l] = l + 1 < p.L ? (p.n[l] + 31) / 32 : 1;
        y.to_b[l] = (p.k[l] + 31) / 32;
        y.wf_off[l] = off;
        off += (size_t)y.ks_f[l] * y.to_f[l] * 1024;
        y.wb_off[l] = off;
        off += (size_t)y.ks_b[l] * y.to_b[l] * 1024;
    }
    y.total = off;
    return y;
}

}  // namespace

bool kact_supported(const FusedPlan& p) {
    if (p.x6 != 2) return false;                 // the fp16x3 planes only
    if (p.n[p.L - 1] > 4) return false;          // head: the compositing's 4 outputs
    if (p.L < 2) return false;
    if (p.kt[0] > 4) return false;               // the encoding stage's 8 K16-steps (k0 <= 128)
    for (int l = 0; l < p.L; ++l)
        if (p.k[l] > 256 || p.n[l] > 256) return false;
    // the packed planes reuse k16's w16 region (3 planes per k16 fragment)
    size_t w16_end = 0;
    for (int l = 0; l < p.L; ++l) {
        const size_t ef = p.w16f_off[l] + (size_t)p.ks16_f[l] * p.to16_f[l] * 3 * 512;
        const size_t eb = p.w16b_off[l] + (size_t)p.ks16_b[l] * p.to16_b[l] * 3 * 512;
        w16_end = ef > w16_end ? ef : w16_end;
        w16_end = eb > w16_end ? eb : w16_end;
    }
    return kact_layout(p).total <= w16_end;
}

void kact_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s) {
    const KactLayout y = kact_layout(p);
    PackArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.k[l] = p.k[l];
        a.n[l] = p.n[l];
        a.ks_f[l] = y.ks_f[l];
        a.ks_b[l] = y.ks_b[l];
        a.to_f[l] = y.to_f[l];
        a.to_b[l] = y.to_b[l];
        a.wf_off[l] = y.wf_off[l];
        a.wb_off[l] = y.wb_off[l];
    }
    a.w_k = p.w_k;
    a.w_n = p.w_n;
    a.W = ws;
    a.B = bs;
    a.w = p.w16;
    a.b16 = p.b16;
    a.wexp = p.wexp16;
    a.wpart = p.wmax_part;
    kact_wmax_kernel<<<dim3(kWmaxParts, p.L), 256, 0, s>>>(a);
    size_t nmax = 0;
    for (int l = 0; l < p.L; ++l) {
        const size_t nel = ((size_t)y.ks_f[l] * y.to_f[l] + (size_t)y.ks_b[l] * y.to_b[l]) * 512 + 256;
        nmax = nel > nmax ? nel : nmax;
    }
    kact_pack_kernel<<<dim3((unsigned)((nmax + 255) / 256), p.L), 256, 0, s>>>(a);
}

void kact_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                 bool want_grad, hipStream_t s) {
    const KactLayout y = kact_layout(p);
    KaArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.ks_f[l] = y.ks_f[l];
        a.ks_b[l] = y.ks_b[l];
        a.to_f[l] = y.to_f[l];
        a.to_b[l] = y.to_b[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = y.wf_off[l];
        a.wb_off[l] = y.wb_off[l];
        a.act_off[l] = p.act_off[l];
        a.grad_off[l] = p.grad_off[l];
    }
    a.kt0 = p.kt[0];
    a.k0 = p.k[0];
    a.w = p.w16;
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
