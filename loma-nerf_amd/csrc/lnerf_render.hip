// lnerf_render.hip -- kr: the forward-only eval render (config 5) on plain bf16 MFMA, with every
// weight fragment read from LDS feeding two MFMAs.
//
// Reference: the eval render of train_nerf.py:558-712 -- get_rays, sampling (:289-306), the
// positional encoding (pos_encoding.py:38-69), the MLP forward (scripts/nerf.py:67-170) and the
// compositing (nerf.py:176-302), forward only, at the config-5 inference precision (bf16 operands,
// fp32 accumulate).
//
// Why a kernel of its own: k16 (lnerf_k16.hip) keeps 16 samples per wave and fp32 activations
// for the training slabs and operand splits; forward-only in one plane, each 16-B fragment read
// there feeds one 16-cycle MFMA, so the LDS reads (4 array cycles per wave instruction, 256 B/clk
// per CU) run as long as the matrix core (MI355X_MICROARCH.md §LDS). Here
//  * a wave owns 32 samples as two 16-sample groups, and every fragment it reads feeds the two
//    groups' MFMAs: half the LDS bytes per MFMA;
//  * the activations live only as the next layer's bf16 B operands (8 k-steps x 4 registers per
//    group), written once per layer by the epilogue in k16's phi order (no data movement between
//    layers), so the two groups' accumulators (128 registers) fit beside them at two waves per
//    SIMD;
//  * one 512-thread workgroup per 256-sample tile of whole rays; the weight stream, its packing
//    (k16_pack with one plane), the LDS-DMA ring and the chunk table are k16's.
#include "lnerf_composite.h"
#include "lnerf_internal.h"

#include <stddef.h>
#include <stdio.h>

#include <utility>

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

constexpr int kWaves = 8;
constexpr int kGroups = 2;                       // 16-sample groups per wave
constexpr int kTile = kWaves * kGroups * 16;     // 256 samples per workgroup
constexpr int kMaxT = 16;                        // 16-wide output tiles of a 256-wide layer
constexpr int kKC = 2;                           // k-steps per chunk
constexpr int kSlot = kKC * kMaxT * 1024;        // one chunk: 2 k-steps x 16 tiles x 1 KiB
constexpr int kMaxChunks = kMaxLayers * 4 + 1;   // <= 4 chunks per forward pass + the end marker
// Staggered wave pairs: waves 4-7 (each the SIMD partner of wave w - 4) meet each chunk's barrier
// half a k-step later than waves 0-3 (in the middle of the chunk's last k-step), so the two waves of
// a SIMD run their chunk prologues and layer epilogues (bias + ReLU + bf16 conversion of 128 values)
// beside the partner's MFMAs instead of in lockstep with them (MI355X_MICROARCH.md, two waves per
// SIMD, item 9). The late waves still read chunk c - 1 while chunk c + 1 lands: three ring slots.
// (Round 5: 63.4 -> 61.6 ms per frame against the unstaggered 2-slot ring, which is gone.)
constexpr int kSlots = 3;
// The head's weights (<= 8 k-steps x one 16-wide tile, 8 KiB) and biases stay resident in LDS,
// loaded at the start beside chunk 0: the head pass runs with no DMA and no barrier, and chunk 0 is
// issued before the encoding (whose scratch sits in ring slot 2) so it lands while the encoding
// runs (round 5: with the in-wave compositing, 55.5 -> 53.7 ms per frame).
constexpr int kOffComp = kSlots * kSlot;         // the ring
constexpr int kOffRay = kOffComp + comp::kCompFloats * kTile * 4;
constexpr int kOffBias = kOffRay + kTile * 4;    // a 3-slot ring of layer biases
constexpr int kOffHead = kOffBias + 3 * 256 * 4; // the resident head: 8 KiB of weights, 1 KiB of biases
constexpr int kLds = kOffHead + 9 * 1024;
static_assert(kLds <= 160 * 1024, "LDS budget");
constexpr int kPePerWave = 16 * 65 * 4;          // the encoding scratch of one wave (16 samples)
// the encoding scratch: from ring slot 2 on into the idle compositing scratch (chunk 0 lands in
// slot 0 meanwhile; slot 2 is first written by chunk 2's DMA, issued after the first chunk barrier)
constexpr int kOffPe = 2 * kSlot;
static_assert(kOffPe + kWaves * kPePerWave <= kOffRay, "encoding scratch");

struct KrArgs {
    int L;
    int ks[kMaxLayers];        // forward k-steps (32 input features) per layer
    int k0;
    const unsigned short* w16;
    const float* b16;          // [L][256] zero-padded biases
    // the chunk stream: per chunk {u16 offset in w16, (bytes / 1024) | (bias layer + 1) << 16},
    // zero past the end; read with scalar loads from the kernel-argument segment
    unsigned chunk_tab[2 * kMaxChunks];
    unsigned head_off;         // u16 offset of the head's packed weights in w16 (not in the chunk
                               // stream: resident)
    int rays, S, rpw, R, input_mode, F;
    float near_t, far_t;
    const float* x;
    const float* dists;
    const float* target;
    float* loss_part;
    float* acc_color;
    // composite_tile's reverse-pass fields (unused: forward only)
    float* d_dists;
    float* d_target;
    float seed;
};

// ---- optional in-kernel phase timing (-DLNERF_PROF=1, `make prof`, never in the product build):
// per-wave s_memtime deltas, lane 0 accumulating in LDS, summed into g_kr_prof at the end
#ifndef LNERF_PROF
#define LNERF_PROF 0
#endif
#if LNERF_PROF
enum { kRpPE, kRpDma0, kRpPass, kRpBar, kRpEpi, kRpHead, kRpComp, kRpTotal, kRpReal, kRpLoop, kRpVm, kRpN };
__device__ unsigned long long g_kr_prof[16];
__device__ __forceinline__ unsigned long long* kr_prof_slots() {
    __shared__ unsigned long long sl[kWaves][16];
    return &sl[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0];
}
// scheduling barriers keep the compiler from moving work across a timer read
#define KR_PROF_T(v)                     \
    __builtin_amdgcn_sched_barrier(0);   \
    const unsigned long long v = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0)
#define KR_PROF_ADD(cat, t0)                                                                   \
    do {                                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                            \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        if ((threadIdx.x & 63) == 0) kr_prof_slots()[cat] += t1_ - (t0);                        \
    } while (0)
#else
#define KR_PROF_T(v)
#define KR_PROF_ADD(cat, t0)
#endif

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// One LDS-DMA wave instruction from inline asm, M0 written in the same statement (no register
// destination; completion counted by the chunk barrier's vmcnt). As lnerf_k16.hip glds16.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc),
                 "s"(__builtin_amdgcn_readfirstlane(lds)));
}

// feature of k-step s in element j of lane group g (k16's phi: the accumulator layout of the
// previous layer is the B operand as it stands)
__host__ __device__ __forceinline__ int phi(int s, int g, int j) {
    return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
}

struct Chunk {
    const char* src;   // nullptr: past the last chunk
    int bytes;
    int bias;          // layer whose biases ride with this chunk, -1: none
};

__device__ __forceinline__ Chunk chunk_at(const KrArgs& a, int ci) {
    const __attribute__((address_space(4))) unsigned* t =
        (const __attribute__((address_space(4))) unsigned*)((const __attribute__((address_space(4))) char*)
                                                                __builtin_amdgcn_kernarg_segment_ptr() +
                                                            offsetof(KrArgs, chunk_tab)) + 2 * ci;
    const unsigned off = t[0], e = t[1];
    const int bytes = (int)(e & 0xFFFFu) * 1024;
    return Chunk{bytes ? (const char*)(a.w16 + off) : nullptr, bytes, (int)(e >> 16) - 1};
}

// This wave's pieces of a chunk (1 KiB each, at byte wave * 1 KiB + p * 8 KiB), plus the bias
// piece from the last wave.
struct Job {
    const char* src = nullptr;
    unsigned char* dst = nullptr;
    int n = 0;
};

__device__ __forceinline__ Job chunk_job(const KrArgs& a, int ci, unsigned char* ring, float* bias_ring) {
    const Chunk c = chunk_at(a, ci);
    const int wave = wave_id(), lane = threadIdx.x & 63;
    Job j;
    const int woff = wave * 1024;
    j.n = (c.src && woff < c.bytes) ? (c.bytes - woff + kWaves * 1024 - 1) / (kWaves * 1024) : 0;
    j.src = c.src + woff + lane * 16;
    j.dst = ring + (ci % kSlots) * kSlot + woff;
    if (c.bias >= 0 && wave == kWaves - 1)
        glds16(a.b16 + (size_t)c.bias * 256 + lane * 4, lds_addr(bias_ring + (c.bias % 3) * 256));
    return j;
}

template <int P>
__device__ __forceinline__ void job_piece(const Job& j) {
    if (P < j.n) glds16(j.src + P * (kWaves * 1024), lds_addr(j.dst + P * (kWaves * 1024)));
}

// the chunk the next k-step reads has landed (every DMA of this wave: vmcnt(0); the pass issues
// no other vector-memory operation), this wave's LDS reads of the slot the next DMA overwrites have
// returned (lgkmcnt(0)), then the workgroup barrier
__device__ __forceinline__ void chunk_barrier() {
    KR_PROF_T(t0);
#if LNERF_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    KR_PROF_ADD(kRpVm, t0);
#endif
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    KR_PROF_ADD(kRpBar, t0);
}

__device__ __forceinline__ fx4 mfma(const bf8& a, const bf8& b, fx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

#ifndef LNERF_KR_DIST
#define LNERF_KR_DIST 2
#endif
constexpr int kDist = LNERF_KR_DIST;   // fragments read ahead of the one the MFMAs consume
// LNERF_KR_SCHED: a scheduling barrier after each tile's fragment read and DMA issue keeps the read
// of tile O + kDist ahead of tile O's MFMAs; without it the machine scheduler sinks every read
// next to its first MFMA (an LDS round trip exposed every two tiles), as in k1
#ifndef LNERF_KR_SCHED
#define LNERF_KR_SCHED 1
#endif

// Output tile O of k-step S: read tile O + kDist's fragment, issue this tile's DMA piece (pieces
// spread one per NTO / pieces tiles), the two groups' MFMAs on tile O's fragment.
template <int NTO, int O>
__device__ __forceinline__ void kr_tile(const unsigned char* base, bf8 (&w)[kDist + 1], const bf8& b0, const bf8& b1,
                                        fx4 (&acc)[kGroups][kMaxT], const Job& job) {
    if constexpr (O + kDist < NTO) w[(O + kDist) % (kDist + 1)] = *(const bf8*)(base + (O + kDist) * 1024);
    // 4 pieces per wave for a whole 16-tile chunk: one every 4 tiles; NTO < 16: all at tile 0
    if constexpr (NTO >= 4) {
        if constexpr (O % (NTO / 4) == 0) job_piece<O / (NTO / 4)>(job);
    } else if constexpr (O == 0) {
        job_piece<0>(job);
        job_piece<1>(job);
        job_piece<2>(job);
        job_piece<3>(job);
    }
    if constexpr (LNERF_KR_SCHED) __builtin_amdgcn_sched_barrier(0);
    const bf8& f = w[O % (kDist + 1)];
    acc[0][O] = mfma(f, b0, acc[0][O]);
    acc[1][O] = mfma(f, b1, acc[1][O]);
}

// tiles B, B + 1, ... of one k-step
template <int NTO, int B, int... O>
__device__ __forceinline__ void kr_tiles_from(std::integer_sequence<int, O...>, const unsigned char* base,
                                              bf8 (&w)[kDist + 1], const bf8& b0, const bf8& b1,
                                              fx4 (&acc)[kGroups][kMaxT], const Job& job) {
    (kr_tile<NTO, B + O>(base, w, b0, b1, acc, job), ...);
}

// k-step S of a pass (S < ks): chunk ci's sub-step S % 2; the first sub-step issues chunk ci + 1's
// DMA, the last meets the barrier that waits for it.
template <int NTO, int S>
__device__ __forceinline__ void kr_step(const KrArgs& a, int ks, int& ci, unsigned char* ring, float* bias_ring,
                                        const bf8 (&B)[kGroups][8], fx4 (&acc)[kGroups][kMaxT]) {
    if (S >= ks) return;
    constexpr int kk = S % kKC;
    const bool last = kk == kKC - 1 || S + 1 == ks;
    Job job;
    if (kk == 0) job = chunk_job(a, ci + 1, ring, bias_ring);
    const int lane = threadIdx.x & 63;
    const unsigned char* base = ring + (ci % kSlots) * kSlot + kk * NTO * 1024 + lane * 16;
    bf8 w[kDist + 1];
#pragma unroll
    for (int o = 0; o < kDist; ++o)
        if (o < NTO) w[o] = *(const bf8*)(base + o * 1024);
    // late waves: the barrier after the first half of the last k-step's tiles
    constexpr int H = NTO / 2;
    const bool late = wave_id() >= 4;
    kr_tiles_from<NTO, 0>(std::make_integer_sequence<int, H>{}, base, w, B[0][S], B[1][S], acc, job);
    if (last && late) chunk_barrier();
    kr_tiles_from<NTO, H>(std::make_integer_sequence<int, NTO - H>{}, base, w, B[0][S], B[1][S], acc, job);
    if (last && !late) chunk_barrier();
    if (last) ++ci;
}

// the head pass from the resident weights (k-step s at head + s KiB): no DMA, no barrier
__device__ __forceinline__ void kr_head_resident(int ks, const unsigned char* head, const bf8 (&B)[kGroups][8],
                                                 fx4 (&acc)[kGroups][kMaxT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (s < ks) {
            const bf8 f = *(const bf8*)(head + s * 1024 + lane * 16);
            acc[0][0] = mfma(f, B[0][s], acc[0][0]);
            acc[1][0] = mfma(f, B[1][s], acc[1][0]);
        }
    }
    // the compiler pads no MFMA hazard on the branch out of the conditional k-steps (tests/test_isa.py
    // found the bias add 7 states after the last MFMA): 16 wait states cover any MFMA result, in
    // place on both accumulators so no MFMA is scheduled below this point
    asm volatile("s_nop 7\n\ts_nop 7" : "+v"(acc[0][0]), "+v"(acc[1][0])::"memory");
}

template <int NTO, int... S>
__device__ __forceinline__ void kr_pass(std::integer_sequence<int, S...>, const KrArgs& a, int ks, int& ci,
                                        unsigned char* ring, float* bias_ring, const bf8 (&B)[kGroups][8],
                                        fx4 (&acc)[kGroups][kMaxT]) {
    (kr_step<NTO, S>(a, ks, ci, ring, bias_ring, B, acc), ...);
}

// Bias + ReLU of a hidden layer's accumulators into the next layer's bf16 B operands: tile o,
// register i of lane group g is feature 16 o + 4 g + i = phi(o / 2, g, 4 (o % 2) + i), so
// B[s][j] takes tile 2s + (j >> 2), register j & 3 (nerf.py:98,125 bias after the sum;
// :141-144 ReLU).
template <int HT>
__device__ __forceinline__ void kr_epilogue(const float* bl, const fx4 (&acc)[kGroups][kMaxT], bf8 (&B)[kGroups][8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (2 * s >= HT) {
            B[0][s] = bf8{};
            B[1][s] = bf8{};
            continue;
        }
        const fx4 b0 = *(const fx4*)(bl + 32 * s);
        const fx4 b1 = *(const fx4*)(bl + 32 * s + 16);
#pragma unroll
        for (int G = 0; G < kGroups; ++G) {
            bf8 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float x0 = acc[G][2 * s][i] + b0[i];
                const float x1 = acc[G][2 * s + 1][i] + b1[i];
                v[i] = (__bf16)(x0 > 0.0f ? x0 : 0.0f);
                v[4 + i] = (__bf16)(x1 > 0.0f ? x1 : 0.0f);
            }
            B[G][s] = v;
        }
    }
}

template <int HT>
__global__ void __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(2, 2)))
kr_fwd_kernel(KrArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
    unsigned char* ring = lds;
    float* comp = (float*)(lds + kOffComp);
    float* rayloss = (float*)(lds + kOffRay);
    float* bias_ring = (float*)(lds + kOffBias);
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), g = lane >> 4, n = lane & 15;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
#if LNERF_PROF
    if (lane < 16) kr_prof_slots()[lane] = 0;
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
#endif
    KR_PROF_T(t_start);
    int ci = 0;
    {
        // chunk 0 (layer 0's weights and biases) and the resident head, issued first: they land
        // while the encoding runs (waited for by the first chunk barrier)
        const Job j0 = chunk_job(a, 0, ring, bias_ring);
        job_piece<0>(j0);
        job_piece<1>(j0);
        job_piece<2>(j0);
        job_piece<3>(j0);
        if (wave < a.ks[a.L - 1])
            glds16((const char*)(a.w16 + a.head_off) + wave * 1024 + lane * 16, lds_addr(lds + kOffHead + wave * 1024));
        if (wave == kWaves - 2)
            glds16(a.b16 + (size_t)(a.L - 1) * 256 + lane * 4, lds_addr(lds + kOffHead + 8 * 1024));
    }

    // ---- layer-0 input (k0 <= 64: two k-steps) as bf16 B operands, group by group, through a
    // per-wave LDS scratch [16 samples][65]: POINTS / RAYS encode one lane per (sample,
    // coordinate), comp::encode_coord (pos_encoding.py:54-66); ENCODED copies loma's layer_input
    bf8 B[kGroups][8];
#pragma unroll
    for (int G = 0; G < kGroups; ++G) {
        constexpr int kStride = 65;
        float* pe = (float*)(lds + kOffPe) + wave * (16 * kStride);
        const int lbase = wave * 32 + G * 16;                 // local sample of the group's row 0
        const int tile_base = wg * tile_samples + lbase;
        if (a.input_mode != LNERF_INPUT_ENCODED) {
            if (lane < 48) {
                const int sl = lane / 3, c = lane - 3 * sl;
                const bool vs = (lbase + sl < tile_samples) && (tile_base + sl < a.R);
                comp::encode_coord(vs ? comp::sample_coord(a, tile_base + sl, c) : 0.0, a.F, pe + sl * kStride, c);
            }
            for (int e = lane; e < 16 * 64; e += 64) {
                const int sl = e >> 6, f = e & 63;
                if (f >= a.k0) pe[sl * kStride + f] = 0.0f;
            }
        } else {
            for (int e = lane; e < 16 * 64; e += 64) {
                const int sl = e >> 6, f = e & 63;
                const bool vs = (lbase + sl < tile_samples) && (tile_base + sl < a.R) && f < a.k0;
                pe[sl * kStride + f] = vs ? a.x[(size_t)(tile_base + sl) * a.k0 + f] : 0.0f;
            }
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            bf8 v = {};
            if (s < 2)
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (__bf16)pe[n * kStride + phi(s, g, j)];
            B[G][s] = v;
        }
    }
    // each wave read only its own scratch rows (LDS operations of a wave complete in order)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    KR_PROF_ADD(kRpPE, t_start);
    KR_PROF_T(t_d);

    chunk_barrier();
    KR_PROF_ADD(kRpDma0, t_d);

    fx4 acc[kGroups][kMaxT];
    KR_PROF_T(t_loop);
    for (int l = 0; l < a.L; ++l) {
        const float* bl = bias_ring + (l % 3) * 256 + g * 4;
        const int ks = a.ks[l];
#pragma unroll
        for (int G = 0; G < kGroups; ++G)
#pragma unroll
            for (int o = 0; o < kMaxT; ++o) acc[G][o] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
        if (l < a.L - 1) {
            KR_PROF_T(t_p);
            kr_pass<HT>(std::make_integer_sequence<int, 8>{}, a, ks, ci, ring, bias_ring, B, acc);
            KR_PROF_ADD(kRpPass, t_p);
            KR_PROF_T(t_e);
            kr_epilogue<HT>(bl, acc, B);
            KR_PROF_ADD(kRpEpi, t_e);
        } else {
            KR_PROF_T(t_h);
            kr_head_resident(ks, lds + kOffHead, B, acc);
            KR_PROF_ADD(kRpHead, t_h);
            // head pre-activations (features 0..3: registers 0..3 of lane group 0), after the sum
            if (g == 0) {
                const fx4 b = *(const fx4*)(lds + kOffHead + 8 * 1024);
#pragma unroll
                for (int G = 0; G < kGroups; ++G) {
                    const int ls = wave * 32 + G * 16 + n;
#pragma unroll
                    for (int i = 0; i < 4; ++i) comp[ls * 4 + i] = acc[G][0][i] + b[i];
                }
            }
        }
    }
    KR_PROF_ADD(kRpLoop, t_loop);
    KR_PROF_T(t_c);
    __syncthreads();
    comp::composite_fwd_wave<kTile>(a, wg, comp, rayloss);
    __syncthreads();
    if (tid == 0) {
        float lsum = 0.0f;
        for (int r = 0; r < a.rpw; ++r) lsum = lsum + rayloss[r];
        a.loss_part[wg] = lsum;
    }
#if LNERF_PROF
    KR_PROF_ADD(kRpComp, t_c);
    KR_PROF_ADD(kRpTotal, t_start);
    if (lane == 0) kr_prof_slots()[kRpReal] += __builtin_amdgcn_s_memrealtime() - rt_start;
    if (lane < kRpN) atomicAdd(&g_kr_prof[lane], kr_prof_slots()[lane]);
#endif
}

}  // namespace

// plain bf16, the NeRF head, whole rays of <= 128 samples, a layer-0 input of <= 64 features
// (PE with F <= 10); anything else renders on k16's forward
// compile-time settings of this object that differ from the product build (lnerf_build_knobs)
unsigned kr_build_knobs() {
    return (LNERF_KR_SCHED != 1 ? kKnobKrSched : 0u) |
           (LNERF_KR_DIST != 2 ? kKnobKrDist : 0u) | (LNERF_PE_DOUBLING != 1 ? kKnobPeDoubling : 0u) |
           (LNERF_PROF != 0 ? kKnobProf : 0u);
}

bool kr_supported(const FusedPlan& p) {
    return p.x6 == 1 && !p.head_fit && p.S <= 128 && p.n[p.L - 1] <= 16 && p.tile == 128 && p.k[0] <= 64;
}

int kr_num_wg(const FusedPlan& p) {
    const int rpw = kTile / p.S;
    return (p.rays + rpw - 1) / rpw;
}

void kr_launch(const FusedPlan& p, const lnerf_batch& b, const lnerf_outputs& out, hipStream_t s) {
    KrArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) a.ks[l] = p.ks16_f[l];
    a.k0 = p.k[0];
    a.w16 = p.w16;
    a.b16 = p.b16;
    a.rays = p.rays;
    a.S = p.S;
    a.rpw = kTile / p.S;
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
    a.seed = 1.0f;
    // the forward chunk stream of k16_pack's one-plane packing: 2 k-steps per chunk
    int ci = 0;
    // the head is not in the chunk stream (the kernel loads it at its start)
    a.head_off = (unsigned)p.w16f_off[p.L - 1];
    for (int l = 0; l < p.L - 1; ++l) {
        const size_t per = (size_t)p.to16_f[l] * 512;   // u16 per k-step
        for (int s2 = 0; s2 < p.ks16_f[l]; s2 += kKC, ++ci) {
            const int nk = p.ks16_f[l] - s2 < kKC ? p.ks16_f[l] - s2 : kKC;
            a.chunk_tab[2 * ci] = (unsigned)(p.w16f_off[l] + (size_t)s2 * per);
            a.chunk_tab[2 * ci + 1] = (unsigned)(nk * per * 2 / 1024) | ((s2 == 0 ? l + 1 : 0) << 16);
        }
    }
    static_assert(sizeof(KrArgs) <= 4096, "kernel arguments");
    const int grid = kr_num_wg(p);
    switch (p.ht16) {
        case 1: kr_fwd_kernel<1><<<grid, 64 * kWaves, 0, s>>>(a); break;
        case 2: kr_fwd_kernel<2><<<grid, 64 * kWaves, 0, s>>>(a); break;
        case 4: kr_fwd_kernel<4><<<grid, 64 * kWaves, 0, s>>>(a); break;
        case 8: kr_fwd_kernel<8><<<grid, 64 * kWaves, 0, s>>>(a); break;
        default: kr_fwd_kernel<16><<<grid, 64 * kWaves, 0, s>>>(a); break;
    }
#if LNERF_PROF
    {
        unsigned long long h[16] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_kr_prof), sizeof(h));
        const char* names[] = {"pe", "dma0", "hidden_pass(incl barrier)", "barrier", "epilogue",
                               "head_pass(incl barrier)", "composite", "total", "realtime_100MHz", "layer_loop", "vmcnt_wait"};
        fprintf(stderr, "LNERF_PROF kr per-wave cycles:");
        for (int i = 0; i < kRpN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / ((double)grid * kWaves));
        fprintf(stderr, " clock_GHz=%.3f\n", h[kRpReal] ? (double)h[kRpTotal] / h[kRpReal] * 0.1 : 0.0);
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kr_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
