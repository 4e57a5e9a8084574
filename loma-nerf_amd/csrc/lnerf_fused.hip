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
#include "lnerf_composite.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

namespace lnerf {

typedef float fx16 __attribute__((ext_vector_type(16)));
typedef float fx4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kWgThreads = 256;
constexpr int kWaves = 4;
constexpr int kTileSamples = comp::kTileSamples;   // samples per fused workgroup
constexpr int kNT = 8;                     // max 32-wide feature tiles (256 features)
constexpr int kChunkMax = 16 * 2 * 256;    // floats per staged weight chunk (r x nt4 x 64 lanes x 4)
constexpr int kCompFloats = comp::kCompFloats;     // per-sample compositing scratch floats in LDS
using comp::composite_tile;
using comp::input_feature;
using comp::sample_coord;

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
    const float* wf;               // f32 MFMA path: fragment-packed weights
    const float* wb;
    const unsigned short* w6;      // bf16x6 path: split-plane packed weights (u16 offsets)
    const float* bp;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    float* act;
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;
    size_t grad_off[kMaxLayers];
    int rays, S, rpw, R, input_mode, F;
    float near_t, far_t;          // RAYS mode sampling range
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
// Weight ring: 2 slots of one contraction tile of one layer (f32: 16 regs x 8 tiles x 64 lanes x
// 4 B = 32 KiB; bf16x6: 2 k-steps x 8 tiles x 3 planes x 64 lanes x 16 B = 48 KiB).
// ReLU masks: per wave and hidden layer, 64 lanes x 16 B of per-lane bits (tile, register).
constexpr int kRingSlotBytes(bool x6) { return x6 ? 2 * kNT * 3 * 1024 : kChunkMax * 4; }
constexpr int kMaskTiles(bool x6) { return x6 ? 64 : 120; }
constexpr int kLdsComp = kTileSamples * kCompFloats;                    // floats
constexpr int kLdsRay = kTileSamples;                                   // per-ray loss partials
constexpr int kLdsTr = kWaves * 32 * 32;                                // per-wave transpose tile
constexpr int kLdsBias = 2 * kNT * 32;                                  // 2 x one layer's biases
constexpr size_t kLdsBytes(bool x6) {
    return (size_t)2 * kRingSlotBytes(x6) + (size_t)kWaves * kMaskTiles(x6) * 16 * 8 +
           (size_t)kLdsComp * 4 + (size_t)kLdsRay * 4 + (size_t)kLdsTr * 4 + (size_t)kLdsBias * 4;
}
static_assert(kLdsBytes(false) <= 160 * 1024, "LDS budget (f32)");
static_assert(kLdsBytes(true) <= 160 * 1024, "LDS budget (bf16x6)");

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
}

// Stage BYTES (a multiple of 16) of packed weights into LDS with LDS-DMA
// (global_load_lds_dwordx4): lane-linear destination, 1 KiB per wave instruction.
// Compile-time size: whole 4-KiB rounds unguarded, one guarded tail round.
template <int BYTES>
__device__ __forceinline__ void stage_bytes_t(const void* __restrict__ src, void* dst) {
    const int tid = threadIdx.x, wave = wave_id();
    constexpr int kRound = kWgThreads * 16, kFull = BYTES / kRound, kTail = BYTES % kRound;
#pragma unroll
    for (int i = 0; i < kFull; ++i) {
        const char* g = (const char*)src + i * kRound + tid * 16;
        char* l = (char*)dst + i * kRound + wave * 1024;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 16, 0, 0);
    }
    if (kTail && tid * 16 < kTail) {
        const char* g = (const char*)src + kFull * kRound + tid * 16;
        char* l = (char*)dst + kFull * kRound + wave * 1024;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 16, 0, 0);
    }
}

// Wait for this wave's LDS-DMA, then s_barrier: afterwards every wave's staged bytes are in LDS.
// vmcnt(0), not vmcnt(N): on CDNA loads and stores share vmcnt and do not retire in order with
// respect to each other, so a partial count cannot single out the DMA behind later stores.
// (__syncthreads would also add lgkmcnt(0); the LDS consumers wait for their own reads.)
// ---- optional in-kernel phase timing (build with -DLNERF_PROF=1; never in the product build):
// per-wave s_memtime deltas accumulated in LDS by lane 0, summed into g_prof at the end.
#ifndef LNERF_PROF
#define LNERF_PROF 0
#endif
#ifndef LNERF_PROF_NOSTORE   // profiling experiments only: drop the slab stores / weight DMA
#define LNERF_PROF_NOSTORE 0
#endif
#ifndef LNERF_X6P   // 1: hand-placed bf16x6 step pipeline (mma_stream_x6p); 0: compiler-scheduled
#define LNERF_X6P 1
#endif
#ifndef LNERF_PROF_NODMA
#define LNERF_PROF_NODMA 0
#endif
#if LNERF_PROF
enum { kPfPE, kPfFwd, kPfWait, kPfComp, kPfBwd, kPfTail, kPfTotal, kPfFwdEpi, kPfBwdEpi,
       kPfChunkPro, kPfSteps, kPfLastStore, kPfLayerPro, kPfChunkBar, kPfN };
__device__ unsigned long long g_prof[16];
__device__ __forceinline__ unsigned long long* prof_slots() {
    __shared__ unsigned long long s[kWaves][16];
    return &s[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0];
}
#define PROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(cat, t0) \
    do { if ((threadIdx.x & 63) == 0) prof_slots()[cat] += __builtin_amdgcn_s_memtime() - (t0); } while (0)
#else
#define PROF_T(v)
#define PROF_ADD(cat, t0)
#endif

template <int N>
__device__ __forceinline__ void dma_barrier_n() {
    static_assert(N == 0, "see above");
    PROF_T(t0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt(7), lgkmcnt(15)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    PROF_ADD(kPfWait, t0);
}
__device__ __forceinline__ void dma_barrier() { dma_barrier_n<0>(); }

// Offset of (feature row, sample) inside a 4-KiB slab tile: two halves of 16 samples, each
// [32 rows][16 samples], so the dW kernel streams a 16-sample half-block as contiguous 2-KiB runs.
__host__ __device__ __forceinline__ int slab_off(int row, int sample) {
    return (sample >> 4) * 512 + row * 16 + (sample & 15);
}

// Store one 32x32 accumulator tile (lane = sample, registers = features in C/D order) as a
// row-major [feature][32 samples] block: transpose through the wave's LDS tile, then 4
// global_store_dwordx4 per lane (each wave instruction writes 8 whole 128-B rows).
__device__ __forceinline__ void store_tile(const fx16& v, float* __restrict__ dst, float* tr) {
    const int lane = threadIdx.x & 63, h = lane >> 5, sl = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) tr[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + sl] = v[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = (lane >> 3) + 8 * q, c4 = (lane & 7) * 4;
        const fx4 x = *(const fx4*)(tr + row * 32 + c4);
        // streaming store (nt): the slabs are read once, by the dW kernel; keep L2 for weights
        __builtin_nontemporal_store(x, (fx4*)(dst + slab_off(row, c4)));
    }
}

// out[o] += sum_{c < nchunks, r} Wpack[c][r][o] (x) in[c][r] for o < NTO: the packed weights of
// one layer streamed chunk by chunk (chunk c = contraction tile c) through a 2-deep LDS ring.
// NTO is compile-time and the chunk loop fully unrolled, so every register index is static (no
// scratch, no per-MFMA branches); a chunk is skipped with one uniform branch.
// While chunk c computes, input tile c-1 (already consumed) is written to its HBM slab
// (`tstore`, nullable), so the slab stores drain under the MFMAs instead of stalling a barrier.
// `bias_src` (nullable) = this layer's fragment-ordered biases, staged into `bias_lds`.
// NCH > 0: compile-time chunk count (drops the per-chunk branch, which makes the compiler copy
// accumulators between AGPRs and VGPRs); NCH = 0: runtime `nchunks`. The call sites use NCH = 0:
// with NCH = HT = 8 the scheduler hoists the next chunks' LDS reads and the kernel spills.
template <int NTO, int NCH = 0>
__device__ __forceinline__ void mma_stream_t(const float* __restrict__ src, int nchunks,
                                             const fx16 (&in)[kNT], fx16 (&out)[kNT], float* ldsw,
                                             float* tstore, float* tr, const float* bias_src,
                                             float* bias_lds) {
    if (NCH > 0) nchunks = NCH;
    const int lane = threadIdx.x & 63;
    constexpr int NT4 = (NTO + 3) / 4;
    constexpr int CF = 16 * NT4 * 256;
    stage_bytes_t<CF * 4>(src, ldsw);
    if (bias_src && wave_id() == 0)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bias_src + lane * 4),
                                         (__attribute__((address_space(3))) void*)bias_lds, 16, 0, 0);
    dma_barrier();
#pragma unroll
    for (int c = 0; c < (NCH > 0 ? NCH : kNT); ++c) {
        if (NCH > 0 || c < nchunks) {
            const float* cur = ldsw + (c & 1) * kChunkMax + lane * 4;
            if (c + 1 < nchunks)
                stage_bytes_t<CF * 4>(src + (size_t)(c + 1) * CF, ldsw + ((c + 1) & 1) * kChunkMax);
            if (tstore && c >= 1) store_tile(in[c - 1], tstore + (c - 1) * 1024, tr);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                fx4 w[NT4];
#pragma unroll
                for (int q = 0; q < NT4; ++q) w[q] = *(const fx4*)(cur + (r * NT4 + q) * 256);
#pragma unroll
                for (int o = 0; o < NTO; ++o)
                    out[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[o >> 2][o & 3], in[c][r], out[o], 0, 0, 0);
            }
            dma_barrier();
            if (tstore && c == nchunks - 1) store_tile(in[c], tstore + c * 1024, tr);
        }
    }
}

// Output-tile counts are rounded up to 1/2/4/8 (the padded tiles of the packed weights are zero).
template <int PREC>
__device__ __forceinline__ void layer_mma_n(const FusedArgs& a, bool fwd, int l, int nchunks, int nto,
                                            const fx16 (&in)[kNT], fx16 (&out)[kNT],
                                            unsigned char* ring, float* tstore, float* tr);

// ---- bf16x6: fp32-accurate products on the bf16 MFMA ---------------------------------------
// x = hi + mid + lo, each a bf16 (8 significant bits; round-to-nearest, the remainders are exact in
// f32), so the three planes carry x's 24 bits. A product keeps the six terms down to 2^-16
// relative (hh, hm, mh, hl, lh, mm): the dropped terms are <= 2^-24 |w x|, fp32 rounding size.
// v_mfma_f32_32x32x16_bf16 does 16x the FLOP/cycle of v_mfma_f32_32x32x2_f32, so six of them
// are 2.67x the f32 rate (MI355X_MICROARCH.md § Matrix cores).
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const fx16& v, int s, bf8& hi, bf8& mid, bf8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = v[8 * s + j];
        const __bf16 h = (__bf16)x;
        const float r = x - (float)h;
        const __bf16 m = (__bf16)r;
        hi[j] = h;
        mid[j] = m;
        lo[j] = (__bf16)(r - (float)m);
    }
}

// One pair (elements 2q, 2q+1) of split3's k-step s: one 32-bit register of each plane.
__device__ __forceinline__ void split3_pair(const fx16& v, int s, int q, bf8& hi, bf8& mid, bf8& lo) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int j = 2 * q + e;
        const float x = v[8 * s + j];
        const __bf16 h = (__bf16)x;
        const float r = x - (float)h;
        const __bf16 m = (__bf16)r;
        hi[j] = h;
        mid[j] = m;
        lo[j] = (__bf16)(r - (float)m);
    }
}

__device__ __forceinline__ fx16 mfma_x6(const bf8& wh, const bf8& wm, const bf8& wl, const bf8& bh,
                                        const bf8& bm, const bf8& bl, fx16 acc) {
    // small terms first (in the order the planes arrive from LDS: hi, mid, lo)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bh, acc, 0, 0, 0);
    return acc;
}

// bf16x6 form of mma_stream_t. Packed chunk c (= contraction tile c) of a layer holds, for k-step
// s (16 of the tile's 32 features), output tile o and plane p, one 16-B A fragment per lane:
// [s][o][p][lane][8 x bf16], the 8 k's of lane half h being the features that accumulator
// registers 8s..8s+7 of the input tile hold (cdna_hip_programming.md "accumulator tile as the
// next MFMA's operand"). The B operand is the input tile itself, split into planes on the fly.
// LDS byte address of a generic pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 outside the compiler's waitcnt bookkeeping (paired with lgkm_wait_for).
template <int OFF>
__device__ __forceinline__ bf8 ds_read_b128_at(unsigned addr) {
    bf8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}

// s_waitcnt lgkmcnt(N) that the fragments depend on (so no use can be scheduled above it).
template <int N>
__device__ __forceinline__ void lgkm_wait_for(bf8& a, bf8& b, bf8& c) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait_for(bf8& a) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}

// bf16 (one plane): round-to-nearest bf16 of the activations, one MFMA per step (inference).
__device__ __forceinline__ void split1(const fx16& v, int s, bf8& hi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = (__bf16)v[8 * s + j];
}

// The fragment-read / MFMA pipeline of one staged chunk, unrolled at compile time (the LDS
// offsets are instruction immediates): reads of steps 0 and 1 first, then per step I the reads
// of step I+2, a wait that leaves those (and step I+1's) in flight, and step I's six MFMAs.
template <int NS, int PL>
__device__ __forceinline__ void x6_prologue(unsigned base, bf8 (&w)[NS][3]) {
    w[0][0] = ds_read_b128_at<0 * 1024>(base);
    if constexpr (PL == 3) {
        w[0][1] = ds_read_b128_at<1 * 1024>(base);
        w[0][2] = ds_read_b128_at<2 * 1024>(base);
    }
    if constexpr (NS > 1) {
        w[1][0] = ds_read_b128_at<(PL + 0) * 1024>(base);
        if constexpr (PL == 3) {
            w[1][1] = ds_read_b128_at<(PL + 1) * 1024>(base);
            w[1][2] = ds_read_b128_at<(PL + 2) * 1024>(base);
        }
    }
}

// A slab tile store spread over the step pipeline: its LDS transpose writes at step 0, the
// transposed reads half way, the global stores at the last step, so neither LDS round trip
// stalls the MFMA stream.
struct TileStore {
    const fx16* v;   // accumulator-layout tile (nullptr: nothing to store)
    float* dst;      // [32 features][32 samples] slab block
    float* tr;       // this wave's 32x32 LDS transpose tile
    fx4 t[4];
};

__device__ __forceinline__ void tile_store_write(TileStore& ts) {
    if (!ts.v) return;
    const int lane = threadIdx.x & 63, h = lane >> 5, sl = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) ts.tr[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + sl] = (*ts.v)[r];
}

__device__ __forceinline__ void tile_store_read(TileStore& ts) {
    if (!ts.v) return;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 4; ++q) ts.t[q] = *(const fx4*)(ts.tr + ((lane >> 3) + 8 * q) * 32 + (lane & 7) * 4);
}

__device__ __forceinline__ void tile_store_global(TileStore& ts) {
    if (!ts.v) return;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        __builtin_nontemporal_store(ts.t[q], (fx4*)(ts.dst + slab_off((lane >> 3) + 8 * q, (lane & 7) * 4)));
}

// The next chunk's LDS-DMA, one 4-KiB round (one 1-KiB instruction per wave) per step, so each
// instruction's issue cost (~60 cycles, MI355X_MICROARCH.md) hides under the MFMAs instead of
// twelve of them stalling the chunk start.
struct ChunkDma {
    const char* src;
    unsigned char* dst;
    bool on;   // (unused: the rounds are unconditional, see mma_stream_x6)
};

template <int CB, int R>
__device__ __forceinline__ void chunk_dma_round(const ChunkDma& d) {
    constexpr int kRound = kWgThreads * 16, kFull = CB / kRound, kTail = CB % kRound;
    if constexpr (!LNERF_PROF_NODMA && (R < kFull || (R == kFull && kTail))) {
        const int tid = threadIdx.x, wave = wave_id();
        if (R < kFull || tid * 16 < kTail) {
            const char* g = d.src + R * kRound + tid * 16;
            unsigned char* l = d.dst + R * kRound + wave * 1024;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                             (__attribute__((address_space(3))) void*)l, 16, 0, 0);
        }
    }
}

template <int CB, int R, int N>
__device__ __forceinline__ void chunk_dma_rest(const ChunkDma& d) {
    if constexpr (R < N) {
        chunk_dma_round<CB, R>(d);
        chunk_dma_rest<CB, R + 1, N>(d);
    }
}

// ---- bf16x6 step pipeline with hand-placed fillers -------------------------------------------
// One wave per SIMD issues in order, and a v_mfma_f32_32x32x16_bf16 gap hides about 24 cycles of
// other issue (MI355X_MICROARCH.md, cycle constants): the six dependent MFMAs of a step leave six
// gaps, and each filler (an LDS-DMA round, a fragment read, half of an operand-pair split, a piece
// of the slab-tile transpose or store) is pinned into one of them with sched_barrier. Every LDS op
// inside the pipeline is inline asm counted by hand, so each step waits for exactly its own
// fragments (lgkmcnt, in-order LDS completion; no SMEM may be outstanding: flushed per layer).
//
// Per chunk c (NS = 2 NTO steps; step I = k-step I / NTO, output tile I % NTO):
//   G1 (after MFMA 1)  LDS-DMA round(s) of chunk c+1 (steps 0..NS-2)
//   G2, G3             fragment reads of step I+2 (planes 0, 1) + halves of an operand-pair split
//                      (k-step 1 of this chunk during steps 0..3, k-step 0 of chunk c+1 during
//                      steps NTO..NTO+3)
//   G4                 fragment read of step I+2 (plane 2)
//   G5, G6             slab tile of input tile c-1: LDS transpose writes (steps 0, 1), transposed
//                      reads (step 2), buffer stores (step 5: early, so their write acks are back
//                      before the chunk-end barrier's vmcnt(0))
//   step NS-1          after its wait: vmcnt(0) + s_barrier (chunk c+1 landed; every wave has
//                      read all of chunk c), then in G6 the fragment reads of chunk c+1's steps 0, 1.
template <int NS>
struct X6Sched {
    static constexpr bool kWide = NS >= 8;
    static constexpr int kWrA = 0, kWrB = kWide ? 1 : 0, kRd = kWide ? 2 : 1;
    static constexpr int kGl = kWide ? 5 : NS - 1;
    static constexpr int tile_ops(int I, bool tile) {
        return !tile || LNERF_PROF_NOSTORE == 3 ? 0 : kWide ? (I <= 1 ? 8 : I == 2 ? 4 : 0) : (I == 0 ? 16 : I == 1 ? 4 : 0);
    }
    static constexpr int reads(int I) { return I + 2 < NS ? 3 : 0; }
    // LDS ops issued after the last fragment read of step I, before step I's wait
    static constexpr int wait(int I, bool tile) {
        const int n = I == 0 ? 3
                      : I == 1 ? reads(0) + tile_ops(0, tile)
                               : tile_ops(I - 2, tile) + reads(I - 1) + tile_ops(I - 1, tile);
        return n > 15 ? 15 : n;
    }
};

typedef unsigned int ux4 __attribute__((ext_vector_type(4)));

template <int OFF>
__device__ __forceinline__ void ds_write_b32_at(unsigned addr, float v) {
    asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(addr), "v"(v), "n"(OFF));
}
template <int OFF>
__device__ __forceinline__ fx4 ds_read_b128_f4(unsigned addr) {
    fx4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
template <int N>
__device__ __forceinline__ void lgkm_wait_t(fx4 (&t)[4]) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(N));
}

#define X6_SB() __builtin_amdgcn_sched_barrier(0)

// One half of split3_pair: A = hi plane and first remainder, B = mid and lo planes.
struct PairSplit {
    float r0, r1;
};
__device__ __forceinline__ void split_pair_a(const fx16& v, int s, int q, bf8& hi, PairSplit& ps) {
    const float x0 = v[8 * s + 2 * q], x1 = v[8 * s + 2 * q + 1];
    const __bf16 h0 = (__bf16)x0, h1 = (__bf16)x1;
    hi[2 * q] = h0;
    hi[2 * q + 1] = h1;
    ps.r0 = x0 - (float)h0;
    ps.r1 = x1 - (float)h1;
}
__device__ __forceinline__ void split_pair_b(int q, const PairSplit& ps, bf8& mid, bf8& lo) {
    const __bf16 m0 = (__bf16)ps.r0, m1 = (__bf16)ps.r1;
    mid[2 * q] = m0;
    mid[2 * q + 1] = m1;
    lo[2 * q] = (__bf16)(ps.r0 - (float)m0);
    lo[2 * q + 1] = (__bf16)(ps.r1 - (float)m1);
}

struct X6Pipe {
    unsigned base;             // this lane's fragment address in the current chunk's slot
    unsigned nbase;            // ... in the next chunk's slot
    unsigned trw, trr;         // transpose tile: write address (lane = sample), read address
    const fx16* tile;          // input tile c-1 (slab store) or nullptr (compile-time per chunk)
    const fx16* cur;           // input tile c (k-step 1 split)
    const fx16* next;          // input tile c+1 (k-step 0 split)
    __amdgpu_buffer_rsrc_t rsrc;   // slab of this layer and block (num_records 0: no store)
    int voff, soff;            // buffer store offsets (lane part, chunk part), bytes
    ChunkDma dma;
    fx4 t[4];                  // transposed tile, in flight from step kRd to kGl
    PairSplit ps;
};

template <int NS, int NTO, bool TILE, int I, int G>
__device__ __forceinline__ void x6p_tile_piece(X6Pipe& p) {
    using S = X6Sched<NS>;
    if constexpr (TILE && LNERF_PROF_NOSTORE != 3) {
        // transpose writes: 4 (wide) or 8 registers per gap
        constexpr int kPer = S::kWide ? 4 : 8;
        constexpr int kFirst = S::kWide ? ((I == S::kWrA ? 0 : 8) + (G == 5 ? 0 : 4)) : (G == 5 ? 0 : 8);
        if constexpr ((I == S::kWrA || I == S::kWrB) && (S::kWide || I == 0)) {
            if constexpr (kFirst + kPer <= 16) {
#define X6_TRW(r) ds_write_b32_at<(((r) & 3) + 8 * ((r) >> 2)) * 128>(p.trw, (*p.tile)[r])
                if constexpr (kFirst + 0 < 16) X6_TRW(kFirst + 0);
                if constexpr (kFirst + 1 < 16) X6_TRW(kFirst + 1);
                if constexpr (kFirst + 2 < 16) X6_TRW(kFirst + 2);
                if constexpr (kFirst + 3 < 16) X6_TRW(kFirst + 3);
                if constexpr (kPer == 8) {
                    X6_TRW(kFirst + 4);
                    X6_TRW(kFirst + 5);
                    X6_TRW(kFirst + 6);
                    X6_TRW(kFirst + 7);
                }
#undef X6_TRW
            }
        }
        if constexpr (I == S::kRd && G == 5) {
            p.t[0] = ds_read_b128_f4<0>(p.trr);
            p.t[1] = ds_read_b128_f4<1024>(p.trr);
            if constexpr (!S::kWide) {
                p.t[2] = ds_read_b128_f4<2048>(p.trr);
                p.t[3] = ds_read_b128_f4<3072>(p.trr);
            }
        }
        if constexpr (S::kWide && I == S::kRd && G == 6) {
            p.t[2] = ds_read_b128_f4<2048>(p.trr);
            p.t[3] = ds_read_b128_f4<3072>(p.trr);
        }
    }
    if constexpr (TILE && LNERF_PROF_NOSTORE != 2) {
        if constexpr (I == S::kGl) {
            if constexpr (!S::kWide && G == 6) lgkm_wait_t<0>(p.t);
            constexpr int q0 = S::kWide ? (G == 5 ? 0 : 2) : 0, nq = S::kWide ? 2 : (G == 6 ? 4 : 0);
#pragma unroll
            for (int q = q0; q < q0 + nq; ++q)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ux4, p.t[q]), p.rsrc,
                                                       p.voff + 512 * q, p.soff, 2 /* nt */);
        }
    }
}

#ifndef LNERF_X6P_DMA_GAP
#define LNERF_X6P_DMA_GAP 1
#endif
// the LDS-DMA round(s) of step I, in gap G = LNERF_X6P_DMA_GAP
template <int NS, int NTO, int I, int G>
__device__ __forceinline__ void x6p_dma(X6Pipe& p) {
    constexpr int CB = 2 * NTO * 3 * 1024;
    constexpr int kRounds = (CB + kWgThreads * 16 - 1) / (kWgThreads * 16);
    if constexpr (G == LNERF_X6P_DMA_GAP && I < NS - 1) {
        if constexpr (I < NS - 2) {
            chunk_dma_round<CB, I>(p.dma);
        } else {
            chunk_dma_rest<CB, I, kRounds>(p.dma);
        }
    }
}

template <int NS, int NTO, bool TILE, int I>
__device__ __forceinline__ void x6p_step(X6Pipe& p, bf8 (&w)[NS][3], bf8 (&bp)[2][3], fx16 (&out)[kNT]) {
    if constexpr (I < NS) {
        using S = X6Sched<NS>;
        constexpr int ks = I / NTO, o = I % NTO;
        constexpr int kW = S::wait(I, TILE);
        if constexpr (TILE && I == S::kGl && S::kWide) lgkm_wait_t<kW>(p.t);
        lgkm_wait_for<kW>(w[I][0], w[I][1], w[I][2]);
        if constexpr (I == NS - 1) {
            // chunk c+1 has landed (this wave's DMA) and, after the barrier, every wave's; every
            // wave has also finished reading chunk c, so its slot may be overwritten from here on
            PROF_T(t_b);
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            PROF_ADD(kPfChunkBar, t_b);
        }
        X6_SB();
        // G1 .. G6 (see above)
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][0], bp[ks][2], out[o], 0, 0, 0);
        X6_SB();
        x6p_dma<NS, NTO, I, 1>(p);
        X6_SB();
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][1], bp[ks][1], out[o], 0, 0, 0);
        X6_SB();
        x6p_dma<NS, NTO, I, 2>(p);
        if constexpr (I + 2 < NS) w[I + 2][0] = ds_read_b128_at<((I + 2) * 3 + 0) * 1024>(p.base);
        if constexpr (NTO >= 4 && I < 4) split_pair_a(*p.cur, 1, I, bp[1][0], p.ps);
        if constexpr (NTO >= 4 && I >= NTO && I < NTO + 4) split_pair_a(*p.next, 0, I - NTO, bp[0][0], p.ps);
        X6_SB();
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][2], bp[ks][0], out[o], 0, 0, 0);
        X6_SB();
        if constexpr (I + 2 < NS) w[I + 2][1] = ds_read_b128_at<((I + 2) * 3 + 1) * 1024>(p.base);
        if constexpr (NTO >= 4 && I < 4) split_pair_b(I, p.ps, bp[1][1], bp[1][2]);
        if constexpr (NTO >= 4 && I >= NTO && I < NTO + 4) split_pair_b(I - NTO, p.ps, bp[0][1], bp[0][2]);
        X6_SB();
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][1], bp[ks][0], out[o], 0, 0, 0);
        X6_SB();
        x6p_dma<NS, NTO, I, 4>(p);
        if constexpr (I + 2 < NS) w[I + 2][2] = ds_read_b128_at<((I + 2) * 3 + 2) * 1024>(p.base);
        X6_SB();
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][0], bp[ks][1], out[o], 0, 0, 0);
        X6_SB();
        x6p_dma<NS, NTO, I, 5>(p);
        x6p_tile_piece<NS, NTO, TILE, I, 5>(p);
        X6_SB();
        out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][0], bp[ks][0], out[o], 0, 0, 0);
        X6_SB();
        x6p_dma<NS, NTO, I, 6>(p);
        x6p_tile_piece<NS, NTO, TILE, I, 6>(p);
        if constexpr (I == NS - 1) {
            // chunk c+1's first two steps (the last chunk reads its re-staged copy; unused)
            w[0][0] = ds_read_b128_at<0 * 1024>(p.nbase);
            w[0][1] = ds_read_b128_at<1 * 1024>(p.nbase);
            w[0][2] = ds_read_b128_at<2 * 1024>(p.nbase);
            w[1][0] = ds_read_b128_at<3 * 1024>(p.nbase);
            w[1][1] = ds_read_b128_at<4 * 1024>(p.nbase);
            w[1][2] = ds_read_b128_at<5 * 1024>(p.nbase);
        }
        X6_SB();
        x6p_step<NS, NTO, TILE, I + 1>(p, w, bp, out);
    }
}

// bf16x6 layer stream on the hand-placed pipeline (see X6Sched).
template <int NTO>
__device__ __forceinline__ void mma_stream_x6p(const unsigned short* __restrict__ src, int nchunks,
                                               const fx16 (&in)[kNT], fx16 (&out)[kNT],
                                               unsigned char* ring, float* tstore, float* tr,
                                               const float* bias_src, float* bias_lds) {
    PROF_T(t_lp);
    const int lane = threadIdx.x & 63;
    constexpr int NS = 2 * NTO;
    constexpr int CB = 2 * NTO * 3 * 1024;
    constexpr int SLOT = kRingSlotBytes(true);
    stage_bytes_t<CB>(src, ring);
    if (bias_src && wave_id() == 0)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bias_src + lane * 4),
                                         (__attribute__((address_space(3))) void*)bias_lds, 16, 0, 0);
    X6Pipe p;
    const int h = lane >> 5, sl = lane & 31;
    p.trw = lds_addr(tr) + (unsigned)((4 * h * 32 + sl) * 4);
    p.trr = lds_addr(tr) + (unsigned)(((lane >> 3) * 32 + (lane & 7) * 4) * 4);
    p.voff = (((lane & 7) >> 2) * 512 + (lane >> 3) * 16 + (lane & 3) * 4) * 4;
    p.rsrc = __builtin_amdgcn_make_buffer_rsrc(tstore, 0, tstore ? nchunks * 4096 : 0, 0x00020000);
    bf8 bp[2][3];
    bf8 w[NS][3];
    dma_barrier();
    // no scalar load may be in flight inside the pipeline (see X6Sched)
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    X6_SB();
    {
        const unsigned b0 = lds_addr(ring) + lane * 16;
        w[0][0] = ds_read_b128_at<0 * 1024>(b0);
        w[0][1] = ds_read_b128_at<1 * 1024>(b0);
        w[0][2] = ds_read_b128_at<2 * 1024>(b0);
        w[1][0] = ds_read_b128_at<3 * 1024>(b0);
        w[1][1] = ds_read_b128_at<4 * 1024>(b0);
        w[1][2] = ds_read_b128_at<5 * 1024>(b0);
    }
    split3(in[0], 0, bp[0][0], bp[0][1], bp[0][2]);
    X6_SB();
    PROF_ADD(kPfLayerPro, t_lp);
#pragma unroll
    for (int c = 0; c < kNT; ++c) {
        if (c < nchunks) {
            PROF_T(t_st);
            p.base = lds_addr(ring + (c & 1) * SLOT) + lane * 16;
            p.nbase = lds_addr(ring + ((c + 1) & 1) * SLOT) + lane * 16;
            // the last chunk re-stages itself into the free slot instead of branching around
            // the per-step DMA rounds (a branch would split the step pipeline into blocks)
            p.dma.src = (const char*)src + (size_t)(c + 1 < nchunks ? c + 1 : c) * CB;
            p.dma.dst = ring + ((c + 1) & 1) * SLOT;
            p.dma.on = true;
            p.cur = &in[c];
            p.tile = c >= 1 ? &in[c - 1] : nullptr;
            // k-step 0 operand of chunk c+1, split under chunk c (junk, unused, after the last)
            p.next = &in[c + 1 < kNT ? c + 1 : c];
            p.soff = (c - 1) * 4096;
            if constexpr (NTO < 4) {
                split3(in[c], 1, bp[1][0], bp[1][1], bp[1][2]);
                X6_SB();
            }
            if (c >= 1 && LNERF_PROF_NOSTORE != 1) {
                x6p_step<NS, NTO, true, 0>(p, w, bp, out);
            } else {
                x6p_step<NS, NTO, false, 0>(p, w, bp, out);
            }
            if constexpr (NTO < 4) {
                split3(*p.next, 0, bp[0][0], bp[0][1], bp[0][2]);
            }
            PROF_ADD(kPfSteps, t_st);
            PROF_T(t_ls);
            if (tstore && c == nchunks - 1) {
                __builtin_amdgcn_s_waitcnt(0xC07F);
                store_tile(in[c], tstore + c * 1024, tr);
            }
            PROF_ADD(kPfLastStore, t_ls);
        }
    }
}

template <int NS, int NTO, int PL, int I>
__device__ __forceinline__ void x6_step(unsigned base, bf8 (&w)[NS][3], bf8 (&bp)[2][3],
                                        fx16 (&out)[kNT], TileStore& ts, const ChunkDma& dma,
                                        const fx16& tile) {
    if constexpr (I < NS) {
        // the second k-step's operand split, one register pair per step under the first
        // k-step's MFMAs (needed from step NTO on)
        if constexpr (PL == 3 && NTO >= 4 && I < 4) split3_pair(tile, 1, I, bp[1][0], bp[1][1], bp[1][2]);
        constexpr int CB = 2 * NTO * PL * 1024;
        constexpr int kRounds = (CB + kWgThreads * 16 - 1) / (kWgThreads * 16);
        // rounds spread over the steps (more rounds than steps: the rest at the last step)
        if constexpr (I < NS - 1) {
            chunk_dma_round<CB, I>(dma);
        } else {
            chunk_dma_rest<CB, I, kRounds>(dma);
        }
        if constexpr (I + 2 < NS) {
            w[I + 2][0] = ds_read_b128_at<((I + 2) * PL + 0) * 1024>(base);
            if constexpr (PL == 3) {
                w[I + 2][1] = ds_read_b128_at<((I + 2) * PL + 1) * 1024>(base);
                w[I + 2][2] = ds_read_b128_at<((I + 2) * PL + 2) * 1024>(base);
            }
        }
        if constexpr (I == 0) tile_store_write(ts);
        if constexpr (I == NS / 2) tile_store_read(ts);
        if constexpr (I == NS - 1) tile_store_global(ts);
        constexpr int ks = I / NTO, o = I % NTO;
        constexpr int kWait = I + 2 < NS ? 2 * PL : (I + 1 < NS ? PL : 0);
        if constexpr (PL == 3) {
            lgkm_wait_for<kWait>(w[I][0], w[I][1], w[I][2]);
            out[o] = mfma_x6(w[I][0], w[I][1], w[I][2], bp[ks][0], bp[ks][1], bp[ks][2], out[o]);
        } else {
            lgkm_wait_for<kWait>(w[I][0]);
            out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[I][0], bp[ks][0], out[o], 0, 0, 0);
        }
        x6_step<NS, NTO, PL, I + 1>(base, w, bp, out, ts, dma, tile);
    }
}

// PL = 3: bf16x6 (fp32-accurate); PL = 1: plain bf16 (one plane, one MFMA per step).
template <int NTO, int PL>
__device__ __forceinline__ void mma_stream_x6(const unsigned short* __restrict__ src, int nchunks,
                                              const fx16 (&in)[kNT], fx16 (&out)[kNT],
                                              unsigned char* ring, float* tstore, float* tr,
                                              const float* bias_src, float* bias_lds) {
#if LNERF_X6P
    if constexpr (PL == 3) {
        mma_stream_x6p<NTO>(src, nchunks, in, out, ring, tstore, tr, bias_src, bias_lds);
        return;
    }
#endif
    const int lane = threadIdx.x & 63;
    constexpr int CB = 2 * NTO * PL * 1024;       // bytes per chunk
    constexpr int SLOT = kRingSlotBytes(true);
    stage_bytes_t<CB>(src, ring);
    if (bias_src && wave_id() == 0)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bias_src + lane * 4),
                                         (__attribute__((address_space(3))) void*)bias_lds, 16, 0, 0);
    dma_barrier();
#pragma unroll
    for (int c = 0; c < kNT; ++c) {
        if (c < nchunks) {
            PROF_T(t_cp);
            const unsigned char* cur = ring + (c & 1) * SLOT + lane * 16;
            ChunkDma dma;
            // the last chunk re-stages itself into the free slot instead of branching around
            // the per-step DMA rounds (a branch would split the step pipeline into blocks)
            dma.src = (const char*)src + (size_t)(c + 1 < nchunks ? c + 1 : c) * CB;
            dma.dst = ring + ((c + 1) & 1) * SLOT;
            dma.on = true;
            TileStore tsx;
            tsx.v = (tstore && c >= 1 && !LNERF_PROF_NOSTORE) ? &in[c - 1] : nullptr;
            tsx.dst = tstore + (c - 1) * 1024;
            tsx.tr = tr;
            // retire any scalar (kernarg) loads still in flight: while one is pending the
            // waitcnt pass can only emit lgkmcnt(0) for the LDS fragment reads below
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt/expcnt untouched
            __builtin_amdgcn_sched_barrier(0);
            // software-pipelined two steps deep: the three planes of step i+2 are read while
            // step i's six MFMAs run. The fragment reads are inline asm with an explicit,
            // dependency-carrying lgkmcnt(N) before each step's MFMAs: the compiler's own waitcnt
            // insertion emits lgkmcnt(0) here, which also waits for the reads just issued.
            constexpr int NS = 2 * NTO;
            const unsigned base = lds_addr(cur);
            bf8 bp[2][3];
            bf8 w[NS][3];
            x6_prologue<NS, PL>(base, w);
            if constexpr (PL == 3) {
                split3(in[c], 0, bp[0][0], bp[0][1], bp[0][2]);
                if constexpr (NTO < 4) split3(in[c], 1, bp[1][0], bp[1][1], bp[1][2]);
            } else {
                split1(in[c], 0, bp[0][0]);
                split1(in[c], 1, bp[1][0]);
            }
            PROF_ADD(kPfChunkPro, t_cp);
            PROF_T(t_st);
            x6_step<NS, NTO, PL, 0>(base, w, bp, out, tsx, dma, in[c]);
            PROF_ADD(kPfSteps, t_st);
            dma_barrier();
            PROF_T(t_ls);
            if (tstore && c == nchunks - 1) store_tile(in[c], tstore + c * 1024, tr);
            PROF_ADD(kPfLastStore, t_ls);
        }
    }
}

// One layer's MMA in the kernel's precision: PREC = bf16 planes per operand (3: bf16x6 split,
// fp32-accurate; 1: plain bf16), PREC = 0: exact f32 MFMA.
template <int NTO, int PREC>
__device__ __forceinline__ void layer_mma(const FusedArgs& a, bool fwd, int l, int nchunks,
                                          const fx16 (&in)[kNT], fx16 (&out)[kNT],
                                          unsigned char* ring, float* tstore, float* tr,
                                          const float* bias_src, float* bias_lds) {
    if constexpr (PREC != 0) {
        const unsigned short* src = a.w6 + (fwd ? a.wf_off[l] : a.wb_off[l]);
        mma_stream_x6<NTO, PREC>(src, nchunks, in, out, ring, tstore, tr, bias_src, bias_lds);
    } else {
        const float* src = fwd ? a.wf + a.wf_off[l] : a.wb + a.wb_off[l];
        mma_stream_t<NTO>(src, nchunks, in, out, (float*)ring, tstore, tr, bias_src, bias_lds);
    }
}

template <int PREC>
__device__ __forceinline__ void layer_mma_n(const FusedArgs& a, bool fwd, int l, int nchunks, int nto,
                                            const fx16 (&in)[kNT], fx16 (&out)[kNT],
                                            unsigned char* ring, float* tstore, float* tr) {
    if (nto <= 1) layer_mma<1, PREC>(a, fwd, l, nchunks, in, out, ring, tstore, tr, nullptr, nullptr);
    else if (nto <= 2) layer_mma<2, PREC>(a, fwd, l, nchunks, in, out, ring, tstore, tr, nullptr, nullptr);
    else if (nto <= 4) layer_mma<4, PREC>(a, fwd, l, nchunks, in, out, ring, tstore, tr, nullptr, nullptr);
    else layer_mma<8, PREC>(a, fwd, l, nchunks, in, out, ring, tstore, tr, nullptr, nullptr);
}

// HT = output tiles of every hidden layer (widths <= 32*HT); the head has <= 32 outputs.
// PREC: 3 = bf16x6 split-plane MFMA (fp32-accurate, 2.67x the f32 MFMA rate), 1 = plain bf16
// (one plane; inference), 0 = exact f32 MFMA.
template <int HT, int PREC>
__global__ void __launch_bounds__(kWgThreads, 1) fused_fwd_bwd_kernel(FusedArgs a) {
    constexpr bool X6 = PREC != 0;   // the bf16 paths share the LDS carve
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kLdsBytes(X6)];
    unsigned char* ring = lds_raw;
    float* ldsw = (float*)lds_raw;
    unsigned long long* masks = (unsigned long long*)(lds_raw + 2 * (size_t)kRingSlotBytes(X6));
    float* comp = (float*)((unsigned char*)masks + (size_t)kWaves * kMaskTiles(X6) * 16 * 8);
    float* rayloss = comp + kLdsComp;
    float* trall = rayloss + kLdsRay;
    float* biasl = trall + kLdsTr;

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), h = lane >> 5;
    const int wg = blockIdx.x;
    const int ls = wave * 32 + (lane & 31);           // local sample 0..127
#if LNERF_PROF
    if (lane < kPfN) prof_slots()[lane] = 0;
    PROF_T(t_start);
#endif
    const int tile_samples = a.rpw * a.S;
    const int gs = wg * tile_samples + ls;            // global sample row (ray*S + j)
    const bool valid = (ls < tile_samples) && (gs < a.R);
    const size_t blk = (size_t)wg * kWaves + wave;    // 32-sample slab index
    // ReLU masks, one bit per (tile, register) and lane: [layer][lane][4 x u32] per wave
    unsigned* wmask = (unsigned*)(masks + (size_t)wave * kMaskTiles(X6) * 16);
    float* tr = trall + wave * 1024;
    const bool st = a.want_grad != 0;

    fx16 act[kNT], out[kNT];
    // ---- layer-0 input: features in accumulator order ----
    // Produced into a per-wave LDS scratch (the weight ring is free before the first layer),
    // then picked up in accumulator order. POINTS mode with 3 + 6F <= 64 (F <= 10) computes
    // each (sample, coordinate, frequency) once with a float64 sincos (pos_encoding.py:54-66:
    // f64 trig of the point, rounded to f32 once); other inputs go tile by tile.
    const int tile_base = wg * tile_samples + wave * 32;
#pragma unroll
    for (int t = 0; t < kNT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) act[t][r] = 0.0f;
    if (a.input_mode != LNERF_INPUT_ENCODED && a.k0 <= 64) {
        constexpr int kStride = 65;
        float* pe = ldsw + (size_t)wave * (32 * kStride);
        const int F = a.F, per = 3 * (F + 1);
        for (int it = lane; it < 32 * per; it += 64) {
            const int sl = it / per, rem = it - sl * per, c = rem % 3, q = rem / 3;
            const bool vs = (wave * 32 + sl < tile_samples) && (tile_base + sl < a.R);
            const double xc = vs ? sample_coord(a, tile_base + sl, c) : 0.0;
            if (q == 0) {
                pe[sl * kStride + c] = (float)xc;
            } else {
                double sn, cs;
                sincos(ldexp(xc, q - 1), &sn, &cs);
                pe[sl * kStride + 3 + 6 * (q - 1) + c] = (float)sn;
                pe[sl * kStride + 6 + 6 * (q - 1) + c] = (float)cs;
            }
        }
        for (int e = lane; e < 32 * 64; e += 64) {        // zero the padded features
            const int sl = e >> 6, f = e & 63;
            if (f >= a.k0) pe[sl * kStride + f] = 0.0f;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
            if (t < a.kt[0]) {
#pragma unroll
                for (int r = 0; r < 16; ++r) act[t][r] = pe[(lane & 31) * kStride + frag_feature(t, r, h)];
            }
        __syncthreads();   // the ring DMA of layer 0 overwrites the scratch
    } else {
        float* pe = ldsw + (size_t)wave * (32 * 33);
#pragma unroll
        for (int t = 0; t < kNT; ++t) {
            if (t < a.kt[0]) {
                for (int e = lane; e < 32 * 32; e += 64) {
                    const int sl = e >> 5, ft = e & 31;
                    const bool vs = (wave * 32 + sl < tile_samples) && (tile_base + sl < a.R);
                    pe[sl * 33 + ft] = input_feature(a, tile_base + sl, vs, 32 * t + ft);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) act[t][r] = pe[(lane & 31) * 33 + (frag_feature(t, r, h) - 32 * t)];
            }
        }
        __syncthreads();
    }

    PROF_ADD(kPfPE, t_start);
    // ---- forward through the layers ----
    for (int l = 0; l < a.L; ++l) {
        PROF_T(t_l);
#pragma unroll
        for (int o = 0; o < kNT; ++o) out[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        // the input tiles of layer l are A_{l-1} (X for l = 0): stored while layer l computes
        float* ts = !st ? nullptr
                        : (l == 0 ? a.act + a.x_off + blk * (size_t)(a.kt[0] * 1024)
                                  : a.act + a.act_off[l - 1] + blk * (size_t)(a.kt[l] * 1024));
        float* bl = biasl + (l & 1) * (kNT * 32);
        // hidden layers l >= 1 and the head contract over HT tiles (k_l = n_{l-1})
        if (l < a.L - 1) layer_mma<HT, PREC>(a, true, l, a.kt[l], act, out, ring, ts, tr, a.bp + a.bp_off[l], bl);
        else layer_mma<1, PREC>(a, true, l, a.kt[l], act, out, ring, ts, tr, a.bp + a.bp_off[l], bl);
        PROF_ADD(kPfFwd, t_l);
        PROF_T(t_e);
        if (l < a.L - 1) {
            unsigned mb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int o = 0; o < HT; ++o) {
                const fx4* bq = (const fx4*)(bl + (o * 2 + h) * 16);
                fx16 bo;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const fx4 b4 = bq[q];
#pragma unroll
                    for (int e = 0; e < 4; ++e) bo[4 * q + e] = b4[e];
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = out[o][r] + bo[r];              // bias after the sum, as loma
                    const bool pos = v > 0.0f;
                    act[o][r] = pos ? v : 0.0f;                     // ReLU nerf.py:141-144
                    mb[o >> 1] |= (pos ? 1u : 0u) << ((o & 1) * 16 + r);
                }
            }
            *(uint4*)(wmask + ((size_t)l * 64 + lane) * 4) = make_uint4(mb[0], mb[1], mb[2], mb[3]);
#pragma unroll
            for (int o = HT; o < kNT; ++o) act[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        } else {
            // head pre-activations (features 0..3 live in regs 0..3 of lane half 0)
            if (h == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) comp[ls * 4 + r] = out[0][r] + bl[r];  // c_z[ls][r]
            }
        }
        PROF_ADD(kPfFwdEpi, t_e);
    }
    PROF_T(t_c);
    __syncthreads();

    // ---- rendering + loss + rendering reverse: one thread per sample, scans along rays ----
    float* c_gz = comp + 512;
    composite_tile(a, wg, comp, rayloss, a.want_grad != 0);
    __syncthreads();
    if (tid == 0) {
        float l = 0.0f;
        for (int r = 0; r < a.rpw; ++r) l = l + rayloss[r];
        a.loss_part[wg] = l;
    }
    PROF_ADD(kPfComp, t_c);
    if (!a.want_grad) return;

    // ---- reverse chain: G_{L-1} from the head, then G_{l-1} = (W_l G_l) * 1[A_{l-1} > 0] ----
    // g (= G_l) is the input of the next reverse MMA, which writes it to its slab chunk by chunk.
    fx16* g = act;
    fx16* go = out;
#pragma unroll
    for (int t = 0; t < kNT; ++t) act[t] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (h == 0 && valid) {
#pragma unroll
        for (int r = 0; r < 4; ++r) act[0][r] = c_gz[ls * 4 + r];
    }
    (void)g;
    (void)go;
    for (int l = a.L - 1; l >= 1; --l) {
        PROF_T(t_b);
#pragma unroll
        for (int o = 0; o < kNT; ++o) out[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        float* ts = a.grad + a.grad_off[l] + blk * (size_t)(a.nt[l] * 1024);
        layer_mma<HT, PREC>(a, false, l, a.nt[l], act, out, ring, ts, tr, nullptr, nullptr);
        PROF_ADD(kPfBwd, t_b);
        PROF_T(t_be);
        const uint4 mq = *(const uint4*)(wmask + ((size_t)(l - 1) * 64 + lane) * 4);
        const unsigned mb[4] = {mq.x, mq.y, mq.z, mq.w};
#pragma unroll
        for (int o = 0; o < HT; ++o) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                act[o][r] = ((mb[o >> 1] >> ((o & 1) * 16 + r)) & 1u) ? out[o][r] : 0.0f;
        }
#pragma unroll
        for (int o = HT; o < kNT; ++o) act[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        PROF_ADD(kPfBwdEpi, t_be);
    }
    PROF_T(t_t);
    // act now holds G_0 (nt[0] tiles)
    float* g0 = a.grad + a.grad_off[0] + blk * (size_t)(a.nt[0] * 1024);
    if (a.d_x) {
        // d_layer_input = G_0 W_0^T (ENCODED mode), written row-major (rows = samples); the MMA
        // also writes G_0's slab
#pragma unroll
        for (int o = 0; o < kNT; ++o) out[o] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        layer_mma_n<PREC>(a, false, 0, a.nt[0], a.kt[0], act, out, ring, g0, tr);
        if (valid) {
#pragma unroll
            for (int o = 0; o < kNT; ++o)
                if (o < a.kt[0]) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int f = frag_feature(o, r, h);
                        if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = out[o][r];
                    }
                }
        }
    } else {
#pragma unroll
        for (int o = 0; o < kNT; ++o)
            if (o < a.nt[0]) store_tile(act[o], g0 + o * 1024, tr);
    }
#if LNERF_PROF
    PROF_ADD(kPfTail, t_t);
    PROF_ADD(kPfTotal, t_start);
    if (lane < kPfN) atomicAdd(&g_prof[lane], prof_slots()[lane]);
#endif
}

// ---------------------------------------------------------------------------------------------
// dW_l = sum_s A_{l-1}[:, s] G_l[:, s]^T (+ db_l = sum_s G_l[:, s]) over a split of the 32-sample
// slabs, fp32 MFMA. Each workgroup streams slab pairs (A: KT*32 feature rows, G: NTo*32 rows, 32
// samples = 128 B per row) into a 2-deep LDS ring with LDS-DMA (global_load_lds_dwordx4). Rows
// are stored with their 16-B chunks XOR-swizzled by ((row >> 1) & 7) -- applied to the per-lane
// global source address, the LDS image stays lane-linear -- so the ds_read_b128 fragment reads
// (one feature row, 4 consecutive samples per lane) are bank-conflict free. Waves own up to 4x4
// blocks of 32x32 output tiles; partials are written per split (deterministic, no atomics).
// ---------------------------------------------------------------------------------------------
constexpr int kDwRows = kNT * 32;                 // max feature rows per slab
constexpr int kDwStageFloats = 2 * kDwRows * 32;  // A + G region of one ring slot

struct DwArgs {
    int L;
    int kt[kMaxLayers], nt[kMaxLayers];
    const float* act;
    size_t a_off[kMaxLayers];   // A_{l-1} slab base per layer (X slab for l = 0)
    const float* grad;
    size_t g_off[kMaxLayers];
    int blocks;
    int splits[kMaxLayers];
    int nl;                     // layers in this launch
    int lid[kMaxLayers];        // their layer ids
    int wg_off[kMaxLayers + 1]; // first workgroup of the i-th layer of this launch
    float* dw_part;
    size_t dwp_off[kMaxLayers];
    float* db_part;
    size_t dbp_off[kMaxLayers];
    int mode[kMaxLayers];       // 0: 4x4-tile blocks per wave; >0: phased (see dw_kernel)
};

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Stage one slab (`rows` x 32 floats) into `dst` (rows x 32, swizzled) with LDS-DMA.
__device__ __forceinline__ void dw_stage(const float* __restrict__ src, float* dst, int rows,
                                         int wave, int lane) {
    // each wave instruction covers 8 rows (1 KiB); lane -> row 8i + (lane >> 3), LDS chunk lane & 7
    for (int i = wave; i < rows / 8; i += kWaves) {
        const int row = i * 8 + (lane >> 3);
        const int c = swz_chunk(row, lane & 7);
        const float* g = src + (row >> 5) * 1024 + slab_off(row & 31, c * 4);
        float* l = dst + i * 256;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)l, 16, 0, 0);
    }
}

__device__ __forceinline__ fx4 dw_frag(const float* base, int row, int g, int h) {
    // samples 8g + 4h .. 8g + 4h + 3 of feature row `row`
    const int c = swz_chunk(row, 2 * g + h);
    return *(const fx4*)(base + row * 32 + c * 4);
}

// One wave's TI x TJ tiles over sample steps g in [g0, g1) of a staged slab pair (a g-step = 8
// samples: lane half h takes samples 8g + 4h + u, u = 0..3, for A and G alike).
template <int TI, int TJ>
__device__ __forceinline__ void dw_block(const float* ca, const float* cg, int kb, int jb, int g0,
                                         int g1, fx16 (&acc)[TI][TJ]) {
    const int lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
#pragma unroll
    for (int g = g0; g < g1; ++g) {
        fx4 af[TI], bf[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = dw_frag(ca, (kb + i) * 32 + rl, g, h);
#pragma unroll
        for (int j = 0; j < TJ; ++j) bf[j] = dw_frag(cg, (jb + j) * 32 + rl, g, h);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][u], bf[j][u], acc[i][j], 0, 0, 0);
    }
}

// bf16x6 form of dw_block: a k-step is 16 samples (lane half h: samples 16ks + 8h + j), the
// fp32 slab values split into hi/mid/lo planes after the LDS read (each split feeds TJ or TI
// tiles x 6 MFMAs). Two k-steps per 32-sample slab.
__device__ __forceinline__ void split3_8(const fx4& x0, const fx4& x1, bf8& hi, bf8& mid, bf8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = j < 4 ? x0[j] : x1[j - 4];
        const __bf16 hh = (__bf16)x;
        const float r = x - (float)hh;
        const __bf16 m = (__bf16)r;
        hi[j] = hh;
        mid[j] = m;
        lo[j] = (__bf16)(r - (float)m);
    }
}

template <int TI, int TJ>
__device__ __forceinline__ void dw_block_x6(const float* ca, const float* cg, int kb, int jb,
                                            fx16 (&acc)[TI][TJ]) {
    const int lane = threadIdx.x & 63, h = lane >> 5, rl = lane & 31;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        bf8 ap[TI][3], gp[TJ][3];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int row = (kb + i) * 32 + rl;
            const fx4 x0 = dw_frag(ca, row, 2 * ks, h), x1 = dw_frag(ca, row, 2 * ks + 1, h);
            // dw_frag(g) reads chunk 2g + h: samples 8g + 4h.. -> here chunks 4ks + h, 4ks + 2 + h
            split3_8(x0, x1, ap[i][0], ap[i][1], ap[i][2]);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int row = (jb + j) * 32 + rl;
            const fx4 x0 = dw_frag(cg, row, 2 * ks, h), x1 = dw_frag(cg, row, 2 * ks + 1, h);
            split3_8(x0, x1, gp[j][0], gp[j][1], gp[j][2]);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                acc[i][j] = mfma_x6(ap[i][0], ap[i][1], ap[i][2], gp[j][0], gp[j][1], gp[j][2], acc[i][j]);
    }
}

// The whole per-workgroup pass for one layer. PHASED = false: wave w owns a 4x4 block of the
// layer's output tiles and every sample; PHASED = true (small layers, TI*TJ <= 16 tiles): every
// wave owns all TI x TJ tiles and one of the 4 sample steps of each slab, writing its own
// partial (4 partials per split). Each instantiation keeps its accumulators to itself.
template <int TI, int TJ, bool PHASED, bool X6>
__device__ __forceinline__ void dw_run(const DwArgs a, int l, int sp, float* lds) {
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KT = a.kt[l], NTo = a.nt[l];
    int kb = 0, jb = 0, ti = TI, tj = TJ;
    bool active = true;
    if (!PHASED) {
        const int nbj = (NTo + 3) >> 2, nblk = ((KT + 3) >> 2) * nbj;
        active = wave < nblk;
        // idle waves repeat block 0 unconditionally and discard it (a branch around the MFMAs
        // would make the compiler shuttle the accumulators out of AGPRs)
        kb = active ? (wave / nbj) * 4 : 0;
        jb = active ? (wave % nbj) * 4 : 0;
        ti = min(TI, KT - kb);
        tj = min(TJ, NTo - jb);
    }
    const int g0 = PHASED ? wave : 0, g1 = PHASED ? wave + 1 : 4;
    const int splits = a.splits[l];
    const int per = (a.blocks + splits - 1) / splits;
    const int b0 = min(a.blocks, sp * per), b1 = min(a.blocks, b0 + per);
    const int a_rows = KT * 32, g_rows = NTo * 32;
    const float* A = a.act + a.a_off[l];
    const float* G = a.grad + a.g_off[l];
    fx16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float dbsum = 0.0f;

    if (b0 < b1) {
        dw_stage(A + (size_t)b0 * a_rows * 32, lds, a_rows, wave, lane);
        dw_stage(G + (size_t)b0 * g_rows * 32, lds + kDwRows * 32, g_rows, wave, lane);
    }
    dma_barrier();
    for (int b = b0; b < b1; ++b) {
        float* cur = lds + ((b - b0) & 1) * kDwStageFloats;
        if (b + 1 < b1) {
            float* nxt = lds + ((b + 1 - b0) & 1) * kDwStageFloats;
            dw_stage(A + (size_t)(b + 1) * a_rows * 32, nxt, a_rows, wave, lane);
            dw_stage(G + (size_t)(b + 1) * g_rows * 32, nxt + kDwRows * 32, g_rows, wave, lane);
        }
        const float* ca = cur;
        const float* cg = cur + kDwRows * 32;
        // (unconditional: a branch around the MFMAs makes the compiler shuttle the accumulators
        // between AGPRs and VGPRs every slab)
        if (X6) dw_block_x6<TI, TJ>(ca, cg, kb, jb, acc);
        else dw_block<TI, TJ>(ca, cg, kb, jb, g0, g1, acc);
        if (tid < g_rows) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const fx4 v = *(const fx4*)(cg + tid * 32 + swz_chunk(tid, c) * 4);
                dbsum += (v[0] + v[1]) + (v[2] + v[3]);
            }
        }
        dma_barrier();
    }
    // partial slab: [split * P + phase][k][j], k < KT*32, j < NTo*32
    if (active) {
        const int ncol = NTo * 32;
        const int part_id = PHASED ? sp * kWaves + wave : sp;
        float* part = a.dw_part + a.dwp_off[l] + (size_t)part_id * (KT * 32) * ncol;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
                if (i < ti && j < tj) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = (kb + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const int jj = (jb + j) * 32 + (lane & 31);
                        part[(size_t)k * ncol + jj] = acc[i][j][r];
                    }
                }
    }
    if (tid < g_rows) a.db_part[a.dbp_off[l] + (size_t)sp * g_rows + tid] = dbsum;
}

// Phased shapes (KT x NTo tiles) with their own instantiation; anything else runs the blocked
// 4x4 path. Mode ids must match dw_mode_for() on the host.
#define LNERF_DW_PHASED_SHAPES(X) X(1, 1, 1) X(2, 1, 2) X(1, 2, 3) X(2, 2, 4) X(2, 4, 5) X(4, 2, 6) \
    X(2, 8, 7) X(8, 1, 8) X(4, 1, 9) X(1, 4, 10) X(8, 2, 11) X(1, 8, 12) X(4, 4, 13)

// Every layer in ONE launch (each workgroup's layer picks its instantiation), so the small
// phased layers fill the machine beside the blocked ones instead of running after them; the
// per-layer splits are balanced by slab bytes (make_layout).
template <bool X6>
__global__ void __launch_bounds__(kWgThreads, 1) dw_all_kernel(DwArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[2 * kDwStageFloats];
    int i = 0;
    while (i + 1 < a.nl && (int)blockIdx.x >= a.wg_off[i + 1]) ++i;
    const int l = a.lid[i], sp = blockIdx.x - a.wg_off[i];
    switch (a.mode[l]) {
#define LNERF_DW_ALL_CASE(I, J, M) \
    case M: dw_run<I, J, true, false>(a, l, sp, lds); break;
        LNERF_DW_PHASED_SHAPES(LNERF_DW_ALL_CASE)
#undef LNERF_DW_ALL_CASE
        default: dw_run<4, 4, false, X6>(a, l, sp, lds); break;
    }
}

void launch_dw_all(int grid, const DwArgs& a, bool x6, hipStream_t s) {
    if (x6) dw_all_kernel<true><<<grid, kWgThreads, 0, s>>>(a);
    else dw_all_kernel<false><<<grid, kWgThreads, 0, s>>>(a);
}

int dw_mode_for(int kt, int nt) {
#define LNERF_DW_MODE_OF(I, J, M) \
    if (kt == I && nt == J) return M;
    LNERF_DW_PHASED_SHAPES(LNERF_DW_MODE_OF)
#undef LNERF_DW_MODE_OF
    return 0;
}

// ---------------------------------------------------------------------------------------------
// weight packing (once per step; weights change every optimizer step)
// ---------------------------------------------------------------------------------------------
struct PackArgs {
    int L;
    int k[kMaxLayers], n[kMaxLayers], kt[kMaxLayers], nt[kMaxLayers];
    int fo[kMaxLayers], bo[kMaxLayers];   // output tiles the kernel's MMA runs (padded, see Layout)
    int w_k, w_n;
    const float* W;
    const float* B;
    float* wf;
    float* wb;
    float* bp;
    unsigned short* w6;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    size_t wf_n[kMaxLayers], wb_n[kMaxLayers], bp_n[kMaxLayers];
    size_t w6f_off[kMaxLayers], w6b_off[kMaxLayers], w6f_n[kMaxLayers], w6b_n[kMaxLayers];
    int planes;                            // bf16 planes packed (3: hi/mid/lo, 1: hi)
};

__global__ void pack_kernel(PackArgs a, int l) {
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const size_t nf = a.wf_n[l], nb = a.wb_n[l], np = a.bp_n[l];
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nf + nb + np;
         e += (size_t)gridDim.x * blockDim.x) {
        if (e < nf) {
            // WF[t][r][jt4][lane][e4] = W[f(t,r,h)][32 jt + lane&31]
            const int nt4 = (a.fo[l] + 3) >> 2;
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
            const int kt4n = (a.bo[l] + 3) >> 2;
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

// bf16x6 planes: forward W6F[t][ks][o][p][lane][j] = plane p of W[f(t, 8ks+j, h)][32o + lane&31],
// backward W6B[t][ks][o][p][lane][j] = plane p of W[32o + lane&31][f(t, 8ks+j, h)] (t = n tile).
__global__ void pack6_kernel(PackArgs a, int l) {
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const size_t nf = a.w6f_n[l], nb = a.w6b_n[l];
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nf + nb;
         e += (size_t)gridDim.x * blockDim.x) {
        const bool fwd = e < nf;
        size_t x = fwd ? e : e - nf;
        const int no = fwd ? a.fo[l] : a.bo[l];
        const int j = x & 7; x >>= 3;
        const int ln = x & 63; x >>= 6;
        const int pl = x % a.planes; x /= a.planes;
        const int o = x % no; x /= no;
        const int ks = x & 1; x >>= 1;
        const int t = (int)x;
        const int f = frag_feature(t, 8 * ks + j, ln >> 5), rr = 32 * o + (ln & 31);
        const int kk = fwd ? f : rr, jj = fwd ? rr : f;
        const float w = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        const __bf16 hi = (__bf16)w;
        const float r = w - (float)hi;
        const __bf16 mid = (__bf16)r;
        const __bf16 lo = (__bf16)(r - (float)mid);
        const __bf16 v = pl == 0 ? hi : (pl == 1 ? mid : lo);
        a.w6[(fwd ? a.w6f_off[l] + e : a.w6b_off[l] + (e - nf))] = __builtin_bit_cast(unsigned short, v);
    }
}

// ---------------------------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------------------------
// Deterministic two-level sum of the per-workgroup partial losses: 256 strided sequential
// sums, then a fixed-order tree in LDS.
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
                v = sum_parts(p, slab, a.nparts[l]);
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

struct Layout {
    int ht;                                   // hidden output tiles, rounded to 1/2/4/8
    int fo[kMaxLayers], bo[kMaxLayers];       // output tiles of each layer's fwd / bwd MMA
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers], bp_off[kMaxLayers];
    size_t wf_n[kMaxLayers], wb_n[kMaxLayers], bp_n[kMaxLayers];
    size_t pack_total;
    size_t w6f_off[kMaxLayers], w6b_off[kMaxLayers], w6f_n[kMaxLayers], w6b_n[kMaxLayers];
    size_t w6_total;                          // u16
    size_t act_off[kMaxLayers], x_off, act_total;
    size_t grad_off[kMaxLayers], grad_total;
    int splits[kMaxLayers], phases[kMaxLayers], mode[kMaxLayers], wg_off[kMaxLayers], dw_grid;
    size_t dwp_off[kMaxLayers], dwp_total, dbp_off[kMaxLayers], dbp_total;
    int num_wg, blocks, rpw;
    // k16 kernel packing (lnerf_k16.hip): 16-wide output tiles, 32-feature k-steps, 3 planes
    int ht16, ks16_f[kMaxLayers], ks16_b[kMaxLayers], to16_f[kMaxLayers], to16_b[kMaxLayers];
    size_t w16f_off[kMaxLayers], w16b_off[kMaxLayers], w16_total;   // u16
    int ht32, to32_f[kMaxLayers], to32_b[kMaxLayers];                // k32: 32-wide output tiles
    size_t w32f_off[kMaxLayers], w32b_off[kMaxLayers];               // u16, in the same region
    size_t b16_total;                                                 // floats
    size_t mask_total;                                                // u64 (k16 ReLU masks)
};

inline int pow2_tiles(int t) { return t <= 1 ? 1 : t <= 2 ? 2 : t <= 4 ? 4 : 8; }

// train = false (render): no slabs or dW partials (the forward-only kernel writes none).
void make_layout(Layout& y, const lnerf_mlp& m, int rays, int S, bool train, int dw_grid,
                 int tile = kTileSamples) {
    const int L = m.num_layers;
    int kt[kMaxLayers], nt[kMaxLayers];
    for (int l = 0; l < L; ++l) {
        kt[l] = (m.k[l] + 31) / 32;
        nt[l] = (m.n[l] + 31) / 32;
    }
    // the kernel runs every hidden layer's forward and every l >= 1 backward with HT output
    // tiles, the head forward with 1 and the dX MMA with pow2(kt0): pack to exactly those
    int mx = 1;
    for (int l = 0; l + 1 < L; ++l) mx = nt[l] > mx ? nt[l] : mx;
    y.ht = pow2_tiles(mx);
    for (int l = 0; l < L; ++l) {
        y.fo[l] = (l < L - 1) ? y.ht : 1;
        y.bo[l] = (l >= 1) ? y.ht : pow2_tiles(kt[0]);
    }
    size_t off = 0;
    for (int l = 0; l < L; ++l) {
        y.wf_n[l] = (size_t)kt[l] * 16 * ((y.fo[l] + 3) / 4) * 256;
        y.wb_n[l] = (size_t)nt[l] * 16 * ((y.bo[l] + 3) / 4) * 256;
        y.bp_n[l] = (size_t)nt[l] * 32;
        y.wf_off[l] = off; off += align_up(y.wf_n[l], 64);
        y.wb_off[l] = off; off += align_up(y.wb_n[l], 64);
        y.bp_off[l] = off; off += align_up(y.bp_n[l], 64);
    }
    y.pack_total = off;
    off = 0;
    for (int l = 0; l < L; ++l) {
        y.w6f_n[l] = (size_t)kt[l] * 2 * y.fo[l] * 3 * 512;
        y.w6b_n[l] = (size_t)nt[l] * 2 * y.bo[l] * 3 * 512;
        y.w6f_off[l] = off; off += align_up(y.w6f_n[l], 512);
        y.w6b_off[l] = off; off += align_up(y.w6b_n[l], 512);
    }
    y.w6_total = off;
    int mx16 = 1;
    for (int l = 0; l + 1 < L; ++l) mx16 = (m.n[l] + 15) / 16 > mx16 ? (m.n[l] + 15) / 16 : mx16;
    y.ht16 = mx16 <= 1 ? 1 : mx16 <= 2 ? 2 : mx16 <= 4 ? 4 : mx16 <= 8 ? 8 : 16;
    const int k0t16 = (m.k[0] + 15) / 16;
    off = 0;
    for (int l = 0; l < L; ++l) {
        y.ks16_f[l] = (m.k[l] + 31) / 32;
        y.ks16_b[l] = (m.n[l] + 31) / 32;
        y.to16_f[l] = (l < L - 1) ? y.ht16 : 1;
        y.to16_b[l] = (l >= 1) ? y.ht16 : (k0t16 <= 1 ? 1 : k0t16 <= 2 ? 2 : k0t16 <= 4 ? 4 : k0t16 <= 8 ? 8 : 16);
        y.w16f_off[l] = off; off += align_up((size_t)y.ks16_f[l] * y.to16_f[l] * 3 * 512, 512);
        y.w16b_off[l] = off; off += align_up((size_t)y.ks16_b[l] * y.to16_b[l] * 3 * 512, 512);
    }
    // k32 (lnerf_k32.hip): per input tile [2 k-steps][32-wide output tiles][planes][1 KiB]
    int mx32 = 1;
    for (int l = 0; l + 1 < L; ++l) mx32 = (m.n[l] + 31) / 32 > mx32 ? (m.n[l] + 31) / 32 : mx32;
    y.ht32 = pow2_tiles(mx32);
    size_t off32 = 0;
    for (int l = 0; l < L; ++l) {
        y.to32_f[l] = (l < L - 1) ? y.ht32 : 1;
        y.to32_b[l] = (l >= 1) ? y.ht32 : pow2_tiles((m.k[0] + 31) / 32);
        y.w32f_off[l] = off32; off32 += align_up((size_t)y.ks16_f[l] * 2 * y.to32_f[l] * 3 * 512, 512);
        y.w32b_off[l] = off32; off32 += align_up((size_t)y.ks16_b[l] * 2 * y.to32_b[l] * 3 * 512, 512);
    }
    y.w16_total = off > off32 ? off : off32;
    y.b16_total = (size_t)L * 256;
    y.rpw = S >= tile ? 1 : tile / S;
    y.num_wg = (rays + y.rpw - 1) / y.rpw;
    y.mask_total = train ? (size_t)y.num_wg * (L > 1 ? L - 1 : 0) * (tile / 16) * 64 : 0;
    y.blocks = y.num_wg * (tile / 32);
    off = 0;
    y.x_off = off; off += (size_t)y.blocks * kt[0] * 1024;
    for (int l = 0; l < L - 1; ++l) { y.act_off[l] = off; off += (size_t)y.blocks * nt[l] * 1024; }
    y.act_total = train ? off : 0;
    off = 0;
    for (int l = 0; l < L; ++l) { y.grad_off[l] = off; off += (size_t)y.blocks * nt[l] * 1024; }
    y.grad_total = train ? off : 0;
    // dW: one launch over every layer, ~dw_grid workgroups (lnerf_ctx_set_option
    // LNERF_OPT_DW_GRID; 512 by default) split between the layers in proportion to the slab bytes
    // each one streams (kt + nt tiles per 32-sample block): the kernel is bandwidth-bound, so
    // equal bytes per workgroup balance it. Phased (small) layers write 4 partials per split.
    const int kDwGrid = dw_grid > 0 ? (dw_grid < 16 ? 16 : dw_grid > 4096 ? 4096 : dw_grid) : kDefaultDwGrid;
    size_t dwp = 0, dbp = 0;
    int tiles_sum = 0;
    for (int l = 0; l < L; ++l) {
        y.mode[l] = dw_mode_for(kt[l], nt[l]);
        tiles_sum += kt[l] + nt[l];
    }
    int wg = 0;
    for (int l = 0; l < L; ++l) {
        int sp = (int)((long long)kDwGrid * (kt[l] + nt[l]) / tiles_sum);
        sp = sp < 1 ? 1 : sp;
        sp = sp > y.blocks ? y.blocks : sp;
        y.splits[l] = sp;
        y.phases[l] = y.mode[l] ? kWaves : 1;
        y.wg_off[l] = wg;
        wg += sp;
        y.dwp_off[l] = dwp;
        dwp += (size_t)sp * y.phases[l] * kt[l] * 32 * nt[l] * 32;
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
    else if (m.n[m.num_layers - 1] > 32) w = "fused path needs a head with <= 32 outputs";
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

static size_t workspace_floats(const lnerf_mlp& m, int rays, int S, bool train, int dw_grid, int tile) {
    Layout y;
    make_layout(y, m, rays, S, train, dw_grid, tile);
    size_t f = align_up(y.pack_total, 64) + align_up((y.w6_total + 1) / 2, 64) +
               align_up(y.act_total, 64) + align_up(y.grad_total, 64) +
               align_up((size_t)y.num_wg, 64) + align_up(y.dwp_total, 64) + align_up(y.dbp_total, 64) +
               64 + align_up((y.w16_total + 1) / 2, 64) + align_up(y.b16_total, 64) +
               align_up(y.mask_total * 2, 64) + 64 +   // + the fp16x3 weight/slab maxima
               align_up((size_t)kMaxLayers * kWmaxParts, 64) +   // + per-block max|W| partials
               (train ? align_up((size_t)m.num_layers * y.num_wg * tile / 2, 64) +   // per-sample shifts
                            align_up((size_t)m.num_layers * y.num_wg * 8, 64) : 0);      // per-wave minima
    return f;
}

// Either tile size (fused_plan runs 64 for k16 under LNERF_K16_W4, 128 otherwise).
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
    Layout y;
    make_layout(y, m, b.rays, b.samples, train, dw_grid, tile);
    p.tile = tile;
    p.L = m.num_layers;
    p.ht = y.ht;
    // The bf16/fp16 planes run on k16 (ReLU masks in HBM, any depth) unless the caller asks for the
    // one-wave kernel pair (LNERF_ONE_WAVE, A/B runs) or the head is wider than one 16-wide tile;
    // only the one-wave kernel keeps its masks in LDS, 1 KiB per hidden layer and wave in the
    // bf16x6 budget: (L-1) <= kMaskTiles / 8. Past that depth it falls back to exact f32 products.
    const bool k16_wanted = !(flags & LNERF_ONE_WAVE) && !(flags & LNERF_MFMA_F32) && m.n[p.L - 1] <= 16;
    const bool bf_ok = k16_wanted || (p.L - 1) <= kMaskTiles(true) / 8;
    p.x6 = (flags & LNERF_MFMA_F32) || !bf_ok ? 0
           : (flags & LNERF_MFMA_BF16)        ? 1
           : (flags & LNERF_MFMA_BF16X6) || !k16_wanted ? 3
                                                        : 2;   // fp16x3 (k16 only)
    for (int l = 0; l < p.L; ++l) {
        p.fo[l] = y.fo[l];
        p.bo[l] = y.bo[l];
        p.w6f_off[l] = y.w6f_off[l];
        p.w6b_off[l] = y.w6b_off[l];
        p.w6f_n[l] = y.w6f_n[l] / 3 * (p.x6 ? p.x6 : 3);   // layout sized for 3 planes
        p.w6b_n[l] = y.w6b_n[l] / 3 * (p.x6 ? p.x6 : 3);
    }
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
        p.dw_mode[l] = y.mode[l];
        p.dw_phases[l] = y.phases[l];
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
    p.w6 = (unsigned short*)(base + off);
    off += align_up((y.w6_total + 1) / 2, 64);
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
    off += 64;
    p.w16 = (unsigned short*)(base + off);
    off += align_up((y.w16_total + 1) / 2, 64);
    p.b16 = base + off;
    off += align_up(y.b16_total, 64);
    p.mask_g = (unsigned long long*)(base + off);
    off += align_up(y.mask_total * 2, 64);
    p.wexp16 = (int*)(base + off);
    p.dw_shift = p.wexp16 + kMaxLayers;
    off += 64;
    p.wmax_part = (int*)(base + off);
    off += align_up((size_t)kMaxLayers * kWmaxParts, 64);
    p.sexp = (signed char*)(base + off);
    if (train) off += align_up((size_t)p.L * y.num_wg * tile / 2, 64);   // L x num_wg x tile x 2 bytes
    p.epart = (int*)(base + off);
    if (train) off += align_up((size_t)p.L * y.num_wg * 8, 64);

    p.x_off = y.x_off;
    p.ht16 = y.ht16;
    for (int l = 0; l < p.L; ++l) {
        p.ks16_f[l] = y.ks16_f[l];
        p.ks16_b[l] = y.ks16_b[l];
        p.to16_f[l] = y.to16_f[l];
        p.to16_b[l] = y.to16_b[l];
        p.w16f_off[l] = y.w16f_off[l];
        p.w16b_off[l] = y.w16b_off[l];
        p.to32_f[l] = y.to32_f[l];
        p.to32_b[l] = y.to32_b[l];
        p.w32f_off[l] = y.w32f_off[l];
        p.w32b_off[l] = y.w32b_off[l];
    }
    p.ht32 = y.ht32;
    p.k16 = k16_wanted && k16_supported(p) ? 1 : 0;
    // k32 (one wave per SIMD, 32 samples per wave) in place of k16 with LNERF_K32
    p.k32 = p.k16 && (flags & LNERF_K32) && k32_supported(p) ? 1 : 0;
    if (p.k32) p.k16 = 0;
    // dW: dw16_kernel after k16 / k32 (it reads their slab layouts and split planes); the
    // one-wave kernel pairs with dw_all_kernel. One partial per split.
    p.dw16 = p.k16 || p.k32;
    if (p.dw16)
        for (int l = 0; l < p.L; ++l) p.dw_phases[l] = 1;
}

void fused_plan(FusedPlan& p, const lnerf_mlp& m, const lnerf_batch& b, void* ws_base, int flags,
                bool train, int dw_grid) {
    fused_plan_tile(p, m, b, ws_base, flags, train, dw_grid, kTileSamples);
    // k16 on 4-wave, 64-sample workgroups (two per CU) with LNERF_K16_W4, where whole rays fit 64
    // samples and the ring fits 80 KiB (fp16x3 / plain bf16). Measured slower than the 8-wave
    // workgroup at cfg3 (the second workgroup doubles the weight stream's LDS-DMA).
    if (p.k16 && p.x6 != 3 && b.samples <= 64 && (flags & LNERF_K16_W4))
        fused_plan_tile(p, m, b, ws_base, flags, train, dw_grid, 64);
    p.head_fit = (flags & LNERF_HEAD_FIT) ? 1 : 0;
}

static void launch_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s) {
    PackArgs a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.k[l] = p.k[l];
        a.n[l] = p.n[l];
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.fo[l] = p.fo[l];
        a.bo[l] = p.bo[l];
        a.wf_off[l] = p.wf_off[l];
        a.wb_off[l] = p.wb_off[l];
        a.bp_off[l] = p.bp_off[l];
        // the x6 path reads only the biases of the f32 region
        a.wf_n[l] = p.x6 ? 0 : (size_t)p.kt[l] * 16 * ((p.fo[l] + 3) / 4) * 256;
        a.wb_n[l] = p.x6 ? 0 : (size_t)p.nt[l] * 16 * ((p.bo[l] + 3) / 4) * 256;
        a.bp_n[l] = (size_t)p.nt[l] * 32;
        a.w6f_off[l] = p.w6f_off[l];
        a.w6b_off[l] = p.w6b_off[l];
        a.w6f_n[l] = p.w6f_n[l];
        a.w6b_n[l] = p.w6b_n[l];
    }
    a.w_k = p.w_k;
    a.w_n = p.w_n;
    a.W = ws;
    a.B = bs;
    a.wf = p.wf;
    a.wb = p.wb;
    a.bp = p.bp;
    a.w6 = p.w6;
    a.planes = p.x6;
    for (int l = 0; l < p.L; ++l) {
        if (p.x6) {
            // biases (and nothing else) through pack_kernel: bp lands after wf_n + wb_n = 0
            const size_t n6 = a.w6f_n[l] + a.w6b_n[l];
            pack6_kernel<<<(unsigned)((n6 + 255) / 256), 256, 0, s>>>(a, l);
        }
        const size_t n = a.wf_n[l] + a.wb_n[l] + a.bp_n[l];
        pack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, l);
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
    if (p.x6) {
        for (int l = 0; l < p.L; ++l) {
            a.wf_off[l] = p.w6f_off[l];
            a.wb_off[l] = p.w6b_off[l];
        }
    }
    a.k0 = p.k[0];
    a.wf = p.wf;
    a.wb = p.wb;
    a.w6 = p.w6;
    a.bp = p.bp;
    a.act = p.act;
    a.x_off = p.x_off;
    a.grad = p.grad;
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
    return a;
}

static void launch_fused(const FusedPlan& p, const FusedArgs& fa, hipStream_t s) {
#define LNERF_FUSED_LAUNCH(HT)                                                         \
    if (p.x6 == 3) fused_fwd_bwd_kernel<HT, 3><<<p.num_wg, kWgThreads, 0, s>>>(fa);    \
    else if (p.x6 == 1) fused_fwd_bwd_kernel<HT, 1><<<p.num_wg, kWgThreads, 0, s>>>(fa); \
    else fused_fwd_bwd_kernel<HT, 0><<<p.num_wg, kWgThreads, 0, s>>>(fa);
    switch (p.ht) {
        case 1: LNERF_FUSED_LAUNCH(1) break;
        case 2: LNERF_FUSED_LAUNCH(2) break;
        case 4: LNERF_FUSED_LAUNCH(4) break;
        default: LNERF_FUSED_LAUNCH(8) break;
    }
#undef LNERF_FUSED_LAUNCH
}

#if LNERF_PROF
static void prof_report(const FusedPlan& p, hipStream_t s) {
    unsigned long long h[16] = {};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof(h));
    const char* names[] = {"pe", "fwd_mma", "barrier_wait", "composite", "bwd_mma", "tail",
                           "total", "fwd_epilogue", "bwd_epilogue", "chunk_prologue", "steps",
                           "last_store", "layer_prologue", "chunk_barrier"};
    const double waves = (double)p.num_wg * kWaves;
    fprintf(stderr, "LNERF_PROF per-wave cycles:");
    for (int i = 0; i < kPfN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / waves);
    fprintf(stderr, "\n");
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));
}
#endif

void fused_train_step(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                      float seed, int flags, const lnerf_outputs& out, hipStream_t s,
                      hipEvent_t* ev) {
    const bool seed_loss = (flags & LNERF_SEED_LOSS) != 0;
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ev[i], s);
    };
    mark(0);
    if (p.k32) k32_pack(p, ws, bs, s);
    else if (p.k16) k16_pack(p, ws, bs, s);
    else launch_pack(p, ws, bs, s);
    mark(1);
    if (p.k32) {
        k32_launch(p, b, seed_loss ? 1.0f : seed, out, true, s);
    } else if (p.k16) {
        k16_launch(p, b, seed_loss ? 1.0f : seed, out, true, s);
    } else {
        FusedArgs fa = make_fused_args(p, b, seed_loss ? 1.0f : seed, out, true);
        launch_fused(p, fa, s);
    }
#if LNERF_PROF
    prof_report(p, s);
#endif
    mark(2);
    k1_reduce_launch(p, out.loss, s);
    mark(3);
    DwArgs da{};
    da.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        da.kt[l] = p.kt[l];
        da.nt[l] = p.nt[l];
        da.a_off[l] = (l == 0) ? p.x_off : p.act_off[l - 1];
        da.g_off[l] = p.grad_off[l];
        da.splits[l] = p.dw_splits[l];
        da.mode[l] = p.dw_mode[l];
        da.dwp_off[l] = p.dwp_off[l];
        da.dbp_off[l] = p.dbp_off[l];
    }
    da.act = p.act;
    da.grad = p.grad;
    da.blocks = p.blocks;
    da.dw_part = p.dw_part;
    da.db_part = p.db_part;
    da.nl = p.L;
    for (int l = 0; l < p.L; ++l) {
        da.lid[l] = l;
        da.wg_off[l] = p.dw_split_off[l];
    }
    da.wg_off[p.L] = p.dw_grid;
    if (p.dw16) dw16_launch(p, s);
    else launch_dw_all(p.dw_grid, da, p.x6 != 0, s);
    mark(4);
    ReduceArgs ra{};
    ra.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        ra.k[l] = p.k[l];
        ra.n[l] = p.n[l];
        ra.kt[l] = p.kt[l];
        ra.nt[l] = p.nt[l];
        ra.nparts[l] = p.dw_splits[l] * p.dw_phases[l];
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
        if (out.d_target)
            k_scale_by_scalar(out.d_target, (size_t)p.rays * (p.head_fit ? p.n[p.L - 1] : 3), p.loss_total, s);
        if (out.d_x) k_scale_by_scalar(out.d_x, (size_t)p.R * p.k[0], p.loss_total, s);
    }
    mark(5);
}

void fused_render(const FusedPlan& p, const float* ws, const float* bs, const lnerf_batch& b,
                  const lnerf_outputs& out, hipStream_t s) {
    if (p.k32) {
        k32_pack(p, ws, bs, s);
        k32_launch(p, b, 1.0f, out, false, s);
    } else if (p.k16) {
        k16_pack(p, ws, bs, s);
        k16_launch(p, b, 1.0f, out, false, s);
    } else {
        launch_pack(p, ws, bs, s);
        FusedArgs fa = make_fused_args(p, b, 1.0f, out, false);
        launch_fused(p, fa, s);
    }
    loss_reduce_kernel<<<1, 256, 0, s>>>(p.loss_part, p.num_wg, p.loss_total, out.loss);
}

}  // namespace lnerf
