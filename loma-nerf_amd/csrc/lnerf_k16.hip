// lnerf_k16.hip -- k1 on wave pairs: the fused PE + MLP + compositing + reverse chain with two
// waves per SIMD (v_mfma_f32_16x16x32_f16 / _bf16), the default fused kernel for every MFMA
// precision but exact f32 (fp16x3 default, bf16x6, plain bf16 for inference).
//
// Same work and outputs as fused_fwd_bwd_kernel (lnerf_fused.hip; reference scripts/nerf.py:1-304
// and its rev_diff, train_nerf.py:325/395), re-tiled so that a CU holds TWO waves per SIMD:
//  * one 512-thread workgroup (8 waves) per 128-sample tile of whole rays; each wave owns 16
//    samples, so a 256-wide layer is 16 accumulator tiles x 4 registers = 64 registers for the
//    activations and 64 for the accumulators, and the kernel fits 256 registers per lane;
//  * the activations stay in the transposed accumulator layout (lane = sample l & 15, registers
//    = features 4(l >> 4) + i of each 16-feature tile), which is the next layer's B operand after
//    a fixed permutation of the contraction order (phi below) baked into the weight packing;
//  * the weights of one k-step (32 input features x every output tile, in the PL planes of the
//    split: fp16 hi/lo for fp16x3, bf16 hi/mid/lo for bf16x6, one plane for plain bf16) stream
//    through a 3-slot LDS ring by LDS-DMA (one chunk in flight while one is computed; the late
//    waves of the staggered pairs still read the previous one), one barrier per k-step;
//  * while one wave of a SIMD issues its LDS reads, operand splits, slab stores, DMA pieces or
//    epilogue, its partner's MFMAs keep the matrix core busy -- the latency hiding that the
//    one-wave-per-SIMD kernel had to hand-schedule.
// The slabs (post-ReLU activations A_l, gradients G_l) are written in the layout the dW kernel
// reads (lnerf_fused.hip slab_off): a wave owns one 16-sample half of a 32-sample block.
#include "lnerf_composite.h"
#include "lnerf_internal.h"

#include <stddef.h>
#include <stdio.h>

#include <utility>

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kTile = comp::kTileSamples;     // 128 samples per workgroup
constexpr int kMaxChunks = 2 * kMaxLayers * 8 + 2;   // <= 2 passes x 8 k-steps per layer + 2 end
constexpr int kMaxT = 16;                     // 16-feature tiles per 256-wide layer
constexpr int kSlotBytes = kMaxT * 3 * 1024;  // one k-step of a 256-output layer, 3 planes
// ring slot of a PL-plane kernel: one k-step of a 256-output layer
template <int PL>
constexpr int slot_bytes() { return kMaxT * PL * 1024; }
// Staggered wave pairs (default): waves 0-3 ("early") meet the per-chunk barrier at the end of
// a chunk, waves 4-7 ("late", each the SIMD partner of an early wave) in its middle, so the two
// waves of a SIMD run their chunk prologues (DMA issue, slab stores, operand split, first
// fragment reads) half a chunk apart, each under its partner's MFMAs. The ring then needs 3
// slots: in one barrier period the late waves still read the previous chunk's second half while
// every wave reads the current chunk and the next one lands (one chunk in flight; every wave
// issues 1/8 of its pieces right after its own prologue).
#ifndef LNERF_K16_STAGGER
#define LNERF_K16_STAGGER 1
#endif
constexpr bool kStagger = LNERF_K16_STAGGER != 0;
#ifndef LNERF_K16_AHEAD
#define LNERF_K16_AHEAD 1
#endif
#ifndef LNERF_K16_LOADERS
#define LNERF_K16_LOADERS 4
#endif
constexpr int kLoaders = kStagger ? 8 : LNERF_K16_LOADERS;   // waves that issue the weight DMA
// timing experiments only (wrong results): drop the slab stores / the weight DMA after chunk 2
#ifndef LNERF_K16_NOSTORE
#define LNERF_K16_NOSTORE 0
#endif
#ifndef LNERF_K16_NODMA
#define LNERF_K16_NODMA 0
#endif
// unstaggered: chunks in flight while one computes: 1 (a 2-slot ring) or 2 (a 3-slot ring;
// measured slower)
constexpr int kAhead = kStagger ? 1 : LNERF_K16_AHEAD;
static_assert(kAhead == 1 || kAhead == 2, "the ring has room for two chunks in flight at most");
constexpr int kSlots = kStagger ? 3 : kAhead + 1;   // ring slots
constexpr int kOffComp = 3 * kSlotBytes;      // room for the deepest ring
constexpr int kCompBytes = 2688 * 4;          // composite_tile's scratch (comp[0, 2688))
constexpr int kOffRay = kOffComp + kCompBytes;
constexpr int kOffBias = kOffRay + kTile * 4;
constexpr int kLdsBytes = kOffBias + 3 * 256 * 4;   // + a 3-slot ring of layer biases
static_assert(kLdsBytes + 1024 <= 160 * 1024, "LDS budget (+1 KiB for the profiling build)");

struct K16Args {
    int L;
    int ks_f[kMaxLayers], ks_b[kMaxLayers];   // k-steps (32 input features) per pass
    int to_f[kMaxLayers], to_b[kMaxLayers];   // 16-wide output tiles per pass
    int kt[kMaxLayers], nt[kMaxLayers];       // 32-wide slab tiles of each layer's input/output
    int k0;
    const unsigned short* w16;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];   // u16 offsets
    const float* b16;                                // [L][256] zero-padded biases
    unsigned long long* mask_g;                      // [wg][L-1][wave][lane] ReLU mask bits
    // the chunk stream (k16_launch): per chunk {u16 offset in w16, (bytes / 1024) | (bias layer + 1)
    // << 16}, zero past the end. Read with scalar loads from the kernel-argument segment.
    unsigned chunk_tab[2 * kMaxChunks];
    float* act;
    size_t act_off[kMaxLayers];
    size_t x_off;
    float* grad;
    size_t grad_off[kMaxLayers];
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
    int planes;
    const int* wexp;   // PL = 2: per-layer max|W| bits of the packed fp16 weight planes (wshift_of)
    float* smax;       // PL = 2, training: per-wave slab maxima [2L][num_wg * 8]: slab l the input
                       // of layer l (X, A_l-1), slab L + l G_l
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---- optional in-kernel phase timing (-DLNERF_PROF=1, never in the product build): per-wave
// s_memtime deltas, lane 0 accumulating in LDS, summed into g_k16_prof at the end.
#ifndef LNERF_PROF
#define LNERF_PROF 0
#endif
#if LNERF_PROF
enum { kPfPE, kPfFwd, kPfFwdEpi, kPfBar, kPfComp, kPfBwd, kPfBwdEpi, kPfTail, kPfTotal, kPfVm, kPfReal, kPfN };
__device__ unsigned long long g_k16_prof[16];
__device__ __forceinline__ unsigned long long* prof_slots() {
    __shared__ unsigned long long sl[kWaves][16];
    return &sl[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0];
}
#define PROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(cat, t0) \
    do { if ((threadIdx.x & 63) == 0) prof_slots()[cat] += __builtin_amdgcn_s_memtime() - (t0); } while (0)
#else
#define PROF_T(v)
#define PROF_ADD(cat, t0)
#endif

// Input feature of k-step s held in element j of a lane in lane group g (the B operand's
// k = 8g + j): tile 2s + (j >> 2), register j & 3 of that lane.
__host__ __device__ __forceinline__ int phi(int s, int g, int j) {
    return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
}

// Chunk `ci` of the kernel's stream (forward passes 0..L-1, then (training) backward L-1..1 and
// backward 0 when d_x is wanted), from K16Args::chunk_tab through the kernel-argument segment
// pointer: a scalar load at a dynamic offset (indexing the by-value argument itself would copy
// it to scratch; a vector load would sit in vmcnt behind the in-flight DMA).
struct ChunkT {
    const unsigned short* src;   // nullptr: past the last chunk
    int bytes;
    int bias;                    // layer whose biases ride with this chunk, -1: none
};

__device__ __forceinline__ ChunkT chunk_at(const K16Args& a, int ci) {
    const __attribute__((address_space(4))) unsigned* t =
        (const __attribute__((address_space(4))) unsigned*)((const __attribute__((address_space(4))) char*)
                                                                __builtin_amdgcn_kernarg_segment_ptr() +
                                                            offsetof(K16Args, chunk_tab)) + 2 * ci;
    const unsigned off = t[0], e = t[1];
    const int bytes = (int)(e & 0xFFFFu) * 1024;
    return ChunkT{bytes ? a.w16 + off : nullptr, bytes, (int)(e >> 16) - 1};
}

// LDS-DMA (global_load_lds_dwordx4) of a chunk into its ring slot: 8 KiB per round of the
// workgroup, each wave instruction 1 KiB (lane-linear); the last wave also stages the biases a
// first forward chunk carries (bias ring slot l % 3). Returns the instructions this wave issued
// (what a later vmcnt must leave outstanding).
__device__ __forceinline__ int dma_chunk(const K16Args& a, const ChunkT& c, unsigned char* dst,
                                         float* bias_ring) {
    const int tid = threadIdx.x, wave = wave_id();
    int n = 0;
    if (!c.src) return 0;
    // loader waves 0..kLoaders-1 (waves w and w+4 share a SIMD: with 4 loaders each SIMD keeps
    // one wave free of DMA issue to feed the matrix core)
    if (wave >= kLoaders) return 0;
    for (int off = wave * 1024; off < c.bytes; off += kLoaders * 1024) {
        const char* g = (const char*)c.src + off + (tid & 63) * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(dst + off), 16, 0, 0);
        ++n;
    }
    if (c.bias >= 0 && wave == kLoaders - 1) {
        const float* g = a.b16 + (size_t)c.bias * 256 + (tid & 63) * 4;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(bias_ring + (c.bias % 3) * 256),
                                         16, 0, 0);
        ++n;
    }
    return n;
}

// The chunk the next k-step reads has landed (this wave's pieces: vector-memory loads return in
// issue order, so at most `pending` outstanding -- the pieces of the chunk after it, issued
// later -- means every older load is done, whatever the stores in between), then s_barrier:
// every wave's pieces are in LDS and every wave is done with the slot the next DMA overwrites.
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt(n) for a wave-uniform n (clamped to the 6-bit counter's 63)
template <int... N>
__device__ __forceinline__ void vm_wait_n(int n, std::integer_sequence<int, N...>) {
    n = n > 63 ? 63 : n;
    ((n == N ? vm_wait<N>() : void()), ...);
}
// pending < 0: this wave has no DMA piece to wait for (only the barrier)
__device__ __forceinline__ void dma_barrier(int pending) {
    PROF_T(t0);
    asm volatile("" ::: "memory");
    if (pending == 0) vm_wait<0>();
    else if (pending == 8) vm_wait<8>();   // kAhead = 1: a loader wave behind its slab stores
    else if (pending > 0) vm_wait_n(pending, std::make_integer_sequence<int, 64>{});
    PROF_ADD(kPfVm, t0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    PROF_ADD(kPfBar, t0);
}

__device__ __forceinline__ fx4 mfma16(const bf8& a, const bf8& b, fx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// the same fragments as fp16 (PL = 2: the fp16x3 planes)
__device__ __forceinline__ fx4 mfma16h(const bf8& a, const bf8& b, fx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
                                                  0);
}

// fp16x3 (PL = 2): x * 2^e = hi + lo, round-to-nearest fp16 of each (the remainder is exact in
// f32); |x 2^e - hi - lo| <= 2^-22 |x 2^e|. The exponent shift keeps the operand's largest value
// in [2^13, 2^14), inside fp16's range (the 3xTF32 split of CUTLASS, on fp16 pieces).
__device__ __forceinline__ void split_h(float xs, _Float16& h, _Float16& l) {
    h = (_Float16)xs;
    l = (_Float16)(xs - (float)h);
}

// the exponent shift ew of a layer from its max|W| bits: max|W| 2^ew in [2^13, 2^14) (0 for an
// all-zero or non-finite layer) -- the weight-side half of the fp16x3 scaling
__device__ __forceinline__ int wshift_of(int maxbits) {
    const float mx = __int_as_float(maxbits);
    if (!(mx > 0.0f) || !(mx < __builtin_inff())) return 0;
    int e;
    (void)__builtin_frexpf(mx, &e);
    return 14 - e;
}

// The same split for a pair (x0, x1) packed as two f16 per register, with v_fma_mix: hi =
// round_f16(x sc) and lo = round_f16(x sc - hi) are fused multiply-adds with one rounding to f16
// (x sc is exact, sc a power of two; x sc - hi is exact), two instructions per value instead of
// scale, convert, widen, subtract and convert.
__device__ __forceinline__ void split_h2(float x0, float x1, float sc, unsigned& hi, unsigned& lo) {
    asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=&v"(hi) : "v"(x0), "v"(sc));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(hi) : "v"(x1), "v"(sc));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(x0), "v"(sc), "v"(hi));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "+v"(lo) : "v"(x1), "v"(sc), "v"(hi));
}

// x = hi + mid + lo (round-to-nearest bf16 of each remainder; every remainder is exact in f32)
__device__ __forceinline__ void split_x(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

// Slab tile store: the 8 features of k-step s that a lane holds (rows phi - 32 s of the
// 32-feature tile) for its sample n, into [32 rows][16 samples] of this wave's half. Each wave
// instruction writes 4 runs of 64 B.
__device__ __forceinline__ void store_slab_step(float* __restrict__ dst, const fx4& t0, const fx4& t1) {
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int row = 16 * (j >> 2) + 4 * g + (j & 3);
        __builtin_nontemporal_store(j < 4 ? t0[j] : t1[j - 4], dst + row * 16 + n);
    }
}

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 with an immediate offset, outside the compiler's waitcnt bookkeeping: the
// matching lgkm_wait below is the only wait, so reads of later tiles stay in flight.
template <int OFF>
__device__ __forceinline__ bf8 ds_read_at(unsigned addr) {
    bf8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}

// s_waitcnt lgkmcnt(N) that the fragments depend on (no use can be scheduled above it). LDS
// reads return in order, so at most N outstanding means every older read has landed.
template <int N>
__device__ __forceinline__ void lgkm_wait(bf8 (&w)[3]) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]) : "n"(N));
}

constexpr int kDist = 2;   // weight tiles read ahead of the one the MFMAs consume

// timing experiments only (wrong results): read one plane per tile / skip the operand split
#ifndef LNERF_K16_HALFLDS
#define LNERF_K16_HALFLDS 0
#endif
#ifndef LNERF_K16_NOSPLIT
#define LNERF_K16_NOSPLIT 0
#endif
template <int PL, int O>
__device__ __forceinline__ void read_tile(unsigned base, bf8 (&w)[3]) {
    w[0] = ds_read_at<(O * PL + 0) * 1024>(base);
    if constexpr (PL >= 2 && LNERF_K16_HALFLDS) w[1] = w[0];
    else if constexpr (PL >= 2) w[1] = ds_read_at<(O * PL + 1) * 1024>(base);
    if constexpr (PL == 3) w[2] = ds_read_at<(O * PL + 2) * 1024>(base);
}

// Output tile O of one k-step: issue the reads of tile O + kDist, wait for tile O's (leaving
// the younger ones in flight), six MFMAs (small terms first).
template <int NTO, int PL, int O>
__device__ __forceinline__ void tile_step(unsigned base, bf8 (&w)[kDist + 1][3], const bf8& bh,
                                          const bf8& bm, const bf8& bl, fx4 (&out)[kMaxT]) {
    if constexpr (O + kDist < NTO) read_tile<PL, O + kDist>(base, w[(O + kDist) % (kDist + 1)]);
    constexpr int ahead = (NTO - 1 - O) < kDist ? (NTO - 1 - O) : kDist;
    bf8(&c)[3] = w[O % (kDist + 1)];
    lgkm_wait<ahead * (LNERF_K16_HALFLDS && PL == 2 ? 1 : PL)>(c);
    fx4 acc = out[O];
    if constexpr (PL == 2) {
        // fp16x3: small terms first (w_hi x_lo, w_lo x_hi), then w_hi x_hi; (bh, bm) = (x_hi, x_lo)
        acc = mfma16h(c[0], bm, acc);
        acc = mfma16h(c[1], bh, acc);
        acc = mfma16h(c[0], bh, acc);
    } else if constexpr (PL == 3) {
        acc = mfma16(c[0], bl, acc);
        acc = mfma16(c[1], bm, acc);
        acc = mfma16(c[2], bh, acc);
        acc = mfma16(c[1], bh, acc);
        acc = mfma16(c[0], bm, acc);
        acc = mfma16(c[0], bh, acc);
    } else {
        acc = mfma16(c[0], bh, acc);
    }
    out[O] = acc;
}

// tiles B, B+1, ... of one k-step
template <int NTO, int PL, int B, int... O>
__device__ __forceinline__ void tile_steps(std::integer_sequence<int, O...>, unsigned base,
                                           bf8 (&w)[kDist + 1][3], const bf8& bh, const bf8& bm,
                                           const bf8& bl, fx4 (&out)[kMaxT]) {
    (tile_step<NTO, PL, B + O>(base, w, bh, bm, bl, out), ...);
}

// The B operand planes of k-step s (the lane's 8 input features phi(s, g, 0..7) of its sample):
// bf16x6 hi/mid/lo, fp16x3 hi/lo (x 2^ex), or plain bf16.
template <int PL>
__device__ __forceinline__ void make_b(const fx4 (&in)[kMaxT], int s, int ex, bf8& bh, bf8& bm, bf8& bl) {
    if constexpr (PL == 2 && !LNERF_K16_NOSPLIT) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        u4 hv, lv;
        const float sc = __builtin_ldexpf(1.0f, ex);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const fx4& t = in[2 * s + (q >> 1)];
            unsigned h2, l2;
            split_h2(t[2 * (q & 1)], t[2 * (q & 1) + 1], sc, h2, l2);
            hv[q] = h2;
            lv[q] = l2;
        }
        bh = __builtin_bit_cast(bf8, hv);
        bm = __builtin_bit_cast(bf8, lv);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float x = j < 4 ? in[2 * s][j] : in[2 * s + 1][j - 4];
            if (PL == 3) {
                __bf16 h, m, l;
                split_x(x, h, m, l);
                bh[j] = h;
                bm[j] = m;
                bl[j] = l;
            } else if (PL == 2) {   // LNERF_K16_NOSPLIT timing experiment
                bh[j] = __builtin_bit_cast(__bf16, (_Float16)x);
                bm[j] = bh[j];
            } else {
                bh[j] = (__bf16)x;
            }
        }
    }
}

// One pass (a layer's forward or backward MMA): out[o] += sum over the pass's k-steps of
// Wpack[s][o] (x) in[2s..2s+1], NTO output tiles. Chunk ci is read from ring slot ci % kSlots
// while chunk ci+kAhead (issued here) lands. `slab` (nullable)
// receives the input tiles (the A_{l-1} or G_l slab of this wave's half-block).
template <int NTO, int PL>
__device__ __forceinline__ void k16_pass(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                         float* bias_ring, const fx4 (&in)[kMaxT], fx4 (&out)[kMaxT],
                                         float* __restrict__ slab, int ex = 0) {
    const int lane = threadIdx.x & 63;
    constexpr int kSB = slot_bytes<PL>();
    bf8 bh = {}, bm = {}, bl = {};
    make_b<PL>(in, 0, ex, bh, bm, bl);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        if (s < ks) {
            const unsigned base = lds_addr(ring + (ci % kSlots) * kSB) + lane * 16;
            // DMA of chunk ci+AHEAD first (its table entry is a scalar load the compiler waits for
            // with lgkmcnt(0), which would also wait for the fragment reads), then the first
            // weight tiles, in flight while the slab stores and the operand split issue
            // The barrier waits for this wave's pieces of chunk ci+1 only: the vector-memory
            // operations younger than them stay in flight -- this k-step's 8 slab stores and
            // (kAhead = 2) chunk ci+2's pieces. A wave that issues no DMA does not wait at all
            // (its slab stores need no completion before the barrier).
            // (register staging -- 16-B loads after the prologue, ds_write_b128 before the barrier
            // -- measured slower: 1.52 vs 1.40 ms)
            const int issued = (LNERF_K16_NODMA && ci >= 2)
                                   ? 0
                                   : dma_chunk(a, chunk_at(a, ci + kAhead),
                                               ring + ((ci + kAhead) % kSlots) * kSB, bias_ring);
            asm volatile("" ::: "memory");   // the slab stores stay younger than the pieces
            const int nst = (slab && !LNERF_K16_NOSTORE) ? 8 : 0;
            const int pending = wave_id() >= kLoaders ? -1
                                : kAhead == 1       ? (issued ? nst : -1)
                                                    : issued + nst;
            const bool late = kStagger && wave_id() >= 4;
            bf8 w[kDist + 1][3];
            read_tile<PL, 0>(base, w[0]);
            if constexpr (NTO > 1) read_tile<PL, 1>(base, w[1]);
            // (an LDS-transposed form -- 8 ds_write_b32 + 2 ds_read_b128 + 2 dwordx4 stores --
            // measured slower: 2.13-2.18 vs 2.02-2.03 ms)
            if (slab && !LNERF_K16_NOSTORE) store_slab_step(slab + s * 1024, in[2 * s], in[2 * s + 1]);
            static_assert(kDist == 2, "the prologue reads kDist tiles");
            // first half of the output tiles, [late waves: barrier], the next k-step's operand
            // split (off the next prologue's critical path), second half, [early: barrier]
            constexpr int H = (NTO + 1) / 2;
            tile_steps<NTO, PL, 0>(std::make_integer_sequence<int, H>{}, base, w, bh, bm, bl, out);
            if (late) dma_barrier(pending);
            bf8 nh = {}, nm = {}, nl = {};
            if (s + 1 < ks) make_b<PL>(in, s + 1 < 8 ? s + 1 : 0, ex, nh, nm, nl);
            tile_steps<NTO, PL, H>(std::make_integer_sequence<int, NTO - H>{}, base, w, bh, bm, bl, out);
            if (!late) dma_barrier(pending);
            bh = nh;
            bm = nm;
            bl = nl;
            ++ci;
        }
    }
}

template <int PL>
__device__ __forceinline__ void k16_pass_n(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                           float* bias_ring, int nto, const fx4 (&in)[kMaxT],
                                           fx4 (&out)[kMaxT], float* slab, int ex) {
    if (nto <= 1) k16_pass<1, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 2) k16_pass<2, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 4) k16_pass<4, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 8) k16_pass<8, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else k16_pass<16, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
}

// PL = 2: the per-sample max|x| of a pass's input (lanes n, n + 16, n + 32, n + 48 hold sample
// n's features), the basis of its exponent shift.
template <int PL>
__device__ __forceinline__ float sample_max(const fx4 (&in)[kMaxT]) {
    if constexpr (PL != 2) return 0.0f;
    float m = 0.0f;
#pragma unroll
    for (int o = 0; o < kMaxT; ++o)
#pragma unroll
        for (int i = 0; i < 4; ++i) m = __builtin_fmaxf(m, __builtin_fabsf(in[o][i]));
    m = __builtin_fmaxf(m, __shfl_xor(m, 16));
    return __builtin_fmaxf(m, __shfl_xor(m, 32));
}

// the exponent shift ex with m 2^ex in [2^13, 2^14); 0 for m = 0 (or non-finite)
__device__ __forceinline__ int shift_of(float m) {
    if (!(m > 0.0f) || !(m < __builtin_inff())) return 0;
    int e;
    (void)__builtin_frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
    return 14 - e;
}

// PL = 2, training: the wave's max of a slab, one plain store per wave and slab into
// smax_part[slab][global wave] (k1_reduce_kernel folds them into dw16's layer-wide exponent
// shifts; an atomic per wave on 2L shared words measured 2.2x slower for the whole kernel).
// Issued before the pass's first DMA, so it is older than every piece a dma_barrier waits for.
__device__ __forceinline__ void slab_max(float* part, int slab, float m) {
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) m = __builtin_fmaxf(m, __shfl_xor(m, d));
    if ((threadIdx.x & 63) == 0)
        part[(size_t)slab * gridDim.x * kWaves + blockIdx.x * kWaves + (threadIdx.x >> 6)] = m;
}

// The layer's biases in the accumulator layout (fx4 = 4 consecutive features of a lane group),
// from its bias ring slot: ds_read_b128 outside the compiler's waitcnt bookkeeping (a plain LDS
// read would make it wait vmcnt(0) for the in-flight weight DMA), one dependent wait per tile.
template <int N>
__device__ __forceinline__ void lgkm_wait4(fx4& v) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}
template <int OFF>
__device__ __forceinline__ fx4 ds_read_f4(unsigned addr) {
    fx4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
template <int NT, int... O>
__device__ __forceinline__ void bias_read(std::integer_sequence<int, O...>, unsigned addr, fx4 (&b)[kMaxT]) {
    ((b[O] = ds_read_f4<O * 64>(addr)), ...);
}
template <int NT, int... O>
__device__ __forceinline__ void bias_wait(std::integer_sequence<int, O...>, fx4 (&b)[kMaxT]) {
    (lgkm_wait4<NT - 1 - O>(b[O]), ...);
}

__device__ __forceinline__ void zero_tiles(fx4 (&t)[kMaxT]) {
#pragma unroll
    for (int o = 0; o < kMaxT; ++o) t[o] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
}

// HT: 16-wide output tiles of every hidden layer (1/2/4/8/16); PL: operand planes (3 = bf16x6,
// 2 = fp16x3, both fp32-class; 1 = plain bf16, inference).
template <int HT, int PL>
__global__ void __launch_bounds__(kThreads, 1) k16_fwd_bwd_kernel(K16Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kLdsBytes];
    unsigned char* ring = lds;
    float* comp = (float*)(lds + kOffComp);
    float* rayloss = (float*)(lds + kOffRay);
    float* bias_ring = (float*)(lds + kOffBias);

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), g = lane >> 4, n = lane & 15;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
    const int ls = wave * 16 + n;                      // local sample 0..127
    const int gs = wg * tile_samples + ls;             // global sample row (ray*S + j)
    const bool valid = (ls < tile_samples) && (gs < a.R);
    const size_t blk = (size_t)wg * 4 + (wave >> 1);   // 32-sample slab block
    const int half = wave & 1;
    const bool st = a.want_grad != 0;
#if LNERF_PROF
    if (lane < 16) prof_slots()[lane] = 0;
    PROF_T(t_start);
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
#endif

    fx4 act[kMaxT], out[kMaxT];
    zero_tiles(act);
    // PL = 2: layer l's weight exponent shift in lane l (read with readlane per pass); a pass's
    // accumulators carry 2^(ex + ew), removed exactly (powers of two) in its epilogue
    const int wexp_lane = (PL == 2 && lane < a.L) ? wshift_of(a.wexp[lane]) : 0;
    auto unscale = [&](int l, int ex) -> int {
        return PL == 2 ? -(ex + __builtin_amdgcn_readlane(wexp_lane, l)) : 0;
    };

    // ---- layer-0 input in the accumulator layout, through a per-wave LDS scratch (the ring is
    // free before the first DMA). POINTS/RAYS with k0 <= 64: one float64 sincos per (sample,
    // coordinate, frequency) (pos_encoding.py:54-66); otherwise tile by tile.
    const int tile_base = wg * tile_samples + wave * 16;
    if (a.input_mode != LNERF_INPUT_ENCODED && a.k0 <= 64) {
        constexpr int kStride = 65;
        float* pe = (float*)ring + wave * (16 * kStride);
        const int F = a.F, per = 3 * (F + 1);
        for (int it = lane; it < 16 * per; it += 64) {
            const int sl = it / per, rem = it - sl * per, c = rem % 3, q = rem / 3;
            const bool vs = (wave * 16 + sl < tile_samples) && (tile_base + sl < a.R);
            const double xc = vs ? comp::sample_coord(a, tile_base + sl, c) : 0.0;
            if (q == 0) {
                pe[sl * kStride + c] = (float)xc;
            } else {
                double sn, cs;
                sincos(ldexp(xc, q - 1), &sn, &cs);
                pe[sl * kStride + 3 + 6 * (q - 1) + c] = (float)sn;
                pe[sl * kStride + 6 + 6 * (q - 1) + c] = (float)cs;
            }
        }
        for (int e = lane; e < 16 * 64; e += 64) {
            const int sl = e >> 6, f = e & 63;
            if (f >= a.k0) pe[sl * kStride + f] = 0.0f;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) act[t][i] = pe[n * kStride + 16 * t + 4 * g + i];
    } else {
        float* pe = (float*)ring + wave * (16 * 17);
#pragma unroll
        for (int t = 0; t < kMaxT; ++t) {
            if (16 * t < a.k0) {
                for (int e = lane; e < 256; e += 64) {
                    const int sl = e >> 4, ft = e & 15;
                    const bool vs = (wave * 16 + sl < tile_samples) && (tile_base + sl < a.R);
                    pe[sl * 17 + ft] = comp::input_feature(a, tile_base + sl, vs, 16 * t + ft);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) act[t][i] = pe[n * 17 + 4 * g + i];
            }
        }
    }
    __syncthreads();   // the first DMA overwrites the scratch

    int ci = 0;   // chunk stream position (chunk_at)
    dma_chunk(a, chunk_at(a, 0), ring, bias_ring);
    dma_barrier(kAhead == 2 ? dma_chunk(a, chunk_at(a, 1), ring + slot_bytes<PL>(), bias_ring) : 0);
    PROF_ADD(kPfPE, t_start);
    // ReLU mask bits of this wave, per hidden layer: [L-1][lane] u64
    unsigned long long* mask_w = a.mask_g + ((size_t)wg * (a.L - 1) * kWaves + wave) * 64 + lane;

    // ---- forward ----
    for (int l = 0; l < a.L; ++l) {
        float* slab = !st ? nullptr
                          : (l == 0 ? a.act + a.x_off + blk * (size_t)(a.kt[0] * 1024)
                                    : a.act + a.act_off[l - 1] + blk * (size_t)(a.kt[l] * 1024)) +
                                half * 512;
        zero_tiles(out);
        const unsigned bl = lds_addr(bias_ring + (l % 3) * 256) + g * 16;
        const float xm = sample_max<PL>(act);
        if (PL == 2 && st) slab_max(a.smax, l, xm);
        const int ex = shift_of(xm);
        const int sh = unscale(l, ex);
        if (l < a.L - 1) {
            PROF_T(t_f);
            k16_pass<HT, PL>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex);
            PROF_ADD(kPfFwd, t_f);
            PROF_T(t_fe);
            // bias after the sum (nerf.py:98,125), ReLU (nerf.py:141-144) and its mask bits
            fx4 bv[kMaxT];
            bias_read<HT>(std::make_integer_sequence<int, HT>{}, bl, bv);
            bias_wait<HT>(std::make_integer_sequence<int, HT>{}, bv);
            unsigned long long mb = 0ull;
#pragma unroll
            for (int o = 0; o < HT; ++o) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float v = (PL == 2 ? __builtin_ldexpf(out[o][i], sh) : out[o][i]) + bv[o][i];
                    const bool pos = v > 0.0f;
                    act[o][i] = pos ? v : 0.0f;
                    mb |= (pos ? 1ull : 0ull) << (4 * o + i);
                }
            }
            if (st) mask_w[(size_t)l * kWaves * 64] = mb;
            PROF_ADD(kPfFwdEpi, t_fe);
        } else {
            k16_pass<1, PL>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex);
            fx4 bv[kMaxT];
            bias_read<1>(std::make_integer_sequence<int, 1>{}, bl, bv);
            bias_wait<1>(std::make_integer_sequence<int, 1>{}, bv);
            // head pre-activations: features 0..3 = registers 0..3 of lane group 0
            if (g == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    comp[ls * 4 + i] = (PL == 2 ? __builtin_ldexpf(out[0][i], sh) : out[0][i]) + bv[0][i];
            }
        }
    }
    PROF_T(t_c);
    __syncthreads();

    // ---- rendering + loss + rendering reverse (one thread per sample, scans along rays) ----
    comp::composite_tile(a, wg, comp, rayloss, st);
    __syncthreads();
    if (tid == 0) {
        float lsum = 0.0f;
        for (int r = 0; r < a.rpw; ++r) lsum = lsum + rayloss[r];
        a.loss_part[wg] = lsum;
    }
    PROF_ADD(kPfComp, t_c);
    if (!st) return;

    // ---- reverse chain: G_{L-1} from the head, G_{l-1} = (W_l G_l) * 1[A_{l-1} > 0] ----
    const float* c_gz = comp + 512;
    zero_tiles(act);
    if (g == 0 && valid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) act[0][i] = c_gz[ls * 4 + i];
    }
    for (int l = a.L - 1; l >= 1; --l) {
        zero_tiles(out);
        float* slab = a.grad + a.grad_off[l] + blk * (size_t)(a.nt[l] * 1024) + half * 512;
        PROF_T(t_b);
        const unsigned long long mb = mask_w[(size_t)(l - 1) * kWaves * 64];   // in flight over the pass
        const float xm = sample_max<PL>(act);
        if (PL == 2) slab_max(a.smax, a.L + l, xm);
        const int ex = shift_of(xm);
        const int sh = unscale(l, ex);
        k16_pass<HT, PL>(a, a.ks_b[l], ci, ring, bias_ring, act, out, slab, ex);
        PROF_ADD(kPfBwd, t_b);
        PROF_T(t_be);
#pragma unroll
        for (int o = 0; o < HT; ++o)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                act[o][i] = ((mb >> (4 * o + i)) & 1ull) ? (PL == 2 ? __builtin_ldexpf(out[o][i], sh) : out[o][i])
                                                         : 0.0f;
        PROF_ADD(kPfBwdEpi, t_be);
    }
    PROF_T(t_t);
    // act holds G_0
    float* g0 = a.grad + a.grad_off[0] + blk * (size_t)(a.nt[0] * 1024) + half * 512;
    if (a.d_x) {
        // d_layer_input = G_0 W_0^T (ENCODED mode); the pass also writes G_0's slab
        zero_tiles(out);
        const float xm = sample_max<PL>(act);
        if (PL == 2) slab_max(a.smax, a.L, xm);
        const int ex = shift_of(xm);
        const int sh = unscale(0, ex);
        k16_pass_n<PL>(a, a.ks_b[0], ci, ring, bias_ring, a.to_b[0], act, out, g0, ex);
        if (valid) {
#pragma unroll
            for (int o = 0; o < kMaxT; ++o)
                if (16 * o < a.k0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int f = 16 * o + 4 * g + i;
                        if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = PL == 2 ? __builtin_ldexpf(out[o][i], sh) : out[o][i];
                    }
                }
        }
    } else {
        if (PL == 2) slab_max(a.smax, a.L, sample_max<PL>(act));
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s < a.ks_b[0]) store_slab_step(g0 + s * 1024, act[2 * s], act[2 * s + 1]);
    }
#if LNERF_PROF
    PROF_ADD(kPfTail, t_t);
    PROF_ADD(kPfTotal, t_start);
    if (lane == 0) prof_slots()[kPfReal] += __builtin_amdgcn_s_memrealtime() - rt_start;
    if (lane < kPfN) atomicAdd(&g_k16_prof[lane], prof_slots()[lane]);
#endif
}

// ---- weight packing: per layer and pass, chunk s = [o][plane][lane 64][8 x bf16] -----------
// forward:  A[m = out 16o + (lane & 15)][k = 8g + j] = W[phi(s, g, j)][16o + m]
// backward: A[m = in  16o + (lane & 15)][k = 8g + j] = W[16o + m][phi(s, g, j)]
struct Pack16Args {
    int L;
    int k[kMaxLayers], n[kMaxLayers];
    int ks_f[kMaxLayers], ks_b[kMaxLayers], to_f[kMaxLayers], to_b[kMaxLayers];
    int w_k, w_n, planes;
    const float* W;
    const float* B;
    unsigned short* w16;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];
    float* b16;
    int* wexp;   // planes = 2: per-layer max|W| bits (pack16_kernel, from wmax16_kernel partials)
    int* wpart;  // [L][kWmaxParts] partial max|W| bits
};

// planes = 2: max|W_l| as the bits of a non-negative float (integer order = float order), one
// partial per block, grid (kWmaxParts, L): plain stores, no zeroing launch and no atomics; the
// packing kernel folds the layer's kWmaxParts partials itself.
__global__ void __launch_bounds__(256) wmax16_kernel(Pack16Args a) {
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
__device__ __forceinline__ int layer_wmax(Pack16Args& a, int l) {
    int mb = 0;
    for (int i = 0; i < kWmaxParts; ++i) mb = max(mb, a.wpart[l * kWmaxParts + i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.wexp[l] = mb;
    return mb;
}


// every layer in one launch: grid (blocks of the largest layer, L)
__global__ void pack16_kernel(Pack16Args a) {
    const int l = blockIdx.y;
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const int wsh = a.planes == 2 ? wshift_of(layer_wmax(a, l)) : 0;
    const size_t nf = (size_t)a.ks_f[l] * a.to_f[l] * 512, nb = (size_t)a.ks_b[l] * a.to_b[l] * 512;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < nf + nb + 256;
         e += (size_t)gridDim.x * blockDim.x) {
        if (e >= nf + nb) {
            const int f = (int)(e - nf - nb);
            a.b16[(size_t)l * 256 + f] = f < N ? a.B[(size_t)l * a.w_n + f] : 0.0f;
            continue;
        }
        const bool fwd = e < nf;
        size_t x = fwd ? e : e - nf;
        const int to = fwd ? a.to_f[l] : a.to_b[l];
        const int j = x & 7; x >>= 3;
        const int ln = x & 63; x >>= 6;
        const int o = (int)(x % to); x /= to;
        const int s = (int)x;
        const int f = phi(s, ln >> 4, j), m = 16 * o + (ln & 15);
        const int kk = fwd ? f : m, jj = fwd ? m : f;
        const float w = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        unsigned short* dst = a.w16 + (fwd ? a.wf_off[l] : a.wb_off[l]) +
                              ((size_t)(s * to + o) * a.planes) * 512 + ln * 8 + j;
        if (a.planes == 2) {
            _Float16 h, lo;
            split_h(__builtin_ldexpf(w, wsh), h, lo);
            dst[0] = __builtin_bit_cast(unsigned short, h);
            dst[512] = __builtin_bit_cast(unsigned short, lo);
            continue;
        }
        __bf16 h, mi, lo;
        split_x(w, h, mi, lo);
        dst[0] = __builtin_bit_cast(unsigned short, h);
        if (a.planes == 3) {
            dst[512] = __builtin_bit_cast(unsigned short, mi);
            dst[1024] = __builtin_bit_cast(unsigned short, lo);
        }
    }
}

}  // namespace

bool k16_supported(const FusedPlan& p) {
    if (p.x6 != 3 && p.x6 != 2 && p.x6 != 1) return false;
    if (p.n[p.L - 1] > 16) return false;       // head: one 16-wide output tile
    return true;
}

void k16_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s) {
    Pack16Args a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.k[l] = p.k[l];
        a.n[l] = p.n[l];
        a.ks_f[l] = p.ks16_f[l];
        a.ks_b[l] = p.ks16_b[l];
        a.to_f[l] = p.to16_f[l];
        a.to_b[l] = p.to16_b[l];
        a.wf_off[l] = p.w16f_off[l];
        a.wb_off[l] = p.w16b_off[l];
    }
    a.w_k = p.w_k;
    a.w_n = p.w_n;
    a.planes = p.x6;
    a.W = ws;
    a.B = bs;
    a.w16 = p.w16;
    a.b16 = p.b16;
    a.wexp = p.wexp16;
    a.wpart = p.wmax_part;
    if (a.planes == 2) wmax16_kernel<<<dim3(kWmaxParts, p.L), 256, 0, s>>>(a);
    size_t nmax = 0;
    for (int l = 0; l < p.L; ++l) {
        const size_t nel = ((size_t)a.ks_f[l] * a.to_f[l] + (size_t)a.ks_b[l] * a.to_b[l]) * 512 + 256;
        nmax = nel > nmax ? nel : nmax;
    }
    pack16_kernel<<<dim3((unsigned)((nmax + 255) / 256), p.L), 256, 0, s>>>(a);
}

void k16_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                bool want_grad, hipStream_t s) {
    K16Args a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.ks_f[l] = p.ks16_f[l];
        a.ks_b[l] = p.ks16_b[l];
        a.to_f[l] = p.to16_f[l];
        a.to_b[l] = p.to16_b[l];
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = p.w16f_off[l];
        a.wb_off[l] = p.w16b_off[l];
        a.act_off[l] = p.act_off[l];
        a.grad_off[l] = p.grad_off[l];
    }
    a.k0 = p.k[0];
    a.w16 = p.w16;
    a.b16 = p.b16;
    a.mask_g = p.mask_g;
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
    a.planes = p.x6;
    a.wexp = p.wexp16;
    a.smax = p.smax_part;
    // the chunk stream: forward 0..L-1, backward L-1..1 (training), backward 0 (d_x)
    {
        int ci = 0;
        auto add = [&](bool fwd, int l) {
            const int ks = fwd ? a.ks_f[l] : a.ks_b[l], to = fwd ? a.to_f[l] : a.to_b[l];
            const size_t per = (size_t)to * a.planes * 512;   // u16
            for (int s2 = 0; s2 < ks; ++s2, ++ci) {
                a.chunk_tab[2 * ci] = (unsigned)((fwd ? a.wf_off[l] : a.wb_off[l]) + (size_t)s2 * per);
                a.chunk_tab[2 * ci + 1] = (unsigned)(per * 2 / 1024) | ((fwd && s2 == 0 ? l + 1 : 0) << 16);
            }
        };
        for (int l = 0; l < p.L; ++l) add(true, l);
        if (want_grad)
            for (int l = p.L - 1; l >= (a.d_x ? 0 : 1); --l) add(false, l);
        // two zero entries past the end (the kernel looks two chunks ahead): a{} zeroed them
    }
    static_assert(sizeof(K16Args) <= 4096, "kernel arguments");
#define LNERF_K16_LAUNCH(HT)                                                              \
    if (p.x6 == 3) k16_fwd_bwd_kernel<HT, 3><<<p.num_wg, kThreads, 0, s>>>(a);            \
    else if (p.x6 == 2) k16_fwd_bwd_kernel<HT, 2><<<p.num_wg, kThreads, 0, s>>>(a);       \
    else k16_fwd_bwd_kernel<HT, 1><<<p.num_wg, kThreads, 0, s>>>(a);
    switch (p.ht16) {
        case 1: LNERF_K16_LAUNCH(1) break;
        case 2: LNERF_K16_LAUNCH(2) break;
        case 4: LNERF_K16_LAUNCH(4) break;
        case 8: LNERF_K16_LAUNCH(8) break;
        default: LNERF_K16_LAUNCH(16) break;
    }
#undef LNERF_K16_LAUNCH
#if LNERF_PROF
    if (want_grad) {
        unsigned long long h[16] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_k16_prof), sizeof(h));
        const char* names[] = {"pe", "fwd_pass", "fwd_epilogue", "barrier", "composite", "bwd_pass",
                               "bwd_epilogue", "tail", "total", "vmcnt_wait", "realtime_100MHz"};
        fprintf(stderr, "LNERF_PROF k16 per-wave cycles:");
        for (int i = 0; i < kPfN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / ((double)p.num_wg * kWaves));
        fprintf(stderr, " clock_GHz=%.3f\n", h[kPfReal] ? (double)h[kPfTotal] / h[kPfReal] * 0.1 : 0.0);
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_k16_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
