// lnerf_k32.hip -- k1 with one wave per SIMD: the fused PE + MLP + compositing + reverse chain on
// v_mfma_f32_32x32x16_{f16,bf16}, 32 samples per wave (fp16x3 default, bf16x6, plain bf16 for
// inference).
//
// Same work and outputs as k16 (lnerf_k16.hip; reference scripts/nerf.py:1-304 and its rev_diff,
// train_nerf.py:325/395), re-tiled so that every weight fragment a wave reads from LDS feeds 32
// samples instead of 16: the LDS bytes per MFMA FLOP halve, which is what bounded k16 (8 waves
// reading the whole 32 KiB weight chunk of every k-step for 16 samples each; SQ counters in
// profiles/r03_sq.json).
//  * one 256-thread workgroup (4 waves, one per SIMD) per 128-sample tile of whole rays; each
//    wave owns 32 samples: a 256-wide layer is 8 accumulator tiles x 16 registers for the
//    activations plus 8 x 16 for the accumulators (256 of the 512 registers a lone wave has);
//  * the activations stay in the 32x32 accumulator layout (lane = sample l & 31, register r of
//    tile t = feature 32 t + (r & 3) + 8 (r >> 2) + 4 (l >> 5)), so registers 8s..8s+7 of a tile
//    are the next layer's B operand for k-step s as they stand; the weight packing bakes in that
//    contraction order (kappa below);
//  * the weights of one input tile (32 features: 2 k-steps x every output tile x the PL split
//    planes, 32 KiB for fp16x3) stream through a 3-slot LDS ring by LDS-DMA, two tiles in flight:
//    the DMA of chunk c + 2 is issued when chunk c starts and waited for at chunk c's barrier, so
//    chunk c + 1 is already visible while chunk c computes and its first weight fragments are
//    read under chunk c's last MFMAs (the barrier exposes no LDS latency);
//  * with a single wave per SIMD every LDS read is issued kD fragments ahead of its MFMAs and the
//    operand splits, slab stores and DMA issue sit in the MFMAs' shadow.
// The slabs (post-ReLU activations A_l, gradients G_l) are written in the layout dw16 reads
// (lnerf_dw16.hip): per 32-sample block (one wave) and 32-feature tile, [q 4][lane 64][4 floats],
// lane l's registers 4q..4q+3 -- four global_store_dwordx4, each wave instruction 1 KiB.
#include "lnerf_composite.h"
#include "lnerf_internal.h"

#include <stddef.h>
#include <stdio.h>

#include <utility>

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef float fx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kTile = comp::kTileSamples;     // 128 samples per workgroup
constexpr int kMaxT = 8;                      // 32-feature tiles per 256-wide layer
constexpr int kMaxChunks = 2 * kMaxLayers * 8 + 2;   // <= 2 passes x 8 input tiles per layer + 2 end
constexpr int kCompBytes = 2688 * 4;          // composite_tile's scratch (comp[0, 2688))
constexpr int kSlots = 3;                     // ring slots: one computed, two in flight / landed
constexpr int kD = 3;                         // weight fragments read ahead of the one consumed
// timing experiments only (wrong results): drop the slab stores / the weight DMA after chunk 2
#ifndef LNERF_K32_NOSTORE
#define LNERF_K32_NOSTORE 0
#endif
#ifndef LNERF_K32_NODMA
#define LNERF_K32_NODMA 0
#endif

template <int PL>
struct Ring {
    static constexpr int slot_bytes = 2 * kMaxT * PL * 1024;   // one input tile of a 256-wide pass
    static constexpr int off_comp = kSlots * slot_bytes;
    static constexpr int off_ray = off_comp + kCompBytes;
    static constexpr int off_bias = off_ray + kTile * 4;
    static constexpr int lds_bytes = off_bias + 3 * 256 * 4;   // + a 3-slot ring of layer biases
    static_assert(lds_bytes + 1024 <= 160 * 1024, "LDS budget (+1 KiB for the profiling build)");
    static_assert((2 * kMaxT - 1) * PL * 1024 + (PL - 1) * 1024 < 65536, "16-bit ds_read offsets");
};

struct K32Args {
    int L;
    int ks_f[kMaxLayers], ks_b[kMaxLayers];   // input tiles (32 features) per pass
    int to_f[kMaxLayers], to_b[kMaxLayers];   // 32-wide output tiles per pass
    int kt[kMaxLayers], nt[kMaxLayers];       // 32-wide slab tiles of each layer's input/output
    int k0;
    const unsigned short* w32;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];   // u16 offsets
    const float* b16;                                // [L][256] zero-padded biases
    unsigned long long* mask_g;                      // [wg][L-1][wave][lane][2] ReLU mask bits
    // the chunk stream (k32_launch): per chunk {u16 offset in w32, (bytes / 1024) | (bias layer
    // + 1) << 16}, zero past the end. Read with scalar loads from the kernel-argument segment.
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
    const int* wexp;   // PL = 2: per-layer max|W| bits of the packed fp16 weight planes
    // training: every sample's exponent shift of each slab row, [l][position][2] int8: byte 0 the
    // input of layer l, byte 1 G_l; position = 32-sample block * 32 + sample
    signed char* sexp;
    int rpad;          // slab positions (num_wg * 128)
    int* epart;        // training: per-wave min over samples of exA + exG, [l][num_wg * 4]
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---- optional in-kernel phase timing (-DLNERF_PROF=1, never in the product build) -------------
#ifndef LNERF_PROF
#define LNERF_PROF 0
#endif
#if LNERF_PROF
enum { kPfPE, kPfFwd, kPfFwdEpi, kPfBar, kPfComp, kPfBwd, kPfBwdEpi, kPfTail, kPfTotal, kPfVm, kPfReal, kPfN };
__device__ unsigned long long g_k32_prof[16];
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

// Input feature of element j of a lane in half h (= lane >> 5) for k-step s of input tile t: the
// 32x32 accumulator's register 8s + j of that lane (the guide's "accumulator as the next MFMA's
// operand": k order permuted inside each k-step, baked into the weight packing).
__host__ __device__ __forceinline__ int kappa(int t, int s, int h, int j) {
    return 32 * t + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
}
// feature held in register r of tile t by a lane in half h
__host__ __device__ __forceinline__ int feat_of(int t, int r, int h) {
    return 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
}

struct ChunkT {
    const unsigned short* src;   // nullptr: past the last chunk
    int bytes;
    int bias;                    // layer whose biases ride with this chunk, -1: none
};

// Chunk `ci` of the kernel's stream from K32Args::chunk_tab through the kernel-argument segment
// pointer (a scalar load at a dynamic offset; indexing the by-value argument would copy it to
// scratch, a vector load would sit in vmcnt behind the in-flight DMA).
__device__ __forceinline__ ChunkT chunk_at(const K32Args& a, int ci) {
    const __attribute__((address_space(4))) unsigned* t =
        (const __attribute__((address_space(4))) unsigned*)((const __attribute__((address_space(4))) char*)
                                                                __builtin_amdgcn_kernarg_segment_ptr() +
                                                            offsetof(K32Args, chunk_tab)) + 2 * ci;
    const unsigned off = t[0], e = t[1];
    const int bytes = (int)(e & 0xFFFFu) * 1024;
    return ChunkT{bytes ? a.w32 + off : nullptr, bytes, (int)(e >> 16) - 1};
}

// LDS-DMA (global_load_lds_dwordx4) of a chunk into its ring slot, each wave instruction 1 KiB
// (lane-linear), the 4 waves taking turns; the last wave also stages the biases a first forward
// chunk carries (bias ring slot l % 3). Returns the instructions this wave issued.
__device__ __forceinline__ int dma_chunk(const K32Args& a, const ChunkT& c, unsigned char* dst,
                                         float* bias_ring) {
    const int tid = threadIdx.x, wave = wave_id();
    int n = 0;
    if (!c.src) return 0;
    for (int off = wave * 1024; off < c.bytes; off += kWaves * 1024) {
        const char* g = (const char*)c.src + off + (tid & 63) * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(dst + off), 16, 0, 0);
        ++n;
    }
    if (c.bias >= 0 && wave == kWaves - 1) {
        const float* g = a.b16 + (size_t)c.bias * 256 + (tid & 63) * 4;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(bias_ring + (c.bias % 3) * 256),
                                         16, 0, 0);
        ++n;
    }
    return n;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int... N>
__device__ __forceinline__ void vm_wait_n(int n, std::integer_sequence<int, N...>) {
    n = n > 63 ? 63 : n;
    ((n == N ? vm_wait<N>() : void()), ...);
}
// The chunk two ahead (this wave's pieces) has landed -- vector-memory operations retire in issue
// order, so at most `pending` outstanding (the slab stores issued after the pieces) means every
// piece is done -- then s_barrier: every wave's pieces are in LDS and every wave is done with
// the slot the next DMA overwrites. pending < 0: nothing to wait for (only the barrier).
__device__ __forceinline__ void dma_barrier(int pending) {
    PROF_T(t0);
    asm volatile("" ::: "memory");
    if (pending == 0) vm_wait<0>();
    else if (pending == 4) vm_wait<4>();
    else if (pending > 0) vm_wait_n(pending, std::make_integer_sequence<int, 64>{});
    PROF_ADD(kPfVm, t0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    PROF_ADD(kPfBar, t0);
}

__device__ __forceinline__ fx16 mfma32(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ fx16 mfma32h(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
                                                  0);
}

// fp16x3: x 2^e = hi + lo, round-to-nearest fp16 of each (the remainder is exact in f32).
__device__ __forceinline__ void split_h(float xs, _Float16& h, _Float16& l) {
    h = (_Float16)xs;
    l = (_Float16)(xs - (float)h);
}
__device__ __forceinline__ int wshift_of(int maxbits) { return fp16x3_shift(__int_as_float(maxbits)); }
__device__ __forceinline__ int shift_of(float m) { return fp16x3_shift(m); }

// The same split for a pair (x0, x1) packed as two f16 per register, by v_fma_mix (one rounding
// each; x sc and x sc - hi are exact): two instructions per value.
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

// The B operand planes of k-step s of an input tile: registers 8s..8s+7 of its accumulator
// (fp16x3 hi/lo x 2^ex, bf16x6 hi/mid/lo x 2^ex, or plain bf16).
struct BOp {
    bf8 h, m, l;
};
template <int PL, int S>
__device__ __forceinline__ BOp make_b(const fx16& x, int ex) {
    BOp b{};
    if constexpr (PL == 2) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        u4 hv, lv;
        const float sc = __builtin_ldexpf(1.0f, ex);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned h2, l2;
            split_h2(x[8 * S + 2 * q], x[8 * S + 2 * q + 1], sc, h2, l2);
            hv[q] = h2;
            lv[q] = l2;
        }
        b.h = __builtin_bit_cast(bf8, hv);
        b.m = __builtin_bit_cast(bf8, lv);
    } else if constexpr (PL == 3) {
        const float sc = __builtin_ldexpf(1.0f, ex);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            __bf16 h, m, l;
            split_x(x[8 * S + j] * sc, h, m, l);
            b.h[j] = h;
            b.m[j] = m;
            b.l[j] = l;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) b.h[j] = (__bf16)x[8 * S + j];
    }
    return b;
}

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_read_b128 with an immediate offset, outside the compiler's waitcnt bookkeeping: the
// matching lgkm_wait below is the only wait, so reads of later fragments stay in flight.
template <int OFF>
__device__ __forceinline__ bf8 ds_read_at(unsigned addr) {
    bf8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
    return r;
}
// s_waitcnt lgkmcnt(N) that the fragment depends on (no use can be scheduled above it). LDS reads
// return in order, so at most N outstanding means every older read has landed.
template <int N, int PL>
__device__ __forceinline__ void lgkm_wait(bf8 (&w)[3]) {
    if constexpr (PL == 1) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(w[0]) : "n"(N));
    else if constexpr (PL == 2) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(w[0]), "+v"(w[1]) : "n"(N));
    else asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]) : "n"(N));
}
// Fragment F of a chunk (k-step F / NTO, output tile F % NTO) = PL planes of 1 KiB, lane-linear.
template <int PL, int F>
__device__ __forceinline__ void read_frag(unsigned base, bf8 (&w)[3]) {
    w[0] = ds_read_at<(F * PL + 0) * 1024>(base);
    if constexpr (PL >= 2) w[1] = ds_read_at<(F * PL + 1) * 1024>(base);
    if constexpr (PL >= 3) w[2] = ds_read_at<(F * PL + 2) * 1024>(base);
}

// Fragment read-ahead distance: 3 fragments, 1 for the head's 2-fragment chunks (the ring of
// kD + 1 register sets must divide a chunk's 2 NTO fragments so that the next chunk's prefetched
// fragments land where it expects them).
template <int NTO>
constexpr int read_ahead() { return NTO == 1 ? 1 : 3; }

// Fragment step F of a chunk of NF = 2 NTO fragments: read fragment F + kD (of this chunk, or the
// first fragments of the next chunk -- landed by the ring's invariant -- at `nbase`, which the
// caller points at a harmless address of this chunk's slot when no chunk of this pass follows),
// wait for fragment F, its MFMAs into output tile F % NTO (small terms first). Every step keeps
// kD younger reads in flight; the pass retires the last ones (k32_pass).
// The chunk's vector-memory work, spread over its fragment steps (LNERF_K32_SPREAD) instead of
// issued as one burst at the chunk's start, where a lone wave's matrix core would idle behind it
// (timing knobs: the pieces cost 0.26 ms and the stores 0.24 ms of a 1.6 ms k1 as bursts): op i
// of the 12 (this wave's <= 8 LDS-DMA pieces of the chunk two ahead, then the 4 slab stores of the
// input tile, younger than every piece so the chunk barrier's vmcnt leaves them in flight) goes
// between the first two (dependent) MFMAs of fragment step i NF / 12, where it issues while the
// first one runs.
#ifndef LNERF_K32_SPREAD
#define LNERF_K32_SPREAD 1
#endif
struct VmJob {
    const char* src = nullptr;      // this lane's address of piece 0
    unsigned char* dst = nullptr;   // LDS address of this wave's piece 0
    int n = 0;                      // this wave's pieces
    float* slab = nullptr;          // the input tile's slab (nullptr: no stores)
    const fx16* tile = nullptr;     // the input tile's registers
};
__device__ __forceinline__ void vm_op(const VmJob& j, int i) {
    if (i < 8) {
        if (i < j.n)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(j.src + i * (kWaves * 1024)),
                                             (__attribute__((address_space(3))) void*)(j.dst + i * (kWaves * 1024)), 16,
                                             0, 0);
    } else if (j.slab) {
        const int q = i - 8, lane = threadIdx.x & 63;
        const fx16& v = *j.tile;
        __builtin_nontemporal_store(fx4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]},
                                    (fx4*)(j.slab + q * 256 + lane * 4));
    }
}
template <int NF, int F, int... I>
__device__ __forceinline__ void vm_ops_at(const VmJob& j, std::integer_sequence<int, I...>) {
    (((I * NF) / 12 == F ? vm_op(j, I) : void()), ...);
}

template <int NTO, int PL, int F>
__device__ __forceinline__ void frag_step(unsigned base, unsigned nbase, bf8 (&w)[4][3], const BOp& b,
                                          fx16 (&out)[kMaxT], const VmJob& vj) {
    constexpr int NF = 2 * NTO, KD = read_ahead<NTO>();
    if constexpr (F + KD < NF) read_frag<PL, F + KD>(base, w[(F + KD) % (KD + 1)]);
    else read_frag<PL, F + KD - NF>(nbase, w[(F + KD) % (KD + 1)]);
    bf8(&c)[3] = w[F % (KD + 1)];
    lgkm_wait<KD * PL, PL>(c);
    fx16 acc = out[F % NTO];
    if constexpr (PL == 2) {
        acc = mfma32h(c[0], b.m, acc);   // w_hi x_lo, w_lo x_hi, then w_hi x_hi
        if constexpr (LNERF_K32_SPREAD) vm_ops_at<NF, F>(vj, std::make_integer_sequence<int, 12>{});
        acc = mfma32h(c[1], b.h, acc);
        acc = mfma32h(c[0], b.h, acc);
    } else if constexpr (PL == 3) {
        acc = mfma32(c[0], b.l, acc);
        acc = mfma32(c[1], b.m, acc);
        acc = mfma32(c[2], b.h, acc);
        acc = mfma32(c[1], b.h, acc);
        acc = mfma32(c[0], b.m, acc);
        acc = mfma32(c[0], b.h, acc);
    } else {
        acc = mfma32(c[0], b.h, acc);
    }
    out[F % NTO] = acc;
}

template <int NTO, int PL, int B, int... F>
__device__ __forceinline__ void frag_steps(std::integer_sequence<int, F...>, unsigned base, unsigned nbase,
                                           bf8 (&w)[4][3], const BOp& b, fx16 (&out)[kMaxT], const VmJob& vj) {
    (frag_step<NTO, PL, B + F>(base, nbase, w, b, out, vj), ...);
}

// Slab tile store: input tile t of this wave's 32-sample block, [q][lane][4] = registers 4q..4q+3
// of every lane; each of the four global_store_dwordx4 covers 1 KiB.
__device__ __forceinline__ void store_slab_tile(float* __restrict__ dst, const fx16& v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        __builtin_nontemporal_store(fx4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]},
                                    (fx4*)(dst + q * 256 + lane * 4));
}

// One chunk = input tile T of a pass (compile-time after unrolling): out[o] += sum over its two
// k-steps of Wpack (x) in[T] registers 8s..8s+7. The chunk is read from ring slot ci % 3; the
// DMA of chunk ci + 2 is issued here and waited for at the chunk's barrier. b holds k-step
// (T, 0)'s B planes on entry and (T + 1, 0)'s on exit; w holds the chunk's first kD fragments on
// entry (the pass's first chunk reads them itself) and the next chunk's on exit (a harmless read
// of this slot when the pass ends here: `more` false).
template <int NTO, int PL, int T>
__device__ __forceinline__ void k32_chunk(const K32Args& a, bool more, int& ci, unsigned char* ring,
                                          float* bias_ring, const fx16 (&in)[kMaxT], fx16 (&out)[kMaxT],
                                          float* __restrict__ slab, int ex, bf8 (&w)[4][3], BOp& b) {
    constexpr int SB = Ring<PL>::slot_bytes;
    constexpr int H = (NTO - 1) / 2;   // the next k-step's split goes after fragment step H
    constexpr int KD = read_ahead<NTO>();
    const int lane = threadIdx.x & 63;
    const unsigned base = lds_addr(ring + (ci % kSlots) * SB) + lane * 16;
    const unsigned nbase = more ? lds_addr(ring + ((ci + 1) % kSlots) * SB) + lane * 16 : base;
    // DMA of chunk ci + 2 first (its table entry is a scalar load the compiler waits for with
    // lgkmcnt(0)), then the slab stores (younger than the pieces: the barrier's vmcnt leaves
    // them in flight)
    constexpr bool spread = LNERF_K32_SPREAD && PL == 2;
    const bool st = slab && !LNERF_K32_NOSTORE;
    VmJob vj;
    int issued;
    {
        const ChunkT c = (LNERF_K32_NODMA && ci >= 2) ? ChunkT{nullptr, 0, -1} : chunk_at(a, ci + 2);
        unsigned char* dst = ring + ((ci + 2) % kSlots) * SB;
        if constexpr (spread) {
            // the pieces go out between the MFMAs below (vm_op); only a first forward chunk's
            // biases are staged now, by the last wave
            const int woff = wave_id() * 1024;
            vj.n = (c.src && woff < c.bytes) ? (c.bytes - woff + kWaves * 1024 - 1) / (kWaves * 1024) : 0;
            vj.src = (const char*)c.src + woff + lane * 16;
            vj.dst = dst + woff;
            vj.slab = st ? slab + T * 1024 : nullptr;
            vj.tile = &in[T];
            issued = vj.n;
            if (c.bias >= 0 && wave_id() == kWaves - 1) {
                const float* g = a.b16 + (size_t)c.bias * 256 + lane * 4;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                                 (__attribute__((address_space(3))) void*)(bias_ring + (c.bias % 3) * 256),
                                                 16, 0, 0);
                ++issued;
            }
        } else {
            issued = dma_chunk(a, c, dst, bias_ring);
        }
    }
    asm volatile("" ::: "memory");
    int pending = issued ? 0 : -1;
    if constexpr (T == 0) {
        read_frag<PL, 0>(base, w[0]);
        if constexpr (KD >= 2) read_frag<PL, 1>(base, w[1]);
        if constexpr (KD >= 3) read_frag<PL, 2>(base, w[2]);
    }
    if (st) {
        if constexpr (!spread) store_slab_tile(slab + T * 1024, in[T]);
        if (pending >= 0) pending += 4;
    }
    // k-step 0: fragments 0..NTO-1; its k-step 1 split after step H
    frag_steps<NTO, PL, 0>(std::make_integer_sequence<int, H + 1>{}, base, nbase, w, b, out, vj);
    const BOp b1 = make_b<PL, 1>(in[T], ex);
    frag_steps<NTO, PL, H + 1>(std::make_integer_sequence<int, NTO - H - 1>{}, base, nbase, w, b, out, vj);
    // k-step 1: fragments NTO..2NTO-1; the next tile's k-step 0 split after step H
    frag_steps<NTO, PL, NTO>(std::make_integer_sequence<int, H + 1>{}, base, nbase, w, b1, out, vj);
    if constexpr (T + 1 < kMaxT) b = make_b<PL, 0>(in[T + 1], ex);
    frag_steps<NTO, PL, NTO + H + 1>(std::make_integer_sequence<int, NTO - H - 1>{}, base, nbase, w, b1, out, vj);
    dma_barrier(pending);
    ++ci;
}

// One pass (a layer's forward or backward MMA) over its ks input tiles.
template <int NTO, int PL, int T>
__device__ __forceinline__ void k32_tiles(const K32Args& a, int ks, int& ci, unsigned char* ring, float* bias_ring,
                                          const fx16 (&in)[kMaxT], fx16 (&out)[kMaxT], float* slab, int ex,
                                          bf8 (&w)[4][3], BOp& b) {
    if constexpr (T < kMaxT) {
        if (T < ks) {
            k32_chunk<NTO, PL, T>(a, T + 1 < ks, ci, ring, bias_ring, in, out, slab, ex, w, b);
            k32_tiles<NTO, PL, T + 1>(a, ks, ci, ring, bias_ring, in, out, slab, ex, w, b);
        }
    }
}

template <int NTO, int PL>
__device__ __forceinline__ void k32_pass(const K32Args& a, int ks, int& ci, unsigned char* ring, float* bias_ring,
                                         const fx16 (&in)[kMaxT], fx16 (&out)[kMaxT], float* __restrict__ slab,
                                         int ex) {
    static_assert(2 * NTO % (read_ahead<NTO>() + 1) == 0, "cross-chunk prefetch keeps the fragment ring aligned");
    bf8 w[4][3];
    BOp b = make_b<PL, 0>(in[0], ex);
    k32_tiles<NTO, PL, 0>(a, ks, ci, ring, bias_ring, in, out, slab, ex, w, b);
    // retire the last chunk's read-ahead (harmless reads of its own slot)
    constexpr int KD = read_ahead<NTO>();
    lgkm_wait<0, PL>(w[0]);
    if constexpr (KD >= 2) lgkm_wait<0, PL>(w[1]);
    if constexpr (KD >= 3) lgkm_wait<0, PL>(w[2]);
    if constexpr (KD >= 3) lgkm_wait<0, PL>(w[3]);
}

template <int PL>
__device__ __forceinline__ void k32_pass_n(const K32Args& a, int ks, int& ci, unsigned char* ring,
                                           float* bias_ring, int nto, const fx16 (&in)[kMaxT],
                                           fx16 (&out)[kMaxT], float* slab, int ex) {
    if (nto <= 1) k32_pass<1, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 2) k32_pass<2, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 4) k32_pass<4, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else k32_pass<8, PL>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
}

// The per-sample max|x| of a pass's input: lanes n and n + 32 hold sample n's features.
__device__ __forceinline__ float sample_max(const fx16 (&in)[kMaxT]) {
    float m = 0.0f;
#pragma unroll
    for (int o = 0; o < kMaxT; ++o)
#pragma unroll
        for (int i = 0; i < 16; ++i) m = __builtin_fmaxf(m, __builtin_fabsf(in[o][i]));
    return __builtin_fmaxf(m, __shfl_xor(m, 32));
}

// Training: this sample's exponent shift of one slab row (-128 for an all-zero row), one byte per
// sample for dw16's per-sample balancing. Returns the byte.
__device__ __forceinline__ int store_sexp(const K32Args& a, int l, int which, float m) {
    const int lane = threadIdx.x & 63;
    const int x = m > 0.0f ? shift_of(m) : -128;
    if (lane < 32) {
        const int p = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * 32 + lane;
        a.sexp[((size_t)l * a.rpad + p) * 2 + which] = (signed char)x;
    }
    return x;
}

// The forward's A-row shifts, one byte per layer packed in 4 registers (selects instead of a
// dynamically indexed register array).
struct ExPack {
    unsigned w[4] = {0u, 0u, 0u, 0u};
    __device__ __forceinline__ void put(int l, int x) {
        const int sh = 8 * (l & 3);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k == (l >> 2)) w[k] = (w[k] & ~(0xFFu << sh)) | ((unsigned)(x & 0xFF) << sh);
    }
    __device__ __forceinline__ int get(int l) const {
        unsigned v = w[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) v = k == (l >> 2) ? w[k] : v;
        return (int)(signed char)((v >> (8 * (l & 3))) & 0xFFu);
    }
};

// Training, after layer l's G-row shift xg: the wave's min over its samples of xa + xg (all-zero
// rows excluded), one plain store per wave into epart[l][global wave].
__device__ __forceinline__ void store_emin(const K32Args& a, int l, int xa, int xg) {
    int v = (xa == -128 || xg == -128) ? (1 << 20) : xa + xg;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) v = min(v, __shfl_xor(v, d));
    if ((threadIdx.x & 63) == 0)
        a.epart[(size_t)l * gridDim.x * kWaves + blockIdx.x * kWaves + (threadIdx.x >> 6)] = v;
}

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
// The biases of output tile o in the accumulator layout: registers 4c..4c+3 hold features
// 32 o + 8 c + 4 h ..+3, one ds_read_b128 each from the bias ring slot (outside the compiler's
// waitcnt bookkeeping: a plain LDS read would wait vmcnt(0) for the in-flight weight DMA).
__device__ __forceinline__ fx16 bias_tile(unsigned addr_h) {
    fx4 b0 = ds_read_f4<0>(addr_h), b1 = ds_read_f4<32>(addr_h), b2 = ds_read_f4<64>(addr_h),
        b3 = ds_read_f4<96>(addr_h);
    lgkm_wait4<3>(b0);
    lgkm_wait4<2>(b1);
    lgkm_wait4<1>(b2);
    lgkm_wait4<0>(b3);
    return fx16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
}

__device__ __forceinline__ void zero_tiles(fx16 (&t)[kMaxT]) {
#pragma unroll
    for (int o = 0; o < kMaxT; ++o)
#pragma unroll
        for (int r = 0; r < 16; ++r) t[o][r] = 0.0f;
}

// HT: 32-wide output tiles of every hidden layer (1/2/4/8); PL: operand planes (3 = bf16x6,
// 2 = fp16x3, both fp32-class; 1 = plain bf16, inference).
template <int HT, int PL>
__global__ void __launch_bounds__(kThreads, 1) k32_fwd_bwd_kernel(K32Args a) {
    using R = Ring<PL>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[R::lds_bytes];
    unsigned char* ring = lds;
    float* comp = (float*)(lds + R::off_comp);
    float* rayloss = (float*)(lds + R::off_ray);
    float* bias_ring = (float*)(lds + R::off_bias);

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), h = lane >> 5, n = lane & 31;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
    const int ls = wave * 32 + n;                      // local sample 0..127
    const int gs = wg * tile_samples + ls;             // global sample row (ray*S + j)
    const bool valid = (ls < tile_samples) && (gs < a.R);
    const size_t blk = (size_t)wg * kWaves + wave;     // this wave's 32-sample slab block
    const bool st = a.want_grad != 0;
#if LNERF_PROF
    if (lane < 16) prof_slots()[lane] = 0;
    PROF_T(t_start);
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
#endif

    fx16 act[kMaxT], out[kMaxT];
    zero_tiles(act);
    ExPack exa;   // training: the forward's A-row shift of this lane's sample, per layer
    // PL = 2: layer l's weight exponent shift in lane l (read with readlane per pass); a pass's
    // accumulators carry 2^(ex + ew), removed exactly (powers of two) in its epilogue
    const int wexp_lane = (PL == 2 && lane < a.L) ? wshift_of(a.wexp[lane]) : 0;
    auto unscale = [&](int l, int ex) -> int {
        return PL == 2 ? -(ex + __builtin_amdgcn_readlane(wexp_lane, l)) : PL == 3 ? -ex : 0;
    };

    // ---- layer-0 input in the accumulator layout, through a per-wave LDS scratch (the ring is
    // free before the first DMA). POINTS/RAYS with k0 <= 64: one float64 sincos per (sample,
    // coordinate, frequency) (pos_encoding.py:54-66); otherwise tile by tile.
    const int tile_base = wg * tile_samples + wave * 32;
    if (a.input_mode != LNERF_INPUT_ENCODED && a.k0 <= 64) {
        constexpr int kStride = 65;
        float* pe = (float*)ring + wave * (32 * kStride);
        const int F = a.F, per = 3 * (F + 1);
        for (int it = lane; it < 32 * per; it += 64) {
            const int sl = it / per, rem = it - sl * per, c = rem % 3, q = rem / 3;
            const bool vs = (wave * 32 + sl < tile_samples) && (tile_base + sl < a.R);
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
        for (int e = lane; e < 32 * 64; e += 64) {
            const int sl = e >> 6, f = e & 63;
            if (f >= a.k0) pe[sl * kStride + f] = 0.0f;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) act[t][r] = pe[n * kStride + feat_of(t, r, h)];
    } else {
        float* pe = (float*)ring + wave * (32 * 33);
#pragma unroll
        for (int t = 0; t < kMaxT; ++t) {
            if (32 * t < a.k0) {
                for (int e = lane; e < 32 * 32; e += 64) {
                    const int sl = e >> 5, ft = e & 31;
                    const bool vs = (wave * 32 + sl < tile_samples) && (tile_base + sl < a.R);
                    pe[sl * 33 + ft] = comp::input_feature(a, tile_base + sl, vs, 32 * t + ft);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) act[t][r] = pe[n * 33 + feat_of(0, r, h)];
            }
        }
    }
    __syncthreads();   // the first DMA overwrites the scratch

    int ci = 0;   // chunk stream position (chunk_at)
    dma_chunk(a, chunk_at(a, 0), ring, bias_ring);
    dma_chunk(a, chunk_at(a, 1), ring + R::slot_bytes, bias_ring);
    dma_barrier(0);
    PROF_ADD(kPfPE, t_start);
    // ReLU mask bits of this wave, per hidden layer: [L-1][lane][2] u64 (bit 16 o + r, o < 4 in
    // the first word, o >= 4 in the second)
    unsigned long long* mask_w = a.mask_g + (((size_t)wg * (a.L - 1) * kWaves + wave) * 64 + lane) * 2;

    // ---- forward ----
    for (int l = 0; l < a.L; ++l) {
        float* slab = !st ? nullptr
                          : (l == 0 ? a.act + a.x_off + blk * (size_t)(a.kt[0] * 1024)
                                    : a.act + a.act_off[l - 1] + blk * (size_t)(a.kt[l] * 1024));
        zero_tiles(out);
        const unsigned bias_h = lds_addr(bias_ring + (l % 3) * 256) + h * 16;
        const float xm = (PL >= 2 || st) ? sample_max(act) : 0.0f;
        if (st) exa.put(l, store_sexp(a, l, 0, xm));
        const int ex = shift_of(xm);
        const int sh = unscale(l, ex);
        if (l < a.L - 1) {
            PROF_T(t_f);
            k32_pass<HT, PL>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex);
            PROF_ADD(kPfFwd, t_f);
            PROF_T(t_fe);
            // bias after the sum (nerf.py:98,125), ReLU (nerf.py:141-144) and its mask bits
            unsigned long long m0 = 0ull, m1 = 0ull;
#pragma unroll
            for (int o = 0; o < HT; ++o) {
                const fx16 bv = bias_tile(bias_h + o * 128);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = (PL >= 2 ? __builtin_ldexpf(out[o][r], sh) : out[o][r]) + bv[r];
                    const bool pos = v > 0.0f;
                    act[o][r] = pos ? v : 0.0f;
                    if (o < 4) m0 |= (pos ? 1ull : 0ull) << (16 * o + r);
                    else m1 |= (pos ? 1ull : 0ull) << (16 * (o - 4) + r);
                }
            }
            if (st) {
                typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
                *(u2*)(mask_w + (size_t)l * kWaves * 128) = u2{m0, m1};
            }
            PROF_ADD(kPfFwdEpi, t_fe);
        } else {
            k32_pass<1, PL>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex);
            const fx16 bv = bias_tile(bias_h);
            // head pre-activations: features 0..3 = registers 0..3 of lane half 0
            if (h == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    comp[ls * 4 + i] = (PL >= 2 ? __builtin_ldexpf(out[0][i], sh) : out[0][i]) + bv[i];
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
    if (h == 0 && valid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) act[0][i] = c_gz[ls * 4 + i];
    }
    for (int l = a.L - 1; l >= 1; --l) {
        zero_tiles(out);
        float* slab = a.grad + a.grad_off[l] + blk * (size_t)(a.nt[l] * 1024);
        PROF_T(t_b);
        typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
        const u2 mb = *(const u2*)(mask_w + (size_t)(l - 1) * kWaves * 128);   // in flight over the pass
        const float xm = sample_max(act);
        const int xg = store_sexp(a, l, 1, xm);
        store_emin(a, l, exa.get(l), xg);
        const int ex = shift_of(xm);
        const int sh = unscale(l, ex);
        k32_pass<HT, PL>(a, a.ks_b[l], ci, ring, bias_ring, act, out, slab, ex);
        PROF_ADD(kPfBwd, t_b);
        PROF_T(t_be);
#pragma unroll
        for (int o = 0; o < HT; ++o)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const unsigned long long word = o < 4 ? mb[0] : mb[1];
                const int bit = 16 * (o & 3) + r;
                act[o][r] = ((word >> bit) & 1ull) ? (PL >= 2 ? __builtin_ldexpf(out[o][r], sh) : out[o][r]) : 0.0f;
            }
        PROF_ADD(kPfBwdEpi, t_be);
    }
    PROF_T(t_t);
    // act holds G_0
    float* g0 = a.grad + a.grad_off[0] + blk * (size_t)(a.nt[0] * 1024);
    if (a.d_x) {
        // d_layer_input = G_0 W_0^T (ENCODED mode); the pass also writes G_0's slab
        zero_tiles(out);
        const float xm = sample_max(act);
        store_emin(a, 0, exa.get(0), store_sexp(a, 0, 1, xm));
        const int ex = shift_of(xm);
        const int sh = unscale(0, ex);
        k32_pass_n<PL>(a, a.ks_b[0], ci, ring, bias_ring, a.to_b[0], act, out, g0, ex);
        if (valid) {
#pragma unroll
            for (int o = 0; o < kMaxT; ++o)
                if (32 * o < a.k0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int f = feat_of(o, r, h);
                        if (f < a.k0) a.d_x[(size_t)gs * a.k0 + f] = PL >= 2 ? __builtin_ldexpf(out[o][r], sh) : out[o][r];
                    }
                }
        }
    } else {
        store_emin(a, 0, exa.get(0), store_sexp(a, 0, 1, sample_max(act)));
#pragma unroll
        for (int t = 0; t < kMaxT; ++t)
            if (t < a.ks_b[0]) store_slab_tile(g0 + t * 1024, act[t]);
    }
#if LNERF_PROF
    PROF_ADD(kPfTail, t_t);
    PROF_ADD(kPfTotal, t_start);
    if (lane == 0) prof_slots()[kPfReal] += __builtin_amdgcn_s_memrealtime() - rt_start;
    if (lane < kPfN) atomicAdd(&g_k32_prof[lane], prof_slots()[lane]);
#endif
}

// ---- weight packing: per layer and pass, input tile t = [s 2][o][plane][lane 64][8 x 16-bit] ----
// forward:  A[m = out 32o + (lane & 31)][k = 8 (lane >> 5) + j] = W[kappa(t, s, lane >> 5, j)][32o + m]
// backward: A[m = in  32o + (lane & 31)][...]                   = W[32o + m][kappa(t, s, lane >> 5, j)]
struct Pack32Args {
    int L;
    int k[kMaxLayers], n[kMaxLayers];
    int ks_f[kMaxLayers], ks_b[kMaxLayers], to_f[kMaxLayers], to_b[kMaxLayers];
    int w_k, w_n, planes;
    const float* W;
    const float* B;
    unsigned short* w32;
    size_t wf_off[kMaxLayers], wb_off[kMaxLayers];
    float* b16;
    int* wexp;   // planes = 2: per-layer max|W| bits (from wmax32_kernel partials)
    int* wpart;  // [L][kWmaxParts] partial max|W| bits
};

// planes = 2: max|W_l| as the bits of a non-negative float, one partial per block, grid
// (kWmaxParts, L): plain stores; the packing kernel folds a layer's partials itself.
__global__ void __launch_bounds__(256) wmax32_kernel(Pack32Args a) {
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
        a.wpart[l * kWmaxParts + blockIdx.x] = __float_as_int(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

__device__ __forceinline__ int layer_wmax(Pack32Args& a, int l) {
    int mb = 0;
    for (int i = 0; i < kWmaxParts; ++i) mb = max(mb, a.wpart[l * kWmaxParts + i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.wexp[l] = mb;
    return mb;
}

// every layer in one launch: grid (blocks of the largest layer, L)
__global__ void pack32_kernel(Pack32Args a) {
    const int l = blockIdx.y;
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const int wsh = a.planes == 2 ? wshift_of(layer_wmax(a, l)) : 0;
    const size_t nf = (size_t)a.ks_f[l] * 2 * a.to_f[l] * 512, nb = (size_t)a.ks_b[l] * 2 * a.to_b[l] * 512;
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
        const int s = (int)(x & 1), t = (int)(x >> 1);
        const int f = kappa(t, s, ln >> 5, j), m = 32 * o + (ln & 31);
        const int kk = fwd ? f : m, jj = fwd ? m : f;
        const float w = (kk < K && jj < N) ? W[(size_t)kk * a.w_n + jj] : 0.0f;
        unsigned short* dst = a.w32 + (fwd ? a.wf_off[l] : a.wb_off[l]) +
                              ((size_t)((2 * t + s) * to + o) * a.planes) * 512 + ln * 8 + j;
        if (a.planes == 2) {
            _Float16 hh, lo;
            split_h(__builtin_ldexpf(w, wsh), hh, lo);
            dst[0] = __builtin_bit_cast(unsigned short, hh);
            dst[512] = __builtin_bit_cast(unsigned short, lo);
            continue;
        }
        __bf16 hh, mi, lo;
        split_x(w, hh, mi, lo);
        dst[0] = __builtin_bit_cast(unsigned short, hh);
        if (a.planes == 3) {
            dst[512] = __builtin_bit_cast(unsigned short, mi);
            dst[1024] = __builtin_bit_cast(unsigned short, lo);
        }
    }
}

// ReLU decisions of the last training k1 as a dense bitmap: out[(l R + r) 32 + f / 8] bit f % 8 =
// feature f of hidden layer l at sample row r was positive (nerf.py:141-144). One thread per
// output byte; feature f = 32 t + (r & 3) + 8 (r >> 2) + 4 h sits in lane h 32 + n, bit 16 t + r
// (t < 4 in word 0, t >= 4 in word 1).
__global__ void k32_masks_kernel(const unsigned long long* __restrict__ mask_g, int L1, int R, int tile_samples,
                                 unsigned char* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)L1 * R * 32) return;
    const int b = (int)(idx & 31);
    const size_t lr = idx >> 5;
    const int l = (int)(lr / R), r = (int)(lr % R);
    const int wg = r / tile_samples, ls = r % tile_samples, wave = ls >> 5, n = ls & 31;
    const unsigned long long* w = mask_g + ((size_t)(wg * L1 + l) * kWaves + wave) * 128;
    unsigned v = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int f = 8 * b + q, t = f >> 5, fr = f & 31;
        const int hh = (fr >> 2) & 1, rr = (fr & 3) + 4 * (fr >> 3);
        const unsigned long long word = w[(hh * 32 + n) * 2 + (t >> 2)];
        v |= (unsigned)((word >> (16 * (t & 3) + rr)) & 1ull) << q;
    }
    out[idx] = (unsigned char)v;
}

}  // namespace

void k32_masks_launch(const FusedPlan& p, unsigned char* out, hipStream_t s) {
    const size_t n = (size_t)(p.L - 1) * p.R * 32;
    if (n == 0) return;
    k32_masks_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(p.mask_g, p.L - 1, p.R, p.rays_per_wg * p.S, out);
}

bool k32_supported(const FusedPlan& p) {
    if (p.x6 != 3 && p.x6 != 2 && p.x6 != 1) return false;
    if (p.n[p.L - 1] > 32) return false;       // head: one 32-wide output tile
    return true;
}

void k32_pack(const FusedPlan& p, const float* ws, const float* bs, hipStream_t s) {
    Pack32Args a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.k[l] = p.k[l];
        a.n[l] = p.n[l];
        a.ks_f[l] = p.ks16_f[l];
        a.ks_b[l] = p.ks16_b[l];
        a.to_f[l] = p.to32_f[l];
        a.to_b[l] = p.to32_b[l];
        a.wf_off[l] = p.w32f_off[l];
        a.wb_off[l] = p.w32b_off[l];
    }
    a.w_k = p.w_k;
    a.w_n = p.w_n;
    a.planes = p.x6;
    a.W = ws;
    a.B = bs;
    a.w32 = p.w16;
    a.b16 = p.b16;
    a.wexp = p.wexp16;
    a.wpart = p.wmax_part;
    if (a.planes == 2) wmax32_kernel<<<dim3(kWmaxParts, p.L), 256, 0, s>>>(a);
    size_t nmax = 0;
    for (int l = 0; l < p.L; ++l) {
        const size_t nel = ((size_t)a.ks_f[l] * 2 * a.to_f[l] + (size_t)a.ks_b[l] * 2 * a.to_b[l]) * 512 + 256;
        nmax = nel > nmax ? nel : nmax;
    }
    pack32_kernel<<<dim3((unsigned)((nmax + 255) / 256), p.L), 256, 0, s>>>(a);
}

void k32_launch(const FusedPlan& p, const lnerf_batch& b, float seed, const lnerf_outputs& out,
                bool want_grad, hipStream_t s) {
    K32Args a{};
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.ks_f[l] = p.ks16_f[l];
        a.ks_b[l] = p.ks16_b[l];
        a.to_f[l] = p.to32_f[l];
        a.to_b[l] = p.to32_b[l];
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.wf_off[l] = p.w32f_off[l];
        a.wb_off[l] = p.w32b_off[l];
        a.act_off[l] = p.act_off[l];
        a.grad_off[l] = p.grad_off[l];
    }
    a.k0 = p.k[0];
    a.w32 = p.w16;
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
    a.sexp = p.sexp;
    a.rpad = p.num_wg * 128;
    a.epart = p.epart;
    // the chunk stream: one chunk per input tile; forward 0..L-1, backward L-1..1 (training),
    // backward 0 (d_x)
    {
        int ci = 0;
        auto add = [&](bool fwd, int l) {
            const int ks = fwd ? a.ks_f[l] : a.ks_b[l], to = fwd ? a.to_f[l] : a.to_b[l];
            const size_t per = (size_t)2 * to * a.planes * 512;   // u16 per input tile
            for (int t = 0; t < ks; ++t, ++ci) {
                a.chunk_tab[2 * ci] = (unsigned)((fwd ? a.wf_off[l] : a.wb_off[l]) + (size_t)t * per);
                a.chunk_tab[2 * ci + 1] = (unsigned)(per * 2 / 1024) | ((fwd && t == 0 ? l + 1 : 0) << 16);
            }
        };
        for (int l = 0; l < p.L; ++l) add(true, l);
        if (want_grad)
            for (int l = p.L - 1; l >= (a.d_x ? 0 : 1); --l) add(false, l);
        // two zero entries past the end (the kernel looks two chunks ahead): a{} zeroed them
    }
    static_assert(sizeof(K32Args) <= 4096, "kernel arguments");
#define LNERF_K32_LAUNCH(HT)                                                              \
    if (p.x6 == 3) k32_fwd_bwd_kernel<HT, 3><<<p.num_wg, kThreads, 0, s>>>(a);            \
    else if (p.x6 == 2) k32_fwd_bwd_kernel<HT, 2><<<p.num_wg, kThreads, 0, s>>>(a);       \
    else k32_fwd_bwd_kernel<HT, 1><<<p.num_wg, kThreads, 0, s>>>(a);
#ifdef LNERF_K32_ONLY_8_2   // compile-time experiments: one instantiation
    k32_fwd_bwd_kernel<8, 2><<<p.num_wg, kThreads, 0, s>>>(a);
#else
    switch (p.ht32) {
        case 1: LNERF_K32_LAUNCH(1) break;
        case 2: LNERF_K32_LAUNCH(2) break;
        case 4: LNERF_K32_LAUNCH(4) break;
        default: LNERF_K32_LAUNCH(8) break;
    }
#endif
#undef LNERF_K32_LAUNCH
#if LNERF_PROF
    if (want_grad) {
        unsigned long long hh[16] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(hh, HIP_SYMBOL(g_k32_prof), sizeof(hh));
        const char* names[] = {"pe", "fwd_pass", "fwd_epilogue", "barrier", "composite", "bwd_pass",
                               "bwd_epilogue", "tail", "total", "vmcnt_wait", "realtime_100MHz"};
        fprintf(stderr, "LNERF_PROF k32 per-wave cycles:");
        for (int i = 0; i < kPfN; ++i) fprintf(stderr, " %s=%.0f", names[i], hh[i] / ((double)p.num_wg * kWaves));
        fprintf(stderr, " clock_GHz=%.3f\n", hh[kPfReal] ? (double)hh[kPfTotal] / hh[kPfReal] * 0.1 : 0.0);
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_k32_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
