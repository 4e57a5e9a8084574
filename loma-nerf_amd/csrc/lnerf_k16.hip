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

// NW = waves per workgroup, 16 samples each: 8 (512 threads, a 128-sample tile, one workgroup
// per CU) or 4 (256 threads, a 64-sample tile, two workgroups per CU: the two waves of a SIMD
// then belong to different workgroups, so one's barrier waits, epilogues and compositing run
// beside the other's MFMAs instead of in lockstep with them)
constexpr int kWaves = 8;                     // the most waves per workgroup
constexpr int kMaxChunks = 2 * kMaxLayers * 8 + 1;   // <= 2 passes x 8 k-steps per layer + 1 end
constexpr int kMaxT = 16;                     // 16-feature tiles per 256-wide layer
constexpr int kCompBytes = 2688 * 4;          // composite_tile's scratch (comp[0, 2688))
// full hidden passes get compile-time step bounds and test-free DMA issue (A/B: 0 = generic only)
#ifndef LNERF_K16_FULLDMA
#define LNERF_K16_FULLDMA 1
#endif

// The weight stream of a PL-plane kernel. A chunk is KC k-steps (32 input features each) x every
// output tile x PL planes, delivered by LDS-DMA into one slot of a ring, one workgroup barrier per
// chunk (the barrier count, not the bytes, is what a 32-deep k-step costs: BK 64 over 32).
//  * fp16x3 / plain bf16 (PL <= 2): KC = 2 (64 KiB per chunk at 16 tiles x 2 planes), two slots:
//    chunk c + 1 lands while chunk c is computed.
//  * bf16x6 (PL = 3): KC = 1 -- two 96 KiB chunks would not fit -- with staggered wave pairs:
//    waves 0-3 meet the per-chunk barrier at the end of a chunk, waves 4-7 (each the SIMD partner
//    of an early wave) in its middle, so the two waves of a SIMD run their chunk prologues half a
//    chunk apart; the ring then needs 3 slots (the late waves still read the previous chunk
//    while every wave reads the current one and the next one lands).
//  * NW = 4 (two workgroups per CU, each within 80 KiB of LDS): KC = 1, two 32 KiB slots.
//  * NG = 2 (two 16-sample groups per wave, NW = 4: one wave per SIMD, a 128-sample tile): every
//    weight fragment read from LDS feeds both groups' MFMAs; the ring as NW = 8 (KC = 2, two 64 KiB
//    slots), 16 pieces per wave per chunk.
template <int PL, int NW = 8, int NG = 1>
struct Ring {
    static constexpr int KC = (PL == 3 || (NW == 4 && NG == 1)) ? 1 : 2;
    static constexpr bool stagger = PL == 3 && NW == 8;
    static constexpr int slots = stagger ? 3 : 2;
    static constexpr int slot_bytes = KC * kMaxT * PL * 1024;
    static constexpr int pieces = slot_bytes / (NW * 1024);   // per wave, a whole chunk
    static constexpr int off_comp = slots * slot_bytes;
    static constexpr int off_ray = off_comp + kCompBytes;
    static constexpr int off_bias = off_ray + 16 * NW * NG * 4;
    static constexpr int lds_bytes = off_bias + 3 * 256 * 4;   // + a 3-slot ring of layer biases
    static_assert(lds_bytes + 1024 <= 160 * 1024, "LDS budget (+1 KiB for the profiling build)");
    static_assert((KC * kMaxT - 1) * PL * 1024 < 65536, "ds_read offsets are 16-bit immediates");
};

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
    const int* hexp;   // PL = 2: the head's per-column max|W| bits (head_col_shift)
    // training: every sample's word per layer (lnerf_internal.h sexp_xa / sexp_xg / sexp_dmax),
    // [l][position] x 4 bytes: byte 0 the exponent shift of layer l's input row (X, A_l-1), byte 2
    // G_l's, byte 3 the row's exceptional-row bound dmax; position = half-block * 16 + sample
    unsigned char* sexp;
    int rpad;          // slab positions (num_wg * 128)
    int* epart;        // training: per-wave min over samples of exA + exG, [l][num_wg * 8]
    int head_fit;      // the mlp_fit head (comp::fit_tile) instead of the NeRF compositing
    int nout;          // head outputs (the mlp_fit head's width)
    int* guard;        // PL = 2 training, nullable: set when a hidden G row fails the floor (kGuardExp)
    const int* gate;   // nullable: the launch exits at once unless *gate != 0 (the guard's re-run)
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

// One LDS-DMA wave instruction (global_load_lds_dwordx4: 16 B per lane, lane-linear into the
// wave-uniform LDS address `lds`), from inline asm with M0 written in the same statement.
// Why asm: an LDS-DMA the compiler can see makes it wait vmcnt(0) before every later LDS read
// (it cannot tell the ring slots apart), which would drain the next chunk's DMA; hidden from it,
// the transfer has no register destination (nothing the compiler could copy or reuse early) and
// its completion is counted by hand (dma_barrier's vmcnt). The `s_nop 0` is the M0-write ->
// LDS-DMA wait state. No compiler code in these kernels reads M0 (tests/test_isa.py checks it).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc),
                 "s"(__builtin_amdgcn_readfirstlane(lds)));
}

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
template <int NW>
__device__ __forceinline__ int dma_chunk(const K16Args& a, const ChunkT& c, unsigned char* dst,
                                         float* bias_ring) {
    const int tid = threadIdx.x, wave = wave_id();
    int n = 0;
    if (!c.src) return 0;
    for (int off = wave * 1024; off < c.bytes; off += NW * 1024) {
        glds16((const char*)c.src + off + (tid & 63) * 16, lds_addr(dst + off));
        ++n;
    }
    if (c.bias >= 0 && wave == NW - 1) {
        glds16(a.b16 + (size_t)c.bias * 256 + (tid & 63) * 4, lds_addr(bias_ring + (c.bias % 3) * 256));
        ++n;
    }
    return n;
}

// The chunk the next k-step reads has landed (this wave's pieces: vector-memory operations retire
// in issue order, so at most `pending` outstanding -- the slab stores issued after the pieces --
// means every piece is done; compiler VM operations in between only make the wait stricter),
// every LDS read this wave issued has returned (lgkmcnt(0): the slot the next DMA overwrites is
// read out -- the compiler may sink the MFMAs that consume those reads below the barrier, not the
// reads), then s_barrier: every wave's pieces are in LDS and every wave is done with that slot.
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
// pending < 0: this wave has no DMA piece to wait for (only the barrier); otherwise the number of
// this wave's vector-memory operations issued after its pieces (the chunk's slab stores)
__device__ __forceinline__ void dma_barrier(int pending) {
    PROF_T(t0);
    asm volatile("" ::: "memory");
    if (pending == 0) vm_wait<0>();
    else if (pending == 2) vm_wait<2>();
    else if (pending == 4) vm_wait<4>();
    else if (pending == 8) vm_wait<8>();
    else if (pending > 0) vm_wait_n(pending, std::make_integer_sequence<int, 64>{});
    PROF_ADD(kPfVm, t0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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

// the exponent shift ew of a layer from its max|W| bits (fp16x3_shift) -- the weight-side half
// of the fp16x3 scaling
__device__ __forceinline__ int wshift_of(int maxbits) { return fp16x3_shift(__int_as_float(maxbits)); }

// The head's per-column weight shift (planes = 2): column n of the head's packed planes is scaled by
// 2^head_col_shift(n) -- its own max|W[:, n]| in [2^13, 2^14) -- instead of the layer's shift, so a
// column far below the others (a sigma output whose weights are 2^-20 or 2^-30 of the rgb ones)
// keeps fp16's normal range. An all-zero column keeps the layer's shift.
__device__ __forceinline__ int head_col_shift(int colmax_bits, int layer_bits) {
    return colmax_bits > 0 ? wshift_of(colmax_bits) : wshift_of(layer_bits);
}


// x = hi + mid + lo (round-to-nearest bf16 of each remainder; every remainder is exact in f32)
__device__ __forceinline__ void split_x(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

// Slab tile store: the 8 features of k-step s that a lane holds for its sample n (registers 0-3 of
// tiles 2s and 2s+1 = features 4g ..+3 and 16 + 4g ..+3 of the 32-feature tile) into this wave's
// sample-major half-block [feature half 2][16 samples][16 features]: two global_store_dwordx4,
// each wave instruction one contiguous 1 KiB (lnerf_dw16.hip reads it back transposed).
__device__ __forceinline__ void store_slab_step(float* __restrict__ dst, const fx4& t0, const fx4& t1) {
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
    __builtin_nontemporal_store(t0, (fx4*)(dst + n * 16 + 4 * g));
    __builtin_nontemporal_store(t1, (fx4*)(dst + 256 + n * 16 + 4 * g));
}

// The same k-step store for an int24 activation slab (lnerf_internal.h a24_slabs): the 8 values
// as y = x 2^(ex + 8) + 1.5 2^23 (round-to-nearest integer q in the mantissa field, |q| < 2^22;
// ex = the sample's row shift), their low 24 bits packed 4 to 12 B by v_perm_b32, two
// global_store_dwordx3 into the 1.5-KiB half-block run [feature half 2][16 samples][16 f] x 3 B.
typedef unsigned u3a __attribute__((ext_vector_type(3), aligned(4)));
struct Packed24 {
    u3a p0, p1;
};
// the 8 values as y = x 2^(ex + 8) + 1.5 2^23, low 24 bits of four y packed into 12 B (v_perm_b32)
__device__ __forceinline__ Packed24 pack_slab_step24(const fx4& t0, const fx4& t1, int ex) {
    constexpr float kMagic = 12582912.0f;   // 1.5 2^23
    auto pack = [&](const fx4& t) {
        unsigned y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = __builtin_bit_cast(unsigned, __builtin_ldexpf(t[i], ex + 8) + kMagic);
        return u3a{__builtin_amdgcn_perm(y[1], y[0], 0x04020100u), __builtin_amdgcn_perm(y[2], y[1], 0x05040201u),
                   __builtin_amdgcn_perm(y[3], y[2], 0x06050402u)};
    };
    return Packed24{pack(t0), pack(t1)};
}
// two global_store_dwordx3 into the 1.5-KiB half-block run [feature half 2][16 samples][16 f] x 3 B
// (4-byte aligned: the 12-B runs sit at 12 g; a plain 3-vector claims 16-B size and alignment,
// which would let the compiler widen the store over the neighbouring lane's bytes)
__device__ __forceinline__ void store_packed24(unsigned char* __restrict__ dst, const Packed24& v) {
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
    __builtin_nontemporal_store(v.p0, (u3a*)(dst + n * 48 + 12 * g));
    __builtin_nontemporal_store(v.p1, (u3a*)(dst + 768 + n * 48 + 12 * g));
}
__device__ __forceinline__ void store_slab_step24(unsigned char* __restrict__ dst, const fx4& t0, const fx4& t1,
                                                  int ex) {
    store_packed24(dst, pack_slab_step24(t0, t1, ex));
}

// Materialise a value here: an empty asm that reads and writes it in place (no instruction; the
// compiler may not compute it later than this point, nor move this point across the
// sched_barriers around it)
template <typename T>
__device__ __forceinline__ void pin(T& v) {
    asm volatile("" : "+v"(v));
}

// A weight fragment: one ds_read_b128 per lane (the compiler counts it and places its wait).
template <int OFF>
__device__ __forceinline__ bf8 lds_frag(const unsigned char* base) {
    return *(const bf8*)(base + OFF);
}

#ifndef LNERF_K16_KDIST
#define LNERF_K16_KDIST 2
#endif
constexpr int kDist = LNERF_K16_KDIST;
// where the next k-step's operand split sits among this k-step's output tiles, in quarters
#ifndef LNERF_K16_SPLIT_AT
#define LNERF_K16_SPLIT_AT 2
#endif   // weight tiles read ahead of the one the MFMAs consume
#ifndef LNERF_K16_SCHED
#define LNERF_K16_SCHED 1
#endif

template <int PL, int O>
__device__ __forceinline__ void read_tile(const unsigned char* base, bf8 (&w)[3]) {
    w[0] = lds_frag<(O * PL + 0) * 1024>(base);
    if constexpr (PL >= 2) w[1] = lds_frag<(O * PL + 1) * 1024>(base);
    if constexpr (PL == 3) w[2] = lds_frag<(O * PL + 2) * 1024>(base);
}

// This wave's share of the next chunk's LDS-DMA, issued piece by piece between the MFMAs of the
// first k-step of a chunk (LNERF_K16_SPREAD) instead of as one burst after the barrier, where
// both waves of a SIMD would issue theirs together with no MFMA to hide behind. Piece p is the
// wave instruction at byte wave * 1 KiB + p * 8 KiB of the chunk (1 KiB, lane-linear).
#ifndef LNERF_K16_PRIO
#define LNERF_K16_PRIO 0
#endif
#ifndef LNERF_K16_SPREAD
#define LNERF_K16_SPREAD 1
#endif
// PIN 2: the next k-step's operand split and this k-step's int24 slab packing run as VALU fillers
// spread over the first 12 of 16 output tiles (FillSpread), each result pinned there by an empty
// asm that "reads and writes" its registers in place; 0: the compiler sinks both next to their
// first use, at the k-step boundary, where both waves of a SIMD issue them together (round 5,
// interleaved A/B with FDSRC: k1 1.33-1.35 ms against 1.36-1.39)
#ifndef LNERF_K16_PIN
#define LNERF_K16_PIN 2
#endif
// FDSRC: a whole chunk of a full pass takes its source address from the pass base (an SGPR the
// layer loop loads once) instead of the chunk table (a scalar load + lgkmcnt(0) per chunk, right
// after the barrier)
#ifndef LNERF_K16_FDSRC
#define LNERF_K16_FDSRC 1
#endif
// ONECHUNK: a one-tile pass (the head's forward; hidden layers <= 16 wide) streams all its <= 8
// k-steps as ONE chunk (<= 8 PL KiB), one barrier instead of ks / KC, each of which waited on a DMA
// issued only a few MFMAs earlier (round 5, in-process interleaved A/B: k1 -0.9 %)
#ifndef LNERF_K16_ONECHUNK
#define LNERF_K16_ONECHUNK 1
#endif
// k-steps per chunk of a pass with NTO output tiles (k16_launch's chunk table follows the same rule)
template <int NTO, int PL, int NW, int NG = 1>
constexpr int pass_kc() {
    return (LNERF_K16_ONECHUNK && NTO == 1) ? 8 : Ring<PL, NW, NG>::KC;
}
// G2: k1 on two 16-sample groups per wave at one wave per SIMD (k16_fwd_bwd_kernel<16, 2, 4, 2>), every
// weight fragment feeding both groups' MFMAs (round 6 A/B)
#ifndef LNERF_K16_G2
#define LNERF_K16_G2 0
#endif
// EPIFMA: the forward epilogue's unscale and bias as one fma (round 5, in-process A/B: k1
// 1.279 -> 1.261 ms; round 4's bench-level A/B had called it neutral)
#ifndef LNERF_K16_EPIFMA
#define LNERF_K16_EPIFMA 1
#endif
// WAVECOMP: the compositing's along-ray scans in-wave (comp::composite_tile_wave: 4 workgroup
// barriers instead of 3 log2 S + 4; round 5: k1 -0.2 %, with ONECHUNK -1.1 %)
#ifndef LNERF_K16_WAVECOMP
#define LNERF_K16_WAVECOMP 1
#endif
constexpr int kPiecesMax = 8;   // pieces per wave of a full chunk (64 KiB / 8 waves, 32 KiB / 4; NG = 2: 16)
struct DmaJob {
    const char* src = nullptr;   // the wave's (uniform) address of piece 0
    unsigned char* dst = nullptr;   // LDS address of this wave's piece 0
    int n = 0;                   // this wave's pieces of the chunk
};
template <int NW>
__device__ __forceinline__ void dma_piece(const DmaJob& j, int p) {
    const int lane = threadIdx.x & 63;
    glds16(j.src + p * (NW * 1024) + lane * 16, lds_addr(j.dst + p * (NW * 1024)));
}
// the pieces that land on output tile O: p with p * NTO / kPiecesMax == O (all on tile 0 when NTO == 1);
// FULL: the chunk is known to be whole (every wave issues kPiecesMax pieces, no per-piece test)
template <int NTO, int O, int NW, bool FULL, int... P>
__device__ __forceinline__ void dma_pieces_at(const DmaJob& j, std::integer_sequence<int, P...>) {
    constexpr int KP = sizeof...(P);
    (((P * NTO) / KP == O ? ((FULL || P < j.n) ? dma_piece<NW>(j, P) : void()) : void()), ...);
}

// Output tile O of one k-step: issue the reads of tile O + kDist, the MFMAs of tile O (small
// terms first; the compiler waits for tile O's reads only, lgkmcnt(N) with the younger ones in
// flight).
// The output tile after which a k-step splits its next operands (and a late wave of a staggered
// pair meets the chunk barrier)
template <int NTO>
constexpr int half_tiles() {
    return NTO >= 4 ? NTO * LNERF_K16_SPLIT_AT / 4 : (NTO + 1) / 2;
}

// The staggered wave pairs (bf16x6) branch on the wave's half right after a k-step's MFMAs (the
// late or the early barrier); on the short side of that branch the compiler's hazard padding has
// come up short (tests/test_isa.py: a VALU write 2 wait states after an MFMA reading the register as
// C, an MFMA result read 4-7 states after issue). 16 wait states here, on every path, cover any
// MFMA of the kernel. The statement takes the last tile's accumulator in place, so that tile's
// MFMAs cannot be scheduled below it (in-place operand, no instruction writes it).
__device__ __forceinline__ void mfma_branch_guard(fx4& acc) { asm volatile("s_nop 7\n\ts_nop 7" : "+v"(acc)::"memory"); }

// no VALU filler between the tiles (see FillSpread)
struct NoFill {
    template <int O>
    __device__ __forceinline__ void at() {}
};

// FDP: how this k-step issues the next chunk's DMA: 0 generic (per-piece tests), 3 a whole chunk's
// 8 pieces (round 5: spreading them over both k-steps of the chunk measured +0.3 % in k1)
template <int NTO, int PL, int NW, int NG, int FDP, int O, typename F = NoFill>
__device__ __forceinline__ void tile_step(const unsigned char* base, bf8 (&w)[kDist + 1][3], const bf8 (&bh)[NG],
                                          const bf8 (&bm)[NG], const bf8 (&bl)[NG], fx4 (&out)[NG][kMaxT],
                                          const DmaJob& job, F& fill) {
    constexpr int KP = Ring<PL, NW, NG>::pieces < kPiecesMax ? kPiecesMax : Ring<PL, NW, NG>::pieces;
    if constexpr (O + kDist < NTO) read_tile<PL, O + kDist>(base, w[(O + kDist) % (kDist + 1)]);
    if constexpr (FDP == 3) dma_pieces_at<NTO, O, NW, true>(job, std::make_integer_sequence<int, KP>{});
    else if (job.n) dma_pieces_at<NTO, O, NW, false>(job, std::make_integer_sequence<int, KP>{});
    // keep tile O + kDist's reads ahead of tile O's MFMAs: the machine scheduler otherwise sinks
    // each read next to its first consumer (one MFMA of slack, an LDS round trip exposed per tile);
    // the compiler still places every wait itself
    if constexpr (LNERF_K16_SCHED) __builtin_amdgcn_sched_barrier(0);
    bf8(&c)[3] = w[O % (kDist + 1)];
    // every group's products from the same fragments (NG = 2: half the LDS bytes per MFMA)
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        fx4 acc = out[q][O];
        if constexpr (PL == 2) {
            // fp16x3: small terms first (w_hi x_lo, w_lo x_hi), then w_hi x_hi; (bh, bm) = (x_hi, x_lo)
            acc = mfma16h(c[0], bm[q], acc);
            acc = mfma16h(c[1], bh[q], acc);
            acc = mfma16h(c[0], bh[q], acc);
        } else if constexpr (PL == 3) {
            acc = mfma16(c[0], bl[q], acc);
            acc = mfma16(c[1], bm[q], acc);
            acc = mfma16(c[2], bh[q], acc);
            acc = mfma16(c[1], bh[q], acc);
            acc = mfma16(c[0], bm[q], acc);
            acc = mfma16(c[0], bh[q], acc);
        } else {
            acc = mfma16(c[0], bh[q], acc);
        }
        out[q][O] = acc;
    }
    fill.template at<O>();
}

// tiles B, B+1, ... of one k-step
template <int NTO, int PL, int NW, int NG, int FDP, int B, typename F, int... O>
__device__ __forceinline__ void tile_steps(std::integer_sequence<int, O...>, const unsigned char* base,
                                           bf8 (&w)[kDist + 1][3], const bf8 (&bh)[NG], const bf8 (&bm)[NG],
                                           const bf8 (&bl)[NG], fx4 (&out)[NG][kMaxT], const DmaJob& job, F& fill) {
    (tile_step<NTO, PL, NW, NG, FDP, B + O>(base, w, bh, bm, bl, out, job, fill), ...);
}

// LNERF_K16_PIN = 2 (fp16x3, 16 output tiles): the next k-step's operand split and this k-step's
// int24 packing as VALU fillers spread over the first 12 tiles, a few instructions after each
// tile's MFMAs (pair q of the split after tile 2q + 1, the two 12-B packs after tiles 9 and 11),
// each result pinned there (in place, no instruction) so the compiler cannot sink it back to the
// k-step boundary
template <int NG>
struct FillSpread {
    const fx4 (*in)[kMaxT];   // the pass input per group (in[q][2 sn], in[q][2 sn + 1]: the next k-step's features)
    int sn;               // the next k-step
    bool split;           // there is a next k-step
    float sc[NG];         // 2^ex per group
    unsigned hv[NG][4], lv[NG][4];
    bool pack;            // this k-step's int24 slab values are packed (stored after the last tile)
    int s, ex[NG];
    Packed24 pk[NG];
    // group q's split pair k after tile 2 k + 1 + q, its two 12-B packs after tiles 9 + q and 11 + q
    template <int O>
    __device__ __forceinline__ void at() {
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            if constexpr (O >= 1 && O <= 7 + NG - 1) {
                if ((O - 1 - q) >= 0 && (O - 1 - q) % 2 == 0 && (O - 1 - q) / 2 < 4) {
                    const int k = (O - 1 - q) / 2;
                    if (split) {
                        const fx4& t = in[q][2 * sn + (k >> 1)];
                        split_h2(t[2 * (k & 1)], t[2 * (k & 1) + 1], sc[q], hv[q][k], lv[q][k]);
                        pin(hv[q][k]);
                        pin(lv[q][k]);
                    }
                }
            }
            if (pack && (O == 9 + q || O == 11 + q)) {
                const Packed24 p = pack_slab_step24(in[q][2 * s], in[q][2 * s + 1], ex[q]);
                if (O == 9 + q) {
                    pk[q].p0 = p.p0;
                    pin(pk[q].p0);
                } else {
                    pk[q].p1 = p.p1;
                    pin(pk[q].p1);
                }
            }
        }
    }
};

// The B operand planes of k-step s (the lane's 8 input features phi(s, g, 0..7) of its sample):
// bf16x6 hi/mid/lo, fp16x3 hi/lo (x 2^ex), or plain bf16.
template <int PL>
__device__ __forceinline__ void make_b(const fx4 (&in)[kMaxT], int s, int ex, bf8& bh, bf8& bm, bf8& bl) {
    if constexpr (PL == 2) {
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
        const float sc = PL == 3 ? __builtin_ldexpf(1.0f, ex) : 1.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float x = j < 4 ? in[2 * s][j] : in[2 * s + 1][j - 4];
            if (PL == 3) {
                __bf16 h, m, l;
                split_x(x * sc, h, m, l);
                bh[j] = h;
                bm[j] = m;
                bl[j] = l;
            } else {
                bh[j] = (__bf16)x;
            }
        }
    }
}

// One k-step s of a pass (compile-time after unrolling): out[o] += Wpack[s][o] (x) in[2s..2s+1]
// from sub-step kk of ring slot ci % slots. The chunk's first k-step (kk = 0) issues the DMA of
// chunk ci + 1 and its last (LAST) meets the barrier that waits for it. (bh, bm, bl) hold k-step
// s's B planes on entry and k-step s + 1's on exit. `slab` (nullable) receives the input tiles
// (the A_{l-1} or G_l slab of this wave's half-block).
// FD: this k-step issues the DMA of a chunk known to be whole (the next chunk of the same full
// pass): kPiecesMax pieces per wave with no per-piece test and no byte arithmetic.
template <int NTO, int PL, int NW, int NG, int FDP = 0, bool A24 = false>
__device__ __forceinline__ void k16_step(const K16Args& a, int ks, int s, int kk, bool last, int& ci,
                                         unsigned char* ring, float* bias_ring, const fx4 (&in)[NG][kMaxT],
                                         fx4 (&out)[NG][kMaxT], float* const (&slab)[NG], const int (&ex)[NG],
                                         bf8 (&bh)[NG], bf8 (&bm)[NG], bf8 (&bl)[NG], int& pending,
                                         const unsigned short* fdsrc) {
    using R = Ring<PL, NW, NG>;
    constexpr int KC_BYTES = R::KC * NTO * PL * 1024;
    constexpr int KP = R::pieces < kPiecesMax ? kPiecesMax : R::pieces;
    const int lane = threadIdx.x & 63;
    const unsigned char* base = ring + (ci % R::slots) * R::slot_bytes + kk * NTO * PL * 1024 + lane * 16;
    const bool st = slab[0] != nullptr;
    constexpr bool spread = LNERF_K16_SPREAD && !R::stagger;
    constexpr bool FD = FDP != 0;
    DmaJob job;
    if (kk == 0) {
        // DMA of chunk ci + 1 (its table entry is a scalar load the compiler waits for with
        // lgkmcnt(0), so it is read before the fragment reads are issued). Unspread: every piece
        // now, before the first weight tiles; spread: one piece per KP-th of the output
        // tiles, between the MFMAs. The barrier waits for this wave's pieces of chunk ci + 1 only:
        // the slab stores issued after them (two per k-step and group) stay in flight.
        // FDSRC: the next chunk of this full pass, whole, no biases (fdsrc = its source)
        const ChunkT c = (FD && LNERF_K16_FDSRC) ? ChunkT{fdsrc, KC_BYTES, -1} : chunk_at(a, ci + 1);
        unsigned char* dst = ring + ((ci + 1) % R::slots) * R::slot_bytes;
        int issued;
        if constexpr (spread) {
            const int wave = wave_id();
            const int woff = wave * 1024;
            job.n = FD ? KP
                       : (c.src && woff < c.bytes) ? (c.bytes - woff + NW * 1024 - 1) / (NW * 1024) : 0;
            job.src = (const char*)c.src + woff;
            job.dst = dst + woff;
            // the biases of a first forward chunk: one more piece from the last wave, now
            issued = job.n;
            if (c.bias >= 0 && wave == NW - 1) {
                glds16(a.b16 + (size_t)c.bias * 256 + lane * 4, lds_addr(bias_ring + (c.bias % 3) * 256));
                ++issued;
            }
        } else {
            issued = dma_chunk<NW>(a, c, dst, bias_ring);
        }
        asm volatile("" ::: "memory");   // the slab stores stay younger than the pieces
        pending = issued ? 0 : -1;
    }
    if (st && pending >= 0) pending += 2 * NG;
    const bool late = R::stagger && wave_id() >= 4;
    bf8 w[kDist + 1][3];
    read_tile<PL, 0>(base, w[0]);
    if constexpr (NTO > 1) read_tile<PL, 1>(base, w[1]);
    if constexpr (NTO > 2 && kDist > 2) read_tile<PL, 2>(base, w[2]);
    static_assert(kDist == 2 || kDist == 3, "the prologue reads kDist tiles");
    auto store = [&]() {
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            if constexpr (A24) {
                store_slab_step24((unsigned char*)slab[q] + s * 3072, in[q][2 * s], in[q][2 * s + 1], ex[q]);
            } else {
                store_slab_step(slab[q] + s * 1024, in[q][2 * s], in[q][2 * s + 1]);
            }
        }
    };
    if (st && !spread) store();
    // first half of the output tiles, [late waves: barrier], the next k-step's operand split (off
    // the next prologue's critical path), second half, [spread: the slab stores, younger than
    // every piece], [early: barrier]
    constexpr int H = half_tiles<NTO>();   // split after tile H
    constexpr bool spread_fill = LNERF_K16_PIN == 2 && PL == 2 && NTO == 16 && !R::stagger;
    // a late wave meets the barrier before this k-step's spread slab stores: they are not pending yet
    const int late_pending = (st && spread && pending >= 2 * NG) ? pending - 2 * NG : pending;
    if constexpr (spread_fill) {
        FillSpread<NG> f;
        f.in = in;
        f.sn = s + 1 < 8 ? s + 1 : 0;
        f.split = s + 1 < ks;
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            f.sc[q] = __builtin_ldexpf(1.0f, ex[q]);
            f.ex[q] = ex[q];
        }
        f.pack = A24 && st && spread;
        f.s = s;
        tile_steps<NTO, PL, NW, NG, FDP, 0>(std::make_integer_sequence<int, H>{}, base, w, bh, bm, bl, out, job, f);
        if (late && last) dma_barrier(late_pending);
        tile_steps<NTO, PL, NW, NG, FDP, H>(std::make_integer_sequence<int, NTO - H>{}, base, w, bh, bm, bl, out, job,
                                            f);
        if (st && spread) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                if constexpr (A24) store_packed24((unsigned char*)slab[q] + s * 3072, f.pk[q]);
                else store_slab_step(slab[q] + s * 1024, in[q][2 * s], in[q][2 * s + 1]);
            }
        }
        if (!late && last) dma_barrier(pending);
        if (last) ++ci;
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            bh[q] = f.split ? __builtin_bit_cast(bf8, u4{f.hv[q][0], f.hv[q][1], f.hv[q][2], f.hv[q][3]}) : bf8{};
            bm[q] = f.split ? __builtin_bit_cast(bf8, u4{f.lv[q][0], f.lv[q][1], f.lv[q][2], f.lv[q][3]}) : bf8{};
        }
        return;
    }
    NoFill nf;
    tile_steps<NTO, PL, NW, NG, FDP, 0>(std::make_integer_sequence<int, H>{}, base, w, bh, bm, bl, out, job, nf);
    if constexpr (R::stagger) mfma_branch_guard(out[0][H > 0 ? H - 1 : 0]);
    if (late && last) dma_barrier(late_pending);
    bf8 nh[NG] = {}, nm[NG] = {}, nl[NG] = {};
    if (s + 1 < ks) {
#pragma unroll
        for (int q = 0; q < NG; ++q) make_b<PL>(in[q], s + 1 < 8 ? s + 1 : 0, ex[q], nh[q], nm[q], nl[q]);
    }
    tile_steps<NTO, PL, NW, NG, FDP, H>(std::make_integer_sequence<int, NTO - H>{}, base, w, bh, bm, bl, out, job, nf);
    if (st && spread) {
        asm volatile("" ::: "memory");
        store();
    }
    if constexpr (R::stagger) mfma_branch_guard(out[0][NTO - 1]);
    if (!late && last) dma_barrier(pending);
    if (last) ++ci;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        bh[q] = nh[q];
        bm[q] = nm[q];
        bl[q] = nl[q];
    }
}

// One k-step S of a pass. FULL: the pass has all 8 k-steps (a 256-wide input), so the step
// bounds are compile-time and, where the chunk after this one belongs to the same pass and is
// whole (KC NTO PL KiB = kPiecesMax pieces per wave), its DMA is issued without per-piece tests.
template <int NTO, int PL, int NW, int NG, bool FULL, bool A24, int S>
__device__ __forceinline__ void k16_pass_step(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                              float* bias_ring, const fx4 (&in)[NG][kMaxT], fx4 (&out)[NG][kMaxT],
                                              float* const (&slab)[NG], const int (&ex)[NG], bf8 (&bh)[NG],
                                              bf8 (&bm)[NG], bf8 (&bl)[NG], int& pending,
                                              const unsigned short* pbase) {
    constexpr int KC = pass_kc<NTO, PL, NW, NG>();
    using R = Ring<PL, NW, NG>;
    if (FULL || S < ks) {
        constexpr int kk = S % KC;
        const bool last = kk == KC - 1 || (FULL ? S == 7 : S + 1 == ks);
        // (a whole chunk is exactly KP pieces per wave: KP = 8, or 16 for NG = 2)
        constexpr int KP = R::pieces < kPiecesMax ? kPiecesMax : R::pieces;
        constexpr bool whole_next = LNERF_K16_FULLDMA && FULL && S / KC + 1 < 8 / KC &&
                                    KC * NTO * PL == KP * NW && LNERF_K16_SPREAD && !R::stagger;
        constexpr int fd = whole_next && kk == 0 ? 3 : 0;
        // the source of the chunk after this one (S / KC + 1 of the pass), for FDSRC
        const unsigned short* fdsrc = pbase + (size_t)(S / KC + 1) * (KC * NTO * PL * 512);
        k16_step<NTO, PL, NW, NG, fd, A24>(a, FULL ? 8 : ks, S, kk, last, ci, ring, bias_ring, in, out, slab, ex,
                                           bh, bm, bl, pending, fdsrc);
    }
}
template <int NTO, int PL, int NW, int NG, bool FULL, bool A24, int... S>
__device__ __forceinline__ void k16_pass_steps(std::integer_sequence<int, S...>, const K16Args& a, int ks, int& ci,
                                               unsigned char* ring, float* bias_ring, const fx4 (&in)[NG][kMaxT],
                                               fx4 (&out)[NG][kMaxT], float* const (&slab)[NG], const int (&ex)[NG],
                                               bf8 (&bh)[NG], bf8 (&bm)[NG], bf8 (&bl)[NG], int& pending,
                                               const unsigned short* pbase) {
    (k16_pass_step<NTO, PL, NW, NG, FULL, A24, S>(a, ks, ci, ring, bias_ring, in, out, slab, ex, bh, bm, bl, pending,
                                                  pbase), ...);
}

// One pass (a layer's forward or backward MMA) over its ks k-steps, Ring::KC k-steps per chunk, for
// the wave's NG sample groups (each its own input, accumulators, slab and shift).
// A24: the pass's input slab (a forward pass's A_{l-1}) is int24 (store_slab_step24).
// pbase: the pass's first chunk in w16 (FULL passes with FDSRC; otherwise unused)
template <int NTO, int PL, int NW, int NG, bool FULL = false, bool A24 = false>
__device__ __forceinline__ void k16_pass(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                         float* bias_ring, const fx4 (&in)[NG][kMaxT], fx4 (&out)[NG][kMaxT],
                                         float* const (&slab)[NG], const int (&ex)[NG],
                                         const unsigned short* pbase = nullptr) {
    bf8 bh[NG] = {}, bm[NG] = {}, bl[NG] = {};
#pragma unroll
    for (int q = 0; q < NG; ++q) make_b<PL>(in[q], 0, ex[q], bh[q], bm[q], bl[q]);
    int pending = 0;
    k16_pass_steps<NTO, PL, NW, NG, FULL, A24>(std::make_integer_sequence<int, 8>{}, a, ks, ci, ring, bias_ring, in,
                                               out, slab, ex, bh, bm, bl, pending, pbase);
}
// a hidden layer's pass: the FULL instantiation for 256-wide inputs (every hidden layer of cfg3)
template <int HT, int PL, int NW, int NG, bool A24 = false>
__device__ __forceinline__ void k16_hidden_pass(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                                float* bias_ring, const fx4 (&in)[NG][kMaxT], fx4 (&out)[NG][kMaxT],
                                                float* const (&slab)[NG], const int (&ex)[NG],
                                                const unsigned short* pbase) {
    if constexpr (LNERF_K16_FULLDMA && HT == 16) {
        if (ks == 8) {
            k16_pass<HT, PL, NW, NG, true, A24>(a, ks, ci, ring, bias_ring, in, out, slab, ex, pbase);
            return;
        }
    }
    k16_pass<HT, PL, NW, NG, false, A24>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
}

template <int PL, int NW, int NG>
__device__ __forceinline__ void k16_pass_n(const K16Args& a, int ks, int& ci, unsigned char* ring,
                                           float* bias_ring, int nto, const fx4 (&in)[NG][kMaxT],
                                           fx4 (&out)[NG][kMaxT], float* const (&slab)[NG], const int (&ex)[NG]) {
    if (nto <= 1) k16_pass<1, PL, NW, NG>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 2) k16_pass<2, PL, NW, NG>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 4) k16_pass<4, PL, NW, NG>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else if (nto <= 8) k16_pass<8, PL, NW, NG>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
    else k16_pass<16, PL, NW, NG>(a, ks, ci, ring, bias_ring, in, out, slab, ex);
}

// The per-sample max|x| of a pass's input (lanes n, n + 16, n + 32, n + 48 hold sample n's
// features), the basis of its exponent shift (PL >= 2) and of dw16's balancing (training).
// KEEP_NAN (activation rows, the forward): NaN-propagating (v_maximum3_f32), so a row holding a NaN
// or an infinity has a non-finite maximum, which store_sexp marks for dw16 (an int24 slab cannot
// carry the value itself; such a row's pre-activations are NaN and its G row is 0 past the ReLU).
// Otherwise (gradient rows, the reverse chain) NaN-dropping: loma's sigmoid adjoint puts NaN into
// an rgb column (nerf.py:157-165) while the row's finite values still need their own shift.
template <bool KEEP_NAN>
__device__ __forceinline__ float sample_max(const fx4 (&in)[kMaxT]) {
    auto mx = [](float a, float b) { return KEEP_NAN ? __builtin_elementwise_maximum(a, b) : __builtin_fmaxf(a, b); };
    float m = 0.0f;
#pragma unroll
    for (int o = 0; o < kMaxT; ++o)
#pragma unroll
        for (int i = 0; i < 4; ++i) m = mx(m, __builtin_fabsf(in[o][i]));
    m = mx(m, __shfl_xor(m, 16));
    return mx(m, __shfl_xor(m, 32));
}

// the exponent shift ex with m 2^ex in [2^13, 2^14) (fp16x3_shift)
__device__ __forceinline__ int shift_of(float m) { return fp16x3_shift(m); }

// Training: this sample's exponent shift of one slab row (the shift its split used, or -128 for an
// all-zero row), for dw16's per-sample balancing of A and G (lnerf_dw16.hip). which = 0: the input
// row of layer l (byte 0 of its word); which = 1: the G_l row, with the row's exceptional-row bound
// dmax (bytes 2, 3). Issued before the pass's first DMA, so it is older than every piece a
// dma_barrier waits for. Returns the shift.
__device__ __forceinline__ int store_sexp(const K16Args& a, int l, int which, float m, int dmax, int lw, int nlw) {
    const int lane = threadIdx.x & 63;
    // -128: an all-zero row; -127 (activation rows only): a row with a non-finite value, int24-encoded
    // at shift 0, whose NaN / infinity codes dw16 turns back into NaN (kSexpNonFinite)
    const bool fin = m < __builtin_inff();
    const int x = (m > 0.0f && fin) ? shift_of(m) : (which == 0 && !(m == 0.0f)) ? kSexpNonFinite : -128;
    if (lane < 16) {
        const int p = (blockIdx.x * nlw + lw) * 16 + lane;   // lw: the 16-sample group's logical wave
        unsigned char* w = a.sexp + ((size_t)l * a.rpad + p) * 4;
        if (which == 0) *w = (unsigned char)x;
        else *(unsigned short*)(w + 2) = (unsigned short)((x & 0xFF) | ((dmax & 0xFF) << 8));
    }
    return x;
}

// The forward's A-row shifts, one byte per layer packed in 4 registers (layer l in byte l % 4 of
// word l / 4), so the backward pass can pair them with the G-row shifts without a memory round
// trip. Selects instead of a dynamically indexed register array.
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

// Training, after layer l's G-row shift xg: the wave's min over its samples of xa + xg (rows
// marked -128 excluded, and every ray's last sample, which dw16 multiplies on the bf16x6 split
// whenever its products exceed E_l: lnerf_internal.h kXrowLast), one plain store per wave into
// epart[l][global wave]; k1_reduce_kernel folds them into dw16's per-layer product shift E_l.
__device__ __forceinline__ void store_emin(const K16Args& a, int l, int xa, int xg, bool excluded, int lw, int nlw) {
    int v = (xa < -126 || xg < -126 || excluded) ? (1 << 20) : xa + xg;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) v = min(v, __shfl_xor(v, d));
    if ((threadIdx.x & 63) == 0)
        a.epart[((size_t)l * gridDim.x + blockIdx.x) * nlw + lw] = v;
}

// The layer's biases in the accumulator layout (fx4 = 4 consecutive features of a lane group),
// from its bias ring slot (plain LDS reads: the bias DMA landed before the pass's last barrier).
template <int NT, int... O>
__device__ __forceinline__ void bias_read(std::integer_sequence<int, O...>, const float* p, fx4 (&b)[kMaxT]) {
    ((b[O] = *(const fx4*)(p + O * 16)), ...);
}

// ReLU and its mask bit in one short dependency chain (nerf.py:141-144): r = v > 0 ? v : 0 (NaN
// and -0 give +0) and bits = 2 bits + (v > 0), through VCC. Written out because the compiler
// otherwise keeps all 64 compare masks of a layer live in SGPRs and spills them to VGPR lanes.
// In place ("+v" only): the statement writes only registers whose last writer was a compiler
// VALU instruction (v, the sum the compiler just formed; bits, the previous statement), never an
// MFMA operand, so no MFMA wait state can fall inside it (hipcc does not pad inside asm).
__device__ __forceinline__ float relu_bit(float v, unsigned& bits) {
    asm("v_cmp_lt_f32_e32 vcc, 0, %0\n\t"
        "v_cndmask_b32_e32 %0, 0, %0, vcc\n\t"
        "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
        : "+v"(v), "+v"(bits) : : "vcc");
    return v;
}

// PL = 2, before the head's backward pass (its B operand is the head's G row): column n scaled by
// 2^(ew - head_col_shift(n)), so that against the column-shifted planes every product carries the
// layer's 2^ew (the pass unscales as any other); a sigma gradient 2^30 above the rgb ones no longer
// pushes them out of fp16's range. Lane group g holds columns 4 g + i.
__device__ __forceinline__ void head_bscale(const K16Args& a, fx4 (&act)[kMaxT]) {
    const int g = (threadIdx.x & 63) >> 4;
    const int lm = a.wexp[a.L - 1];
    const int ew = wshift_of(lm);
#pragma unroll
    for (int i = 0; i < 4; ++i) act[0][i] = __builtin_ldexpf(act[0][i], ew - head_col_shift(a.hexp[4 * g + i], lm));
}

// the floor guard (lnerf_internal.h kGuardExp): the smallest frexp exponent over a lane's four head
// values (zeros give 0)
__device__ __forceinline__ int head_floor(const fx4& h) {
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) m = min(m, __builtin_amdgcn_frexp_expf(h[i]));
    return m;
}

__device__ __forceinline__ void zero_tiles(fx4 (&t)[kMaxT]) {
#pragma unroll
    for (int o = 0; o < kMaxT; ++o) t[o] = fx4{0.0f, 0.0f, 0.0f, 0.0f};
}

// HT: 16-wide output tiles of every hidden layer (1/2/4/8/16); PL: operand planes (3 = bf16x6,
// 2 = fp16x3, both fp32-class; 1 = plain bf16, inference).
// NW: waves per workgroup; NG: 16-sample groups per wave. (8, 1): 128-sample tiles, one workgroup per
// CU, two waves per SIMD with at most 256 registers each; (4, 1): 64-sample tiles, two workgroups per
// CU; (4, 2): 128-sample tiles, ONE wave per SIMD with the whole 512-entry register file, each weight
// fragment read from LDS feeding both groups' MFMAs (half the LDS bytes per MFMA; fp16x3, HT = 16).
// A group's logical wave lw = wave NG + group owns samples 16 lw ..+15 of the tile: every slab,
// shift word, mask word and per-wave minimum keeps the (8, 1) layout, so k2 and the mask readback
// see the same data whatever NG.
template <int HT, int PL, int NW, int NG = 1>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NG == 2 ? 1 : 2, NG == 2 ? 1 : 2)))
k16_fwd_bwd_kernel(K16Args a) {
    using R = Ring<PL, NW, NG>;
    constexpr int LW = NW * NG;   // logical waves (16-sample groups) per workgroup
    __shared__ __attribute__((aligned(16))) unsigned char lds[R::lds_bytes];
    unsigned char* ring = lds;
    float* comp = (float*)(lds + R::off_comp);
    float* rayloss = (float*)(lds + R::off_ray);
    float* bias_ring = (float*)(lds + R::off_bias);

    if (a.gate && *a.gate == 0) return;   // the floor guard's re-run, not needed this step
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), g = lane >> 4, n = lane & 15;
    const int wg = blockIdx.x;
    const int tile_samples = a.rpw * a.S;
#if LNERF_K16_PRIO
    // static priority for the second-dispatched half (MI355X_MICROARCH.md, two waves per SIMD 4)
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    const bool st = a.want_grad != 0;
    int lw[NG], ls[NG], gs[NG];
    bool valid[NG], tail[NG];
    size_t blk[NG];
    int half[NG], dmax[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        lw[q] = wave * NG + q;
        ls[q] = lw[q] * 16 + n;                          // local sample 0..127
        gs[q] = wg * tile_samples + ls[q];               // global sample row (ray*S + j)
        valid[q] = (ls[q] < tile_samples) && (gs[q] < a.R);
        blk[q] = (size_t)wg * (LW / 2) + (lw[q] >> 1);   // 32-sample slab block
        half[q] = lw[q] & 1;
        // training: this sample is its ray's last (the delta = 1e8 row, train_nerf.py:306-311): kept
        // out of every layer's product scale E_l and an exceptional row only above it (lnerf_internal.h
        // kXrowLast); every other row may fall kXrowD0 binades short of E_l before it is one
        tail[q] = st && valid[q] && !a.head_fit && (ls[q] % a.S) == a.S - 1;
        dmax[q] = tail[q] ? kXrowLast : kXrowD0;
    }
#if LNERF_PROF
    if (lane < 16) prof_slots()[lane] = 0;
    PROF_T(t_start);
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
#endif

    fx4 act[NG][kMaxT], out[NG][kMaxT];
#pragma unroll
    for (int q = 0; q < NG; ++q) zero_tiles(act[q]);
    ExPack exa[NG];   // training: the forward's A-row shift of this lane's sample, per layer
    // PL = 2: layer l's weight exponent shift in lane l (read with readlane per pass); a pass's
    // accumulators carry 2^(ex + ew), removed exactly (powers of two) in its epilogue
    const int wexp_lane = (PL == 2 && lane < a.L) ? wshift_of(a.wexp[lane]) : 0;
    // PL = 3 (bf16x6): the activations carry the per-sample shift too (bf16 spans fp32's range,
    // but the mid / lo planes of values below ~2^-110 would be subnormal); the weights do not
    auto unscale = [&](int l, int ex) -> int {
        return PL == 2 ? -(ex + __builtin_amdgcn_readlane(wexp_lane, l)) : PL == 3 ? -ex : 0;
    };

    // ---- layer-0 input in the accumulator layout, through a per-group LDS scratch (the ring is
    // free before the first DMA). POINTS/RAYS with k0 <= 64: one lane per (sample, coordinate),
    // comp::encode_coord (pos_encoding.py:54-66); otherwise tile by tile.
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        const int tile_base = wg * tile_samples + lw[q] * 16;
        if (a.input_mode != LNERF_INPUT_ENCODED && a.k0 <= 64) {
            constexpr int kStride = 65;
            float* pe = (float*)ring + lw[q] * (16 * kStride);
            if (lane < 48) {
                const int sl = lane / 3, c = lane - 3 * sl;
                const bool vs = (lw[q] * 16 + sl < tile_samples) && (tile_base + sl < a.R);
                comp::encode_coord(vs ? comp::sample_coord(a, tile_base + sl, c) : 0.0, a.F, pe + sl * kStride, c);
            }
            for (int e = lane; e < 16 * 64; e += 64) {
                const int sl = e >> 6, f = e & 63;
                if (f >= a.k0) pe[sl * kStride + f] = 0.0f;
            }
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) act[q][t][i] = pe[n * kStride + 16 * t + 4 * g + i];
        } else {
            float* pe = (float*)ring + lw[q] * (16 * 17);
#pragma unroll
            for (int t = 0; t < kMaxT; ++t) {
                if (16 * t < a.k0) {
                    for (int e = lane; e < 256; e += 64) {
                        const int sl = e >> 4, ft = e & 15;
                        const bool vs = (lw[q] * 16 + sl < tile_samples) && (tile_base + sl < a.R);
                        pe[sl * 17 + ft] = comp::input_feature(a, tile_base + sl, vs, 16 * t + ft);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) act[q][t][i] = pe[n * 17 + 4 * g + i];
                }
            }
        }
    }
    __syncthreads();   // the first DMA overwrites the scratch

    int ci = 0;   // chunk stream position (chunk_at)
    dma_chunk<NW>(a, chunk_at(a, 0), ring, bias_ring);
    dma_barrier(0);
    PROF_ADD(kPfPE, t_start);
    // ReLU mask bits of each group, per hidden layer: [L-1][logical wave][lane] u64
    unsigned long long* mask_w[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) mask_w[q] = a.mask_g + ((size_t)wg * (a.L - 1) * LW + lw[q]) * 64 + lane;

    // ---- forward ----
    for (int l = 0; l < a.L; ++l) {
        constexpr int AT = a_tile_floats(PL);   // float slots per activation tile-block (int24: 768)
        float* slab[NG];
        int ex[NG], sh[NG];
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            slab[q] = !st ? nullptr
                          : (l == 0 ? a.act + a.x_off + blk[q] * (size_t)(a.kt[0] * AT)
                                    : a.act + a.act_off[l - 1] + blk[q] * (size_t)(a.kt[l] * AT)) +
                                half[q] * (AT / 2);
            zero_tiles(out[q]);
            const float xm = (PL >= 2 || st) ? sample_max<true>(act[q]) : 0.0f;
            if (st) exa[q].put(l, store_sexp(a, l, 0, xm, 0, lw[q], LW));
            ex[q] = shift_of(xm);
            sh[q] = unscale(l, ex[q]);
        }
        const float* bl = bias_ring + (l % 3) * 256 + g * 4;
        if (l < a.L - 1) {
            PROF_T(t_f);
            k16_hidden_pass<HT, PL, NW, NG, a24_slabs(PL)>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex,
                                                           a.w16 + a.wf_off[l]);
            PROF_ADD(kPfFwd, t_f);
            PROF_T(t_fe);
            // bias after the sum (nerf.py:98,125), ReLU (nerf.py:141-144) and its mask bits
            fx4 bv[kMaxT];
            bias_read<HT>(std::make_integer_sequence<int, HT>{}, bl, bv);
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                // values in descending bit order (feature 4o + i ends in bit 4o + i of lo / hi)
                unsigned mlo = 0u, mhi = 0u;
                // EPIFMA: unscale and bias as one fma (the scale is a power of two, so out 2^sh is
                // exact and the sum rounds once either way; only a subnormal out 2^sh would differ, in
                // fma's favour)
                const float shs = __builtin_ldexpf(1.0f, sh[q]);
#pragma unroll
                for (int o = HT - 1; o >= 0; --o) {
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        const float v = LNERF_K16_EPIFMA && PL >= 2
                                            ? __builtin_fmaf(out[q][o][i], shs, bv[o][i])
                                            : (PL >= 2 ? __builtin_ldexpf(out[q][o][i], sh[q]) : out[q][o][i]) + bv[o][i];
                        act[q][o][i] = relu_bit(v, o >= 8 ? mhi : mlo);
                    }
                }
                const unsigned long long mb = ((unsigned long long)mhi << 32) | mlo;
                if (st) mask_w[q][(size_t)l * LW * 64] = mb;
            }
            PROF_ADD(kPfFwdEpi, t_fe);
        } else {
            k16_pass<1, PL, NW, NG, false, a24_slabs(PL)>(a, a.ks_f[l], ci, ring, bias_ring, act, out, slab, ex);
            fx4 bv[kMaxT];
            bias_read<1>(std::make_integer_sequence<int, 1>{}, bl, bv);
            // head pre-activations: features 0..3 = registers 0..3 of lane group 0; PL = 2 unscales
            // each column by its own weight shift (head_col_shift)
            if (g == 0) {
#pragma unroll
                for (int q = 0; q < NG; ++q)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int shi = PL == 2 ? -(ex[q] + head_col_shift(a.hexp[i], a.wexp[l])) : sh[q];
                        comp[ls[q] * 4 + i] = (PL >= 2 ? __builtin_ldexpf(out[q][0][i], shi) : out[q][0][i]) + bv[0][i];
                    }
            }
        }
    }
    PROF_T(t_c);
    __syncthreads();

    // ---- rendering + loss + rendering reverse (one thread per sample, scans along rays) ----
    if (a.head_fit) comp::fit_tile(a, wg, comp, rayloss, st, a.nout);
    else if (LNERF_K16_WAVECOMP) comp::composite_tile_wave<comp::kTileSamples>(a, wg, comp, rayloss, st);
    else comp::composite_tile(a, wg, comp, rayloss, st);
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
    // PL = 2, the floor guard (lnerf_internal.h kGuardExp): the smallest frexp exponent over this lane's
    // elements of the G row the last epilogue produced (zeros give 0), tested against the row's shift
    // once sample_max has it
    int gmin[NG];
    bool below = false;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        gmin[q] = 0;
        zero_tiles(act[q]);
        if (g == 0 && valid[q]) {
#pragma unroll
            for (int i = 0; i < 4; ++i) act[q][0][i] = c_gz[ls[q] * 4 + i];
        }
    }
    for (int l = a.L - 1; l >= 1; --l) {
        float* slab[NG];
        int ex[NG], sh[NG];
        unsigned long long mb[NG];
        PROF_T(t_b);
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            zero_tiles(out[q]);
            slab[q] = a.grad + a.grad_off[l] + blk[q] * (size_t)(a.nt[l] * 1024) + half[q] * 512;
            mb[q] = mask_w[q][(size_t)(l - 1) * LW * 64];   // in flight over the pass
            const float xm = sample_max<false>(act[q]);
            store_emin(a, l, exa[q].get(l), store_sexp(a, l, 1, xm, dmax[q], lw[q], LW), tail[q], lw[q], LW);
            ex[q] = shift_of(xm);
            if (PL == 2 && l < a.L - 1) below |= valid[q] && gmin[q] + ex[q] <= kGuardExp;
            if (PL == 2 && l == a.L - 1) {
                // the head: G's slab as it is (one k-step), then the pass on the column-scaled G row
                store_slab_step(slab[q], act[q][0], act[q][1]);
                slab[q] = nullptr;
                head_bscale(a, act[q]);
                ex[q] = shift_of(sample_max<false>(act[q]));
                // the floor guard on the head row as this pass splits it (column-scaled): an rgb
                // adjoint 2^40 below a sigma one (delta = 1e8) is gone from every G row below the head
                below |= valid[q] && head_floor(act[q][0]) + ex[q] <= kGuardExp;
            }
            sh[q] = unscale(l, ex[q]);
        }
        k16_hidden_pass<HT, PL, NW, NG>(a, a.ks_b[l], ci, ring, bias_ring, act, out, slab, ex, a.w16 + a.wb_off[l]);
        PROF_ADD(kPfBwd, t_b);
        PROF_T(t_be);
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            // the forward's decision as an all-ones / zero lane mask (v_bfe_i32), one AND per value
            const int mlo = (int)(unsigned)mb[q], mhi = (int)(unsigned)(mb[q] >> 32);
            gmin[q] = 0;
#pragma unroll
            for (int o = 0; o < HT; ++o)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int keep = __builtin_amdgcn_sbfe(o >= 8 ? mhi : mlo, (4 * o + i) & 31, 1);
                    const float gv = PL >= 2 ? __builtin_ldexpf(out[q][o][i], sh[q]) : out[q][o][i];
                    act[q][o][i] = __int_as_float(__float_as_int(gv) & keep);
                    if constexpr (PL == 2 && LNERF_GUARD)
                        gmin[q] = min(gmin[q], __builtin_amdgcn_frexp_expf(act[q][o][i]));
                }
        }
        PROF_ADD(kPfBwdEpi, t_be);
    }
    PROF_T(t_t);
    // act holds G_0
    float* g0[NG];
#pragma unroll
    for (int q = 0; q < NG; ++q) g0[q] = a.grad + a.grad_off[0] + blk[q] * (size_t)(a.nt[0] * 1024) + half[q] * 512;
    if (a.d_x) {
        // d_layer_input = G_0 W_0^T (ENCODED mode); the pass also writes G_0's slab
        float* g0s[NG];
        int ex[NG], sh[NG];
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            zero_tiles(out[q]);
            const float xm = sample_max<false>(act[q]);
            store_emin(a, 0, exa[q].get(0), store_sexp(a, 0, 1, xm, dmax[q], lw[q], LW), tail[q], lw[q], LW);
            ex[q] = shift_of(xm);
            if (PL == 2 && a.L > 1) below |= valid[q] && gmin[q] + ex[q] <= kGuardExp;
            g0s[q] = g0[q];
            if (PL == 2 && a.L == 1) {
                // a head-only MLP: layer 0 is the head (its column-shifted planes, as above)
                store_slab_step(g0[q], act[q][0], act[q][1]);
                g0s[q] = nullptr;
                head_bscale(a, act[q]);
                ex[q] = shift_of(sample_max<false>(act[q]));
                below |= valid[q] && head_floor(act[q][0]) + ex[q] <= kGuardExp;
            }
            sh[q] = unscale(0, ex[q]);
        }
        k16_pass_n<PL, NW, NG>(a, a.ks_b[0], ci, ring, bias_ring, a.to_b[0], act, out, g0s, ex);
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            if (valid[q]) {
#pragma unroll
                for (int o = 0; o < kMaxT; ++o)
                    if (16 * o < a.k0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int f = 16 * o + 4 * g + i;
                            if (f < a.k0)
                                a.d_x[(size_t)gs[q] * a.k0 + f] =
                                    PL >= 2 ? __builtin_ldexpf(out[q][o][i], sh[q]) : out[q][o][i];
                        }
                    }
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < NG; ++q) {
            const float xm = sample_max<false>(act[q]);
            store_emin(a, 0, exa[q].get(0), store_sexp(a, 0, 1, xm, dmax[q], lw[q], LW), tail[q], lw[q], LW);
            if (PL == 2 && a.L > 1) below |= valid[q] && gmin[q] + shift_of(xm) <= kGuardExp;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < a.ks_b[0]) store_slab_step(g0[q] + s * 1024, act[q][2 * s], act[q][2 * s + 1]);
        }
    }
    // one plain store per wave that met an element below the floor (every writer stores 1)
    if (PL == 2 && LNERF_GUARD && a.guard && __builtin_amdgcn_ballot_w64(below) != 0 && lane == 0)
        *a.guard = 1;
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
    int* hexp;   // planes = 2: the head's per-column max|W| bits [kHeadCols] (pack16_kernel)
    int* hpart;  // [kWmaxParts][kHeadCols] their partials (wmax16_kernel)
    int* guard_reset;   // nullable: the floor guard's word, zeroed before k1 (lnerf_internal.h kGuardExp)
    unsigned short* w16x;   // nullable (planes = 2): also the bf16x6 planes of the guard's re-run, three planes
    const int* gate;    // nullable: the launch exits at once unless *gate != 0 (the guard's re-run)
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
    // the head's per-column partials (thread j: column j over this block's rows)
    if (l == a.L - 1 && threadIdx.x < kHeadCols) {
        const int j = threadIdx.x;
        float mc = 0.0f;
        if (j < N)
            for (int k = blockIdx.x; k < K; k += gridDim.x) mc = fmaxf(mc, fabsf(W[(size_t)k * a.w_n + j]));
        a.hpart[blockIdx.x * kHeadCols + j] = __float_as_int(mc);
    }
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
    if (a.gate && *a.gate == 0) return;
    if (a.guard_reset && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.guard_reset = 0;
    const int l = blockIdx.y;
    const float* W = a.W + (size_t)l * a.w_k * a.w_n;
    const int K = a.k[l], N = a.n[l];
    const int lmax = a.planes == 2 ? layer_wmax(a, l) : 0;
    const int wsh = a.planes == 2 ? wshift_of(lmax) : 0;
    const bool head = a.planes == 2 && l == a.L - 1;
    __shared__ int hsh[kHeadCols];   // the head's per-column shifts
    if (head) {
        if (threadIdx.x < kHeadCols) {
            int mb = 0;
            for (int i = 0; i < kWmaxParts; ++i) mb = max(mb, a.hpart[i * kHeadCols + threadIdx.x]);
            hsh[threadIdx.x] = head_col_shift(mb, lmax);
            if (blockIdx.x == 0) a.hexp[threadIdx.x] = mb;
        }
        __syncthreads();
    }
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
            split_h(__builtin_ldexpf(w, head && jj < kHeadCols ? hsh[jj] : wsh), h, lo);
            dst[0] = __builtin_bit_cast(unsigned short, h);
            dst[512] = __builtin_bit_cast(unsigned short, lo);
            if (a.w16x) {
                // the floor guard's re-run reads these (no pack launch of its own)
                unsigned short* dx = a.w16x + (fwd ? a.wf_off[l] : a.wb_off[l]) + ((size_t)(s * to + o) * 3) * 512 +
                                     ln * 8 + j;
                __bf16 xh, xm, xl;
                split_x(w, xh, xm, xl);
                dx[0] = __builtin_bit_cast(unsigned short, xh);
                dx[512] = __builtin_bit_cast(unsigned short, xm);
                dx[1024] = __builtin_bit_cast(unsigned short, xl);
            }
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

// ReLU decisions of the last training k1 as a dense bitmap: out[(l R + r) 32 + f / 8] bit f % 8 =
// feature f of hidden layer l at sample row r was positive (nerf.py:141-144). One thread per
// output byte; the bits come from two lanes' u64 mask words (lane g 16 + n holds features
// 16 o + 4 g + i in bits 4 o + i).
__global__ void k16_masks_kernel(const unsigned long long* __restrict__ mask_g, int L1, int R, int tile_samples,
                                 int nw, unsigned char* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (size_t)L1 * R * 32) return;
    const int b = (int)(idx & 31);
    const size_t lr = idx >> 5;
    const int l = (int)(lr / R), r = (int)(lr % R);
    const int wg = r / tile_samples, ls = r % tile_samples, wave = ls >> 4, n = ls & 15;
    const int o = b >> 1, g0 = 2 * (b & 1);
    const unsigned long long* w = mask_g + ((size_t)(wg * L1 + l) * nw + wave) * 64;
    const unsigned lo = (unsigned)(w[g0 * 16 + n] >> (4 * o)) & 0xFu;
    const unsigned hi = (unsigned)(w[(g0 + 1) * 16 + n] >> (4 * o)) & 0xFu;
    out[idx] = (unsigned char)(lo | (hi << 4));
}

}  // namespace

// Compile-time settings of this object that differ from the product build (lnerf_build_knobs):
// 0 for the shipped library; an A/B variant built with -D... reports which knob it moved.
unsigned k16_build_knobs() {
    return (LNERF_K16_FULLDMA != 1 ? kKnobK16FullDma : 0u) | (LNERF_K16_KDIST != 2 ? kKnobK16KDist : 0u) |
           (LNERF_K16_SPLIT_AT != 2 ? kKnobK16SplitAt : 0u) | (LNERF_K16_SCHED != 1 ? kKnobK16Sched : 0u) |
           (LNERF_K16_PRIO != 0 ? kKnobK16Prio : 0u) | (LNERF_K16_SPREAD != 1 ? kKnobK16Spread : 0u) |
           (LNERF_PROF != 0 ? kKnobProf : 0u) | (LNERF_A24 != 1 ? kKnobA24 : 0u) |
           (LNERF_K16_PIN != 2 ? kKnobK16Pin : 0u) | (LNERF_K16_FDSRC != 1 ? kKnobK16FdSrc : 0u) |
           (LNERF_K16_ONECHUNK != 1 ? kKnobK16OneChunk : 0u) | (LNERF_K16_WAVECOMP != 1 ? kKnobK16WaveComp : 0u) |
           (LNERF_K16_EPIFMA != 1 ? kKnobK16EpiFma : 0u) | (LNERF_K16_G2 != 0 ? kKnobK16G2 : 0u) |
           (LNERF_PE_DOUBLING != 1 ? kKnobPeDoubling : 0u) | (LNERF_GUARD != 1 ? kKnobGuard : 0u)
#ifdef LNERF_K16_ONLY_16_2
           | kKnobK16Only
#endif
        ;
}

void k16_masks_launch(const FusedPlan& p, unsigned char* out, hipStream_t s) {
    const size_t n = (size_t)(p.L - 1) * p.R * 32;
    if (n == 0) return;
    k16_masks_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(p.mask_g, p.L - 1, p.R, p.rays_per_wg * p.S,
                                                                 p.tile / 16, out);
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
    a.hexp = p.hexp16;
    a.hpart = p.wmax_part + (size_t)kMaxLayers * kWmaxParts;
    a.guard_reset = p.guard;
    a.gate = p.gate;
    a.w16x = p.x6 == 2 ? p.w16x : nullptr;
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
    a.head_fit = p.head_fit;
    a.nout = p.n[p.L - 1];
    a.planes = p.x6;
    a.wexp = p.wexp16;
    a.hexp = p.hexp16;
    a.sexp = (unsigned char*)p.sexp;
    a.rpad = p.num_wg * p.tile;
    a.epart = p.epart;
    a.guard = want_grad && p.x6 == 2 ? p.guard : nullptr;
    a.gate = p.gate;
    // the chunk stream: forward 0..L-1, backward L-1..1 (training), backward 0 (d_x); chunks of
    // KC k-steps (Ring: 2 for fp16x3 / bf16, 1 for bf16x6), the pack layout's consecutive k-steps
    {
        const int KC0 = (p.x6 == 3 || p.tile == 64) ? 1 : 2;
        int ci = 0;
        auto add = [&](bool fwd, int l) {
            const int ks = fwd ? a.ks_f[l] : a.ks_b[l], to = fwd ? a.to_f[l] : a.to_b[l];
            const int KC = (LNERF_K16_ONECHUNK && to == 1) ? 8 : KC0;   // pass_kc
            const size_t per = (size_t)to * a.planes * 512;   // u16 per k-step
            for (int s2 = 0; s2 < ks; s2 += KC, ++ci) {
                const int nk = ks - s2 < KC ? ks - s2 : KC;
                a.chunk_tab[2 * ci] = (unsigned)((fwd ? a.wf_off[l] : a.wb_off[l]) + (size_t)s2 * per);
                a.chunk_tab[2 * ci + 1] = (unsigned)(nk * per * 2 / 1024) | ((fwd && s2 == 0 ? l + 1 : 0) << 16);
            }
        };
        for (int l = 0; l < p.L; ++l) add(true, l);
        if (want_grad)
            for (int l = p.L - 1; l >= (a.d_x ? 0 : 1); --l) add(false, l);
        // a zero entry past the end (the kernel looks one chunk ahead): a{} zeroed it
    }
    static_assert(sizeof(K16Args) <= 4096, "kernel arguments");
#if LNERF_K16_G2
    // two 16-sample groups per wave, one wave per SIMD (fp16x3, 256-wide hidden layers, 128-sample tiles)
    if (p.x6 == 2 && p.tile == 128 && p.ht16 == 16) {
        k16_fwd_bwd_kernel<16, 2, 4, 2><<<p.num_wg, 256, 0, s>>>(a);
        return;
    }
#endif
#ifdef LNERF_K16_ONLY_16_2   // compile-time experiments: one instantiation
    if (p.tile == 64) k16_fwd_bwd_kernel<16, 2, 4><<<p.num_wg, 256, 0, s>>>(a);
    else k16_fwd_bwd_kernel<16, 2, 8><<<p.num_wg, 512, 0, s>>>(a);
    return;
#endif
// bf16x6 (three planes) always runs the 8-wave workgroup (its ring does not fit two per CU)
#define LNERF_K16_LAUNCH(HT)                                                                 \
    if (p.x6 == 3) k16_fwd_bwd_kernel<HT, 3, 8><<<p.num_wg, 512, 0, s>>>(a);                 \
    else if (p.tile == 64 && p.x6 == 2) k16_fwd_bwd_kernel<HT, 2, 4><<<p.num_wg, 256, 0, s>>>(a); \
    else if (p.tile == 64) k16_fwd_bwd_kernel<HT, 1, 4><<<p.num_wg, 256, 0, s>>>(a);         \
    else if (p.x6 == 2) k16_fwd_bwd_kernel<HT, 2, 8><<<p.num_wg, 512, 0, s>>>(a);            \
    else k16_fwd_bwd_kernel<HT, 1, 8><<<p.num_wg, 512, 0, s>>>(a);
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
        for (int i = 0; i < kPfN; ++i) fprintf(stderr, " %s=%.0f", names[i], h[i] / ((double)p.num_wg * (p.tile / 16)));
        fprintf(stderr, " clock_GHz=%.3f\n", h[kPfReal] ? (double)h[kPfTotal] / h[kPfReal] * 0.1 : 0.0);
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_k16_prof), z, sizeof(z));
    }
#endif
}

}  // namespace lnerf
