// lnerf_dw16.hip -- k2 on wave pairs: dW_l = sum_s A_{l-1}[s]^T G_l[s] and db_l = sum_s G_l[s]
// from the slabs k1 wrote, in k1's split (fp16x3 on v_mfma_f32_32x32x16_f16 with the slabs'
// layer-wide exponent shifts, or bf16x6 on v_mfma_f32_32x32x16_bf16), two waves per SIMD.
//
// Reference: the weight/bias adjoints of nerf.py's reverse pass (reverse_diff.py:492-559;
// dW_l += A_{l-1}^T G_l, db_l += sum_rows G_l). One workgroup (8 waves)
// streams a contiguous range of 16-sample half-blocks of one layer:
//  * global -> registers: the half-block's A rows (kt*32) and G rows (nt*32), 64 B per row, read
//    as fully coalesced 16-B loads two half-blocks ahead (no LDS staging of fp32);
//  * split once, cooperatively: every value is split into its hi/mid/lo bf16 planes exactly
//    once per workgroup and written to a double-buffered LDS plane image [plane][row][16 samples]
//    (the MFMA operand layout: 8 consecutive samples of a row = one 16-B fragment);
//  * each wave owns a 64 x 128 block of the layer's output (2 x 4 tiles of 32 x 32, 128
//    accumulator registers) and runs 6 MFMAs per tile pair and half-block;
//  * db from the same registers (per-row partial sums, reduced in LDS at the end);
//  * partials per split, summed in order by grad_reduce_kernel (deterministic, no atomics).
#include "lnerf_internal.h"

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef float fx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf4 __attribute__((ext_vector_type(4)));

// timing experiments only (wrong results): skip the MFMAs / the slab loads
#ifndef LNERF_DW16_NOMMA
#define LNERF_DW16_NOMMA 0
#endif
#ifndef LNERF_DW16_NOLOAD
#define LNERF_DW16_NOLOAD 0
#endif

constexpr int kThreads = 512;
constexpr int kRows = 512;                  // A rows [0, 256) and G rows [256, 512) of the image
constexpr int kPlaneBytes = kRows * 32;     // one plane of a half-block: [row][16 samples] 16-bit
// PL planes per operand: 3 = bf16x6, 2 = fp16x3 (x 2^e = hi + lo, the slab's layer-wide shift)
template <int PL>
constexpr int image_bytes() { return PL * kPlaneBytes; }

struct Dw16Args {
    int kt[kMaxLayers], nt[kMaxLayers];
    const float* act;
    size_t a_off[kMaxLayers];   // A_{l-1} slab base per layer (X slab for l = 0)
    const float* grad;
    size_t g_off[kMaxLayers];
    int blocks;                 // 32-sample blocks
    int splits[kMaxLayers];
    int nl;                     // layers in the launch
    int lid[kMaxLayers];
    int wg_off[kMaxLayers + 1]; // first workgroup of the i-th layer
    float* dw_part;
    size_t dwp_off[kMaxLayers];
    float* db_part;
    size_t dbp_off[kMaxLayers];
    const int* smax;            // PL = 2: slab max bits, [l] layer l's input, [L + l] G_l
    int L;
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// the exponent shift e with max 2^e in [2^13, 2^14) from a slab max's bits (0: zero/non-finite)
__device__ __forceinline__ int shift_of_bits(int bits) {
    const float m = __int_as_float(bits);
    if (!(m > 0.0f) || !(m < __builtin_inff())) return 0;
    int e;
    (void)__builtin_frexpf(m, &e);
    return 14 - e;
}

// The 16 B that thread t loads in round i (0..3) of a half-block: image row r = 128 i + t / 4
// (rounds 0, 1: A rows; 2, 3: G rows), samples 4 (t % 4) .. +3. A slab block is
// [tile][half][32 rows][16 samples]; a half-block is one half of one 32-sample block. The
// per-thread part of the offset is fixed (RowMap), the half-block part is wave-uniform.
struct RowMap {
    int lane;        // per-thread float offset inside a tile's half: row (t/4) % 32, samples 4 (t % 4)
    int tile[4];     // wave-uniform: the 32-row tile of round i (tile 0 for rows past the layer)
    bool ok[4];      // wave-uniform: the row exists in this layer (else it is never split)
};

__device__ __forceinline__ RowMap row_map(int kt, int nt) {
    RowMap m;
    const int t = threadIdx.x;
    m.lane = ((t >> 2) & 31) * 16 + 4 * (t & 3);
    // a round's 16 rows of a wave lie in one tile: tile = (128 (i & 1) + t / 4) / 32 = 4 (i & 1) + wave / 2
    const int w2 = wave_id() >> 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int tl = 4 * (i & 1) + w2;
        m.ok[i] = tl < (i < 2 ? kt : nt);
        m.tile[i] = m.ok[i] ? tl : 0;
    }
    return m;
}

struct Loads {
    fx4 v[4];
};

// Always four loads from valid addresses and no select on the data (nothing waits for it before
// its use): rows past the layer's tiles are never split, half-blocks past the split land in the
// idle image and add nothing to db (the callers' hb < hb1 guards).
__device__ __forceinline__ void issue_loads(const float* A, const float* G, int kt, int nt, const RowMap& m,
                                            int hb, int hb_end, Loads& L) {
    const bool in = hb < hb_end;
    const int hbc = in ? hb : max(0, hb_end - 1);
    const int blk = hbc >> 1, half = hbc & 1;
    const float* pa = A + (size_t)blk * kt * 1024 + half * 512;
    const float* pg = G + (size_t)blk * nt * 1024 + half * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const fx4* p = (const fx4*)((i < 2 ? pa : pg) + m.tile[i] * 1024 + m.lane);
        L.v[i] = LNERF_DW16_NOLOAD ? fx4{1.0f, 2.0f, 3.0f, (float)i} : __builtin_nontemporal_load(p);
    }
}

// x = hi + mid + lo, round-to-nearest bf16 of each remainder (every remainder is exact in f32).
__device__ __forceinline__ void split4(const fx4& x, bf4& h, bf4& m, bf4& lo) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const __bf16 hh = (__bf16)x[e];
        const float r = x[e] - (float)hh;
        const __bf16 mm = (__bf16)r;
        h[e] = hh;
        m[e] = mm;
        lo[e] = (__bf16)(r - (float)mm);
    }
}

// The pair (x0, x1) as packed f16 hi = round(x sc), lo = round(x sc - hi) by v_fma_mix (one
// rounding each; x sc and x sc - hi are exact): two instructions per value.
__device__ __forceinline__ void split_h2(float x0, float x1, float sc, unsigned& hi, unsigned& lo) {
    asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=&v"(hi) : "v"(x0), "v"(sc));
    asm("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(hi) : "v"(x1), "v"(sc));
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(x0), "v"(sc), "v"(hi));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "+v"(lo) : "v"(x1), "v"(sc), "v"(hi));
}

// Split round i of the thread's values into the plane image (8 B per plane and row); rounds 0, 1
// are A rows (shift ea), 2, 3 G rows (shift eg).
template <int PL>
__device__ __forceinline__ void write_planes_row(const fx4& v, int i, unsigned char* img, int ea, int eg) {
    const int t = threadIdx.x, q = t & 3;
    const int r = 128 * i + (t >> 2);
    unsigned char* p = img + r * 32 + q * 8;
    if constexpr (PL == 2) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const float sc = __builtin_ldexpf(1.0f, i < 2 ? ea : eg);
        unsigned h0, l0, h1, l1;
        split_h2(v[0], v[1], sc, h0, l0);
        split_h2(v[2], v[3], sc, h1, l1);
        *(u2*)(p) = u2{h0, h1};
        *(u2*)(p + kPlaneBytes) = u2{l0, l1};
    } else {
        bf4 h, m, lo;
        split4(v, h, m, lo);
        *(bf4*)(p) = h;
        *(bf4*)(p + kPlaneBytes) = m;
        *(bf4*)(p + 2 * kPlaneBytes) = lo;
    }
}

template <int PL>
__device__ __forceinline__ void write_planes(const Loads& L, unsigned char* img, int ea, int eg) {
#pragma unroll
    for (int i = 0; i < 4; ++i) write_planes_row<PL>(L.v[i], i, img, ea, eg);
}

__device__ __forceinline__ fx16 mfma32(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ fx16 mfma32h(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
                                                  0);
}

// The wave's TI x TJ tile block (TI 32-row tiles of A, TJ of G) on one half-block image (per
// tile a fragment is one ds_read_b128 per plane; lane: row l & 31, samples 8 (l >> 5) .. +7),
// with the split of the next half-block interleaved (round k beside output column tile k), so
// the VALU split issues under the MFMAs. Branch-free (ACTIVE is a template parameter; past the
// split's last half-block the zeroed loads land in the idle image buffer).
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void block_mma(const unsigned char* img, int a0, int g0, fx16 (&acc)[TI][TJ],
                                          const Loads& nl, unsigned char* nxt, const RowMap& m, int ea,
                                          int eg) {
    const int lane = threadIdx.x & 63, fo = (lane & 31) * 32 + (lane >> 5) * 16;
    bf8 ap[TI][PL];
    if constexpr (ACTIVE) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int p = 0; p < PL; ++p) ap[i][p] = *(const bf8*)(img + p * kPlaneBytes + (a0 + 32 * i) * 32 + fo);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // rows past the layer's tiles are never read: skip their split (wave-uniform: a wave's
        // 16 rows of a round lie in one 32-row tile); FULL layers need no branch
        if (FULL || m.ok[k]) write_planes_row<PL>(nl.v[k], k, nxt, ea, eg);
        if constexpr (ACTIVE) {
            if (k < TJ) {
                const int j = k < TJ ? k : 0;
                bf8 gp[PL];
#pragma unroll
                for (int p = 0; p < PL; ++p) gp[p] = *(const bf8*)(img + p * kPlaneBytes + (256 + g0 + 32 * j) * 32 + fo);
#pragma unroll
                for (int i = 0; i < TI; ++i) {
                    fx16 c = acc[i][j];
                    if constexpr (PL == 2) {
                        c = mfma32h(ap[i][0], gp[1], c);   // small terms first
                        c = mfma32h(ap[i][1], gp[0], c);
                        c = mfma32h(ap[i][0], gp[0], c);
                    } else {
                        c = mfma32(ap[i][0], gp[2], c);   // small terms first
                        c = mfma32(ap[i][1], gp[1], c);
                        c = mfma32(ap[i][2], gp[0], c);
                        c = mfma32(ap[i][1], gp[0], c);
                        c = mfma32(ap[i][0], gp[1], c);
                        c = mfma32(ap[i][0], gp[0], c);
                    }
                    acc[i][j] = c;
                }
            }
        }
    }
}

// The half-block loop of one split: L0 holds hb0 (already in the image), L1 hb0 + 1.
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void hb_loop(const float* A, const float* G, int kt, int nt, const RowMap& m,
                                        int hb0, int hb1, int a0, int g0, fx16 (&acc)[TI][TJ], Loads& L0,
                                        Loads& L1, float (&dbs)[2], unsigned char* lds, int ea, int eg) {
    constexpr int kIB = image_bytes<PL>();
    for (int hb = hb0; hb < hb1; ++hb) {
        const int cur = (hb - hb0) & 1;
        // L1 holds hb + 1; L0 receives hb + 2
        issue_loads(A, G, kt, nt, m, hb + 2, hb1, L0);
        if (hb + 1 < hb1) {
            dbs[0] += (L1.v[2][0] + L1.v[2][1]) + (L1.v[2][2] + L1.v[2][3]);
            dbs[1] += (L1.v[3][0] + L1.v[3][1]) + (L1.v[3][2] + L1.v[3][3]);
        }
        block_mma<PL, TI, TJ, ACTIVE, FULL>(lds + cur * kIB, a0, g0, acc, L1, lds + (cur ^ 1) * kIB, m, ea, eg);
        __syncthreads();
        Loads t = L0;
        L0 = L1;
        L1 = t;
    }
}

// Three half-blocks in flight (LNERF_DW16_DEPTH=3): step I of a 3-step rotation over the load
// register sets (images alternate at run time). Entering half-block hb: its planes are in image
// (hb - hb0) & 1, the set after I holds hb + 1 (split now into the other image), the one after
// that hb + 2 (in flight) and set I is free: it receives hb + 3.
#ifndef LNERF_DW16_DEPTH
#define LNERF_DW16_DEPTH 3
#endif
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL, int I>
__device__ __forceinline__ void hb_step3(const float* A, const float* G, int kt, int nt, const RowMap& m, int hb,
                                         int hb0, int hb1, int a0, int g0, fx16 (&acc)[TI][TJ], Loads& L0,
                                         Loads& L1, Loads& L2, float (&dbs)[2], unsigned char* lds, int ea,
                                         int eg) {
    constexpr int kIB = image_bytes<PL>();
    Loads& fr = I == 0 ? L0 : I == 1 ? L1 : L2;
    const Loads& nx = I == 0 ? L1 : I == 1 ? L2 : L0;
    issue_loads(A, G, kt, nt, m, hb + 3, hb1, fr);
    if (hb + 1 < hb1) {
        dbs[0] += (nx.v[2][0] + nx.v[2][1]) + (nx.v[2][2] + nx.v[2][3]);
        dbs[1] += (nx.v[3][0] + nx.v[3][1]) + (nx.v[3][2] + nx.v[3][3]);
    }
    const int cur = (hb - hb0) & 1;
    block_mma<PL, TI, TJ, ACTIVE, FULL>(lds + cur * kIB, a0, g0, acc, nx, lds + (cur ^ 1) * kIB, m, ea, eg);
    __syncthreads();
}

template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void hb_loop3(const float* A, const float* G, int kt, int nt, const RowMap& m,
                                         int hb0, int hb1, int a0, int g0, fx16 (&acc)[TI][TJ], Loads& L0,
                                         Loads& L1, Loads& L2, float (&dbs)[2], unsigned char* lds, int ea,
                                         int eg) {
    int hb = hb0;
    for (; hb + 3 <= hb1; hb += 3) {
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 0>(A, G, kt, nt, m, hb, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 1>(A, G, kt, nt, m, hb + 1, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 2>(A, G, kt, nt, m, hb + 2, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
    }
    if (hb < hb1) hb_step3<PL, TI, TJ, ACTIVE, FULL, 0>(A, G, kt, nt, m, hb, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
    if (hb + 1 < hb1) hb_step3<PL, TI, TJ, ACTIVE, FULL, 1>(A, G, kt, nt, m, hb + 1, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
}

// One split of layer l with TI x TJ tile blocks per wave (the layer's ceil(KT/TI) x ceil(NT/TJ)
// blocks on waves 0.., at most 8).
template <int PL, int TI, int TJ>
__device__ __forceinline__ void dw_split(const Dw16Args& a, int l, int sp, unsigned char* lds) {
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int KT = a.kt[l], NT = a.nt[l];
    const int nbg = (NT + TJ - 1) / TJ, nblk = ((KT + TI - 1) / TI) * nbg;
    const bool active = wave < nblk && !LNERF_DW16_NOMMA;
    const int a0 = active ? (wave / nbg) * 32 * TI : 0, g0 = active ? (wave % nbg) * 32 * TJ : 0;
    // half-block range of this split
    const int hbs = 2 * a.blocks, splits = a.splits[l];
    const int per = (hbs + splits - 1) / splits;
    const int hb0 = min(hbs, sp * per), hb1 = min(hbs, hb0 + per);

    fx16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = fx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // db: this thread's G rows are image rows 128 i + t/4 for i = 2, 3 (4 samples each)
    float dbs[2] = {0.0f, 0.0f};

    const float* A = a.act + a.a_off[l];
    const float* G = a.grad + a.g_off[l];
    const RowMap m = row_map(KT, NT);
    // PL = 2: the layer-wide exponent shifts of the A_{l-1} and G_l slabs (k1's slab maxima); the
    // partials are shifted back by -(ea + eg) (exact)
    const int ea = PL == 2 ? shift_of_bits(a.smax[l]) : 0, eg = PL == 2 ? shift_of_bits(a.smax[a.L + l]) : 0;
    const bool full = KT == 8 && NT == 8;
    if constexpr (LNERF_DW16_DEPTH == 3) {
        Loads L0, L1, L2;
        issue_loads(A, G, KT, NT, m, hb0, hb1, L0);
        issue_loads(A, G, KT, NT, m, hb0 + 1, hb1, L1);
        issue_loads(A, G, KT, NT, m, hb0 + 2, hb1, L2);
        if (hb0 < hb1) {
            dbs[0] += (L0.v[2][0] + L0.v[2][1]) + (L0.v[2][2] + L0.v[2][3]);
            dbs[1] += (L0.v[3][0] + L0.v[3][1]) + (L0.v[3][2] + L0.v[3][3]);
            write_planes<PL>(L0, lds, ea, eg);
        }
        __syncthreads();
        if (active && full) hb_loop3<PL, TI, TJ, true, true>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
        else if (active) hb_loop3<PL, TI, TJ, true, false>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
        else if (full) hb_loop3<PL, TI, TJ, false, true>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
        else hb_loop3<PL, TI, TJ, false, false>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, ea, eg);
    } else {
        Loads L0, L1;
        issue_loads(A, G, KT, NT, m, hb0, hb1, L0);
        issue_loads(A, G, KT, NT, m, hb0 + 1, hb1, L1);
        if (hb0 < hb1) {
            dbs[0] += (L0.v[2][0] + L0.v[2][1]) + (L0.v[2][2] + L0.v[2][3]);
            dbs[1] += (L0.v[3][0] + L0.v[3][1]) + (L0.v[3][2] + L0.v[3][3]);
            write_planes<PL>(L0, lds, ea, eg);
        }
        __syncthreads();
        if (active && full) hb_loop<PL, TI, TJ, true, true>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, ea, eg);
        else if (active) hb_loop<PL, TI, TJ, true, false>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, ea, eg);
        else if (full) hb_loop<PL, TI, TJ, false, true>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, ea, eg);
        else hb_loop<PL, TI, TJ, false, false>(A, G, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, ea, eg);
    }

    // partial [split][k][j], k < KT*32, j < NT*32 (32x32 C/D layout: row (r&3)+8(r>>2)+4h, col l&31)
    if (active) {
        const int ncol = NT * 32, h = lane >> 5;
        float* part = a.dw_part + a.dwp_off[l] + (size_t)sp * (KT * 32) * ncol;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int kb = a0 + 32 * i, jb = g0 + 32 * j;
                if (kb < KT * 32 && jb < ncol) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = kb + (r & 3) + 8 * (r >> 2) + 4 * h;
                        part[(size_t)k * ncol + jb + (lane & 31)] =
                            PL == 2 ? __builtin_ldexpf(acc[i][j][r], -(ea + eg)) : acc[i][j][r];
                    }
                }
            }
    }
    // db: 4 threads per G row -> in-order sum through LDS
    float* red = (float*)lds;
#pragma unroll
    for (int i = 0; i < 2; ++i) red[(i * 128 + (tid >> 2)) * 4 + (tid & 3)] = dbs[i];
    __syncthreads();
    if (tid < NT * 32) {
        const float* q = red + tid * 4;
        a.db_part[a.dbp_off[l] + (size_t)sp * NT * 32 + tid] = (q[0] + q[1]) + (q[2] + q[3]);
    }
}

// Block shape per layer: the smallest of 1x1, 1x2, 2x4 tiles that needs at most 8 waves, so
// small layers (the head, layer 0) spread over all SIMDs instead of a few waves.
__host__ __device__ __forceinline__ int dw_shape(int kt, int nt) {
    if (kt * nt <= 8) return 0;
    if (kt * ((nt + 1) / 2) <= 8) return 1;
    return 2;
}

template <int PL>
__global__ void __launch_bounds__(kThreads, 1) dw16_kernel(Dw16Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * image_bytes<PL>()];
    int li = 0;
    while (li + 1 < a.nl && (int)blockIdx.x >= a.wg_off[li + 1]) ++li;
    const int l = a.lid[li], sp = blockIdx.x - a.wg_off[li];
    switch (dw_shape(a.kt[l], a.nt[l])) {
        case 0: dw_split<PL, 1, 1>(a, l, sp, lds); break;
        case 1: dw_split<PL, 1, 2>(a, l, sp, lds); break;
        default: dw_split<PL, 2, 4>(a, l, sp, lds); break;
    }
}

// The reductions between k1 and dw16 in one launch (1024 threads per block):
//  * blocks [0, nslab): PL = 2, slab b's layer-wide max from k1's per-wave maxima (n per slab), as
//    the bits of a non-negative float in smax[b] (the exponent shifts dw16 splits with);
//  * block nslab: the batch loss, the same deterministic 256-lane tree as loss_reduce_kernel
//    (lnerf_fused.hip), into *total (the loss seed) and *out_loss.
__global__ void __launch_bounds__(1024) k1_reduce_kernel(const float* __restrict__ part, int n,
                                                         int* __restrict__ smax, int nslab,
                                                         const float* __restrict__ loss_part, int nwg,
                                                         float* total, float* out_loss) {
    __shared__ float red[1024];
    const int t = threadIdx.x;
    if ((int)blockIdx.x < nslab) {
        const float* q = part + (size_t)blockIdx.x * n;
        float m = 0.0f;
        if ((n & 3) == 0) {
            const float4* q4 = reinterpret_cast<const float4*>(q);
            for (int i = t; i < (n >> 2); i += 1024) {
                const float4 v = q4[i];
                m = fmaxf(fmaxf(m, fmaxf(v.x, v.y)), fmaxf(v.z, v.w));
            }
        } else {
            for (int i = t; i < n; i += 1024) m = fmaxf(m, q[i]);
        }
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        if ((t & 63) == 0) red[t >> 6] = m;
        __syncthreads();
        if (t == 0) {
            float r = red[0];
            for (int w = 1; w < 16; ++w) r = fmaxf(r, red[w]);
            smax[blockIdx.x] = __float_as_int(r);
        }
        return;
    }
    float s = 0.0f;
    if (t < 256)
        for (int i = t; i < nwg; i += 256) s += loss_part[i];
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

}  // namespace

void dw16_launch(const FusedPlan& p, hipStream_t s) {
    Dw16Args a{};
    for (int l = 0; l < p.L; ++l) {
        a.kt[l] = p.kt[l];
        a.nt[l] = p.nt[l];
        a.a_off[l] = (l == 0) ? p.x_off : p.act_off[l - 1];
        a.g_off[l] = p.grad_off[l];
        a.splits[l] = p.dw_splits[l];
        a.dwp_off[l] = p.dwp_off[l];
        a.dbp_off[l] = p.dbp_off[l];
        a.lid[l] = l;
        a.wg_off[l] = p.dw_split_off[l];
    }
    a.wg_off[p.L] = p.dw_grid;
    a.nl = p.L;
    a.act = p.act;
    a.grad = p.grad;
    a.blocks = p.blocks;
    a.dw_part = p.dw_part;
    a.db_part = p.db_part;
    a.smax = p.smax16;
    a.L = p.L;
    // PL = 2 needs the slab maxima of k1_reduce_launch (launched right after k1)
    if (p.x6 == 2) dw16_kernel<2><<<p.dw_grid, kThreads, 0, s>>>(a);
    else dw16_kernel<3><<<p.dw_grid, kThreads, 0, s>>>(a);
}

void k1_reduce_launch(const FusedPlan& p, float* out_loss, hipStream_t s) {
    const int nslab = (p.dw16 && p.x6 == 2) ? 2 * p.L : 0;
    k1_reduce_kernel<<<nslab + 1, 1024, 0, s>>>(p.smax_part, p.num_wg * 8, p.smax16, nslab, p.loss_part,
                                                p.num_wg, p.loss_total, out_loss);
}

}  // namespace lnerf
