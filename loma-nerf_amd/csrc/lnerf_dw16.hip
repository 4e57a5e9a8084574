// lnerf_dw16.hip -- k2 on wave pairs: dW_l = sum_s A_{l-1}[s]^T G_l[s] and db_l = sum_s G_l[s]
// from the slabs k1 wrote, in k1's split (fp16x3 on v_mfma_f32_32x32x16_f16, bf16x6 / bf16 on
// v_mfma_f32_32x32x16_bf16, with per-sample balanced exponent shifts), two waves per SIMD.
//
// Reference: the weight/bias adjoints of nerf.py's reverse pass (reverse_diff.py:492-559;
// dW_l += A_{l-1}^T G_l, db_l += sum_rows G_l). One workgroup (8 waves)
// streams a contiguous range of 16-sample half-blocks of one layer:
//  * global -> registers: a slab tile's half-block is sample-major, [feature half 2][16 samples]
//    [16 features] (G: fp32, 1 KiB per wave-store of k1; A under fp16x3: int24, 768 B,
//    lnerf_internal.h a24_slabs), read as fully coalesced 16-B (12-B) loads, 4 features of one
//    sample per thread, three half-blocks ahead;
//  * split once, cooperatively: every value is scaled and split into its hi/lo (fp16x3) or
//    hi/mid/lo (bf16x6) planes exactly once per workgroup and written to a double-buffered LDS
//    image [plane][16 samples][512 features] (A rows 0..255, G rows 256..511), 8 B per plane and
//    thread (one ds_write_b64), the 8-B feature quads XOR-swizzled per sample row (swz) so that
//    these writes and the fragment reads are both bank-conflict-free;
//  * MFMA operands come out of that sample-major image transposed by ds_read_b64_tr_b16: lane
//    (feature l & 31, samples 8 (l >> 5) ..+7) takes two 4-sample x 16-feature blocks;
//  * each wave owns a TI x TJ block of 32 x 32 output tiles (2 x 4 for the hidden layers);
//  * db from the same registers (per-feature partial sums, reduced in LDS at the end);
//  * partials per split, summed in order by grad_reduce_kernel (deterministic, no atomics);
//  * under fp16x3, the exceptional rows of the split's range (lnerf_internal.h kXrowD0: rows far
//    below or above the layer's product scale, every ray's last sample) are dropped from the fp16x3
//    products and multiplied afterwards on the bf16x6 split, gathered 16 to a group, into the same
//    accumulators (xrow_pass).
#include "lnerf_internal.h"

namespace lnerf {

namespace {

typedef float fx4 __attribute__((ext_vector_type(4)));
typedef float fx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf4 __attribute__((ext_vector_type(4)));

// split round k after column k's MFMAs (1): dW 0.733-0.737 -> 0.722-0.726 ms interleaved; 0 = before them
#ifndef LNERF_DW16_SPLIT_LATE
#define LNERF_DW16_SPLIT_LATE 1
#endif
// half-blocks of slab loads in flight per thread (3: default; 2: 17 fewer registers)
#ifndef LNERF_DW16_DEPTH
#define LNERF_DW16_DEPTH 3
#endif

// XROW: the exceptional-row pass under fp16x3 (A/B: 0 = round 5's plain balanced split for every row)
#ifndef LNERF_DW16_XROW
#define LNERF_DW16_XROW 1
#endif

// WAVES: waves per dW workgroup. 8 (round 5): two per SIMD, 256 registers each -- a 2 x 4 tile block
// per wave, three half-blocks of loads in flight that the compiler partly spills to scratch (and
// then waits for with vmcnt(0)); 4 (round 6 A/B): one wave per SIMD with the whole 512-entry
// register file -- a 4 x 4 tile block per wave and the same loads in registers (no spills), twice the
// rounds per thread. Measured in-process on the bench batch: k2 0.866-0.899 ms against 0.765 for 8
// waves (k1 unchanged): without a partner wave the split VALU, the image writes and the
// per-half-block barrier no longer issue under another wave's MFMAs; the spills were not the bound.
#ifndef LNERF_DW16_WAVES
#define LNERF_DW16_WAVES 8
#endif
constexpr int kWavesDw = LNERF_DW16_WAVES;
static_assert(kWavesDw == 16 || kWavesDw == 8 || kWavesDw == 4, "dW workgroups of 16, 8 or 4 waves");
constexpr int kThreads = 64 * kWavesDw;
// a 32-feature tile's half-block is 128 threads' loads (4 features of one sample each); the
// workgroup's kTileGroups thread groups take kRPO tiles of an operand each: rounds 0 .. kRPO - 1
// load A tiles, kRPO .. 2 kRPO - 1 G tiles, round i tile kTileGroups (i % kRPO) + t / 128
constexpr int kTileGroups = kWavesDw / 2;
constexpr int kRPO = 8 / kTileGroups;
constexpr int kRounds = 2 * kRPO;
constexpr int kRows = 512;                  // A rows [0, 256) and G rows [256, 512) of the image
// one plane of a half-block: [16 samples][512 features] 16-bit, each sample's row padded by 64 B
// so that the 4 sample rows one ds_read_b64_tr_b16 lane group reads start 16 banks apart
// (conflict-free reads; the ds_write_b64 image writes see a 2-way conflict)
#ifndef LNERF_DW16_SWZ
#define LNERF_DW16_SWZ 1
#endif
// SWZ: rows of exactly 1 KiB with the 8-B feature quads XOR-swizzled per row (conflict-free writes
// and reads); else rows padded by 64 B (conflict-free reads, 2-way conflicted writes)
constexpr int kImgRow = kRows * 2 + (LNERF_DW16_SWZ ? 0 : 64);
__host__ __device__ constexpr int swz(int row) { return LNERF_DW16_SWZ ? (0x18140C00 >> (8 * (row & 3))) & 0xFF : 0; }
constexpr int kPlaneBytes = 16 * kImgRow;
// PL: the split of a dW launch -- 3 = bf16x6, 2 = fp16x3, 1 = bf16 (all x 2^e, per-sample shifts)
// -- and kX6A24 = 4: the bf16x6 split of an fp16x3 training's int24 activation slabs, which the
// exceptional rows take (xrow_pass): bf16 planes keep fp32's exponent range
constexpr int kX6A24 = 4;
__host__ __device__ constexpr int nplanes(int PL) { return PL == kX6A24 ? 3 : PL; }
__host__ __device__ constexpr bool a24k(int PL) { return PL == kX6A24 || a24_slabs(PL); }
// the split of the exceptional rows under fp16x3 training
constexpr int kXrowPL = a24_slabs(2) ? kX6A24 : 3;
template <int PL>
constexpr int image_bytes() { return nplanes(PL) * kPlaneBytes; }

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
    const unsigned* sexp;       // k1's per-sample words [l][position] (sexp_xa / sexp_xg / sexp_dmax)
    int* xcount;                // per workgroup: the exceptional rows it multiplied, of them last samples
    int rpad;                   // slab positions per layer
    const int* eshift;          // per-layer product shift E_l (k1_reduce_kernel)
    int L;
    const int* gate;            // nullable: the launch exits at once unless *gate != 0 (the floor guard's
                                // re-run, lnerf_internal.h kGuardExp)
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// The 16 B that thread t loads in round i of a half-block (8 waves: rounds 0, 1 are A tiles 0-3 and
// 4-7, rounds 2, 3 G tiles 0-3 and 4-7; tile 4 (i & 1) + t / 128 -- generally kTileGroups (i % kRPO)
// + t / 128, A for i < kRPO), and inside the tile's 512-float
// half-block [h][n][16 f] (k16's sample-major layout) the floats 4 (t % 128) ..+3 = features
// 16 h + 4 (t % 4) ..+3 of sample n, with h = (t / 64) % 2 and n = (t % 64) / 4. A slab block is
// [tile][half-block 2][512]. The per-thread part of the offset is fixed (RowMap), the half-block
// part is wave-uniform.
struct RowMap {
    int lane;        // per-thread float offset inside a tile's half-block
    int hstride;     // floats between the two half-blocks of a 32-sample block's tile
    int rowo;        // the thread's first feature inside its 32-feature tile (4 consecutive)
    int isamp;       // the thread's sample inside the half-block (its LDS image row)
    int tile[kRounds];   // wave-uniform: the 32-feature tile of round i (tile 0 for tiles past the layer)
    bool ok[kRounds];    // wave-uniform: the tile exists in this layer (else it is never split)
};

__device__ __forceinline__ RowMap row_map(int kt, int nt) {
    RowMap m;
    const int t = threadIdx.x, u = t & 127;
    m.lane = 4 * u;
    m.hstride = 512;
    m.rowo = 16 * ((t >> 6) & 1) + 4 * (t & 3);
    m.isamp = (t & 63) >> 2;
    const int w2 = wave_id() >> 1;
#pragma unroll
    for (int i = 0; i < kRounds; ++i) {
        const int tl = kTileGroups * (i % kRPO) + w2;
        m.ok[i] = tl < (i < kRPO ? kt : nt);
        m.tile[i] = m.ok[i] ? tl : 0;
    }
    return m;
}

// image feature row of round i's 4 values for thread t (A rows 0..255, G rows 256..511)
__device__ __forceinline__ int image_row(int i, const RowMap& m) {
    return (i < kRPO ? 0 : 256) + 32 * (kTileGroups * (i % kRPO) + (threadIdx.x >> 7)) + m.rowo;
}

struct Loads {
    fx4 v[kRounds];
    unsigned e;   // the sample's k1 word (sexp_xa, sexp_xg, sexp_dmax)
};

// Per-sample balancing of the split: the product of a sample's A row and G row is what dW sums,
// so a sample's A row is scaled by 2^ea and its G row by 2^eg with ea + eg = E_l for every sample
// (E_l = min over samples of exA + exG, the row shifts k1 used; k1_reduce_kernel): the products
// keep one layer-wide scale while each operand sits within D/2 binades of its own ideal shift,
// D = exA + exG - E_l -- a sample whose A is tiny and G huge (tiny sigma behind the 1e8 delta)
// no longer pushes every other sample's G toward fp16's subnormals. Neither operand exceeds its
// own ideal shift, so nothing overflows. -128 marks an all-zero row: its partner keeps its own
// shift (the zero products stay zero). kSexpNonFinite marks an activation row holding a NaN or an
// infinity (k1 store_sexp, encoded at shift 0): its G row keeps its own shift and the A row takes
// the rest of E, so the product scale stays 2^E; its terms are non-finite anyway.
__device__ __forceinline__ void sample_shifts(unsigned e, int E, int& ea, int& eg) {
    const int xa = sexp_xa(e), xg = sexp_xg(e);
    if (xa == -128 || xg == -128) {
        ea = xa < -126 ? 0 : xa;
        eg = xg == -128 ? 0 : xg;
        return;
    }
    if (xa == kSexpNonFinite) {
        eg = xg;
        ea = E - xg;
        return;
    }
    const int d = xa + xg - E;   // >= 0
    ea = xa - (d >> 1);
    eg = xg - ((d + 1) >> 1);
}

// Always four loads from valid addresses and no select on the data (nothing waits for it before
// its use): rows past the layer's tiles are never split, half-blocks past the split land in the
// idle image and add nothing to db (the callers' hb < hb1 guards).
template <bool A24>
__device__ __forceinline__ void issue_loads(const float* A, const float* G, const unsigned* se, int kt,
                                            int nt, const RowMap& m, int hb, int hb_end, Loads& L) {
    const bool in = hb < hb_end;
    const int hbc = in ? hb : max(0, hb_end - 1);
    L.e = se[hbc * 16 + m.isamp];
    const int blk = hbc >> 1, half = hbc & 1;
    const float* pg = G + (size_t)blk * nt * 1024 + half * m.hstride;
    if constexpr (A24) {
        // int24 A slab (k1 store_slab_step24): a tile-block is 3 KiB, its half-blocks 1.5 KiB
        // [h][n][16 f] x 3 B, so thread u's 4 values are the 12 B at 12 u
        // (three dword loads the compiler merges into one global_load_dwordx3: a nontemporal load
        // of a 3-element vector type keeps only its first element)
        const unsigned char* pa = (const unsigned char*)A + ((size_t)blk * kt * 3072 + half * 1536 + 12 * (threadIdx.x & 127));
#pragma unroll
        for (int i = 0; i < kRPO; ++i) {
            const unsigned* q = (const unsigned*)(pa + m.tile[i] * 3072);
            L.v[i] = fx4{__builtin_bit_cast(float, __builtin_nontemporal_load(q)),
                         __builtin_bit_cast(float, __builtin_nontemporal_load(q + 1)),
                         __builtin_bit_cast(float, __builtin_nontemporal_load(q + 2)), 0.0f};
        }
    } else {
        const float* pa = A + (size_t)blk * kt * 1024 + half * m.hstride;
#pragma unroll
        for (int i = 0; i < kRPO; ++i) L.v[i] = __builtin_nontemporal_load((const fx4*)(pa + m.tile[i] * 1024 + m.lane));
    }
#pragma unroll
    for (int i = kRPO; i < kRounds; ++i) L.v[i] = __builtin_nontemporal_load((const fx4*)(pg + m.tile[i] * 1024 + m.lane));
}

// The 4 values of an int24 A round (k1 store_slab_step24): 3 dwords holding the low 24 bits of
// y_i = 1.5 2^23 + q_i (q_i = rint(x_i 2^(xa + 8)), |q_i| < 2^22, so y_i lies in [2^23, 2^24)
// where its mantissa field is y_i - 2^23): q_i = float(0x4B000000 | bits) - 1.5 2^23, exact.
__device__ __forceinline__ fx4 decode_a24(const fx4& raw) {
    // bit_cast the whole vector: __builtin_bit_cast of an ext_vector element (raw[1]) yields
    // element 0 in this compiler (ROCm 7.2 clang), which decoded three quarters of A from the
    // wrong dword
    typedef unsigned ux4 __attribute__((ext_vector_type(4)));
    const ux4 d = __builtin_bit_cast(ux4, raw);
    const unsigned d0 = d[0], d1 = d[1], d2 = d[2];
    const unsigned m0 = d0 & 0xFFFFFFu;
    const unsigned m1 = __builtin_amdgcn_alignbit(d1, d0, 24) & 0xFFFFFFu;
    const unsigned m2 = __builtin_amdgcn_alignbit(d2, d1, 16) & 0xFFFFFFu;
    const unsigned m3 = d2 >> 8;
    constexpr float kMagic = 12582912.0f;   // 1.5 2^23
    return fx4{__builtin_bit_cast(float, 0x4B000000u | m0) - kMagic, __builtin_bit_cast(float, 0x4B000000u | m1) - kMagic,
               __builtin_bit_cast(float, 0x4B000000u | m2) - kMagic, __builtin_bit_cast(float, 0x4B000000u | m3) - kMagic};
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


// Split round i of the thread's values (4 features of sample n) into the plane image: 8 B per
// plane at [plane][n][row .. row + 3]; rounds 0, 1 are A rows (shift ea), 2, 3 G rows (shift eg).
template <int PL>
__device__ __forceinline__ void write_planes_row(const fx4& v, int i, unsigned char* img, float sa, float sg,
                                                 const RowMap& m) {
    unsigned char* p = img + m.isamp * kImgRow + 8 * ((image_row(i, m) >> 2) ^ swz(m.isamp));
    const float sc = i < kRPO ? sa : sg;
    if constexpr (PL == 2) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        unsigned h0, l0, h1, l1;
        split_h2(v[0], v[1], sc, h0, l0);
        split_h2(v[2], v[3], sc, h1, l1);
        *(u2*)(p) = u2{h0, h1};
        *(u2*)(p + kPlaneBytes) = u2{l0, l1};
    } else if constexpr (PL == 1) {
        const fx4 x = v * sc;
        *(bf4*)(p) = bf4{(__bf16)x[0], (__bf16)x[1], (__bf16)x[2], (__bf16)x[3]};
    } else {
        bf4 h, m, lo;
        split4(v * sc, h, m, lo);
        *(bf4*)(p) = h;
        *(bf4*)(p + kPlaneBytes) = m;
        *(bf4*)(p + 2 * kPlaneBytes) = lo;
    }
}

// the split scales 2^ea (A rows) and 2^eg (G rows) of a half-block's sample (sample_shifts); with
// int24 A slabs the A values arrive as q = x 2^(xa + 8), so their scale is 2^(ea - xa - 8) (1 for an
// all-zero row, whose q are 0)
// An exceptional row (lnerf_internal.h kXrowD0): a live row (neither all-zero, -128, nor a non-finite
// activation row, kSexpNonFinite) whose deficit d = xa + xg - E_l is negative (products above the
// layer's scale: a ray's last sample, which k1 keeps out of E_l) or above the row's dmax (kXrowD0;
// kXrowLast = 127 for every ray's last sample: exceptional only above the scale)
__device__ __forceinline__ bool xrow(unsigned e, int E) {
    const int xa = sexp_xa(e), xg = sexp_xg(e);
    const int d = xa + xg - E;
    return xa > -127 && xg > -127 && (d < 0 || d > sexp_dmax(e));
}

template <int PL>
__device__ __forceinline__ void sample_scales(unsigned e, int E, float& sa, float& sg) {
    int ea, eg;
    sample_shifts(e, E, ea, eg);
    if constexpr (a24k(PL)) {
        const int xa = sexp_xa(e);
        ea = xa == -128 ? 0 : ea - (xa == kSexpNonFinite ? 0 : xa) - 8;
    }
    sa = __builtin_ldexpf(1.0f, ea);
    sg = __builtin_ldexpf(1.0f, eg);
    if constexpr (PL == 2 && LNERF_DW16_XROW) {
        // the fp16x3 products skip the exceptional rows (xrow_pass multiplies them)
        const bool x = xrow(e, E);
        sa = x ? 0.0f : sa;
        sg = x ? 0.0f : sg;
    }
}

// round i's values as the split takes them (int24 A rounds decoded). A row k1 marked non-finite
// (kSexpNonFinite) turns its out-of-range codes (|q| >= 2^22: NaN and +-infinity) back into NaN;
// the test is one wave-uniform branch, taken only when some lane's sample is marked.
template <int PL>
__device__ __forceinline__ fx4 round_values(const Loads& L, int i) {
    if constexpr (a24k(PL)) {
        if (i >= kRPO) return L.v[i];
        fx4 v = decode_a24(L.v[i]);
        const bool marked = sexp_xa(L.e) == kSexpNonFinite;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(marked) != 0, 0)) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (marked && __builtin_fabsf(v[j]) >= 4194304.0f) v[j] = __builtin_nanf("");
            // a volatile statement cannot be speculated, so the block stays a branch whatever the
            // compiler's cost model (measured: the dynamic VALU count per wave is the same as
            // without it, i.e. the compiler had kept the branch; k2 time unchanged)
            asm volatile("" : "+v"(v));
        }
        return v;
    }
    return L.v[i];
}

template <int PL>
__device__ __forceinline__ void write_planes(const Loads& L, unsigned char* img, int E, const RowMap& m) {
    float sa, sg;
    sample_scales<PL>(L.e, E, sa, sg);
#pragma unroll
    for (int i = 0; i < kRounds; ++i) write_planes_row<PL>(round_values<PL>(L, i), i, img, sa, sg, m);
}

__device__ __forceinline__ fx16 mfma32(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ fx16 mfma32h(const bf8& a, const bf8& b, fx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hf8, a), __builtin_bit_cast(hf8, b), c, 0, 0,
                                                  0);
}

typedef short s4 __attribute__((ext_vector_type(4)));

// One MFMA operand fragment (32 features x 16 samples, one plane) from the sample-major image:
// two ds_read_b64_tr_b16, samples 8 h .. +3 and 8 h + 4 .. +7 of lane l's feature (h = l >> 5).
// `addr` is this lane's byte address of the fragment's first feature in the plane.
__device__ __forceinline__ bf8 read_frag(unsigned char* addr) {
    typedef __attribute__((address_space(3))) s4* lp;
    const s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(__attribute__((address_space(3))) void*)addr);
    const s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lp)(__attribute__((address_space(3))) void*)(addr + 4 * kImgRow));
    typedef short s8 __attribute__((ext_vector_type(8)));
    return __builtin_bit_cast(bf8, s8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]});
}

// This lane's byte offset inside a plane for a fragment starting at feature 0: lane 4 q + p of
// each 16-lane group supplies sample row 8 (l >> 5) + q, features 16 ((l >> 4) & 1) + 4 p ..+3
// (ds_read_b64_tr_b16 hands lane i of the group feature i of the 4 rows).
__device__ __forceinline__ int frag_off(int f0) {
    const int l = threadIdx.x & 63;
    const int row = 8 * (l >> 5) + ((l >> 2) & 3);
    const int quad = (f0 >> 2) + 4 * ((l >> 4) & 1) + (l & 3);
    return row * kImgRow + 8 * (quad ^ swz(row));
}

// One 32 x 32 output tile's products of a half-block: A fragment planes ap, G fragment planes gp
// (small terms first)
template <int PL>
__device__ __forceinline__ fx16 mma_tile(const bf8 (&ap)[nplanes(PL)], const bf8 (&gp)[nplanes(PL)], fx16 c) {
    if constexpr (PL == 2) {
        c = mfma32h(ap[0], gp[1], c);
        c = mfma32h(ap[1], gp[0], c);
        c = mfma32h(ap[0], gp[0], c);
    } else if constexpr (PL == 1) {
        c = mfma32(ap[0], gp[0], c);
    } else {
        c = mfma32(ap[0], gp[2], c);
        c = mfma32(ap[1], gp[1], c);
        c = mfma32(ap[2], gp[0], c);
        c = mfma32(ap[1], gp[0], c);
        c = mfma32(ap[0], gp[1], c);
        c = mfma32(ap[0], gp[0], c);
    }
    return c;
}

// One output column tile j's products for all TI row tiles, product-major: the TI accumulators
// take their k-th product in turn, so consecutive MFMAs never wait on each other's result (a
// dependent 32x32x16 MFMA pair stalls for the first one's passes; two waves per SIMD hide that with
// the partner's MFMAs, one wave per SIMD has only its own other tiles). Round-6 default for every
// wave count: the same sums per accumulator bit for bit; 8 waves measured k2 0.761 ms against
// 0.765 tile-major (in-process A/B).
#ifndef LNERF_DW16_PMAJOR
#define LNERF_DW16_PMAJOR 1
#endif
template <int PL, int TI, int TJ>
__device__ __forceinline__ void mma_col(const bf8 (&ap)[TI][nplanes(PL)], const bf8 (&gp)[nplanes(PL)],
                                        fx16 (&acc)[TI][TJ], int j) {
    if constexpr (!LNERF_DW16_PMAJOR) {
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mma_tile<PL>(ap[i], gp, acc[i][j]);
    } else if constexpr (PL == 2) {
        // (a_hi g_lo, a_lo g_hi, a_hi g_hi): small terms first, as mma_tile
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma32h(ap[i][0], gp[1], acc[i][j]);
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma32h(ap[i][1], gp[0], acc[i][j]);
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma32h(ap[i][0], gp[0], acc[i][j]);
    } else if constexpr (PL == 1) {
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma32(ap[i][0], gp[0], acc[i][j]);
    } else {
        constexpr int pa[6] = {0, 1, 2, 1, 0, 0}, pg[6] = {2, 1, 0, 0, 1, 0};
#pragma unroll
        for (int k = 0; k < 6; ++k)
#pragma unroll
            for (int i = 0; i < TI; ++i) acc[i][j] = mfma32(ap[i][pa[k]], gp[pg[k]], acc[i][j]);
    }
}

// The wave's TI x TJ tile block (TI 32-row tiles of A, TJ of G) on one half-block image, with
// the split of the next half-block interleaved (round k beside output column tile k), so the
// VALU split issues under the MFMAs. Branch-free (ACTIVE is a template parameter; past the
// split's last half-block the zeroed loads land in the idle image buffer).
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void block_mma(const unsigned char* img, int a0, int g0, fx16 (&acc)[TI][TJ],
                                          const Loads& nl, unsigned char* nxt, const RowMap& m, int E,
                                          bool live = true) {
    float sa, sg;
    sample_scales<PL>(nl.e, E, sa, sg);
    sa = live ? sa : 0.0f;
    sg = live ? sg : 0.0f;
    const unsigned char* fl = img;
    constexpr int NP = nplanes(PL);
    bf8 ap[TI][NP];
    if constexpr (ACTIVE) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int p = 0; p < NP; ++p) ap[i][p] = read_frag((unsigned char*)fl + p * kPlaneBytes + frag_off(a0 + 32 * i));
    }
    // RPS split rounds beside each output column tile (8 waves: one; 4 waves: kRounds / TJ)
    constexpr int RPS = (kWavesDw == 8 || TJ >= kRounds) ? 1 : (kRounds + TJ - 1) / TJ;
    constexpr int NR = (kRounds + RPS - 1) / RPS;
    constexpr int NK = NR > TJ ? NR : TJ;
    auto split = [&](int k) {
        // rows past the layer's tiles are never read: skip their split (wave-uniform: a wave's
        // values of a round lie in one 32-feature tile); FULL layers need no branch
#pragma unroll
        for (int r = 0; r < RPS; ++r) {
            const int i = k * RPS + r;
            if (i < kRounds && (FULL || m.ok[i])) write_planes_row<PL>(round_values<PL>(nl, i), i, nxt, sa, sg, m);
        }
    };
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        if (!LNERF_DW16_SPLIT_LATE) split(k);
        if constexpr (ACTIVE) {
            if (k < TJ) {
                const int j = k < TJ ? k : 0;
                bf8 gp[NP];
#pragma unroll
                for (int p = 0; p < NP; ++p) gp[p] = read_frag((unsigned char*)fl + p * kPlaneBytes + frag_off(256 + g0 + 32 * j));
                mma_col<PL, TI, TJ>(ap, gp, acc, j);
            }
        }
        if (LNERF_DW16_SPLIT_LATE) split(k);
    }
}

// Three half-blocks in flight: step I of a 3-step rotation over the load
// register sets (images alternate at run time). Entering half-block hb: its planes are in image
// (hb - hb0) & 1, the set after I holds hb + 1 (split now into the other image), the one after
// that hb + 2 (in flight) and set I is free: it receives hb + 3.
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL, int I>
__device__ __forceinline__ void hb_step3(const float* A, const float* G, const unsigned* se, int kt, int nt,
                                         const RowMap& m, int hb, int hb0, int hb1, int a0, int g0,
                                         fx16 (&acc)[TI][TJ], Loads& L0, Loads& L1, Loads& L2, fx4 (&dbs)[kRPO],
                                         unsigned char* lds, int E, bool& xany) {
    constexpr int kIB = image_bytes<PL>();
    Loads& fr = I == 0 ? L0 : I == 1 ? L1 : L2;
    const Loads& nx = I == 0 ? L1 : I == 1 ? L2 : L0;
    issue_loads<a24k(PL)>(A, G, se, kt, nt, m, hb + 3, hb1, fr);
    if (hb + 1 < hb1) {
#pragma unroll
        for (int i = 0; i < kRPO; ++i) dbs[i] += nx.v[kRPO + i];
    }
    const int cur = (hb - hb0) & 1;
    block_mma<PL, TI, TJ, ACTIVE, FULL>(lds + cur * kIB, a0, g0, acc, nx, lds + (cur ^ 1) * kIB, m, E, hb + 1 < hb1);
    // (after the split of hb + 1, which already waited for its k1 word)
    if constexpr (PL == 2 && LNERF_DW16_XROW) xany |= hb + 1 < hb1 && xrow(nx.e, E);
    __syncthreads();
}

template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void hb_loop3(const float* A, const float* G, const unsigned* se, int kt, int nt,
                                         const RowMap& m, int hb0, int hb1, int a0, int g0, fx16 (&acc)[TI][TJ],
                                         Loads& L0, Loads& L1, Loads& L2, fx4 (&dbs)[kRPO], unsigned char* lds,
                                         int E, bool& xany) {
    // whole triples only (one loop body; remainder copies make the compiler spill the
    // accumulators): the steps past hb1 split zero-scaled (zero) planes and add nothing
    for (int hb = hb0; hb < hb1; hb += 3) {
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 0>(A, G, se, kt, nt, m, hb, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 1>(A, G, se, kt, nt, m, hb + 1, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
        hb_step3<PL, TI, TJ, ACTIVE, FULL, 2>(A, G, se, kt, nt, m, hb + 2, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
    }
}

// Two half-blocks in flight (LNERF_DW16_DEPTH = 2): the same rotation over two register sets --
// entering hb, set I held hb (split last step, free: it receives hb + 2), set I ^ 1 holds hb + 1
// (split now). 17 fewer registers than the 3-deep rotation.
template <int PL, int TI, int TJ, bool ACTIVE, bool FULL, int I>
__device__ __forceinline__ void hb_step2(const float* A, const float* G, const unsigned* se, int kt, int nt,
                                         const RowMap& m, int hb, int hb0, int hb1, int a0, int g0,
                                         fx16 (&acc)[TI][TJ], Loads& L0, Loads& L1, fx4 (&dbs)[kRPO],
                                         unsigned char* lds, int E, bool& xany) {
    constexpr int kIB = image_bytes<PL>();
    Loads& fr = I == 0 ? L0 : L1;
    const Loads& nx = I == 0 ? L1 : L0;
    issue_loads<a24k(PL)>(A, G, se, kt, nt, m, hb + 2, hb1, fr);
    if (hb + 1 < hb1) {
#pragma unroll
        for (int i = 0; i < kRPO; ++i) dbs[i] += nx.v[kRPO + i];
    }
    const int cur = (hb - hb0) & 1;
    block_mma<PL, TI, TJ, ACTIVE, FULL>(lds + cur * kIB, a0, g0, acc, nx, lds + (cur ^ 1) * kIB, m, E, hb + 1 < hb1);
    // (after the split of hb + 1, which already waited for its k1 word)
    if constexpr (PL == 2 && LNERF_DW16_XROW) xany |= hb + 1 < hb1 && xrow(nx.e, E);
    __syncthreads();
}

template <int PL, int TI, int TJ, bool ACTIVE, bool FULL>
__device__ __forceinline__ void hb_loop2(const float* A, const float* G, const unsigned* se, int kt, int nt,
                                         const RowMap& m, int hb0, int hb1, int a0, int g0, fx16 (&acc)[TI][TJ],
                                         Loads& L0, Loads& L1, fx4 (&dbs)[kRPO], unsigned char* lds, int E,
                                         bool& xany) {
    for (int hb = hb0; hb < hb1; hb += 2) {
        hb_step2<PL, TI, TJ, ACTIVE, FULL, 0>(A, G, se, kt, nt, m, hb, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
        hb_step2<PL, TI, TJ, ACTIVE, FULL, 1>(A, G, se, kt, nt, m, hb + 1, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
    }
}

// ---- exceptional rows (lnerf_internal.h kXrowD0) ----------------------------------------------
// The four rounds of loads of ONE sample row at slab position p (p < 0: position 0, whose values
// the caller scales by 0): the thread's [h][sample][4-feature quad] offset inside the row's
// half-block with the sample index replaced by p's.
template <bool A24>
__device__ __forceinline__ void gather_loads(const float* A, const float* G, const unsigned* se, int kt, int nt,
                                             const RowMap& m, int p, Loads& L) {
    const int pc = p < 0 ? 0 : p;
    L.e = se[pc];
    const int hb = pc >> 4, blk = hb >> 1, half = hb & 1;
    const int u = ((int)threadIdx.x & 127 & ~0x3C) | ((pc & 15) << 2);
    const float* pg = G + (size_t)blk * nt * 1024 + half * 512 + 4 * u;
    if constexpr (A24) {
        const unsigned char* pa = (const unsigned char*)A + ((size_t)blk * kt * 3072 + half * 1536 + 12 * u);
#pragma unroll
        for (int i = 0; i < kRPO; ++i) {
            const unsigned* q = (const unsigned*)(pa + m.tile[i] * 3072);
            L.v[i] = fx4{__builtin_bit_cast(float, q[0]), __builtin_bit_cast(float, q[1]),
                         __builtin_bit_cast(float, q[2]), 0.0f};
        }
    } else {
        const float* pa = A + (size_t)blk * kt * 1024 + half * 512 + 4 * u;
#pragma unroll
        for (int i = 0; i < kRPO; ++i) L.v[i] = *(const fx4*)(pa + m.tile[i] * 1024);
    }
#pragma unroll
    for (int i = kRPO; i < kRounds; ++i) L.v[i] = *(const fx4*)(pg + m.tile[i] * 1024);
}

// the wave's TI x TJ tile block of one image (no split interleaved)
template <int PL, int TI, int TJ>
__device__ __forceinline__ void mma_block(const unsigned char* img, int a0, int g0, fx16 (&acc)[TI][TJ]) {
    constexpr int NP = nplanes(PL);
    bf8 ap[TI][NP];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p) ap[i][p] = read_frag((unsigned char*)img + p * kPlaneBytes + frag_off(a0 + 32 * i));
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        bf8 gp[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) gp[p] = read_frag((unsigned char*)img + p * kPlaneBytes + frag_off(256 + g0 + 32 * j));
        mma_col<PL, TI, TJ>(ap, gp, acc, j);
    }
}

// After the fp16x3 half-blocks of a split: its exceptional rows -- found by a scan of its
// positions' k1 words (the same xrow test that zeroed their scales in the main loop), listed in
// position order into an LDS ring and multiplied 16 at a time on the bf16x6 split into the same
// accumulators (products at the layer's scale 2^E: the per-sample balanced shifts, which bf16's
// exponent range carries at any deficit); each group's gathered loads are issued before the
// previous group is split. `any`: some thread's main loop met an exceptional row; a split that met
// none (the bench batch: all but a handful) skips the scan after two barriers. Deterministic: the
// groups follow position order. Returns the rows multiplied and, of them, rays' last samples.
constexpr int kXrowRing = 8 * kThreads;   // > 15 pending + 4 x kThreads listed per scan step
template <int TI, int TJ>
__device__ __forceinline__ int2 xrow_pass(const float* A, const float* G, const unsigned* se, int KT, int NT,
                                          const RowMap& m, int hb0, int hb1, int a0, int g0, bool active,
                                          fx16 (&acc)[TI][TJ], unsigned char* lds, int E, bool any) {
    constexpr int PX = kXrowPL;
    int* ring = (int*)(lds + image_bytes<PX>());
    int* wcnt = ring + kXrowRing;   // [2: rows, last samples][4 scan rounds][waves], then the any flags
    constexpr int W = kWavesDw;
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int p0 = hb0 * 16, p1 = hb1 * 16;
    const bool wany = __builtin_amdgcn_ballot_w64(any) != 0;
    __syncthreads();   // every wave is done with the fp16x3 images
    if (lane == 0) wcnt[8 * W + wave] = wany ? 1 : 0;
    __syncthreads();
    int anyw = 0;
#pragma unroll
    for (int w = 0; w < kWavesDw; ++w) anyw |= wcnt[8 * W + w];
    if (!anyw) return int2{0, 0};
    int head = 0, tail = 0, ntail = 0;   // workgroup-uniform (ring slot = index % kXrowRing)
    for (int base = p0; base < p1; base += 4 * kThreads) {
        bool f[4], tl[4];
        unsigned long long bal[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = base + k * kThreads + tid;
            const unsigned e = se[p < p1 ? p : p0];
            f[k] = p < p1 && xrow(e, E);
            tl[k] = f[k] && sexp_dmax(e) == kXrowLast;
        }
        __syncthreads();   // the previous step's counts are read
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bal[k] = __builtin_amdgcn_ballot_w64(f[k]);
            const unsigned long long bt = __builtin_amdgcn_ballot_w64(tl[k]);
            if (lane == 0) {
                wcnt[k * W + wave] = __builtin_popcountll(bal[k]);
                wcnt[4 * W + k * W + wave] = __builtin_popcountll(bt);
            }
        }
        __syncthreads();
        int off = tail;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int mine = off;
            for (int w = 0; w < kWavesDw; ++w) {
                const int c = wcnt[k * W + w];
                mine += w < wave ? c : 0;
                off += c;
                ntail += wcnt[4 * W + k * W + w];
            }
            if (f[k]) {
                const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(bal[k] >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal[k], 0u));
                ring[(mine + r) % kXrowRing] = base + k * kThreads + tid;
            }
        }
        tail = off;
        __syncthreads();
        // the whole groups now in the ring (every remaining entry after the last scan step)
        const bool last = base + 4 * kThreads >= p1;
        const int ng = last ? (tail - head + 15) / 16 : (tail - head) / 16;
        if (ng > 0) {
            auto pos = [&](int gi) {
                const int at = head + 16 * gi + m.isamp;
                return at < tail ? ring[at % kXrowRing] : -1;
            };
            int pc = pos(0);
            Loads Lc;
            gather_loads<a24k(PX)>(A, G, se, KT, NT, m, pc, Lc);
            for (int gi = 0; gi < ng; ++gi) {
                const int pn = gi + 1 < ng ? pos(gi + 1) : -1;
                Loads Ln;
                if (gi + 1 < ng) gather_loads<a24k(PX)>(A, G, se, KT, NT, m, pn, Ln);
                float sa, sg;
                sample_scales<PX>(Lc.e, E, sa, sg);
                sa = pc < 0 ? 0.0f : sa;
                sg = pc < 0 ? 0.0f : sg;
#pragma unroll
                for (int i = 0; i < kRounds; ++i)
                    if (m.ok[i]) write_planes_row<PX>(round_values<PX>(Lc, i), i, lds, sa, sg, m);
                __syncthreads();
                if (active) mma_block<PX, TI, TJ>(lds, a0, g0, acc);
                __syncthreads();
                Lc = Ln;
                pc = pn;
            }
            head = head + 16 * ng < tail ? head + 16 * ng : tail;
        }
    }
    return int2{tail, ntail};
}

// One split of layer l with TI x TJ tile blocks per wave (the layer's ceil(KT/TI) x ceil(NT/TJ)
// blocks on waves 0.., at most 8).
template <int PL, int TI, int TJ>
__device__ __forceinline__ void dw_split(const Dw16Args& a, int l, int sp, unsigned char* lds) {
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int KT = a.kt[l], NT = a.nt[l];
    const int nbg = (NT + TJ - 1) / TJ, nblk = ((KT + TI - 1) / TI) * nbg;
    const bool active = wave < nblk;
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
    // db: this thread's G values are features image_row(i) - 256 ..+3 of one sample, i = 2, 3
    fx4 dbs[kRPO];
#pragma unroll
    for (int i = 0; i < kRPO; ++i) dbs[i] = fx4{0.0f, 0.0f, 0.0f, 0.0f};

    const float* A = a.act + a.a_off[l];
    const float* G = a.grad + a.g_off[l];
    const RowMap m = row_map(KT, NT);
    // the per-sample balanced shifts (sample_shifts): every product carries 2^E, removed from the
    // partials at the end (exact)
    const unsigned* se = a.sexp + (size_t)l * a.rpad;
    const int E = a.eshift[l];
    const bool full = KT == 8 && NT == 8;
#if LNERF_DW16_DEPTH == 2
    Loads L0, L1;
    bool xany = false;   // this thread split an exceptional row (fp16x3: xrow_pass)
    issue_loads<a24k(PL)>(A, G, se, KT, NT, m, hb0, hb1, L0);
    issue_loads<a24k(PL)>(A, G, se, KT, NT, m, hb0 + 1, hb1, L1);
    if (hb0 < hb1) {
#pragma unroll
        for (int i = 0; i < kRPO; ++i) dbs[i] += L0.v[kRPO + i];
        write_planes<PL>(L0, lds, E, m);
        if constexpr (PL == 2 && LNERF_DW16_XROW) xany = xrow(L0.e, E);
    }
    __syncthreads();
    if (active && full) hb_loop2<PL, TI, TJ, true, true>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
    else if (active) hb_loop2<PL, TI, TJ, true, false>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
    else if (full) hb_loop2<PL, TI, TJ, false, true>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
    else hb_loop2<PL, TI, TJ, false, false>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, dbs, lds, E, xany);
#else
    Loads L0, L1, L2;
    bool xany = false;   // this thread split an exceptional row (fp16x3: xrow_pass)
    issue_loads<a24k(PL)>(A, G, se, KT, NT, m, hb0, hb1, L0);
    issue_loads<a24k(PL)>(A, G, se, KT, NT, m, hb0 + 1, hb1, L1);
    issue_loads<a24k(PL)>(A, G, se, KT, NT, m, hb0 + 2, hb1, L2);
    if (hb0 < hb1) {
#pragma unroll
        for (int i = 0; i < kRPO; ++i) dbs[i] += L0.v[kRPO + i];
        write_planes<PL>(L0, lds, E, m);
        if constexpr (PL == 2 && LNERF_DW16_XROW) xany = xrow(L0.e, E);
    }
    __syncthreads();
    if (active && full) hb_loop3<PL, TI, TJ, true, true>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
    else if (active) hb_loop3<PL, TI, TJ, true, false>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
    else if (full) hb_loop3<PL, TI, TJ, false, true>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
    else hb_loop3<PL, TI, TJ, false, false>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, acc, L0, L1, L2, dbs, lds, E, xany);
#endif

    if constexpr (PL == 2 && LNERF_DW16_XROW) {
        const int2 nx = xrow_pass<TI, TJ>(A, G, se, KT, NT, m, hb0, hb1, a0, g0, active, acc, lds, E, xany);
        if (threadIdx.x == 0 && a.xcount) {
            a.xcount[2 * blockIdx.x] = nx.x;
            a.xcount[2 * blockIdx.x + 1] = nx.y;
        }
    } else {
        if (threadIdx.x == 0 && a.xcount) a.xcount[2 * blockIdx.x] = a.xcount[2 * blockIdx.x + 1] = 0;
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
                            __builtin_ldexpf(acc[i][j][r], -E);
                    }
                }
            }
    }
    // db: 16 threads (one per sample n) per G feature -> in-order sum through LDS [feature][n]
    float* red = (float*)lds;
    __syncthreads();   // the image buffers are free: every wave is past its last MFMA reads
#pragma unroll
    for (int i = 0; i < kRPO; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(image_row(kRPO + i, m) - 256 + j) * 16 + m.isamp] = dbs[i][j];
    __syncthreads();
    if (tid < NT * 32) {
        const float* q = red + tid * 16;
        float s0 = 0.0f;
#pragma unroll
        for (int n = 0; n < 16; ++n) s0 += q[n];
        a.db_part[a.dbp_off[l] + (size_t)sp * NT * 32 + tid] = s0;
    }
}

// Block shape per layer: the smallest tile block that needs at most kWavesDw waves, so small
// layers (the head, layer 0) spread over all SIMDs instead of a few waves. 8 waves: 1x1, 1x2, 2x4;
// 4 waves: 1x1, 2x1, 1x2, 2x2, 4x4 (the 8 x 8 hidden layers).
__host__ __device__ __forceinline__ int dw_shape(int kt, int nt) {
    auto fits = [&](int ti, int tj) { return ((kt + ti - 1) / ti) * ((nt + tj - 1) / tj) <= kWavesDw; };
    if (kWavesDw == 8) {
        if (fits(1, 1)) return 0;
        if (fits(1, 2)) return 1;
        return 2;
    }
    if (kWavesDw == 16) {
        if (fits(1, 1)) return 0;
        if (fits(1, 2)) return 1;
        if (fits(2, 1)) return 3;
        return 4;
    }
    if (fits(1, 1)) return 0;
    if (fits(2, 1)) return 3;
    if (fits(1, 2)) return 1;
    if (fits(2, 2)) return 4;
    return 5;
}

// LDS of a dW workgroup: the two half-block images; under fp16x3 the exceptional rows' bf16x6 image
// and position ring (xrow_pass) reuse and extend them
template <int PL>
constexpr int dw_lds_bytes() {
    constexpr int main = 2 * image_bytes<PL>();
    constexpr int xr = PL == 2 && LNERF_DW16_XROW ? image_bytes<kXrowPL>() + (kXrowRing + 9 * kWavesDw) * 4 : 0;
    return main > xr ? main : xr;
}

template <int PL>
__global__ void __launch_bounds__(kThreads, 1) __attribute__((amdgpu_waves_per_eu(kWavesDw / 4, kWavesDw / 4)))
dw16_kernel(Dw16Args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[dw_lds_bytes<PL>()];
    if (a.gate && *a.gate == 0) return;
    int li = 0;
    while (li + 1 < a.nl && (int)blockIdx.x >= a.wg_off[li + 1]) ++li;
    const int l = a.lid[li], sp = blockIdx.x - a.wg_off[li];
    if constexpr (kWavesDw == 8) {
        switch (dw_shape(a.kt[l], a.nt[l])) {
            case 0: dw_split<PL, 1, 1>(a, l, sp, lds); break;
            case 1: dw_split<PL, 1, 2>(a, l, sp, lds); break;
            default: dw_split<PL, 2, 4>(a, l, sp, lds); break;
        }
    } else if constexpr (kWavesDw == 16) {
        switch (dw_shape(a.kt[l], a.nt[l])) {
            case 0: dw_split<PL, 1, 1>(a, l, sp, lds); break;
            case 1: dw_split<PL, 1, 2>(a, l, sp, lds); break;
            case 3: dw_split<PL, 2, 1>(a, l, sp, lds); break;
            default: dw_split<PL, 2, 2>(a, l, sp, lds); break;
        }
    } else {
        switch (dw_shape(a.kt[l], a.nt[l])) {
            case 0: dw_split<PL, 1, 1>(a, l, sp, lds); break;
            case 3: dw_split<PL, 2, 1>(a, l, sp, lds); break;
            case 1: dw_split<PL, 1, 2>(a, l, sp, lds); break;
            case 4: dw_split<PL, 2, 2>(a, l, sp, lds); break;
            default: dw_split<PL, 4, 4>(a, l, sp, lds); break;
        }
    }
}

// The reductions between k1 and dw16 in one launch (1024 threads per block):
//  * blocks [0, nl): layer l's product shift E_l = min over samples of exA + exG (k1's per-sample
//    shifts of the layer's A and G rows), from k1's per-wave minima (n per layer; all-zero rows
//    excluded; 0 if every row is), the scale dw16's per-sample balancing keeps uniform;
//  * block nl: the batch loss, the same deterministic 256-lane tree as loss_reduce_kernel
//    (lnerf_fused.hip), into *total (the loss seed) and *out_loss.
__global__ void __launch_bounds__(1024) k1_reduce_kernel(const int* __restrict__ epart, int n,
                                                         int* __restrict__ eshift, int nl,
                                                         const float* __restrict__ loss_part, int nwg,
                                                         float* total, float* out_loss, const int* gate) {
    __shared__ float red[1024];
    if (gate && *gate == 0) return;
    const int t = threadIdx.x;
    if ((int)blockIdx.x < nl) {
        const int* q = epart + (size_t)blockIdx.x * n;
        int m = 1 << 20;
        for (int i = t; i < n; i += 1024) m = min(m, q[i]);
        for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
        int* ired = (int*)red;
        if ((t & 63) == 0) ired[t >> 6] = m;
        __syncthreads();
        if (t == 0) {
            int r = ired[0];
            for (int w = 1; w < 16; ++w) r = min(r, ired[w]);
            eshift[blockIdx.x] = r == (1 << 20) ? 0 : r;
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

// compile-time settings of this object that differ from the product build (lnerf_build_knobs)
unsigned dw16_build_knobs() {
    return (LNERF_DW16_SPLIT_LATE != 1 ? kKnobDwSplitLate : 0u) | (LNERF_DW16_DEPTH != 3 ? kKnobDwDepth : 0u) |
           (LNERF_DW16_SWZ != 1 ? kKnobDwSwz : 0u) | (LNERF_A24 != 1 ? kKnobA24 : 0u) |
           (LNERF_DW16_XROW != 1 ? kKnobDwXrow : 0u) |
           (LNERF_DW16_WAVES != 8 || !LNERF_DW16_PMAJOR ? kKnobDwWaves : 0u);
}

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
    a.sexp = p.sexp;
    a.xcount = p.xcount;
    a.rpad = p.num_wg * p.tile;
    a.eshift = p.dw_shift;
    a.L = p.L;
    a.gate = p.gate;
    // the guard's re-run leaves the primary step's exceptional-row counts (lnerf_ctx_exceptional_rows)
    if (p.gate) a.xcount = nullptr;
    static_assert(sizeof(Dw16Args) <= 4096, "kernel arguments");
    // the per-layer product shifts of k1_reduce_launch (launched right after k1)
    if (p.x6 == 2) dw16_kernel<2><<<p.dw_grid, kThreads, 0, s>>>(a);
    else if (p.x6 == 3) dw16_kernel<3><<<p.dw_grid, kThreads, 0, s>>>(a);
    else dw16_kernel<1><<<p.dw_grid, kThreads, 0, s>>>(a);
}

void k1_reduce_launch(const FusedPlan& p, float* out_loss, hipStream_t s) {
    // k1's per-wave minima: tile / 16 waves per workgroup
    k1_reduce_kernel<<<p.L + 1, 1024, 0, s>>>(p.epart, p.num_wg * (p.tile / 16), p.dw_shift, p.L, p.loss_part,
                                              p.num_wg, p.loss_total, out_loss, p.gate);
}

}  // namespace lnerf
