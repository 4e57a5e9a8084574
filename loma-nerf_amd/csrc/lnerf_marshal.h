// lnerf_marshal.h -- host-only marshalling of the loma ABI's nested pointer tables (no HIP): the
// shapes and extents of one call and the gather / scatter between the caller's row-allocated
// tables (mlp_utils.py:33-118, convert_ndim_array_to_ndim_ctypes) and flat rectangles.
//
// Used by lnerf_api.cpp (the compat entry points stage through it into pinned memory) and built
// on its own under AddressSanitizer / UBSan by tests/native/marshal_check.cpp: the extents are the
// reference's loop bounds, and every row the reference's loops touch --
// and no other byte -- is read or written.
#pragma once

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "lnerf.h"

namespace lnerf {

constexpr int kMaxLayers = LNERF_MAX_LAYERS;

// One loma call on flat rectangles. Field meaning follows scripts/nerf.py:1-22.
struct LgDims {
    int L;                    // num_weights
    int in_h, in_w;           // layer_input_h / layer_input_w
    int th, tw;               // target_image_h / target_image_w
    int S;                    // num_samples
    int wsh1[kMaxLayers];     // weight_shapes[l][1]
    int ios0[kMaxLayers];     // intermediate_output_shapes[l][0]
    int ios1[kMaxLayers];     // intermediate_output_shapes[l][1]
    int x_cols;               // strides of the flat rectangles
    int w_k, w_n, b_n;
    int io_rows, io_cols;
    int t_cols, acc_cols;
    int nerf_head;            // 1: nerf.py head (sigma ReLU on channel 3); 0: mlp_fit (all sigmoid)
};

namespace marshal {

// A malformed call (null table or row, out-of-range shape): the entry points turn it into
// lnerf_last_error() and a NaN loss / untouched gradients.
struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    throw Error(buf);
}

// ---- nested-pointer gather / scatter (mlp_utils.py:33-118 layouts) ---------------------------
inline void gather2(float* dst, float** src, int rows, int cols, int ld) {
    if (rows > 0 && cols > 0 && !src) fail("null array argument");
    for (int i = 0; i < rows; ++i) {
        if (!src[i]) fail("null row pointer");
        std::memcpy(dst + (size_t)i * ld, src[i], sizeof(float) * cols);
    }
}
inline void scatter2(float** dst, const float* src, int rows, int cols, int ld) {
    for (int i = 0; i < rows; ++i) std::memcpy(dst[i], src + (size_t)i * ld, sizeof(float) * cols);
}
// rgba (th, S, 4)
inline void gather3(float* dst, float*** src, int d0, int d1, int d2) {
    if (d0 > 0 && d1 > 0 && !src) fail("null array argument");
    for (int i = 0; i < d0; ++i)
        for (int j = 0; j < d1; ++j) std::memcpy(dst + ((size_t)i * d1 + j) * d2, src[i][j], sizeof(float) * d2);
}
inline void scatter3(float*** dst, const float* src, int d0, int d1, int d2) {
    for (int i = 0; i < d0; ++i)
        for (int j = 0; j < d1; ++j) std::memcpy(dst[i][j], src + ((size_t)i * d1 + j) * d2, sizeof(float) * d2);
}

// Shapes and extents of one loma call (the reference's loop bounds).
struct CallShape {
    LgDims d{};
    int K[kMaxLayers];        // contraction length of layer l
    int rows[kMaxLayers];     // touched rows of io[l]
    int cols[kMaxLayers];     // touched cols of io[l]
    int bcols[kMaxLayers];    // touched cols of bs[l]
};

inline CallShape make_shape(bool nerf, int in_h, int in_w, int th, int tw, int L, int** weight_shapes,
                     int** ios, int S) {
    CallShape c;
    LgDims& d = c.d;
    if (L < 1 || L > kMaxLayers) fail("num_weights=%d out of range 1..%d", L, kMaxLayers);
    if (in_h < 0 || in_w < 0 || th < 0 || tw < 0 || S < 0) fail("negative dimension");
    if (!weight_shapes || !ios) fail("null shape table");
    d.L = L;
    d.in_h = in_h;
    d.in_w = in_w;
    d.th = th;
    d.tw = tw;
    d.S = nerf ? S : 0;
    d.nerf_head = nerf ? 1 : 0;
    for (int l = 0; l < L; ++l) {
        if (!weight_shapes[l] || !ios[l]) fail("null shape row");
        d.wsh1[l] = weight_shapes[l][1];
        d.ios0[l] = ios[l][0];
        d.ios1[l] = ios[l][1];
        if (d.wsh1[l] < 0 || d.ios0[l] < 0 || d.ios1[l] < 0) fail("negative shape entry");
    }
    int w_k = 1, w_n = 1, b_n = 1, io_r = 1, io_c = 4;
    for (int l = 0; l < L; ++l) {
        c.K[l] = (l == 0) ? in_w : d.ios1[l - 1];
        const int mm_rows = (l == 0) ? in_h : d.ios0[l - 1];
        int r = std::max(mm_rows, d.ios0[l]);
        int cc = std::max(d.wsh1[l], d.ios1[l]);
        if (l == L - 1) {
            if (nerf) {
                r = std::max(r, th * S);
                cc = std::max(cc, 4);
            } else {
                r = std::max(r, th);
                cc = std::max(cc, tw);
            }
        }
        c.rows[l] = r;
        c.cols[l] = cc;
        c.bcols[l] = d.ios1[l];
        w_k = std::max(w_k, c.K[l]);
        w_n = std::max(w_n, d.wsh1[l]);
        b_n = std::max(b_n, d.ios1[l]);
        io_r = std::max(io_r, r);
        io_c = std::max(io_c, cc);
    }
    d.x_cols = std::max(in_w, 1);
    d.w_k = w_k;
    d.w_n = w_n;
    d.b_n = b_n;
    d.io_rows = io_r;
    d.io_cols = io_c;
    d.t_cols = std::max(tw, 1);
    d.acc_cols = std::max(3, tw);
    return c;
}

inline void gather_w(float* dst, float*** ws, const CallShape& c) {
    const LgDims& d = c.d;
    if (!ws) fail("null ws");
    for (int l = 0; l < d.L; ++l) {
        if (c.K[l] > 0 && d.wsh1[l] > 0 && !ws[l]) fail("null ws[%d]", l);
        for (int k = 0; k < c.K[l]; ++k)
            std::memcpy(dst + ((size_t)l * d.w_k + k) * d.w_n, ws[l][k], sizeof(float) * d.wsh1[l]);
    }
}
inline void scatter_w(float*** ws, const float* src, const CallShape& c) {
    const LgDims& d = c.d;
    for (int l = 0; l < d.L; ++l)
        for (int k = 0; k < c.K[l]; ++k)
            std::memcpy(ws[l][k], src + ((size_t)l * d.w_k + k) * d.w_n, sizeof(float) * d.wsh1[l]);
}
inline void gather_b(float* dst, float** bs, const CallShape& c) {
    const LgDims& d = c.d;
    if (!bs) fail("null bs");
    for (int l = 0; l < d.L; ++l)
        if (c.bcols[l] > 0) std::memcpy(dst + (size_t)l * d.b_n, bs[l], sizeof(float) * c.bcols[l]);
}
inline void scatter_b(float** bs, const float* src, const CallShape& c) {
    const LgDims& d = c.d;
    for (int l = 0; l < d.L; ++l)
        if (c.bcols[l] > 0) std::memcpy(bs[l], src + (size_t)l * d.b_n, sizeof(float) * c.bcols[l]);
}
inline void gather_io(float* dst, float*** io, const CallShape& c) {
    const LgDims& d = c.d;
    if (!io) fail("null intermediate_outputs");
    for (int l = 0; l < d.L; ++l)
        for (int i = 0; i < c.rows[l]; ++i)
            std::memcpy(dst + ((size_t)l * d.io_rows + i) * d.io_cols, io[l][i], sizeof(float) * c.cols[l]);
}
inline void scatter_io(float*** io, const float* src, const CallShape& c) {
    const LgDims& d = c.d;
    for (int l = 0; l < d.L; ++l)
        for (int i = 0; i < c.rows[l]; ++i)
            std::memcpy(io[l][i], src + ((size_t)l * d.io_rows + i) * d.io_cols, sizeof(float) * c.cols[l]);
}

}  // namespace marshal
}  // namespace lnerf
