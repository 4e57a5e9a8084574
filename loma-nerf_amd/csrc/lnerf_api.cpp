// lnerf_api.cpp -- the C ABI of libloma_nerf.so (declared in include/lnerf.h).
//
// loma-compat entry points: the reference passes nested host pointer tables built by
// mlp_utils.convert_ndim_array_to_ndim_ctypes (mlp_utils.py:33-118). We read exactly the elements
// the reference's loops touch (extents derived from the same loop bounds), gather them into one
// pinned staging block, run the loma-order HIP kernels (lnerf_generic.hip) on the calling
// thread's stream, and scatter the mutated buffers back. No CPU compute path exists: if the HIP
// runtime or device is unavailable the call fails loudly (NaN / error string).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <sys/syscall.h>
#include <unistd.h>

#include "lnerf_internal.h"

using namespace lnerf;

namespace {

thread_local std::string g_last_error;

using marshal::fail;
using namespace marshal;

#define HIP_OK(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) fail("%s failed: %s", #expr, hipGetErrorString(_e));          \
    } while (0)

void check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) fail("%s: kernel launch failed: %s", what, hipGetErrorString(e));
}

// Grow-only device / pinned buffers.
struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    void* get(size_t bytes) {
        if (bytes > n) {
            if (p) HIP_OK(hipFree(p));
            p = nullptr;
            n = 0;
            HIP_OK(hipMalloc(&p, bytes));
            n = bytes;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HostBuf {
    void* p = nullptr;
    size_t n = 0;
    void* get(size_t bytes) {
        if (bytes > n) {
            if (p) HIP_OK(hipHostFree(p));
            p = nullptr;
            n = 0;
            HIP_OK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
            n = bytes;
        }
        return p;
    }
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// Per-thread engine state for the loma-compat ABI (ctypes drops the GIL, so calls may come from
// several threads at once; each gets its own stream and staging).
struct CompatCtx {
    hipStream_t stream = nullptr;
    DevBuf dev;
    HostBuf host;
    CompatCtx() {
        int n = 0;
        HIP_OK(hipGetDeviceCount(&n));
        if (n < 1) fail("no HIP device visible");
        HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }
    ~CompatCtx() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};
// One CompatCtx per calling thread, freed when that thread exits (its stream and staging go with
// it). The main thread's context is left to process teardown: at exit() its thread_local
// destructor may run after the HIP runtime has begun shutting down, where hipStreamDestroy is
// not safe. The main thread is the one whose kernel thread id is the process id (whichever
// thread happened to load the library).
bool on_main_thread() { return (pid_t)syscall(SYS_gettid) == getpid(); }
struct CompatHolder {
    CompatCtx* ctx = nullptr;
    ~CompatHolder() {
        if (ctx && !on_main_thread()) delete ctx;
    }
};
thread_local CompatHolder tl_compat;
CompatCtx& compat() {
    if (!tl_compat.ctx) tl_compat.ctx = new CompatCtx();
    return *tl_compat.ctx;
}

// Carves one contiguous region into float arrays (same offsets on host and device).
struct Carve {
    size_t off = 0;
    size_t take(size_t nfloats) {
        size_t o = off;
        off += (nfloats + 63) / 64 * 64;
        return o;
    }
};

struct Offsets {
    size_t X, W, B, T, IO, rgba, dists, alpha, cp, wsamp, acc, loss, seed;
    size_t zpre, cpC, cpP;
    size_t dX, dW, dB, dT, dIO, drgba, ddists, dalpha, dcp, dwsamp, dacc;
    size_t total;
};

Offsets carve(const CallShape& c, bool grad) {
    const LgDims& d = c.d;
    Carve k;
    Offsets o{};
    const size_t nS = (size_t)d.th * d.S;
    o.X = k.take((size_t)d.in_h * d.x_cols);
    o.W = k.take((size_t)d.L * d.w_k * d.w_n);
    o.B = k.take((size_t)d.L * d.b_n);
    o.T = k.take((size_t)d.th * d.t_cols);
    o.IO = k.take((size_t)d.L * d.io_rows * d.io_cols);
    o.rgba = k.take(nS * 4);
    o.dists = k.take(nS);
    o.alpha = k.take(nS);
    o.cp = k.take(nS);
    o.wsamp = k.take(nS);
    o.acc = k.take((size_t)d.th * d.acc_cols);
    o.loss = k.take(1);
    o.seed = k.take(1);
    if (grad) {
        o.zpre = k.take((size_t)d.L * d.io_rows * d.io_cols);
        o.cpC = k.take(nS);
        o.cpP = k.take(nS);
        o.dX = k.take((size_t)d.in_h * d.x_cols);
        o.dW = k.take((size_t)d.L * d.w_k * d.w_n);
        o.dB = k.take((size_t)d.L * d.b_n);
        o.dT = k.take((size_t)d.th * d.t_cols);
        o.dIO = k.take((size_t)d.L * d.io_rows * d.io_cols);
        o.drgba = k.take(nS * 4);
        o.ddists = k.take(nS);
        o.dalpha = k.take(nS);
        o.dcp = k.take(nS);
        o.dwsamp = k.take(nS);
        o.dacc = k.take((size_t)d.th * d.acc_cols);
    }
    o.total = k.off;
    return o;
}

LgBuffers dev_buffers(float* base, const Offsets& o, bool grad) {
    LgBuffers b{};
    b.X = base + o.X;
    b.W = base + o.W;
    b.B = base + o.B;
    b.T = base + o.T;
    b.IO = base + o.IO;
    b.rgba = base + o.rgba;
    b.dists = base + o.dists;
    b.alpha = base + o.alpha;
    b.cp = base + o.cp;
    b.wsamp = base + o.wsamp;
    b.acc = base + o.acc;
    if (grad) {
        b.zpre = base + o.zpre;
        b.cpC = base + o.cpC;
        b.cpP = base + o.cpP;
    }
    return b;
}
LgAdjoints dev_adjoints(float* base, const Offsets& o, bool want_dx) {
    LgAdjoints a{};
    a.dX = want_dx ? base + o.dX : nullptr;
    a.dW = base + o.dW;
    a.dB = base + o.dB;
    a.dT = base + o.dT;
    a.dIO = base + o.dIO;
    a.drgba = base + o.drgba;
    a.ddists = base + o.ddists;
    a.dalpha = base + o.dalpha;
    a.dcp = base + o.dcp;
    a.dwsamp = base + o.dwsamp;
    a.dacc = base + o.dacc;
    return a;
}

template <class F>
float guard_float(F&& f) {
    try {
        g_last_error.clear();
        return f();
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return std::numeric_limits<float>::quiet_NaN();
    }
}
template <class F>
int guard_int(F&& f) {
    try {
        g_last_error.clear();
        f();
        return 0;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -1;
    }
}

}  // namespace

// =============================================================================================
// loma-compat ABI
// =============================================================================================
extern "C" float nerf_evaluate_and_march(float** layer_input, int layer_input_h, int layer_input_w,
                                         float*** ws, float** bs, float** target_image,
                                         int target_image_h, int target_image_w, int num_weights,
                                         int** weight_shapes, int** bias_shapes,
                                         int** intermediate_output_shapes,
                                         float*** intermediate_outputs,
                                         float*** img_sample_rgba_arr, int num_samples,
                                         float** dists, float** alpha, float** cumprod_alpha,
                                         float** weights_samples, float** accumulated_color) {
    (void)bias_shapes;  // never read by nerf.py
    return guard_float([&]() -> float {
        CallShape c = make_shape(true, layer_input_h, layer_input_w, target_image_h, target_image_w,
                                 num_weights, weight_shapes, intermediate_output_shapes, num_samples);
        const LgDims& d = c.d;
        Offsets o = carve(c, false);
        CompatCtx& cx = compat();
        float* h = (float*)cx.host.get(o.total * sizeof(float));
        float* g = (float*)cx.dev.get(o.total * sizeof(float));
        std::memset(h, 0, o.total * sizeof(float));
        gather2(h + o.X, layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.W, ws, c);
        gather_b(h + o.B, bs, c);
        gather2(h + o.T, target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.IO, intermediate_outputs, c);
        gather2(h + o.dists, dists, d.th, d.S, d.S);
        gather2(h + o.acc, accumulated_color, d.th, d.acc_cols, d.acc_cols);
        HIP_OK(hipMemcpyAsync(g, h, o.total * sizeof(float), hipMemcpyHostToDevice, cx.stream));
        LgBuffers b = dev_buffers(g, o, false);
        lg_nerf_forward(d, b, g + o.loss, cx.stream);
        check_launch("nerf_evaluate_and_march");
        // everything from IO to the loss is contiguous in the carve
        HIP_OK(hipMemcpyAsync(h + o.IO, g + o.IO, (o.seed - o.IO) * sizeof(float),
                              hipMemcpyDeviceToHost, cx.stream));
        HIP_OK(hipStreamSynchronize(cx.stream));
        scatter_io(intermediate_outputs, h + o.IO, c);
        if (d.th > 0 && d.S > 0) {
            scatter3(img_sample_rgba_arr, h + o.rgba, d.th, d.S, 4);
            scatter2(alpha, h + o.alpha, d.th, d.S, d.S);
            scatter2(cumprod_alpha, h + o.cp, d.th, d.S, d.S);
            scatter2(weights_samples, h + o.wsamp, d.th, d.S, d.S);
        }
        scatter2(accumulated_color, h + o.acc, d.th, 3, d.acc_cols);
        return h[o.loss];
    });
}

extern "C" void grad_nerf_evaluate_and_march(
    float** layer_input, float** d_layer_input, int layer_input_h, int* d_layer_input_h,
    int layer_input_w, int* d_layer_input_w, float*** ws, float*** d_ws, float** bs, float** d_bs,
    float** target_image, float** d_target_image, int target_image_h, int* d_target_image_h,
    int target_image_w, int* d_target_image_w, int num_weights, int* d_num_weights,
    int** weight_shapes, int** d_weight_shapes, int** bias_shapes, int** d_bias_shapes,
    int** intermediate_output_shapes, int** d_intermediate_output_shapes,
    float*** intermediate_outputs, float*** d_intermediate_outputs, float*** img_sample_rgba_arr,
    float*** d_img_sample_rgba_arr, int num_samples, int* d_num_samples, float** dists,
    float** d_dists, float** alpha, float** d_alpha, float** cumprod_alpha,
    float** d_cumprod_alpha, float** weights_samples, float** d_weights_samples,
    float** accumulated_color, float** d_accumulated_color, float _dreturn) {
    // int adjoints are never written by loma (reverse_diff.py:146-147)
    (void)d_layer_input_h; (void)d_layer_input_w; (void)d_target_image_h; (void)d_target_image_w;
    (void)d_num_weights; (void)d_weight_shapes; (void)d_bias_shapes;
    (void)d_intermediate_output_shapes; (void)d_num_samples; (void)bias_shapes;
    (void)img_sample_rgba_arr; (void)alpha; (void)cumprod_alpha; (void)weights_samples;
    guard_int([&]() {
        CallShape c = make_shape(true, layer_input_h, layer_input_w, target_image_h, target_image_w,
                                 num_weights, weight_shapes, intermediate_output_shapes, num_samples);
        const LgDims& d = c.d;
        Offsets o = carve(c, true);
        CompatCtx& cx = compat();
        float* h = (float*)cx.host.get(o.total * sizeof(float));
        float* g = (float*)cx.dev.get(o.total * sizeof(float));
        std::memset(h, 0, o.total * sizeof(float));
        const bool S_ok = d.th > 0 && d.S > 0;
        // primal inputs the re-executed forward reads (the rest is overwritten before use)
        gather2(h + o.X, layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.W, ws, c);
        gather_b(h + o.B, bs, c);
        gather2(h + o.T, target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.IO, intermediate_outputs, c);
        if (S_ok) gather2(h + o.dists, dists, d.th, d.S, d.S);
        gather2(h + o.acc, accumulated_color, d.th, d.acc_cols, d.acc_cols);
        h[o.seed] = _dreturn;
        // adjoints (accumulated into)
        const bool want_dx = d_layer_input != nullptr;
        if (want_dx) gather2(h + o.dX, d_layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.dW, d_ws, c);
        gather_b(h + o.dB, d_bs, c);
        gather2(h + o.dT, d_target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.dIO, d_intermediate_outputs, c);
        if (S_ok) {
            gather3(h + o.drgba, d_img_sample_rgba_arr, d.th, d.S, 4);
            gather2(h + o.ddists, d_dists, d.th, d.S, d.S);
            gather2(h + o.dalpha, d_alpha, d.th, d.S, d.S);
            gather2(h + o.dcp, d_cumprod_alpha, d.th, d.S, d.S);
            gather2(h + o.dwsamp, d_weights_samples, d.th, d.S, d.S);
        }
        gather2(h + o.dacc, d_accumulated_color, d.th, d.acc_cols, d.acc_cols);
        HIP_OK(hipMemcpyAsync(g, h, o.total * sizeof(float), hipMemcpyHostToDevice, cx.stream));
        lg_nerf_grad(d, dev_buffers(g, o, true), dev_adjoints(g, o, want_dx), g + o.seed, cx.stream);
        check_launch("grad_nerf_evaluate_and_march");
        HIP_OK(hipMemcpyAsync(h + o.dX, g + o.dX, (o.total - o.dX) * sizeof(float),
                              hipMemcpyDeviceToHost, cx.stream));
        HIP_OK(hipStreamSynchronize(cx.stream));
        if (want_dx) scatter2(d_layer_input, h + o.dX, d.in_h, d.in_w, d.x_cols);
        scatter_w(d_ws, h + o.dW, c);
        scatter_b(d_bs, h + o.dB, c);
        scatter2(d_target_image, h + o.dT, d.th, d.tw, d.t_cols);
        scatter_io(d_intermediate_outputs, h + o.dIO, c);
        if (S_ok) {
            scatter3(d_img_sample_rgba_arr, h + o.drgba, d.th, d.S, 4);
            scatter2(d_dists, h + o.ddists, d.th, d.S, d.S);
            scatter2(d_alpha, h + o.dalpha, d.th, d.S, d.S);
            scatter2(d_cumprod_alpha, h + o.dcp, d.th, d.S, d.S);
            scatter2(d_weights_samples, h + o.dwsamp, d.th, d.S, d.S);
        }
        scatter2(d_accumulated_color, h + o.dacc, d.th, d.acc_cols, d.acc_cols);
    });
}

extern "C" float mlp_fit(float** layer_input, int layer_input_h, int layer_input_w,
                         float** layer_output, float*** ws, float** bs, float** target_image,
                         int target_image_h, int target_image_w, int num_weights,
                         int** weight_shapes, int** bias_shapes, int** intermediate_output_shapes,
                         float*** intermediate_outputs) {
    (void)layer_output;  // unused by mlp_fit.py
    (void)bias_shapes;
    return guard_float([&]() -> float {
        CallShape c = make_shape(false, layer_input_h, layer_input_w, target_image_h, target_image_w,
                                 num_weights, weight_shapes, intermediate_output_shapes, 0);
        const LgDims& d = c.d;
        Offsets o = carve(c, false);
        CompatCtx& cx = compat();
        float* h = (float*)cx.host.get(o.total * sizeof(float));
        float* g = (float*)cx.dev.get(o.total * sizeof(float));
        std::memset(h, 0, o.total * sizeof(float));
        gather2(h + o.X, layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.W, ws, c);
        gather_b(h + o.B, bs, c);
        gather2(h + o.T, target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.IO, intermediate_outputs, c);
        HIP_OK(hipMemcpyAsync(g, h, o.total * sizeof(float), hipMemcpyHostToDevice, cx.stream));
        lg_mlp_fit_forward(d, dev_buffers(g, o, false), g + o.loss, cx.stream);
        check_launch("mlp_fit");
        HIP_OK(hipMemcpyAsync(h + o.IO, g + o.IO, (o.seed - o.IO) * sizeof(float),
                              hipMemcpyDeviceToHost, cx.stream));
        HIP_OK(hipStreamSynchronize(cx.stream));
        scatter_io(intermediate_outputs, h + o.IO, c);
        return h[o.loss];
    });
}

extern "C" void grad_mlp_fit(float** layer_input, float** d_layer_input, int layer_input_h,
                             int* d_layer_input_h, int layer_input_w, int* d_layer_input_w,
                             float** layer_output, float** d_layer_output, float*** ws,
                             float*** d_ws, float** bs, float** d_bs, float** target_image,
                             float** d_target_image, int target_image_h, int* d_target_image_h,
                             int target_image_w, int* d_target_image_w, int num_weights,
                             int* d_num_weights, int** weight_shapes, int** d_weight_shapes,
                             int** bias_shapes, int** d_bias_shapes,
                             int** intermediate_output_shapes,
                             int** d_intermediate_output_shapes, float*** intermediate_outputs,
                             float*** d_intermediate_outputs, float _dreturn) {
    (void)d_layer_input_h; (void)d_layer_input_w; (void)layer_output; (void)d_layer_output;
    (void)d_target_image_h; (void)d_target_image_w; (void)d_num_weights; (void)d_weight_shapes;
    (void)bias_shapes; (void)d_bias_shapes; (void)d_intermediate_output_shapes;
    guard_int([&]() {
        CallShape c = make_shape(false, layer_input_h, layer_input_w, target_image_h, target_image_w,
                                 num_weights, weight_shapes, intermediate_output_shapes, 0);
        const LgDims& d = c.d;
        Offsets o = carve(c, true);
        CompatCtx& cx = compat();
        float* h = (float*)cx.host.get(o.total * sizeof(float));
        float* g = (float*)cx.dev.get(o.total * sizeof(float));
        std::memset(h, 0, o.total * sizeof(float));
        gather2(h + o.X, layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.W, ws, c);
        gather_b(h + o.B, bs, c);
        gather2(h + o.T, target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.IO, intermediate_outputs, c);
        h[o.seed] = _dreturn;
        const bool want_dx = d_layer_input != nullptr;
        if (want_dx) gather2(h + o.dX, d_layer_input, d.in_h, d.in_w, d.x_cols);
        gather_w(h + o.dW, d_ws, c);
        gather_b(h + o.dB, d_bs, c);
        gather2(h + o.dT, d_target_image, d.th, d.tw, d.t_cols);
        gather_io(h + o.dIO, d_intermediate_outputs, c);
        HIP_OK(hipMemcpyAsync(g, h, o.total * sizeof(float), hipMemcpyHostToDevice, cx.stream));
        lg_mlp_fit_grad(d, dev_buffers(g, o, true), dev_adjoints(g, o, want_dx), g + o.seed, cx.stream);
        check_launch("grad_mlp_fit");
        HIP_OK(hipMemcpyAsync(h + o.dX, g + o.dX, (o.total - o.dX) * sizeof(float),
                              hipMemcpyDeviceToHost, cx.stream));
        HIP_OK(hipStreamSynchronize(cx.stream));
        if (want_dx) scatter2(d_layer_input, h + o.dX, d.in_h, d.in_w, d.x_cols);
        scatter_w(d_ws, h + o.dW, c);
        scatter_b(d_bs, h + o.dB, c);
        scatter2(d_target_image, h + o.dT, d.th, d.tw, d.t_cols);
        scatter_io(d_intermediate_outputs, h + o.dIO, c);
    });
}

extern "C" void mult_a_b(float** a, int a_h, int a_w, float** b, int b_h, int b_w, float** c) {
    (void)b_h;
    guard_int([&]() {
        if (a_h < 0 || a_w < 0 || b_w < 0) fail("negative dimension");
        CompatCtx& cx = compat();
        Carve k;
        const size_t oa = k.take((size_t)a_h * a_w), ob = k.take((size_t)a_w * b_w),
                     oc = k.take((size_t)a_h * b_w);
        float* h = (float*)cx.host.get(k.off * sizeof(float));
        float* g = (float*)cx.dev.get(k.off * sizeof(float));
        gather2(h + oa, a, a_h, a_w, a_w);
        gather2(h + ob, b, a_w, b_w, b_w);  // mult_a_b reads b[k][j] for k < a_w
        gather2(h + oc, c, a_h, b_w, b_w);
        HIP_OK(hipMemcpyAsync(g, h, k.off * sizeof(float), hipMemcpyHostToDevice, cx.stream));
        lg_mult_a_b(g + oa, a_h, a_w, g + ob, b_w, g + oc, cx.stream);
        check_launch("mult_a_b");
        HIP_OK(hipMemcpyAsync(h + oc, g + oc, (size_t)a_h * b_w * sizeof(float),
                              hipMemcpyDeviceToHost, cx.stream));
        HIP_OK(hipStreamSynchronize(cx.stream));
        scatter2(c, h + oc, a_h, b_w, b_w);
    });
}

// =============================================================================================
// native batched API
// =============================================================================================
struct lnerf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf fused_ws;
    DevBuf generic_ws;
    std::mutex mu;
    hipEvent_t ev[7] = {};
    bool timed = false;
    int last_path = 0;   // lnerf_ctx_last_path
    int dw_grid = 0;     // LNERF_OPT_DW_GRID (0: default_dw_grid)
    FusedPlan last_plan{};   // the last fused training step's plan (lnerf_ctx_relu_masks)
    bool last_k16_train = false;
};

static int path_bits(const FusedPlan& p, bool train) {
    return LNERF_PATH_FUSED | LNERF_PATH_K16 | (p.tile == 64 ? LNERF_PATH_K16_W4 : 0) |
           (train ? LNERF_PATH_DW16 : 0) | (train && a24_slabs(p.x6) ? LNERF_PATH_A24 : 0) | (p.x6 << 8);
}

// Flags that ask for a fused-path kernel or precision: an explicit request that cannot be served
// is an error, never a silent substitute.
constexpr int kFusedRequests = LNERF_MFMA_BF16 | LNERF_MFMA_F16X3 | LNERF_MFMA_BF16X6 | LNERF_K16_W4 |
                               LNERF_RENDER_K16;

// At most one MFMA precision flag; the round-1..3 kernel selectors are gone (lnerf.h).
static void check_precision_flags(int flags) {
    if (flags & (LNERF_MFMA_F32 | LNERF_ONE_WAVE | LNERF_K32))
        fail("flags 0x%x select a removed kernel (LNERF_MFMA_F32 / LNERF_ONE_WAVE / LNERF_K32): the fused "
             "path is k16 + dw16; exact fp32 arithmetic is LNERF_GENERIC",
             flags & (LNERF_MFMA_F32 | LNERF_ONE_WAVE | LNERF_K32));
    const int prec = flags & (LNERF_MFMA_BF16 | LNERF_MFMA_F16X3 | LNERF_MFMA_BF16X6);
    if (prec & (prec - 1)) fail("conflicting MFMA precision flags 0x%x (set at most one)", prec);
    if ((flags & LNERF_GENERIC) && (flags & kFusedRequests))
        fail("LNERF_GENERIC conflicts with the fused-path flags 0x%x", flags & kFusedRequests);
}

extern "C" const char* lnerf_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* lnerf_version(void) { return "loma-nerf-amd 0.5 (gfx950)"; }

extern "C" unsigned lnerf_build_knobs(void) {
    return lnerf::k16_build_knobs() | lnerf::dw16_build_knobs() | lnerf::kr_build_knobs();
}

extern "C" int lnerf_ctx_create(lnerf_ctx** out, int device) {
    return guard_int([&]() {
        if (!out) fail("null out");
        int n = 0;
        HIP_OK(hipGetDeviceCount(&n));
        if (device < 0 || device >= n) fail("device %d not visible (%d devices)", device, n);
        HIP_OK(hipSetDevice(device));
        lnerf_ctx* c = new lnerf_ctx();
        c->device = device;
        HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        for (auto& e : c->ev) HIP_OK(hipEventCreate(&e));
        *out = c;
    });
}

extern "C" void lnerf_ctx_destroy(lnerf_ctx* ctx) {
    if (!ctx) return;
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    for (auto& e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    delete ctx;
}

static void validate(const lnerf_mlp* m, const lnerf_batch* b) {
    if (!m || !b) fail("null mlp/batch");
    if (m->num_layers < 1 || m->num_layers > kMaxLayers) fail("num_layers out of range");
    for (int l = 0; l < m->num_layers; ++l) {
        if (m->k[l] < 1 || m->n[l] < 1) fail("layer %d has an empty shape", l);
        if (m->k[l] > m->w_k || m->n[l] > m->w_n) fail("layer %d exceeds padded layout", l);
        if (l > 0 && m->k[l] != m->n[l - 1]) fail("k[%d] != n[%d]", l, l - 1);
    }
    if (b->rays < 1 || b->samples < 1) fail("empty batch");
    if (!b->x || !b->target) fail("null batch pointer");
    if (b->input_mode == LNERF_INPUT_POINTS || b->input_mode == LNERF_INPUT_RAYS) {
        if (b->num_freqs < 0 || m->k[0] != 3 + 6 * b->num_freqs)
            fail("POINTS/RAYS mode needs k[0] == 3 + 6F");
    } else if (b->input_mode != LNERF_INPUT_ENCODED) {
        fail("unknown input_mode");
    }
}

// NeRF head (rgb + sigma) needs dists (unless RAYS) and >= 4 outputs; the mlp_fit head
// (LNERF_HEAD_FIT) runs only on the fused k16 path, one row per "ray", without dists.
static void validate_head(const lnerf_mlp* m, const lnerf_batch* b, int flags) {
    if (!(flags & LNERF_HEAD_FIT)) {
        if (m->n[m->num_layers - 1] < 4) fail("head needs >= 4 outputs");
        if (b->input_mode != LNERF_INPUT_RAYS && !b->dists) fail("null dists");
        return;
    }
    if (flags & (LNERF_GENERIC | LNERF_MFMA_BF16X6))
        fail("LNERF_HEAD_FIT runs on the k16 kernel in fp16x3 or bf16 only");
    if (b->samples != 1 || b->input_mode != LNERF_INPUT_ENCODED || m->n[m->num_layers - 1] > 4)
        fail("LNERF_HEAD_FIT needs samples == 1, ENCODED input and 1..4 outputs");
}

extern "C" size_t lnerf_workspace_bytes(const lnerf_mlp* mlp, int rays, int samples) {
    if (!mlp) return 0;
    return fused_workspace_bytes(*mlp, rays, samples);
}

// Standard-semantics generic call: io rows = R, zero-initialised buffers (train_nerf.py builds
// fresh zero arrays for every call, :313-317, :370-392).
static void generic_step(lnerf_ctx* ctx, const lnerf_mlp& m, const float* ws, const float* bs,
                         const lnerf_batch& bt, float seed, int flags, const lnerf_outputs& out,
                         bool want_grad, hipStream_t s) {
    const int L = m.num_layers, R = bt.rays * bt.samples, S = bt.samples, th = bt.rays;
    if (want_grad && (flags & LNERF_ACCUMULATE))
        fail("LNERF_ACCUMULATE is only supported on the fused path");
    LgDims d{};
    d.L = L;
    d.in_h = R;
    d.in_w = m.k[0];
    d.th = th;
    d.tw = 3;
    d.S = S;
    d.nerf_head = 1;
    int maxn = 4;
    for (int l = 0; l < L; ++l) {
        d.wsh1[l] = m.n[l];
        d.ios0[l] = R;
        d.ios1[l] = m.n[l];
        maxn = std::max(maxn, m.n[l]);
    }
    d.x_cols = m.k[0];
    d.w_k = m.w_k;
    d.w_n = m.w_n;
    d.b_n = m.w_n;
    d.io_rows = R;
    d.io_cols = maxn;
    d.t_cols = 3;
    d.acc_cols = 3;
    Carve k;
    const size_t nio = (size_t)L * R * maxn, nS = (size_t)R;
    const size_t oX = k.take((size_t)R * m.k[0]), oIO = k.take(nio), oZ = k.take(nio),
                 odIO = k.take(nio), org = k.take(nS * 4), oal = k.take(nS), ocp = k.take(nS),
                 ows = k.take(nS), ocC = k.take(nS), ocP = k.take(nS), oacc = k.take((size_t)th * 3),
                 odrg = k.take(nS * 4), odal = k.take(nS), odcp = k.take(nS), odws = k.take(nS),
                 odd = k.take(nS), odacc = k.take((size_t)th * 3), odT = k.take((size_t)th * 3),
                 odW = k.take((size_t)L * m.w_k * m.w_n), odB = k.take((size_t)L * m.w_n),
                 oloss = k.take(1), oseed = k.take(1), odX = k.take((size_t)R * m.k[0]),
                 odist = k.take(nS);
    float* g = (float*)ctx->generic_ws.get(k.off * sizeof(float));
    const float* X = bt.x;
    const float* dists = bt.dists;
    if (bt.input_mode == LNERF_INPUT_POINTS) {
        k_positional_encoding(bt.x, R, bt.num_freqs, g + oX, m.k[0], s);
        X = g + oX;
    } else if (bt.input_mode == LNERF_INPUT_RAYS) {
        k_positional_encoding_rays(bt.x, bt.rays, S, bt.near_t, bt.far_t, bt.num_freqs, g + oX,
                                   m.k[0], s);
        k_ray_dists(bt.rays, S, bt.near_t, bt.far_t, g + odist, s);
        X = g + oX;
        dists = g + odist;
    }
    // forward call (nerf_evaluate_and_march)
    HIP_OK(hipMemsetAsync(g + oIO, 0, nio * sizeof(float), s));
    HIP_OK(hipMemsetAsync(g + oacc, 0, (size_t)th * 3 * sizeof(float), s));
    LgBuffers b{};
    b.X = X;
    b.W = ws;
    b.B = bs;
    b.T = bt.target;
    b.IO = g + oIO;
    b.rgba = g + org;
    b.dists = dists;
    b.alpha = g + oal;
    b.cp = g + ocp;
    b.wsamp = g + ows;
    b.acc = g + oacc;
    lg_nerf_forward(d, b, g + oloss, s);
    if (out.loss) HIP_OK(hipMemcpyAsync(out.loss, g + oloss, 4, hipMemcpyDeviceToDevice, s));
    if (out.acc_color)
        HIP_OK(hipMemcpyAsync(out.acc_color, g + oacc, (size_t)th * 3 * 4, hipMemcpyDeviceToDevice, s));
    if (!want_grad) return;
    // grad call on fresh zero buffers, seeded with the loss or the constant
    HIP_OK(hipMemsetAsync(g + oIO, 0, (oloss - oIO) * sizeof(float), s));  // primal + adjoints
    HIP_OK(hipMemsetAsync(g + odX, 0, (size_t)R * m.k[0] * sizeof(float), s));
    const float* seed_dev = g + oloss;
    if (!(flags & LNERF_SEED_LOSS)) {
        k_fill(g + oseed, seed, 1, s);
        seed_dev = g + oseed;
    }
    b.zpre = g + oZ;
    b.cpC = g + ocC;
    b.cpP = g + ocP;
    LgAdjoints a{};
    a.dX = out.d_x ? g + odX : nullptr;
    a.dW = g + odW;
    a.dB = g + odB;
    a.dT = g + odT;
    a.dIO = g + odIO;
    a.drgba = g + odrg;
    a.ddists = g + odd;
    a.dalpha = g + odal;
    a.dcp = g + odcp;
    a.dwsamp = g + odws;
    a.dacc = g + odacc;
    lg_nerf_grad(d, b, a, seed_dev, s);
    const size_t nW = (size_t)L * m.w_k * m.w_n, nB = (size_t)L * m.w_n;
    auto emit = [&](float* dst, const float* src, size_t n) {
        if (dst) HIP_OK(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, s));
    };
    emit(out.d_ws, g + odW, nW);
    emit(out.d_bs, g + odB, nB);
    emit(out.d_dists, g + odd, nS);
    emit(out.d_target, g + odT, (size_t)th * 3);
    emit(out.d_x, g + odX, (size_t)R * m.k[0]);
}

static bool use_fused(const lnerf_mlp& m, const lnerf_batch& b, int flags) {
    if (flags & LNERF_GENERIC) return false;
    const char* why = nullptr;
    const bool fit = (flags & LNERF_HEAD_FIT) != 0;
    const bool ok = fused_supported(m, b.rays, b.samples, b.input_mode, &why, fit);
    if (fit && !ok) fail("mlp_fit head: %s", why);
    if (!ok && (flags & LNERF_FAST)) fail("fused path unavailable: %s", why);
    if (!ok && (flags & kFusedRequests))
        fail("flags 0x%x ask for the fused path, which is unavailable: %s", flags & kFusedRequests, why);
    if (ok && (flags & LNERF_WANT_DX) && b.input_mode != LNERF_INPUT_ENCODED)
        fail("LNERF_WANT_DX needs ENCODED input");
    return ok;
}

extern "C" int lnerf_train_step(lnerf_ctx* ctx, const lnerf_mlp* mlp, const float* ws,
                                const float* bs, const lnerf_batch* batch, float seed, int flags,
                                const lnerf_outputs* out, void* stream) {
    return guard_int([&]() {
        if (!ctx) fail("null ctx");
        validate(mlp, batch);
        validate_head(mlp, batch, flags);
        if (!ws || !bs) fail("null weights");
        lnerf_outputs o = out ? *out : lnerf_outputs{};
        if (!(flags & LNERF_WANT_DX)) o.d_x = nullptr;
        if (flags & LNERF_HEAD_FIT) o.d_dists = nullptr;
        check_precision_flags(flags);
        std::lock_guard<std::mutex> lock(ctx->mu);
        // any failure below leaves the masks unreadable: the workspace (mask_g) may be reallocated
        // before the step fails
        ctx->last_k16_train = false;
        HIP_OK(hipSetDevice(ctx->device));
        hipStream_t s = (hipStream_t)stream;   // NULL: the device's default (null) stream
        if (use_fused(*mlp, *batch, flags)) {
            const size_t bytes = fused_workspace_bytes(*mlp, batch->rays, batch->samples, true, ctx->dw_grid);
            FusedPlan p{};
            void* wsb = ctx->fused_ws.get(bytes);
            fused_plan(p, *mlp, *batch, wsb, flags, true, ctx->dw_grid);
            // the fp16x3 floor guard (lnerf_internal.h kGuardExp) under the default precision: the
            // bf16x6 plan of the same step, run on the device only if k1 finds a hidden G element
            // below fp16x3's floor (an explicit LNERF_MFMA_F16X3 asks for fp16x3 exactly; the mlp_fit
            // head and the 64-sample workgroups have no bf16x6 k1)
            const bool guarded = LNERF_GUARD && p.x6 == 2 && !(flags & (LNERF_MFMA_F16X3 | LNERF_K16_W4 | LNERF_HEAD_FIT));
            FusedPlan px{};
            if (guarded) {
                fused_plan(px, *mlp, *batch, wsb, flags | LNERF_MFMA_BF16X6, true, ctx->dw_grid);
                px.guard = nullptr;
                px.gate = p.guard;
                px.w16 = p.w16x;   // packed by p's own pack launch, beside its fp16x3 planes
                px.w16x = nullptr;
            } else {
                p.guard = nullptr;
                p.w16x = nullptr;
            }
            const bool timed = (flags & LNERF_TIMING) != 0;
            fused_train_step(p, ws, bs, *batch, seed, flags, o, s, timed ? ctx->ev : nullptr, guarded ? &px : nullptr);
            check_launch("lnerf_train_step");
            ctx->timed = timed;
            ctx->last_path = path_bits(p, true);
            ctx->last_plan = p;
            ctx->last_k16_train = true;
        } else {
            generic_step(ctx, *mlp, ws, bs, *batch, seed, flags, o, true, s);
            ctx->timed = false;
            ctx->last_path = LNERF_PATH_GENERIC;
        }
        check_launch("lnerf_train_step");
    });
}

extern "C" int lnerf_get_rays(int width, const double* K, const double* c2w, float* rays,
                              void* stream) {
    return guard_int([&]() {
        if (width < 1 || !K || !c2w || !rays) fail("lnerf_get_rays: bad arguments");
        k_get_rays(width, K, c2w, rays, (hipStream_t)stream);
        check_launch("lnerf_get_rays");
    });
}

extern "C" int lnerf_render(lnerf_ctx* ctx, const lnerf_mlp* mlp, const float* ws, const float* bs,
                            const lnerf_batch* batch, int flags, const lnerf_outputs* out,
                            void* stream) {
    return guard_int([&]() {
        if (!ctx) fail("null ctx");
        validate(mlp, batch);
        validate_head(mlp, batch, flags);
        lnerf_outputs o = out ? *out : lnerf_outputs{};
        check_precision_flags(flags);
        std::lock_guard<std::mutex> lock(ctx->mu);
        ctx->last_k16_train = false;   // a render reuses the workspace the masks live in
        HIP_OK(hipSetDevice(ctx->device));
        hipStream_t s = (hipStream_t)stream;   // NULL: the device's default (null) stream
        if (use_fused(*mlp, *batch, flags & ~LNERF_WANT_DX)) {
            const size_t bytes = fused_workspace_bytes(*mlp, batch->rays, batch->samples, false, ctx->dw_grid);
            FusedPlan p{};
            fused_plan(p, *mlp, *batch, ctx->fused_ws.get(bytes), flags, false, ctx->dw_grid);
            p.guard = nullptr;   // (the floor guard is a training-step feature)
            p.w16x = nullptr;
            const bool timed = (flags & LNERF_TIMING) != 0;
            fused_render(p, ws, bs, *batch, o, s, flags, timed ? ctx->ev : nullptr);
            ctx->timed = timed;
            ctx->last_path = path_bits(p, false) | (fused_render_uses_kr(p, flags) ? LNERF_PATH_KR : 0);
        } else {
            ctx->timed = false;
            generic_step(ctx, *mlp, ws, bs, *batch, 1.0f, 0, o, false, s);
            ctx->last_path = LNERF_PATH_GENERIC;
        }
        check_launch("lnerf_render");
    });
}

extern "C" int lnerf_ctx_timings(lnerf_ctx* ctx, float* ms_out, int n) {
    int written = 0;
    const int rc = guard_int([&]() {
        if (!ctx || !ms_out) fail("null argument");
        if (!ctx->timed) return;
        HIP_OK(hipEventSynchronize(ctx->ev[5]));
        float v[6];
        for (int i = 0; i < 5; ++i) HIP_OK(hipEventElapsedTime(&v[i], ctx->ev[i], ctx->ev[i + 1]));
        HIP_OK(hipEventElapsedTime(&v[5], ctx->ev[0], ctx->ev[5]));
        for (int i = 0; i < 6 && i < n; ++i) ms_out[written++] = v[i];
    });
    return rc != 0 ? rc : written;
}

extern "C" int lnerf_ctx_last_path(lnerf_ctx* ctx) {
    int path = 0;
    const int rc = guard_int([&]() {
        if (!ctx) fail("null ctx");
        std::lock_guard<std::mutex> lock(ctx->mu);
        path = ctx->last_path;
    });
    return rc != 0 ? rc : path;
}

extern "C" int lnerf_ctx_relu_masks(lnerf_ctx* ctx, unsigned char* out, size_t out_bytes, void* stream) {
    return guard_int([&]() {
        if (!ctx || !out) fail("null argument");
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!ctx->last_k16_train) fail("no k16 training step has run on this context since the last other call");
        const FusedPlan& p = ctx->last_plan;
        const size_t need = (size_t)(p.L - 1) * p.R * 32;
        if (out_bytes < need) fail("relu mask buffer holds %zu bytes, needs %zu", out_bytes, need);
        HIP_OK(hipSetDevice(ctx->device));
        k16_masks_launch(p, out, (hipStream_t)stream);
        check_launch("lnerf_ctx_relu_masks");
    });
}

extern "C" int lnerf_ctx_exceptional_rows(lnerf_ctx* ctx, long long* rows, long long* last_samples) {
    return guard_int([&]() {
        if (!ctx || !rows) fail("null argument");
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!ctx->last_k16_train) fail("no k16 training step has run on this context since the last other call");
        const FusedPlan& p = ctx->last_plan;
        *rows = 0;
        if (last_samples) *last_samples = 0;
        if (p.x6 != 2) return;   // only the fp16x3 split has exceptional rows
        HIP_OK(hipSetDevice(ctx->device));
        std::vector<int> c((size_t)2 * p.dw_grid);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(c.data(), p.xcount, c.size() * sizeof(int), hipMemcpyDeviceToHost));
        long long t = 0, l = 0;
        for (int i = 0; i < p.dw_grid; ++i) {
            t += c[2 * i];
            l += c[2 * i + 1];
        }
        *rows = t;
        if (last_samples) *last_samples = l;
    });
}

extern "C" int lnerf_ctx_guard_fired(lnerf_ctx* ctx, int* fired) {
    return guard_int([&]() {
        if (!ctx || !fired) fail("null argument");
        std::lock_guard<std::mutex> lock(ctx->mu);
        *fired = -1;   // no guard on the last call (the generic path, a render, an explicit precision)
        if (!ctx->last_k16_train) return;
        const FusedPlan& p = ctx->last_plan;
        if (!p.guard) return;
        HIP_OK(hipSetDevice(ctx->device));
        HIP_OK(hipDeviceSynchronize());
        int w = 0;
        HIP_OK(hipMemcpy(&w, p.guard, sizeof(int), hipMemcpyDeviceToHost));
        *fired = w != 0 ? 1 : 0;
    });
}

extern "C" int lnerf_ctx_set_option(lnerf_ctx* ctx, int option, int value) {
    return guard_int([&]() {
        if (!ctx) fail("null ctx");
        std::lock_guard<std::mutex> lock(ctx->mu);
        switch (option) {
            case LNERF_OPT_DW_GRID:
                if (value != 0 && (value < 16 || value > 4096)) fail("LNERF_OPT_DW_GRID %d outside 16..4096", value);
                ctx->dw_grid = value;
                break;
            default:
                fail("unknown option %d", option);
        }
    });
}

extern "C" int lnerf_scale_by_device_scalar(float* buf, size_t n, const float* scale, void* stream) {
    return guard_int([&]() {
        k_scale_by_scalar(buf, n, scale, (hipStream_t)stream);
        check_launch("lnerf_scale_by_device_scalar");
    });
}

extern "C" int lnerf_adam_update(float* params, const float* grads, float* m, float* v, size_t n,
                                 int t, float lr, float beta1, float beta2, float eps,
                                 void* stream) {
    return guard_int([&]() {
        if (t < 1) fail("adam step t must be >= 1");
        k_adam(params, grads, m, v, n, t, lr, beta1, beta2, eps, (hipStream_t)stream);
        check_launch("lnerf_adam_update");
    });
}
