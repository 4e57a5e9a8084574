// marshal_check.cpp -- host-only check of the loma-ABI marshalling, built with AddressSanitizer and
// UBSan (tests/native/Makefile, run by tests/test_sanitize.py; no GPU, no HIP).
//
//  1. The product's gather / scatter (loma-nerf_amd/csrc/lnerf_marshal.h, what the compat entry
//     points run before and after their kernels) on nested tables allocated the way the
//     reference's ctypes marshalling allocates them -- every row its own exactly-sized heap block
//     (mlp_utils.py:33-118) -- for the train_nerf chunk with its 256-row fake trace
//     (train_nerf.py:216-241, 296-317), the "real rows" variant, and an mlp_fit call
//     (fit_img.py:423-470). A read or write one element outside what the reference's loops touch
//     is a heap-buffer-overflow report; the checks below also require that every touched element
//     round-trips and no untouched one changes.
//  2. The oracle behind the same tables (oracle/nerf_oracle_abi.c: its own gather + the C
//     restatement) under the same sanitizers, forward + grad, against the flat oracle on the
//     gathered rectangles: bit-identical.
//  3. Malformed calls (null row, negative shape, too many layers) raise the marshalling error.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lnerf_marshal.h"
#include "nerf_oracle.h"

using lnerf::marshal::CallShape;

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                                      \
    do {                                                      \
        if (!(cond)) {                                        \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                \
            std::fprintf(stderr, "\n");                       \
            ++g_fail;                                         \
        }                                                     \
    } while (0)

// deterministic values in [-1, 1)
struct Rng {
    unsigned long long s;
    float next() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (float)((s >> 40) & 0xFFFFFF) / (float)(1 << 23) - 1.0f;
    }
};

// A ctypes-style 2-D table: `rows` separately allocated rows of `cols` floats.
struct T2 {
    std::vector<float*> rows;
    int r = 0, c = 0;
    T2(int r_, int c_, Rng& g, float scale = 1.0f) : rows(r_), r(r_), c(c_) {
        for (auto& p : rows) {
            p = (float*)std::malloc(sizeof(float) * (c ? c : 1));
            for (int j = 0; j < c; ++j) p[j] = g.next() * scale;
        }
    }
    T2(const T2&) = delete;
    ~T2() {
        for (auto p : rows) std::free(p);
    }
    float** ptr() { return rows.data(); }
    std::vector<float> snapshot() const {
        std::vector<float> v;
        for (auto p : rows) v.insert(v.end(), p, p + c);
        return v;
    }
};
struct T3 {
    std::vector<T2*> planes;
    std::vector<float**> ptrs;
    T3(int d0, int r, int c, Rng& g, float scale = 1.0f) {
        for (int i = 0; i < d0; ++i) {
            planes.push_back(new T2(r, c, g, scale));
            ptrs.push_back(planes.back()->ptr());
        }
    }
    T3(const T3&) = delete;
    ~T3() {
        for (auto p : planes) delete p;
    }
    float*** ptr() { return ptrs.data(); }
    std::vector<float> snapshot() const {
        std::vector<float> v;
        for (auto p : planes) {
            auto s = p->snapshot();
            v.insert(v.end(), s.begin(), s.end());
        }
        return v;
    }
};
struct I2 {
    std::vector<int*> rows;
    explicit I2(const std::vector<std::vector<int>>& v) {
        for (auto& r : v) {
            int* p = (int*)std::malloc(sizeof(int) * r.size());
            std::memcpy(p, r.data(), sizeof(int) * r.size());
            rows.push_back(p);
        }
    }
    ~I2() {
        for (auto p : rows) std::free(p);
    }
    int** ptr() { return rows.data(); }
};

// One train_nerf chunk call: L layers (K_l x N_l), N rays x S samples, io allocated io_alloc^2.
struct NerfChunk {
    int L, N, S, in_w, io_alloc;
    std::vector<int> K, Nn;
    std::vector<std::vector<int>> wsh, bsh, ios;
    int kmax = 0, nmax = 0;
};

NerfChunk chunk_shape(bool fake_trace) {
    NerfChunk c;
    c.L = 3, c.N = 4, c.S = 30, c.in_w = 33, c.io_alloc = 256;
    c.K = {33, 30, 30};
    c.Nn = {30, 30, 4};
    for (int l = 0; l < c.L; ++l) {
        c.wsh.push_back({c.K[l], c.Nn[l]});
        c.bsh.push_back({c.Nn[l], 1});
        c.ios.push_back({fake_trace ? 256 : c.N * c.S, c.Nn[l]});
        c.kmax = std::max(c.kmax, c.K[l]);
        c.nmax = std::max(c.nmax, c.Nn[l]);
    }
    return c;
}

// 1. gather every table into the flat layout, compare with the touched elements, scatter changed
// values back into the same tables and check exactly the touched elements changed
void check_gather_scatter(const char* name, bool nerf, const NerfChunk& ch, int th, int tw) {
    Rng g{12345};
    const int R = ch.N * ch.S;
    T2 X(nerf ? R : th, ch.in_w, g);
    T3 W(ch.L, ch.kmax, ch.nmax, g);
    T2 B(ch.L, ch.nmax, g);
    T3 IO(ch.L, ch.io_alloc, ch.io_alloc, g);
    I2 wsh(ch.wsh), ios(ch.ios);
    const CallShape c = lnerf::marshal::make_shape(nerf, X.r, ch.in_w, th, tw, ch.L, wsh.ptr(), ios.ptr(),
                                                   nerf ? ch.S : 0);
    const lnerf::LgDims& d = c.d;
    std::vector<float> fx((size_t)d.in_h * d.x_cols), fw((size_t)d.L * d.w_k * d.w_n), fb((size_t)d.L * d.b_n),
        fio((size_t)d.L * d.io_rows * d.io_cols);
    lnerf::marshal::gather2(fx.data(), X.ptr(), d.in_h, d.in_w, d.x_cols);
    lnerf::marshal::gather_w(fw.data(), W.ptr(), c);
    lnerf::marshal::gather_b(fb.data(), B.ptr(), c);
    lnerf::marshal::gather_io(fio.data(), IO.ptr(), c);
    for (int i = 0; i < d.in_h; ++i)
        for (int k = 0; k < d.in_w; ++k) CHECK(fx[(size_t)i * d.x_cols + k] == X.rows[i][k], "%s X[%d][%d]", name, i, k);
    int touched_io = 0;
    for (int l = 0; l < d.L; ++l) {
        for (int k = 0; k < c.K[l]; ++k)
            for (int j = 0; j < d.wsh1[l]; ++j)
                CHECK(fw[((size_t)l * d.w_k + k) * d.w_n + j] == W.planes[l]->rows[k][j], "%s W[%d][%d][%d]", name, l, k,
                      j);
        for (int j = 0; j < c.bcols[l]; ++j) CHECK(fb[(size_t)l * d.b_n + j] == B.rows[l][j], "%s B[%d][%d]", name, l, j);
        for (int i = 0; i < c.rows[l]; ++i)
            for (int j = 0; j < c.cols[l]; ++j, ++touched_io)
                CHECK(fio[((size_t)l * d.io_rows + i) * d.io_cols + j] == IO.planes[l]->rows[i][j], "%s IO[%d][%d][%d]",
                      name, l, i, j);
    }
    // the reference's loops: every io row the matmul, bias, activation and (nerf) reshape touch
    for (int l = 0; l < d.L; ++l) {
        int need_r = std::max(l == 0 ? d.in_h : d.ios0[l - 1], d.ios0[l]);
        if (l == d.L - 1) need_r = std::max(need_r, nerf ? th * ch.S : th);
        CHECK(c.rows[l] == need_r, "%s rows[%d] = %d, loops touch %d", name, l, c.rows[l], need_r);
    }
    // scatter: add 1 to every gathered value, write back, compare
    const auto io_before = IO.snapshot();
    for (auto& v : fio) v += 1.0f;
    lnerf::marshal::scatter_io(IO.ptr(), fio.data(), c);
    const auto io_after = IO.snapshot();
    int changed = 0;
    for (int l = 0; l < d.L; ++l)
        for (int i = 0; i < ch.io_alloc; ++i)
            for (int j = 0; j < ch.io_alloc; ++j) {
                const size_t e = ((size_t)l * ch.io_alloc + i) * ch.io_alloc + j;
                const bool in = i < c.rows[l] && j < c.cols[l];
                if (in) {
                    CHECK(io_after[e] == io_before[e] + 1.0f, "%s scatter IO[%d][%d][%d]", name, l, i, j);
                    ++changed;
                } else {
                    CHECK(io_after[e] == io_before[e], "%s untouched IO[%d][%d][%d] changed", name, l, i, j);
                }
            }
    CHECK(changed == touched_io, "%s: %d scattered vs %d gathered", name, changed, touched_io);
    for (auto& v : fw) v = -v;
    lnerf::marshal::scatter_w(W.ptr(), fw.data(), c);
    for (int l = 0; l < d.L; ++l)
        for (int k = 0; k < c.K[l]; ++k)
            for (int j = 0; j < d.wsh1[l]; ++j)
                CHECK(W.planes[l]->rows[k][j] == fw[((size_t)l * d.w_k + k) * d.w_n + j], "%s scatter W", name);
    std::printf("ok %-28s io rows %d/%d/%d, %d io elements\n", name, c.rows[0], c.rows[1], c.rows[d.L - 1],
                touched_io);
}

// 2. the oracle through the nested tables vs the flat oracle on the same values
void check_oracle_abi(bool fake_trace) {
    const NerfChunk ch = chunk_shape(fake_trace);
    Rng g{777};
    const int R = ch.N * ch.S, th = ch.N;
    T2 X(R, ch.in_w, g), T(th, 3, g), dists(th, ch.S, g, 0.0f), alpha(th, ch.S, g, 0.0f), cp(th, ch.S, g, 0.0f),
        wsamp(th, ch.S, g, 0.0f), acc(th, 3, g, 0.0f);
    for (int i = 0; i < th; ++i)
        for (int j = 0; j < ch.S; ++j) dists.rows[i][j] = j + 1 < ch.S ? 4.0f / (ch.S - 1) : 1e8f;
    for (int i = 0; i < th; ++i)
        for (int k = 0; k < 3; ++k) T.rows[i][k] = 0.5f * (T.rows[i][k] + 1.0f);
    T3 W(ch.L, ch.kmax, ch.nmax, g, 0.3f), IO(ch.L, ch.io_alloc, ch.io_alloc, g, 0.0f), rgba(th, ch.S, 4, g, 0.0f);
    T2 B(ch.L, ch.nmax, g, 0.5f);
    I2 wsh(ch.wsh), bsh(ch.bsh), ios(ch.ios);
    // flat copies (the gathered rectangles) before the call
    const CallShape c = lnerf::marshal::make_shape(true, R, ch.in_w, th, 3, ch.L, wsh.ptr(), ios.ptr(), ch.S);
    oracle_dims d{};
    d.num_weights = ch.L, d.layer_input_h = R, d.layer_input_w = ch.in_w, d.target_image_h = th,
    d.target_image_w = 3, d.num_samples = ch.S;
    for (int l = 0; l < ch.L; ++l) {
        d.weight_shapes[l][0] = ch.wsh[l][0], d.weight_shapes[l][1] = ch.wsh[l][1];
        d.bias_shapes[l][0] = ch.bsh[l][0], d.bias_shapes[l][1] = 1;
        d.intermediate_output_shapes[l][0] = ch.ios[l][0], d.intermediate_output_shapes[l][1] = ch.ios[l][1];
    }
    d.x_cols = ch.in_w, d.w_k = ch.kmax, d.w_n = ch.nmax, d.b_n = ch.nmax, d.io_rows = ch.io_alloc,
    d.io_cols = ch.io_alloc, d.t_cols = 3, d.acc_cols = 3;
    auto fX = X.snapshot(), fW = W.snapshot(), fB = B.snapshot(), fT = T.snapshot(), fIO = IO.snapshot(),
         fr = rgba.snapshot(), fd = dists.snapshot(), fa = alpha.snapshot(), fc = cp.snapshot(),
         fs = wsamp.snapshot(), fac = acc.snapshot();
    const float want = oracle_nerf_forward(&d, fX.data(), fW.data(), fB.data(), fT.data(), fIO.data(), fr.data(),
                                           fd.data(), fa.data(), fc.data(), fs.data(), fac.data());
    const float got = oracle_abi_nerf_evaluate_and_march(X.ptr(), R, ch.in_w, W.ptr(), B.ptr(), T.ptr(), th, 3, ch.L,
                                                         wsh.ptr(), bsh.ptr(), ios.ptr(), IO.ptr(), rgba.ptr(), ch.S,
                                                         dists.ptr(), alpha.ptr(), cp.ptr(), wsamp.ptr(), acc.ptr());
    CHECK(std::isfinite(want) && got == want, "oracle abi forward %g vs flat %g", got, want);
    const auto accv = acc.snapshot();
    for (size_t e = 0; e < accv.size(); ++e) CHECK(accv[e] == fac[e], "oracle abi acc[%zu]", e);
    const auto iov = IO.snapshot();
    for (size_t e = 0; e < iov.size(); ++e) CHECK(iov[e] == fIO[e], "oracle abi io[%zu]", e);
    // grad on zeroed adjoints, seeded with the loss (train_nerf.py:477), primals as after the
    // forward (the tables now hold them)
    Rng z{1};
    T2 dX(R, ch.in_w, z, 0.0f), dB(ch.L, ch.nmax, z, 0.0f), dT(th, 3, z, 0.0f), dd(th, ch.S, z, 0.0f),
        dal(th, ch.S, z, 0.0f), dcp(th, ch.S, z, 0.0f), dws(th, ch.S, z, 0.0f), dacc(th, 3, z, 0.0f);
    T3 dW(ch.L, ch.kmax, ch.nmax, z, 0.0f), dIO(ch.L, ch.io_alloc, ch.io_alloc, z, 0.0f), drgba(th, ch.S, 4, z, 0.0f);
    std::vector<int> zi(8, 0);
    I2 dwsh(ch.wsh), dbsh(ch.bsh), dios(ch.ios);
    std::vector<float> gX(fX.size(), 0.0f), gW(fW.size(), 0.0f), gB(fB.size(), 0.0f), gT(fT.size(), 0.0f),
        gIO(fIO.size(), 0.0f), gr(fr.size(), 0.0f), gd(fd.size(), 0.0f), ga(fa.size(), 0.0f), gc(fc.size(), 0.0f),
        gs(fs.size(), 0.0f), gac(fac.size(), 0.0f);
    oracle_nerf_grad(&d, fX.data(), gX.data(), fW.data(), gW.data(), fB.data(), gB.data(), fT.data(), gT.data(),
                     fIO.data(), gIO.data(), fr.data(), gr.data(), fd.data(), gd.data(), fa.data(), ga.data(),
                     fc.data(), gc.data(), fs.data(), gs.data(), fac.data(), gac.data(), want);
    oracle_abi_grad_nerf_evaluate_and_march(
        X.ptr(), dX.ptr(), R, &zi[0], ch.in_w, &zi[1], W.ptr(), dW.ptr(), B.ptr(), dB.ptr(), T.ptr(), dT.ptr(), th,
        &zi[2], 3, &zi[3], ch.L, &zi[4], wsh.ptr(), dwsh.ptr(), bsh.ptr(), dbsh.ptr(), ios.ptr(), dios.ptr(), IO.ptr(),
        dIO.ptr(), rgba.ptr(), drgba.ptr(), ch.S, &zi[5], dists.ptr(), dd.ptr(), alpha.ptr(), dal.ptr(), cp.ptr(),
        dcp.ptr(), wsamp.ptr(), dws.ptr(), acc.ptr(), dacc.ptr(), want);
    const auto dWv = dW.snapshot(), dXv = dX.snapshot(), ddv = dd.snapshot();
    double mx = 0.0;
    for (size_t e = 0; e < dWv.size(); ++e) {
        CHECK(dWv[e] == gW[e], "oracle abi dW[%zu] %g vs %g", e, dWv[e], gW[e]);
        mx = std::max(mx, (double)std::fabs(gW[e]));
    }
    for (size_t e = 0; e < dXv.size(); ++e) CHECK(dXv[e] == gX[e], "oracle abi dX[%zu]", e);
    for (size_t e = 0; e < ddv.size(); ++e) CHECK(ddv[e] == gd[e], "oracle abi d_dists[%zu]", e);
    for (int i = 0; i < 8; ++i) CHECK(zi[i] == 0, "int adjoint %d written", i);
    CHECK(mx > 0.0, "zero gradient");
    (void)c;
    std::printf("ok oracle abi (%s)          loss %.6f, max|dW| %.4g\n", fake_trace ? "fake trace" : "real rows", got,
                mx);
}

void check_errors() {
    const NerfChunk ch = chunk_shape(true);
    I2 wsh(ch.wsh), ios(ch.ios);
    int thrown = 0;
    try {
        lnerf::marshal::make_shape(true, 120, 33, 4, 3, 17, wsh.ptr(), ios.ptr(), 30);
    } catch (const lnerf::marshal::Error&) {
        ++thrown;
    }
    try {
        lnerf::marshal::make_shape(true, -1, 33, 4, 3, 3, wsh.ptr(), ios.ptr(), 30);
    } catch (const lnerf::marshal::Error&) {
        ++thrown;
    }
    try {
        lnerf::marshal::make_shape(true, 120, 33, 4, 3, 3, nullptr, ios.ptr(), 30);
    } catch (const lnerf::marshal::Error&) {
        ++thrown;
    }
    try {
        float* rows[2] = {nullptr, nullptr};
        float buf[4];
        lnerf::marshal::gather2(buf, rows, 2, 2, 2);
    } catch (const lnerf::marshal::Error&) {
        ++thrown;
    }
    CHECK(thrown == 4, "%d of 4 malformed calls raised", thrown);
    std::printf("ok malformed calls raise     %d/4\n", thrown);
}

}  // namespace

int main() {
    check_gather_scatter("nerf chunk, fake trace", true, chunk_shape(true), 4, 3);
    check_gather_scatter("nerf chunk, real rows", true, chunk_shape(false), 4, 3);
    {
        // mlp_fit (fit_img.py:423-470): 256 rows of 22 PE inputs, 22 -> 16 -> 16 -> 3, ios rows 256
        NerfChunk m;
        m.L = 3, m.N = 256, m.S = 1, m.in_w = 22, m.io_alloc = 256;
        m.K = {22, 16, 16};
        m.Nn = {16, 16, 3};
        for (int l = 0; l < 3; ++l) {
            m.wsh.push_back({m.K[l], m.Nn[l]});
            m.bsh.push_back({m.Nn[l], 1});
            m.ios.push_back({256, m.Nn[l]});
            m.kmax = std::max(m.kmax, m.K[l]);
            m.nmax = std::max(m.nmax, m.Nn[l]);
        }
        check_gather_scatter("mlp_fit chunk", false, m, 256, 3);
    }
    check_oracle_abi(true);
    check_oracle_abi(false);
    check_errors();
    if (g_fail) {
        std::printf("%d checks FAILED\n", g_fail);
        return 1;
    }
    std::printf("all marshalling checks passed\n");
    return 0;
}
