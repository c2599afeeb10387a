// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// ORACLE — test infrastructure only. Never linked into the product.
// Run-time binding of the MKL runtime (or plain loops); see cpu_blas.hpp.
#include "cpu_blas.hpp"

#include <dlfcn.h>

#include <cmath>
#include <cstdlib>
#include <atomic>
#include <mutex>

namespace oracle {

namespace {

MklApi g_api;
MklApi g_off;  // loaded = false: the loop kernels
std::atomic<bool> g_force_loops{false};
// the loop kernels' summation of fp32 operands (force_loops(mode)):
// kSumF64 fp32 products summed in fp64 in index order, rounded once (the HIP
// kernels' default class); kSumSeq32 every partial sum an fp32 value, one
// sequential chain in index order (a scalar CPU BLAS); kSumPair32 fp32
// partial sums in pairwise (tree) order over the long reductions -- the
// shape of a GPU reduction (cublasSdot / Sgemv, the HIP kernels under
// accum f32) -- and sequentially over the short ones (a row of A, the k+1
// basis columns of one gemv row)
std::atomic<int> g_sum{kSumF64};
std::once_flag g_once;

template <class F>
void bind(void* h, F& fn, const char* name, bool& ok) {
    fn = reinterpret_cast<F>(dlsym(h, name));
    if (!fn) ok = false;
}

void load() {
    const char* force = std::getenv("MPG_ORACLE_BACKEND");
    if (force && std::string(force) == "loops") return;
    const char* env = std::getenv("MPG_MKL_PATH");
    const char* candidates[] = {env, "/opt/conda/lib/libmkl_rt.so.1", "/opt/conda/lib/libmkl_rt.so", "libmkl_rt.so.1",
                                "libmkl_rt.so"};
    void* h = nullptr;
    std::string used;
    for (const char* c : candidates) {
        if (!c) continue;
        h = dlopen(c, RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            used = c;
            break;
        }
    }
    if (!h) return;
    // GNU OpenMP threading layer, as the reference links mkl_gnu_thread (Makefile:13)
    if (auto set_layer = reinterpret_cast<int (*)(int)>(dlsym(h, "MKL_Set_Threading_Layer"))) set_layer(3);
    bool ok = true;
    MklApi& a = g_api;
    bind(h, a.ddot, "cblas_ddot", ok);
    bind(h, a.sdot, "cblas_sdot", ok);
    bind(h, a.dnrm2, "cblas_dnrm2", ok);
    bind(h, a.snrm2, "cblas_snrm2", ok);
    bind(h, a.daxpy, "cblas_daxpy", ok);
    bind(h, a.saxpy, "cblas_saxpy", ok);
    bind(h, a.dscal, "cblas_dscal", ok);
    bind(h, a.sscal, "cblas_sscal", ok);
    bind(h, a.drotg, "cblas_drotg", ok);
    bind(h, a.srotg, "cblas_srotg", ok);
    bind(h, a.drot, "cblas_drot", ok);
    bind(h, a.srot, "cblas_srot", ok);
    bind(h, a.dgemv, "cblas_dgemv", ok);
    bind(h, a.sgemv, "cblas_sgemv", ok);
    bind(h, a.dtrsv, "cblas_dtrsv", ok);
    bind(h, a.strsv, "cblas_strsv", ok);
    bind(h, a.d_create_csr, "mkl_sparse_d_create_csr", ok);
    bind(h, a.s_create_csr, "mkl_sparse_s_create_csr", ok);
    bind(h, a.d_mv, "mkl_sparse_d_mv", ok);
    bind(h, a.s_mv, "mkl_sparse_s_mv", ok);
    bind(h, a.d_trsv, "mkl_sparse_d_trsv", ok);
    bind(h, a.s_trsv, "mkl_sparse_s_trsv", ok);
    bind(h, a.destroy, "mkl_sparse_destroy", ok);
    bind(h, a.set_num_threads, "MKL_Set_Num_Threads", ok);
    bind(h, a.get_max_threads, "MKL_Get_Max_Threads", ok);
    // conditional numerical reproducibility (MKL_CBWR in the environment,
    // read by MKL at its first call): the branch it runs, for the record
    a.cbwr_get = reinterpret_cast<int (*)(int)>(dlsym(h, "MKL_CBWR_Get"));  // (mkl_cbwr_get is the by-reference Fortran entry)
    a.loaded = ok;
    a.path = used;
}

// classic reference-BLAS ?rotg for the loop backend
template <class T>
void rotg_loops(T* a, T* b, T* c, T* s) {
    const T av = *a, bv = *b;
    const T roe = std::fabs(av) > std::fabs(bv) ? av : bv;
    const T scale = std::fabs(av) + std::fabs(bv);
    T r, z;
    if (scale == T(0)) {
        *c = 1;
        *s = 0;
        r = 0;
        z = 0;
    } else {
        const T as = av / scale, bs = bv / scale;
        r = scale * std::sqrt(as * as + bs * bs);
        r = roe >= T(0) ? r : -r;
        *c = av / r;
        *s = bv / r;
        z = 1;
        if (std::fabs(av) > std::fabs(bv)) z = *s;
        if (std::fabs(bv) >= std::fabs(av) && *c != T(0)) z = T(1) / *c;
    }
    *a = r;
    *b = z;
}

// fp32 sums of a[i] * b[i] (products rounded to fp32; the oracle is built
// with -ffp-contract=off, so no fused multiply-add)
float sum_seq32(int n, const float* a, const float* b) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}
float sum_pair32(int n, const float* a, const float* b) {
    if (n <= 8) return sum_seq32(n, a, b);
    const int h = n / 2;
    return sum_pair32(h, a, b) + sum_pair32(n - h, a + h, b + h);
}
float sum32(int n, const float* a, const float* b) {
    return g_sum.load(std::memory_order_relaxed) == kSumPair32 ? sum_pair32(n, a, b) : sum_seq32(n, a, b);
}

template <class T>
void gemv_loops(bool trans, int rows, int cols, T alpha, const T* A, int lda, const T* x, T beta, T* y) {
    if constexpr (sizeof(T) == 4) {
        if (g_sum.load(std::memory_order_relaxed) != kSumF64) {
            if (trans) {  // one fp32 reduction over the rows per column
#pragma omp parallel for schedule(static)
                for (int j = 0; j < cols; ++j) {
                    const T t = sum32(rows, A + (size_t)j * lda, x);
                    y[j] = beta == T(0) ? alpha * t : alpha * t + beta * y[j];
                }
            } else {  // each row: the k+1 column terms in order in fp32
#pragma omp parallel for schedule(static)
                for (int i = 0; i < rows; ++i) {
                    T t = 0;
                    for (int j = 0; j < cols; ++j) t += A[(size_t)j * lda + i] * x[j];
                    y[i] = beta == T(0) ? alpha * t : alpha * t + beta * y[i];
                }
            }
            return;
        }
    }
    if (trans) {
#pragma omp parallel for schedule(static)
        for (int j = 0; j < cols; ++j) {
            double acc = 0;
            for (int i = 0; i < rows; ++i) acc += (double)A[(size_t)j * lda + i] * x[i];
            const T t = (T)acc;
            y[j] = beta == T(0) ? alpha * t : alpha * t + beta * y[j];
        }
    } else {
#pragma omp parallel for schedule(static)
        for (int i = 0; i < rows; ++i) {
            double acc = 0;
            for (int j = 0; j < cols; ++j) acc += (double)A[(size_t)j * lda + i] * x[j];
            const T t = (T)acc;
            y[i] = beta == T(0) ? alpha * t : alpha * t + beta * y[i];
        }
    }
}

template <class T>
void trsv_upper_loops(int n, const T* A, int lda, T* x) {
    for (int j = n - 1; j >= 0; --j) {
        if (x[j] == T(0)) continue;
        x[j] = x[j] / A[(size_t)j * lda + j];
        const T t = x[j];
        for (int i = j - 1; i >= 0; --i) x[i] = x[i] - t * A[(size_t)j * lda + i];
    }
}

}  // namespace

const MklApi& mkl() {
    std::call_once(g_once, load);
    return g_force_loops.load(std::memory_order_relaxed) ? g_off : g_api;
}

void force_loops(bool on) { force_loops_mode(on ? kSumF64 : -1); }
void force_loops_mode(int mode) {
    g_force_loops.store(mode >= 0, std::memory_order_relaxed);
    g_sum.store(mode >= 0 ? mode : kSumF64, std::memory_order_relaxed);
}
int loop_sum_mode() { return g_sum.load(std::memory_order_relaxed); }

const char* backend_name() { return mkl().loaded ? "mkl" : "loops"; }

void set_threads(int threads) {
    if (threads <= 0) return;
    if (mkl().loaded) mkl().set_num_threads(threads);
}

int max_threads() { return mkl().loaded ? mkl().get_max_threads() : 1; }
int cbwr_branch() { return mkl().loaded && mkl().cbwr_get ? mkl().cbwr_get(1) : -1; }

double dot(int n, const double* x, const double* y) {
    if (mkl().loaded) return mkl().ddot(n, x, 1, y, 1);
    double s = 0;
    for (int i = 0; i < n; ++i) s += x[i] * y[i];
    return s;
}
float dot(int n, const float* x, const float* y) {
    if (mkl().loaded) return mkl().sdot(n, x, 1, y, 1);
    if (g_sum.load(std::memory_order_relaxed) != kSumF64) return sum32(n, x, y);
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)x[i] * y[i];
    return (float)s;
}
double nrm2(int n, const double* x) {
    if (mkl().loaded) return mkl().dnrm2(n, x, 1);
    double s = 0;
    for (int i = 0; i < n; ++i) s += x[i] * x[i];
    return std::sqrt(s);
}
float nrm2(int n, const float* x) {
    if (mkl().loaded) return mkl().snrm2(n, x, 1);
    if (g_sum.load(std::memory_order_relaxed) != kSumF64) return std::sqrt(sum32(n, x, x));
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)x[i] * x[i];
    return (float)std::sqrt(s);
}
void axpy(int n, double a, const double* x, double* y) {
    if (mkl().loaded) return mkl().daxpy(n, a, x, 1, y, 1);
    for (int i = 0; i < n; ++i) y[i] += a * x[i];
}
void axpy(int n, float a, const float* x, float* y) {
    if (mkl().loaded) return mkl().saxpy(n, a, x, 1, y, 1);
    for (int i = 0; i < n; ++i) y[i] += a * x[i];
}
void scal(int n, double a, double* x) {
    if (mkl().loaded) return mkl().dscal(n, a, x, 1);
    for (int i = 0; i < n; ++i) x[i] *= a;
}
void scal(int n, float a, float* x) {
    if (mkl().loaded) return mkl().sscal(n, a, x, 1);
    for (int i = 0; i < n; ++i) x[i] *= a;
}
void rotg(double* a, double* b, double* c, double* s) {
    if (mkl().loaded) return mkl().drotg(a, b, c, s);
    rotg_loops(a, b, c, s);
}
void rotg(float* a, float* b, float* c, float* s) {
    if (mkl().loaded) return mkl().srotg(a, b, c, s);
    rotg_loops(a, b, c, s);
}
void rot1(double* x, double* y, double c, double s) {
    if (mkl().loaded) return mkl().drot(1, x, 1, y, 1, c, s);
    const double t = c * *x + s * *y;
    *y = c * *y - s * *x;
    *x = t;
}
void rot1(float* x, float* y, float c, float s) {
    if (mkl().loaded) return mkl().srot(1, x, 1, y, 1, c, s);
    const float t = c * *x + s * *y;
    *y = c * *y - s * *x;
    *x = t;
}
void gemv(bool trans, int rows, int cols, double alpha, const double* A, int lda, const double* x, double beta,
          double* y) {
    if (mkl().loaded)
        return mkl().dgemv(kColMajor, trans ? kTrans : kNoTrans, rows, cols, alpha, A, lda, x, 1, beta, y, 1);
    gemv_loops(trans, rows, cols, alpha, A, lda, x, beta, y);
}
void gemv(bool trans, int rows, int cols, float alpha, const float* A, int lda, const float* x, float beta, float* y) {
    if (mkl().loaded)
        return mkl().sgemv(kColMajor, trans ? kTrans : kNoTrans, rows, cols, alpha, A, lda, x, 1, beta, y, 1);
    gemv_loops(trans, rows, cols, alpha, A, lda, x, beta, y);
}
void trsv_upper(int n, const double* A, int lda, double* x) {
    if (mkl().loaded) return mkl().dtrsv(kColMajor, kUpper, kNoTrans, kNonUnit, n, A, lda, x, 1);
    trsv_upper_loops(n, A, lda, x);
}
void trsv_upper(int n, const float* A, int lda, float* x) {
    if (mkl().loaded) return mkl().strsv(kColMajor, kUpper, kNoTrans, kNonUnit, n, A, lda, x, 1);
    trsv_upper_loops(n, A, lda, x);
}

}  // namespace oracle
