// ORACLE — test infrastructure only. Never linked into the product.
//
// Host BLAS / sparse-BLAS layer of the CPU oracle: the arithmetic of the
// reference's CPU backend (kernels_mkl.cpp:73-352) comes from Intel MKL
// (cblas_* and mkl_sparse_?_mv). The image ships the MKL 2021.4.0 runtime
// (/opt/conda/lib/libmkl_rt.so.1) but no MKL headers, so the entry points
// are bound at run time with dlopen/dlsym using the documented LP64 C
// prototypes and enum values. When the runtime is absent (or
// MPG_ORACLE_BACKEND=loops) the same operations run as plain loops with
// fp64 accumulation — the oracle reports which backend it used.
#ifndef MPG_ORACLE_CPU_BLAS_HPP
#define MPG_ORACLE_CPU_BLAS_HPP

#include <cstddef>
#include <string>

namespace oracle {

// CBLAS / MKL sparse enum values (LP64 interface)
enum { kColMajor = 102, kNoTrans = 111, kTrans = 112, kUpper = 121, kLower = 122, kNonUnit = 131 };
enum { kSparseOpNoTrans = 10, kSparseTypeGeneral = 20, kSparseTypeTriangular = 23, kSparseIndexZero = 0 };
enum { kSparseFillLower = 40, kSparseFillUpper = 41, kSparseDiagNonUnit = 50, kSparseDiagUnit = 51 };
struct SparseDescr {
    int type, mode, diag;
};

struct MklApi {
    bool loaded = false;
    std::string path;
    double (*ddot)(int, const double*, int, const double*, int) = nullptr;
    float (*sdot)(int, const float*, int, const float*, int) = nullptr;
    double (*dnrm2)(int, const double*, int) = nullptr;
    float (*snrm2)(int, const float*, int) = nullptr;
    void (*daxpy)(int, double, const double*, int, double*, int) = nullptr;
    void (*saxpy)(int, float, const float*, int, float*, int) = nullptr;
    void (*dscal)(int, double, double*, int) = nullptr;
    void (*sscal)(int, float, float*, int) = nullptr;
    void (*drotg)(double*, double*, double*, double*) = nullptr;
    void (*srotg)(float*, float*, float*, float*) = nullptr;
    void (*drot)(int, double*, int, double*, int, double, double) = nullptr;
    void (*srot)(int, float*, int, float*, int, float, float) = nullptr;
    void (*dgemv)(int, int, int, int, double, const double*, int, const double*, int, double, double*, int) = nullptr;
    void (*sgemv)(int, int, int, int, float, const float*, int, const float*, int, float, float*, int) = nullptr;
    void (*dtrsv)(int, int, int, int, int, const double*, int, double*, int) = nullptr;
    void (*strsv)(int, int, int, int, int, const float*, int, float*, int) = nullptr;
    int (*d_create_csr)(void**, int, int, int, int*, int*, int*, double*) = nullptr;
    int (*s_create_csr)(void**, int, int, int, int*, int*, int*, float*) = nullptr;
    int (*d_mv)(int, double, void*, SparseDescr, const double*, double, double*) = nullptr;
    int (*s_mv)(int, float, void*, SparseDescr, const float*, float, float*) = nullptr;
    int (*d_trsv)(int, double, void*, SparseDescr, const double*, double*) = nullptr;
    int (*s_trsv)(int, float, void*, SparseDescr, const float*, float*) = nullptr;
    int (*destroy)(void*) = nullptr;
    void (*set_num_threads)(int) = nullptr;
    int (*get_max_threads)() = nullptr;
    int (*cbwr_get)(int) = nullptr;  // mkl_cbwr_get (optional)
};

// Loaded once per process; `loaded` false means the loop backend.
const MklApi& mkl();
// Use the loop kernels (fp32 products summed in fp64, in index order) while
// on, whether or not MKL loaded: a machine-independent summation order.
void force_loops(bool on);
// the loop kernels with a summation mode for fp32 operands (cpu_blas.cpp:
// kSumF64, kSumSeq32, kSumPair32); -1: MKL again
enum { kSumF64 = 0, kSumSeq32 = 1, kSumPair32 = 2 };
void force_loops_mode(int mode);
int loop_sum_mode();
const char* backend_name();
void set_threads(int threads);
int max_threads();
// MKL's conditional-numerical-reproducibility branch (mkl_cbwr_get(MKL_CBWR_BRANCH)); -1 without MKL
int cbwr_branch();

// ---- typed BLAS used by the restated algorithm ----
double dot(int n, const double* x, const double* y);
float dot(int n, const float* x, const float* y);
double nrm2(int n, const double* x);
float nrm2(int n, const float* x);
void axpy(int n, double a, const double* x, double* y);
void axpy(int n, float a, const float* x, float* y);
void scal(int n, double a, double* x);
void scal(int n, float a, float* x);
void rotg(double* a, double* b, double* c, double* s);
void rotg(float* a, float* b, float* c, float* s);
void rot1(double* x, double* y, double c, double s);  // one-element ?rot
void rot1(float* x, float* y, float c, float s);
// column-major y = alpha*op(A) x + beta*y, A is rows x cols with lda
void gemv(bool trans, int rows, int cols, double alpha, const double* A, int lda, const double* x, double beta,
          double* y);
void gemv(bool trans, int rows, int cols, float alpha, const float* A, int lda, const float* x, float beta, float* y);
// upper, non-transposed, non-unit triangular solve
void trsv_upper(int n, const double* A, int lda, double* x);
void trsv_upper(int n, const float* A, int lda, float* x);

}  // namespace oracle

#endif  // MPG_ORACLE_CPU_BLAS_HPP
