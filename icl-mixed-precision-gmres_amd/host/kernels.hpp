// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Operator surface of the GMRES hot path — the plugin boundary.
//
// Same operator set, names, argument order and <Type, Device> templating as
// the reference kernels.hpp:9-169 (dot / nrm2 with host or device result,
// axpy, naxpy, scal (x5), copy with cast, fill, rotg, rot (scalar and
// column), gemv, trsv, gdmv, spmv). A backend drops in by providing a Device
// tag (types.hpp) and explicit specialisations of these templates in its own
// translation unit — kernels_hip.cpp for `Hip`, the way kernels_mkl.cpp /
// kernels_cuda.cpp do for `MKL` / `Cuda` in the reference. The generic
// conveniences (scalar-type casting overloads, fill on any handle) are
// written once here on top of two backend primitives: fill_strided and
// jacobi_diag.
#ifndef MPGMRES_KERNELS_HPP
#define MPGMRES_KERNELS_HPP

#include <cassert>

#include "types.hpp"

// ---- copy with cast (kernels.hpp:11-30) ----
template <class Type1, class Type2, class Device>
void copy(Vect<Type1, Device> x, Vect<Type2, Device> y);
template <class Type1, class Type2, class Device>
void copy(Scalar<Type1, Device> x, Scalar<Type2, Device> y);

// ---- reductions ----
template <class Type, class Device>
Type dot(Vect<Type, Device> x, Vect<Type, Device> y);
template <class Type, class Device>
void dot(Vect<Type, Device> x, Vect<Type, Device> y, Scalar<Type, Device> result);
template <class Type, class Device>
Type nrm2(Vect<Type, Device> x);
template <class Type, class Device>
void nrm2(Vect<Type, Device> x, Scalar<Type, Device> result);

// ---- axpy family ----
template <class Type, class Device>
void axpy(Type alpha, Vect<Type, Device> x, Vect<Type, Device> y);
template <class Type, class Device>
void axpy(Scalar<Type, Device> alpha, Vect<Type, Device> x, Vect<Type, Device> y);
template <class ScalarType, class Type, class Device>
void axpy(ScalarType alpha, Vect<Type, Device> x, Vect<Type, Device> y) {
    axpy(Type(alpha), x, y);
}
// y <- y - alpha*x, alpha in device memory
template <class Type, class Device>
void naxpy(Scalar<Type, Device> alpha, Vect<Type, Device> x, Vect<Type, Device> y);

// ---- scal family ----
template <class Type, class Device>
void scal(Type alpha, Vect<Type, Device> x);
template <class Type, class Device>
void scal(Type alpha, Vect<Type, Device> x, Vect<Type, Device> y);
template <class ScalarType, class Type, class Device>
void scal(ScalarType alpha, Vect<Type, Device> x, Vect<Type, Device> y) {
    scal(Type(alpha), x, y);
}
template <class Type, class Device>
void scal(Scalar<Type, Device> alpha, Vect<Type, Device> x, Vect<Type, Device> y);
template <class Type, class Device>
void scal(Type alpha, Scalar<Type, Device> x, Scalar<Type, Device> y);
template <class ScalarType, class Type, class Device>
void scal(ScalarType alpha, Scalar<Type, Device> x, Scalar<Type, Device> y) {
    scal(Type(alpha), x, y);
}
template <class Type, class Device>
void scal(Scalar<Type, Device> alpha, Scalar<Type, Device> x, Scalar<Type, Device> y);
// y = (1/alpha) x with the reciprocal formed in Type where alpha lives: the
// reference's `inv = 1/h.access(); scal(inv, w, v)` (Orthogonalization.hpp:
// 51-60) without the host read (the same two roundings, so bit-identical).
// Addition to the reference surface; a backend without a device form can
// define it as exactly that host read.
template <class Type, class Device>
void scal_recip(Scalar<Type, Device> alpha, Vect<Type, Device> x, Vect<Type, Device> y);

// ---- fill (kernels.hpp:88-101) ----
// backend primitive: x[c*ld + r] = value for r < rows, c < cols
template <class Type, class Device>
void fill_strided(Type* x, size_t rows, size_t cols, size_t ld, Type value);

template <class Type, class Device, class ScalarType>
void fill(ScalarType alpha, Scalar<Type, Device> x) {
    fill_strided<Type, Device>(x.data(), 1, 1, 1, Type(alpha));
}
template <class Type, class Device, class ScalarType>
void fill(ScalarType alpha, Vect<Type, Device> x) {
    fill_strided<Type, Device>(x.data(), x.n(), 1, x.n(), Type(alpha));
}
template <class Type, class Device, class ScalarType>
void fill(ScalarType alpha, MultiVect<Type, Device> x) {
    fill_strided<Type, Device>(x.data(), x.nrows_base(), x.ncols_base(), x.stride(), Type(alpha));
}

// ---- Givens ----
template <class Type, class Device>
void rotg(Scalar<Type, Device> a, Scalar<Type, Device> b, Scalar<Type, Device> c, Scalar<Type, Device> s);
template <class Type, class Device>
void rot(Scalar<Type, Device> a, Scalar<Type, Device> b, Scalar<Type, Device> c, Scalar<Type, Device> s);
// apply rotations j = 0..c.n()-1 to the pairs (a[j], a[j+1])
template <class Type, class Device>
void rot(Vect<Type, Device> a, Vect<Type, Device> c, Vect<Type, Device> s);

// ---- BLAS-2 ----
template <class Type, class Device>
void gemv(Type alpha, MultiVect<Type, Device> matrix, Vect<Type, Device> x, Type beta, Vect<Type, Device> y);
template <class ScalarType, class Type, class Device>
void gemv(ScalarType alpha, MultiVect<Type, Device> matrix, Vect<Type, Device> x, ScalarType beta,
          Vect<Type, Device> y) {
    gemv(Type(alpha), matrix, x, Type(beta), y);
}
template <class Type, class Device>
void trsv(const char* upper, MultiVect<Type, Device> matrix, Vect<Type, Device> x);

// y = beta*y + alpha*diag∘x (kernels.hpp:131-151)
template <class Type, class Device>
void gdmv(Type alpha, Vect<Type, Device> diag, Vect<Type, Device> x, Type beta, Vect<Type, Device> y);
template <class ScalarType, class Type, class Device>
void gdmv(ScalarType alpha, Vect<Type, Device> diag, Vect<Type, Device> x, ScalarType beta, Vect<Type, Device> y) {
    gdmv(Type(alpha), diag, x, Type(beta), y);
}

// ---- sparse ----
template <class Type, class Device>
void spmv(Type alpha, SparseMatrix<Type, Device> matrix, Vect<Type, Device> x, Type beta, Vect<Type, Device> y);
template <class ScalarType, class Type, class Device>
void spmv(ScalarType alpha, SparseMatrix<Type, Device> matrix, Vect<Type, Device> x, ScalarType beta,
          Vect<Type, Device> y) {
    spmv(Type(alpha), matrix, x, Type(beta), y);
}

// backend primitive: Jacobi inverse diagonal with the eps_f32 * ||A||_inf
// boost of types.hpp:393-431
template <class Type, class Device>
void jacobi_diag(SparseMatrix<Type, Device> A, Vect<Type, Device> diag);

// ILU(0) of the fp64 matrix in precision Type (kernels.hpp:155-156), its
// triangular solves (kernels.hpp:168-169) and the Jacobi-sweep
// approximation of them (ilusv_jacobi, kernels.hpp:219-248).
template <class Type, class Device>
ILU<Type, Device> ilu0(SparseMatrix<double, Device> matrix);
template <class Type, class Device>
void ilusv(ILU<Type, Device> ilu, Vect<Type, Device> rhs);
template <class Type, class Device>
void ilusv_jacobi(ILU_Jacobi<Type, Device> ilu, Vect<Type, Device> x);

// Jacobi preconditioner M = D^-1 (types.hpp:381-448).
template <class Type, class Device>
class Jacobi : public LinearOperator<Type, Device> {
    Vect<Type, Device> diag_;

public:
    explicit Jacobi(SparseMatrix<Type, Device> A) : diag_(A.nrows()) { jacobi_diag(A, diag_); }
    int n() const { return (int)diag_.n(); }
    Type* diag_data() { return diag_.data(); }
    Vect<Type, Device> diag_vect() { return diag_; }
    void apply(Vect<Type, Device> rhs) override { gdmv(1.0, diag_, rhs, 0.0, rhs); }
};

#endif  // MPGMRES_KERNELS_HPP
