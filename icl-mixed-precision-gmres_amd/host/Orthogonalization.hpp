// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Arnoldi basis and Gram-Schmidt kernels, Kokkos-free.
//
// Behaviour follows the reference Orthogonalization.hpp:
//   GS::first_vector      :36-45  v0 = w * (1/beta)  (zero fill when beta == 0)
//   GS::add_vector        :51-60  orthogonalize; h(k+1,k) = ||w|| (device);
//                                 v_{k+1} = w * (1/h), the reciprocal formed on
//                                 the device (the reference reads h to the host)
//   GS::update_x          :62-73  x += V y  /  x_hi += hi(V y)
//   CGS_Kernel            :76-89  h = V^T w ; w -= V h
//   MGS_Kernel            :91-107 per column: h_j = <w, v_j> ; w -= h_j v_j
//   CGSR_Kernel<., ., 2>  :109-136 CGS, then a second CGS pass accumulated into h
// The reciprocal-then-multiply normalisation is kept on purpose: it changes
// the rounding compared with a division.
#ifndef MPGMRES_ORTHOGONALIZATION_HPP
#define MPGMRES_ORTHOGONALIZATION_HPP

#include <utility>

#include "kernels.hpp"

namespace Orthogonalization {

template <class Type, class Device>
class Orth {
public:
    virtual MultiVect<Type, Device> basis() = 0;
    virtual ~Orth() {}
};

template <class Type, class GS_Kernel, class Device>
class GS : public Orth<Type, Device> {
    GS_Kernel kernel_;

public:
    using value_type = Type;
    using kernel_type = GS_Kernel;

    MultiVect<Type, Device> v;  // n x (m+1) Krylov basis, column-major

    GS(size_t n, size_t restart_length) : kernel_(n, restart_length), v(n, restart_length + 1) {}

    MultiVect<Type, Device> basis() override { return v; }

    Type first_vector(const Vect<Type, Device> w) {
        const Type beta = nrm2(w);
        Vect<Type, Device> v0(v, mpg::ALL, 0);
        if (beta == Type(0)) {
            fill(0.0, v0);
        } else {
            const Type inv = Type(1) / beta;
            scal(inv, w, v0);
        }
        return beta;
    }

    Vect<Type, Device> previous_krylov_vector(size_t k) { return Vect<Type, Device>(v, mpg::ALL, k); }

    void add_vector(const size_t k, Vect<Type, Device> w, MultiVect<Type, Device> h) {
        kernel_.orthogonalize(v, k, w, h);
        Scalar<Type, Device> h_next = h(k + 1, k);
        nrm2(w, h_next);
        // v_{k+1} = w * (1/h): the reference reads h to the host and forms
        // the reciprocal there (:56-59); scal_recip forms the same Type
        // reciprocal on the device, so the step has no host read.
        scal_recip(h_next, w, Vect<Type, Device>(v, mpg::ALL, k + 1));
    }

    // x += V(:, 0:k) y, all in Type
    void update_x(const size_t k, const Vect<Type, Device> y, Vect<Type, Device> x) const {
        MultiVect<Type, Device> vk(v, mpg::ALL, std::make_pair(size_t(0), k));
        gemv(1.0, vk, y, 1.0, x);
    }

    // x_hi += High(V(:, 0:k) y): the low-precision product is formed in
    // x_inc_temp, widened into x_temp, then added in High (gmres.cpp:276-290)
    template <class High>
    void update_x(const size_t k, const Vect<Type, Device> y, Vect<High, Device> x, Vect<Type, Device> x_inc_temp,
                  Vect<High, Device> x_temp) const {
        MultiVect<Type, Device> vk(v, mpg::ALL, std::make_pair(size_t(0), k));
        gemv(1.0, vk, y, 0.0, x_inc_temp);
        copy(x_inc_temp, x_temp);
        axpy(1.0, x_temp, x);
    }
};

template <class Type, class Device>
class CGS_Kernel {
public:
    CGS_Kernel(size_t, size_t) {}

    void orthogonalize(MultiVect<Type, Device> v, const size_t k, Vect<Type, Device> w,
                       MultiVect<Type, Device> h) const {
        const auto cols = std::make_pair(size_t(0), k + 1);
        MultiVect<Type, Device> vk(v, mpg::ALL, cols);
        Vect<Type, Device> hk(h, cols, k);
        gemv(1.0, vk.transpose_matrix(), w, 0.0, hk);  // h = V^T w
        gemv(-1.0, vk, hk, 1.0, w);                    // w = w - V h
    }
};

template <class Type, class Device>
class MGS_Kernel {
public:
    MGS_Kernel(size_t, size_t) {}

    void orthogonalize(MultiVect<Type, Device> v, size_t k, Vect<Type, Device> w,
                       MultiVect<Type, Device> h) const {
        for (size_t j = 0; j <= k; ++j) {
            Vect<Type, Device> vj(v, mpg::ALL, j);
            Scalar<Type, Device> hjk = h(j, k);
            dot(w, vj, hjk);
            naxpy(hjk, vj, w);
        }
    }
};

template <class Type, class Device, size_t orth_steps>
class CGSR_Kernel {
    Vect<Type, Device> weights_;

public:
    CGSR_Kernel(size_t, size_t restart_length) : weights_(restart_length) {}

    void orthogonalize(MultiVect<Type, Device> v, const size_t k, Vect<Type, Device> w,
                       MultiVect<Type, Device> h) const {
        const auto cols = std::make_pair(size_t(0), k + 1);
        MultiVect<Type, Device> vk(v, mpg::ALL, cols);
        Vect<Type, Device> hk(h, cols, k);
        Vect<Type, Device> corr(weights_, cols);
        gemv(1.0, vk.transpose_matrix(), w, 0.0, hk);
        gemv(-1.0, vk, hk, 1.0, w);
        for (size_t pass = 1; pass < orth_steps; ++pass) {
            gemv(1.0, vk.transpose_matrix(), w, 0.0, corr);
            gemv(-1.0, vk, corr, 1.0, w);
            axpy(1.0, corr, hk);
        }
    }
};

}  // namespace Orthogonalization

#endif  // MPGMRES_ORTHOGONALIZATION_HPP
