// Restarted GMRES(m) drivers (reference gmres.hpp:14-57, gmres.cpp:24-303).
//
//  gmres_baseline<Orth, Device, Type, PrecType>
//      everything in Type; the preconditioner may run in PrecType through a
//      cast wrapper (gmres.cpp:12-22). Modes: baseline (double,double),
//      single-prec (double,float), single (float,float).
//  gmres_singleUpdate<Orth, Device>
//      mixed precision: true residual r = b - A x and the update x += V y
//      in fp64, the Arnoldi cycle (SpMV, Gram-Schmidt, Givens) in fp32.
//
// The drivers are templates over the Device, so they are "driven
// unchanged" by any backend that specialises kernels.hpp; instantiations for
// Hip live in gmres.cpp.
#ifndef MPGMRES_GMRES_HPP
#define MPGMRES_GMRES_HPP

#include <iostream>
#include <utility>

#include "IterUtil.hpp"
#include "types.hpp"

namespace mpg {
// Stream the drivers print their progress lines to (std::cout unless
// silenced); the lines are those of gmres.cpp:73-77 / 186-190.
std::ostream& out();
void set_quiet(bool quiet);
}  // namespace mpg

template <class Orth, class Device, class Type, class PrecType>
void gmres_baseline(Convergence<Type, Device>& convergence, SparseMatrix<Type, Device> A,
                    LinearOperator<PrecType, Device>* M, Vect<Type, Device> b, Vect<Type, Device> x);

template <class Orth, class Device>
void gmres_singleUpdate(Convergence<float, Device>& convergence, SparseMatrix<double, Device> A,
                        SparseMatrix<float, Device> A_single, LinearOperator<float, Device>* M,
                        Vect<double, Device> b, Vect<double, Device> x);

// x_hi += V(:,0:k) * (H(0:k,0:k)^-1 s(0:k)) with a low-precision basis
template <class Orth, class Device>
void solution_update(Orth& orth, Vect<double, Device>& x, const size_t k, const MultiVect<float, Device> h,
                     const Vect<float, Device> s, Vect<float, Device> x_inc_temp, Vect<double, Device> x_temp);

// x += V(:,0:k) * (H(0:k,0:k)^-1 s(0:k)) in one precision
template <class Orth, class Device, class Type>
void solution_update(Orth& orth, Vect<Type, Device>& x, const size_t k, const MultiVect<Type, Device> h,
                     const Vect<Type, Device> s);

#include "gmres_impl.hpp"

#endif  // MPGMRES_GMRES_HPP
