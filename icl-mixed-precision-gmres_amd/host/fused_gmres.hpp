// Fused Arnoldi engine (see fused_gmres.cpp).
#ifndef MPGMRES_FUSED_GMRES_HPP
#define MPGMRES_FUSED_GMRES_HPP

#include "mpgmres/solve.h"

namespace mpg {
int solve_fused(const mpg_solve_args& args, mpg_solve_result* result);
}  // namespace mpg

#endif  // MPGMRES_FUSED_GMRES_HPP
