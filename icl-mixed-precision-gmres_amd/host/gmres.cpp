// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Explicit instantiations of the GMRES drivers for the Hip backend —
// the counterpart of CREATE_TEST_CONFIGS(MKL) / (Cuda) in the reference
// (gmres.cpp:306-360): {CGS, MGS, CGSR(2)} x {double/double baseline,
// double/float single-prec, float/float single, mixed}.
#include "gmres.hpp"

#include <fstream>

#include "kernels.hpp"
#include "types_hip.hpp"

namespace mpg {
namespace {
bool g_quiet = false;
struct NullBuf : std::streambuf {
    int overflow(int c) override { return c; }
};
NullBuf g_null_buf;
std::ostream g_null(&g_null_buf);
}  // namespace
std::ostream& out() { return g_quiet ? g_null : std::cout; }
void set_quiet(bool q) { g_quiet = q; }
}  // namespace mpg

using namespace Orthogonalization;

#define MPG_BASELINE(DEV, KERNEL, T, P)                                                                  \
    template void gmres_baseline<GS<T, KERNEL, DEV>, DEV, T, P>(Convergence<T, DEV>&, SparseMatrix<T, DEV>, \
                                                                LinearOperator<P, DEV>*, Vect<T, DEV>,  \
                                                                Vect<T, DEV>);
#define MPG_MIXED(DEV, KERNEL)                                                                        \
    template void gmres_singleUpdate<GS<float, KERNEL, DEV>, DEV>(                                    \
        Convergence<float, DEV>&, SparseMatrix<double, DEV>, SparseMatrix<float, DEV>,               \
        LinearOperator<float, DEV>*, Vect<double, DEV>, Vect<double, DEV>);

#define MPG_ORTH_CONFIGS(DEV, KD, KS) \
    MPG_BASELINE(DEV, KD, double, double) \
    MPG_BASELINE(DEV, KD, double, float)  \
    MPG_BASELINE(DEV, KS, float, float)   \
    MPG_MIXED(DEV, KS)

namespace {
using CgsD = CGS_Kernel<double, Hip>;
using CgsS = CGS_Kernel<float, Hip>;
using MgsD = MGS_Kernel<double, Hip>;
using MgsS = MGS_Kernel<float, Hip>;
using CgsrD = CGSR_Kernel<double, Hip, 2>;
using CgsrS = CGSR_Kernel<float, Hip, 2>;
}  // namespace

MPG_ORTH_CONFIGS(Hip, CgsD, CgsS)
MPG_ORTH_CONFIGS(Hip, MgsD, MgsS)
MPG_ORTH_CONFIGS(Hip, CgsrD, CgsrS)
