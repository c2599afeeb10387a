// fp32-accumulation build of the fused Arnoldi phases (mpg_arnoldi_set_accum,
// include/mpgmres/arnoldi.h): the launch code of arnoldi_launch.hpp with A =
// float, for the fp32-Arnoldi type combinations (single, mixed, mixed-half).
// Its own translation unit, so it compiles beside arnoldi.hip.
#include "arnoldi_launch.hpp"

namespace mpg_acc32 {
int reduce(mpg_arnoldi* a, int ncols) { return reduce_run<float>(a, ncols); }
int spmv(mpg_arnoldi* a, int k, int fold, bool dots) { return spmv_run<float>(a, k, fold, dots); }
int dots(mpg_arnoldi* a, int k, bool combine) { return dots_run<float>(a, k, combine); }
int cgs(mpg_arnoldi* a, int k, int pass, bool givens, bool from_partials, bool no_next) {
    return cgs_run<float>(a, k, pass, givens, from_partials, no_next);
}
int mgs(mpg_arnoldi* a, int k, int j, bool from_partials) { return mgs_run<float>(a, k, j, from_partials); }
int givens(mpg_arnoldi* a, int k, bool from_partials) { return givens_run<float>(a, k, from_partials); }
int update(mpg_arnoldi* a, int k) { return update_run<float>(a, k); }
}  // namespace mpg_acc32
