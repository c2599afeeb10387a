#include "fused_gmres.hpp"

#include <stdexcept>

namespace mpg {
int solve_fused(const mpg_solve_args&, mpg_solve_result*) {
    throw std::invalid_argument("fused engine not built yet");
}
}  // namespace mpg
