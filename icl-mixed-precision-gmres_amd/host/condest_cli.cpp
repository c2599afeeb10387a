// Command-line condition-number estimator with the reference's flags and
// stdout lines (condest.cpp:181-227), on MI355X through mpg_condest.
//
// Reference flags: --Apath --rand --gpu --max-iters. The reference runs only
// with --gpu and otherwise prints "CPU not currently supported"; this build
// does the same. Additions: --matrix SPEC (synthetic input instead of
// --Apath, mpg_gen_spec), --device D.
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "mpgmres/condest.h"
#include "mpgmres/problems.h"

int main(int argc, char* argv[]) {
    const char* a_path = nullptr;
    const char* synthetic = nullptr;
    int rand_seed = 42;
    bool use_gpu = false;
    long long max_iters = 100000;
    int device = 0;

    for (int i = 1; i < argc; i++) {
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::cout << "Missing value for " << argv[i] << std::endl;
                std::exit(1);
            }
            return argv[++i];
        };
        if (std::strcmp("--Apath", argv[i]) == 0) a_path = next();
        else if (std::strcmp("--rand", argv[i]) == 0) rand_seed = std::stoi(next());
        else if (std::strcmp("--gpu", argv[i]) == 0) use_gpu = true;
        else if (std::strcmp("--max-iters", argv[i]) == 0) max_iters = std::stoll(next());
        else if (std::strcmp("--matrix", argv[i]) == 0) synthetic = next();
        else if (std::strcmp("--device", argv[i]) == 0) device = std::stoi(next());
        else {
            std::cout << "Unknown flag" << argv[i] << std::endl;
            return 1;
        }
    }
    if (a_path == nullptr && synthetic == nullptr) {
        std::cout << "No value suplied for A" << std::endl;
        return 1;
    }

    mpg_host_csr A{};
    char err[256];
    if (a_path ? mpg_load_mtx(a_path, &A, err, sizeof err) : mpg_gen_spec(synthetic, &A, err, sizeof err)) {
        std::cerr << err << std::endl;
        return 1;
    }
    if (!use_gpu) {
        std::cout << "CPU not currently supported" << std::endl;
        mpg_host_csr_free(&A);
        return 0;
    }
    if (A.nrows != A.ncols) {
        std::cerr << "condest needs a square matrix" << std::endl;
        mpg_host_csr_free(&A);
        return 1;
    }
    mpg_condest_args a{};
    a.n = (int32_t)A.nrows;
    a.nnz = A.nnz;
    a.rowptr = A.rowptr;
    a.col = A.col;
    a.val = A.val;
    a.rand_seed = rand_seed;
    a.max_iters = max_iters;
    a.verbose = 1;
    a.device = device;
    mpg_condest_result r{};
    const int st = mpg_condest(&a, &r);
    mpg_host_csr_free(&A);
    if (st != 0) {
        std::cerr << "mpg_condest failed: " << r.message << std::endl;
        return 1;
    }
    return 0;
}
