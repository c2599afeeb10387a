// Givens operators and the scalar program (mpg_scalar_program) as device
// code shared by its own one-wave kernel (blas1.hip) and the SELL SpMV,
// which can run a program in one extra workgroup of its launch (sell.hip).
#pragma once

#include "internal.hpp"
#include "mpgmres/capi.h"

namespace mpg {

// ---------------- Givens (single lane; O(1)/O(k) scalar work) ----------------
// Exact IEEE order: products rounded separately, no FMA contraction, so the
// results equal the reference BLAS formulas evaluated in T.
#pragma clang fp contract(off)
template <class T>
__device__ void rotg_dev(T* a, T* b, T* c, T* s) {
    // Reference BLAS xROTG (classic netlib form), then b := 0
    // (kernels_mkl.cpp:214-226 zeroes b after cblas_?rotg).
    T av = *a, bv = *b;
    T roe = fabs(av) > fabs(bv) ? av : bv;
    T scale = fabs(av) + fabs(bv);
    T cc, ss, r;
    if (scale == T(0)) {
        cc = T(1); ss = T(0); r = T(0);
    } else {
        T as = av / scale, bs = bv / scale;
        r = scale * sqrt(as * as + bs * bs);
        r = roe >= T(0) ? r : -r;
        cc = av / r;
        ss = bv / r;
    }
    *a = r;
    *b = T(0);
    *c = cc;
    *s = ss;
}

template <class T>
__device__ void rot_pair(T* a, T* b, T c, T s) {
    T a1 = *a, a2 = *b;
    *a = c * a1 + s * a2;
    *b = c * a2 - s * a1;
}
#pragma clang fp contract(on)

// A scalar program in call order with the single-operator kernels'
// arithmetic, on one wave: lane 0 runs every operator; a rot_vec first
// stages its column and rotations in LDS with all 64 lanes (one memory
// latency instead of one per rotation: the chain stores a[j+1] before it
// loads it back), rotates there, and writes the column back with all lanes.
struct ScalarProgram {
    mpg_scalar_op ops[MPG_SCALAR_PROGRAM_MAX];
    int count;
};

// the wave's earlier stores (LDS and global) before its later loads: the
// program runs on one wave, in a workgroup that may hold other waves
__device__ __forceinline__ void program_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// STAGE: rotations staged in LDS per pass (lds: 3 STAGE + 1 elements of T)
template <int STAGE, class T>
__device__ void scalar_op(const mpg_scalar_op& o, T* lds) {
    T* p0 = static_cast<T*>(o.p[0]);
    T* p1 = static_cast<T*>(o.p[1]);
    T* p2 = static_cast<T*>(o.p[2]);
    T* p3 = static_cast<T*>(o.p[3]);
    const int lane = threadIdx.x & (kWave - 1);
    if (o.op == MPG_SOP_ROT_VEC) {
        // the column a[0..k] and c, s never overlap in the drivers; if they
        // do, run the chain from memory like k_rot_vec
        const bool disjoint = (p0 + o.k + 1 <= p2 || p2 + o.k <= p0) && (p0 + o.k + 1 <= p3 || p3 + o.k <= p0);
        if (!disjoint) {
            if (lane == 0)
                for (int j = 0; j < o.k; ++j) rot_pair(p0 + j, p0 + j + 1, p2[j], p3[j]);
            program_sync();
            return;
        }
        T* la = lds;
        T* lc = lds + STAGE + 1;
        T* ls = lc + STAGE;
        for (int j0 = 0; j0 < o.k; j0 += STAGE) {
            const int kk = o.k - j0 < STAGE ? o.k - j0 : STAGE;
            for (int j = lane; j <= kk; j += kWave) la[j] = p0[j0 + j];
            for (int j = lane; j < kk; j += kWave) {
                lc[j] = p2[j0 + j];
                ls[j] = p3[j0 + j];
            }
            program_sync();
            if (lane == 0)
                for (int j = 0; j < kk; ++j) rot_pair(la + j, la + j + 1, lc[j], ls[j]);
            program_sync();
            for (int j = lane; j <= kk; j += kWave) p0[j0 + j] = la[j];
            program_sync();
        }
        return;
    }
    if (lane == 0) {
        switch (o.op) {
            case MPG_SOP_ROTG: rotg_dev(p0, p1, p2, p3); break;
            case MPG_SOP_ROT: rot_pair(p0, p1, *p2, *p3); break;
            case MPG_SOP_COPY: *p1 = *p0; break;
            case MPG_SOP_SCAL: *p1 = T(o.alpha) * *p0; break;
            case MPG_SOP_SCAL_DEV: *p1 = *p2 * *p0; break;
            default: break;
        }
    }
    program_sync();
}

// the whole program on the calling wave (lds: 3 STAGE + 1 doubles)
template <int STAGE>
__device__ void run_scalar_program(const ScalarProgram& prog, double* lds) {
    for (int i = 0; i < prog.count; ++i) {
        if (prog.ops[i].f64) scalar_op<STAGE, double>(prog.ops[i], lds);
        else scalar_op<STAGE, float>(prog.ops[i], reinterpret_cast<float*>(lds));
    }
}

// validate and copy a program (MPG_ERR_ARG on a bad count or opcode)
inline int make_scalar_program(const mpg_scalar_op* ops, int count, ScalarProgram& prog) {
    if (count < 0 || count > MPG_SCALAR_PROGRAM_MAX || (count && !ops)) return MPG_ERR_ARG;
    prog = ScalarProgram{};
    for (int i = 0; i < count; ++i) {
        if (ops[i].op < MPG_SOP_ROTG || ops[i].op > MPG_SOP_SCAL_DEV) return MPG_ERR_ARG;
        prog.ops[i] = ops[i];
    }
    prog.count = count;
    return MPG_OK;
}

}  // namespace mpg
