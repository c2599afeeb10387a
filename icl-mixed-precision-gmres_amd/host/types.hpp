// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Kokkos-free data handles of the GMRES hot path.
//
// Mirrors the handle surface of the reference types.hpp:15-228 (Scalar,
// Vect, MultiVect: shallow, reference-counted aliases with sub-view
// constructors, column-major MultiVect with a `transposed` flag and an
// explicit leading dimension) without Kokkos: storage is a shared owner of a
// Device allocation plus pointer/extent/stride. Device allocations are
// zero-filled, as Kokkos views are.
//
// A Device tag provides:
//   static constexpr bool host_accessible;
//   static void* allocate(size_t bytes);           // zero-filled
//   static void  deallocate(void*);
//   static void  to_host(void* dst, const void* src, size_t bytes);
//   static void  to_device(void* dst, const void* src, size_t bytes);
//   static void  fence();                          // execution_space().fence()
#ifndef MPGMRES_TYPES_HPP
#define MPGMRES_TYPES_HPP

#include <cassert>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <utility>

namespace mpg {

// Stand-ins for Kokkos::ALL and Kokkos::pair in sub-view constructors.
struct all_t {};
constexpr all_t ALL{};
using range_t = std::pair<size_t, size_t>;

template <class A, class B>
inline range_t make_range(std::pair<A, B> p) {
    return range_t(static_cast<size_t>(p.first), static_cast<size_t>(p.second));
}

template <class Device>
std::shared_ptr<void> device_alloc(size_t bytes) {
    if (bytes == 0) return std::shared_ptr<void>();
    void* p = Device::allocate(bytes);
    return std::shared_ptr<void>(p, [](void* q) { Device::deallocate(q); });
}

// The Arnoldi steps of one restart cycle when nothing inside them reads the
// device (the driver's deferred |s(k+1)| path): a backend may record them once
// and replay the recording every later cycle. Generic form: run them as given.
template <class Device>
class CycleProgram {
public:
    explicit CycleProgram(bool /*counted*/ = true) {}
    template <class F>
    void run(F&& steps) {
        steps();
    }
};

}  // namespace mpg

template <class Type, class Device> class Vect;
template <class Type, class Device> class MultiVect;

// One element living in Device memory (types.hpp:15-55).
template <class Type, class Device>
class Scalar {
    std::shared_ptr<void> owner_;
    Type* ptr_ = nullptr;

public:
    Scalar() : owner_(mpg::device_alloc<Device>(sizeof(Type))), ptr_(static_cast<Type*>(owner_.get())) {}
    explicit Scalar(Type value) : Scalar() { Device::to_device(ptr_, &value, sizeof(Type)); }
    Scalar(const std::shared_ptr<void>& owner, Type* ptr) : owner_(owner), ptr_(ptr) {}
    Scalar(Vect<Type, Device> v, size_t i) : owner_(v.owner()), ptr_(v.data() + i) { assert(i < v.n()); }
    Scalar(MultiVect<Type, Device> m, size_t row, size_t col)
        : owner_(m.owner()), ptr_(m.data() + row + col * m.stride()) {
        assert(row < m.nrows_base() && col < m.ncols_base());
    }

    // Host read; a device->host copy when Device memory is not host visible
    // (types.hpp:39-46).
    Type access() const {
        if (Device::host_accessible) return *ptr_;
        Type v;
        Device::to_host(&v, ptr_, sizeof(Type));
        return v;
    }
    Type* data() const { return ptr_; }
    const std::shared_ptr<void>& owner() const { return owner_; }
};

// Contiguous 1-D vector (types.hpp:57-113).
template <class Type, class Device>
class Vect {
    std::shared_ptr<void> owner_;
    Type* ptr_ = nullptr;
    size_t n_ = 0;

public:
    Vect() = default;
    explicit Vect(size_t n)
        : owner_(mpg::device_alloc<Device>(n * sizeof(Type))), ptr_(static_cast<Type*>(owner_.get())), n_(n) {}
    Vect(const std::shared_ptr<void>& owner, Type* ptr, size_t n) : owner_(owner), ptr_(ptr), n_(n) {}

    // sub-range of a vector
    template <class A, class B>
    Vect(Vect v, std::pair<A, B> rows) : owner_(v.owner_) {
        mpg::range_t r = mpg::make_range(rows);
        assert(r.first <= r.second && r.second <= v.n_);
        ptr_ = v.ptr_ + r.first;
        n_ = r.second - r.first;
    }
    // whole column `col` of the underlying (untransposed) storage
    Vect(MultiVect<Type, Device> m, mpg::all_t, size_t col)
        : owner_(m.owner()), ptr_(m.data() + col * m.stride()), n_(m.nrows_base()) {
        assert(col < m.ncols_base());
    }
    // rows [first, second) of column `col`
    template <class A, class B>
    Vect(MultiVect<Type, Device> m, std::pair<A, B> rows, size_t col) : owner_(m.owner()) {
        mpg::range_t r = mpg::make_range(rows);
        assert(col < m.ncols_base() && r.second <= m.nrows_base());
        ptr_ = m.data() + col * m.stride() + r.first;
        n_ = r.second - r.first;
    }

    Scalar<Type, Device> operator()(size_t i) const { return Scalar<Type, Device>(*this, i); }
    template <class A, class B>
    Vect operator()(std::pair<A, B> rows) const { return Vect(*this, rows); }

    Type* data() const { return ptr_; }
    size_t n() const { return n_; }
    const std::shared_ptr<void>& owner() const { return owner_; }

    Type access(size_t i) const { return Scalar<Type, Device>(*this, i).access(); }
};

// Column-major 2-D block with leading dimension stride() (types.hpp:115-228).
// nrows()/ncols() are the logical (possibly transposed) extents;
// nrows_base()/ncols_base() those of the storage.
template <class Type, class Device>
class MultiVect {
    std::shared_ptr<void> owner_;
    Type* ptr_ = nullptr;
    size_t rows_ = 0, cols_ = 0, ld_ = 0;
    bool transposed_ = false;

    // Pad tall panels (the Krylov basis) to a 256-byte leading dimension so
    // every column starts on a 16-B granule boundary for vector loads.
    static size_t padded_ld(size_t m) {
        const size_t q = 256 / sizeof(Type);
        return m > q ? (m + q - 1) / q * q : m;
    }

public:
    MultiVect() = default;
    MultiVect(size_t m, size_t n) : rows_(m), cols_(n), ld_(padded_ld(m)) {
        owner_ = mpg::device_alloc<Device>(ld_ * n * sizeof(Type));
        ptr_ = static_cast<Type*>(owner_.get());
        if (ld_ == 0) ld_ = 1;
    }
    MultiVect(const std::shared_ptr<void>& owner, Type* ptr, size_t rows, size_t cols, size_t ld, bool tr)
        : owner_(owner), ptr_(ptr), rows_(rows), cols_(cols), ld_(ld), transposed_(tr) {}

    // logical row range, all logical columns
    template <class A, class B>
    MultiVect(MultiVect m, std::pair<A, B> rows, mpg::all_t) : MultiVect(m) {
        mpg::range_t r = mpg::make_range(rows);
        if (transposed_) select_cols(r); else select_rows(r);
        assert(nrows() == r.second - r.first && ncols() == m.ncols());
    }
    // all logical rows, logical column range
    template <class A, class B>
    MultiVect(MultiVect m, mpg::all_t, std::pair<A, B> cols) : MultiVect(m) {
        mpg::range_t c = mpg::make_range(cols);
        if (transposed_) select_rows(c); else select_cols(c);
        assert(ncols() == c.second - c.first && nrows() == m.nrows());
    }
    template <class A, class B, class C, class D>
    MultiVect(MultiVect m, std::pair<A, B> rows, std::pair<C, D> cols) : MultiVect(m) {
        mpg::range_t r = mpg::make_range(rows), c = mpg::make_range(cols);
        if (transposed_) { select_cols(r); select_rows(c); }
        else { select_rows(r); select_cols(c); }
        assert(nrows() == r.second - r.first && ncols() == c.second - c.first);
    }

    size_t nrows() const { return transposed_ ? cols_ : rows_; }
    size_t ncols() const { return transposed_ ? rows_ : cols_; }
    size_t nrows_base() const { return rows_; }
    size_t ncols_base() const { return cols_; }
    size_t n() const { return rows_; }
    size_t stride() const { return ld_; }
    bool transposed() const { return transposed_; }
    Type* data() const { return ptr_; }
    const std::shared_ptr<void>& owner() const { return owner_; }

    MultiVect transpose_matrix() const { return MultiVect(owner_, ptr_, rows_, cols_, ld_, !transposed_); }

    Scalar<Type, Device> operator()(size_t i, size_t j) const {
        return transposed_ ? Scalar<Type, Device>(*this, j, i) : Scalar<Type, Device>(*this, i, j);
    }
    template <class A, class B>
    Vect<Type, Device> operator()(std::pair<A, B> rows, size_t col) const {
        return Vect<Type, Device>(*this, rows, col);
    }

private:
    void select_rows(mpg::range_t r) {
        assert(r.first <= r.second && r.second <= rows_);
        ptr_ += r.first;
        rows_ = r.second - r.first;
    }
    void select_cols(mpg::range_t c) {
        assert(c.first <= c.second && c.second <= cols_);
        ptr_ += c.first * ld_;
        cols_ = c.second - c.first;
    }
};

// Preconditioner interface (types.hpp:230-237).
template <class Type, class Device>
class LinearOperator {
public:
    virtual ~LinearOperator() {}
    virtual void apply(Vect<Type, Device> rhs) = 0;
};

// Device-specialised CSR matrix (types_mkl.hpp:17-107, types_cuda.hpp:47-152).
template <class Type, class Device>
class SparseMatrix {};

// Device-specialised ILU(0) factors and their Jacobi-sweep variant
// (types.hpp:243-372; types_mkl.hpp:110-240; types_cuda.hpp:155-260).
template <class Type, class Device>
class ILU {};
template <class Type, class Device>
class ILU_Jacobi {};

// M = I (types.hpp:374-378).
template <class Type, class Device>
class Identity : public LinearOperator<Type, Device> {
public:
    void apply(Vect<Type, Device>) override {}
};

#endif  // MPGMRES_TYPES_HPP
