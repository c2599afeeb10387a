// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Host-side problem construction (include/mpgmres/problems.h).
#include "mpgmres/problems.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

namespace {

template <class T>
T* dup_array(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(std::max<size_t>(1, v.size()) * sizeof(T)));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

int emit(mpg_host_csr* out, int32_t nrows, int32_t ncols, const std::vector<int32_t>& rp,
         const std::vector<int32_t>& ci, const std::vector<double>& va) {
    out->nrows = nrows;
    out->ncols = ncols;
    out->nnz = (int64_t)ci.size();
    out->rowptr = dup_array(rp);
    out->col = dup_array(ci);
    out->val = dup_array(va);
    if (!out->rowptr || !out->col || !out->val) {
        mpg_host_csr_free(out);
        return -3;
    }
    return 0;
}

// splitmix64 finaliser: a counter-based stream, so any row slice of a band
// matrix can be generated independently (weak-scaling partitions).
inline uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
inline double unit_double(uint64_t seed, int64_t row, int32_t off) {
    uint64_t key = mix64(seed ^ mix64((uint64_t)row * 64u + (uint64_t)(off + 32)));
    return (double)(key >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
}

void set_err(char* err, int errlen, const std::string& msg) {
    if (err && errlen > 0) {
        std::strncpy(err, msg.c_str(), (size_t)errlen - 1);
        err[errlen - 1] = '\0';
    }
}

// Minimal Matrix Market banner / size parsing (NIST format).
struct MMHeader {
    bool coordinate = false, array = false;
    bool real = false, integer = false, pattern = false, complex_ = false;
    bool general = false, symmetric = false;
};

bool read_banner(FILE* f, MMHeader& h, std::string& why) {
    char line[1025];
    if (!std::fgets(line, sizeof line, f)) { why = "Missing values in banner"; return false; }
    char banner[64], object[64], format[64], field[64], symm[64];
    if (std::sscanf(line, "%63s %63s %63s %63s %63s", banner, object, format, field, symm) != 5) {
        why = "Missing values in banner";
        return false;
    }
    auto lower = [](char* s) { for (; *s; ++s) *s = (char)std::tolower((unsigned char)*s); };
    lower(object); lower(format); lower(field); lower(symm);
    if (std::strcmp(banner, "%%MatrixMarket") != 0) { why = "Banner is missing"; return false; }
    if (std::strcmp(object, "matrix") != 0) { why = "Unrecognized description"; return false; }
    h.coordinate = !std::strcmp(format, "coordinate");
    h.array = !std::strcmp(format, "array");
    h.real = !std::strcmp(field, "real") || !std::strcmp(field, "double");
    h.integer = !std::strcmp(field, "integer");
    h.pattern = !std::strcmp(field, "pattern");
    h.complex_ = !std::strcmp(field, "complex");
    h.general = !std::strcmp(symm, "general");
    h.symmetric = !std::strcmp(symm, "symmetric");
    if (!(h.coordinate || h.array) || !(h.real || h.integer || h.pattern || h.complex_) ||
        !(h.general || h.symmetric || !std::strcmp(symm, "skew-symmetric") || !std::strcmp(symm, "hermitian"))) {
        why = "Unrecognized description";
        return false;
    }
    return true;
}

// skip comment lines, return the first data line
bool next_data_line(FILE* f, char* buf, int len) {
    while (std::fgets(buf, len, f)) {
        if (buf[0] == '%') continue;
        bool blank = true;
        for (char* p = buf; *p; ++p)
            if (!std::isspace((unsigned char)*p)) { blank = false; break; }
        if (!blank) return true;
    }
    return false;
}

}  // namespace

extern "C" {

void mpg_host_csr_free(mpg_host_csr* a) {
    if (!a) return;
    std::free(a->rowptr);
    std::free(a->col);
    std::free(a->val);
    a->rowptr = nullptr;
    a->col = nullptr;
    a->val = nullptr;
    a->nnz = 0;
}

int mpg_gen_band(int64_t n, int32_t lo, int32_t hi, uint64_t seed, int64_t row_begin, int64_t row_end,
                 mpg_host_csr* out) {
    if (!out || n <= 0 || n > INT32_MAX || lo < 0 || hi < 0 || lo > 31 || hi > 31 || row_begin < 0 ||
        row_end > n || row_begin > row_end)
        return -2;
    const int64_t rows = row_end - row_begin;
    std::vector<int32_t> rp((size_t)rows + 1), ci;
    std::vector<double> va;
    ci.reserve((size_t)rows * (lo + hi + 1));
    va.reserve((size_t)rows * (lo + hi + 1));
    for (int64_t r = 0; r < rows; ++r) {
        const int64_t i = row_begin + r;
        rp[(size_t)r] = (int32_t)ci.size();
        double offsum = 0.0;
        size_t diag_slot = 0;
        for (int32_t d = -lo; d <= hi; ++d) {
            const int64_t c = i + d;
            if (c < 0 || c >= n) continue;
            ci.push_back((int32_t)c);
            if (d == 0) {
                diag_slot = va.size();
                va.push_back(0.0);
            } else {
                const double v = -unit_double(seed, i, d);
                offsum += std::fabs(v);
                va.push_back(v);
            }
        }
        va[diag_slot] = 1.0 + offsum;
    }
    rp[(size_t)rows] = (int32_t)ci.size();
    if (ci.size() > (size_t)INT32_MAX) return -2;
    return emit(out, (int32_t)rows, (int32_t)n, rp, ci, va);
}

int mpg_gen_laplace3d(int32_t nx, int32_t ny, int32_t nz, mpg_host_csr* out) {
    if (!out || nx <= 0 || ny <= 0 || nz <= 0) return -2;
    const int64_t n = (int64_t)nx * ny * nz;
    if (n > INT32_MAX / 7) return -2;
    std::vector<int32_t> rp((size_t)n + 1), ci;
    std::vector<double> va;
    ci.reserve((size_t)n * 7);
    va.reserve((size_t)n * 7);
    for (int32_t z = 0; z < nz; ++z)
        for (int32_t y = 0; y < ny; ++y)
            for (int32_t x = 0; x < nx; ++x) {
                const int64_t i = x + (int64_t)nx * (y + (int64_t)ny * z);
                rp[(size_t)i] = (int32_t)ci.size();
                auto add = [&](int64_t c, double v) {
                    ci.push_back((int32_t)c);
                    va.push_back(v);
                };
                if (z > 0) add(i - (int64_t)nx * ny, -1.0);
                if (y > 0) add(i - nx, -1.0);
                if (x > 0) add(i - 1, -1.0);
                add(i, 6.0);
                if (x + 1 < nx) add(i + 1, -1.0);
                if (y + 1 < ny) add(i + nx, -1.0);
                if (z + 1 < nz) add(i + (int64_t)nx * ny, -1.0);
            }
    rp[(size_t)n] = (int32_t)ci.size();
    return emit(out, (int32_t)n, (int32_t)n, rp, ci, va);
}

int mpg_gen_stencil27(int32_t nx, int32_t ny, int32_t nz, int32_t dof, uint64_t seed, mpg_host_csr* out) {
    if (!out || nx <= 0 || ny <= 0 || nz <= 0 || dof <= 0 || dof > 8) return -2;
    const int64_t nodes = (int64_t)nx * ny * nz, n = nodes * dof;
    if (n > INT32_MAX || n * 27 * dof > INT32_MAX) return -2;
    std::vector<int32_t> rp((size_t)n + 1), ci;
    std::vector<double> va;
    ci.reserve((size_t)n * 27 * dof);
    va.reserve((size_t)n * 27 * dof);
    for (int32_t z = 0; z < nz; ++z)
        for (int32_t y = 0; y < ny; ++y)
            for (int32_t x = 0; x < nx; ++x) {
                const int64_t node = x + (int64_t)nx * (y + (int64_t)ny * z);
                for (int32_t d = 0; d < dof; ++d) {
                    const int64_t i = node * dof + d;
                    rp[(size_t)i] = (int32_t)ci.size();
                    double offsum = 0.0;
                    size_t diag_slot = 0;
                    // neighbours in lexicographic order (z, y, x), so columns come sorted
                    for (int dz = -1; dz <= 1; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                const int32_t X = x + dx, Y = y + dy, Z = z + dz;
                                if (X < 0 || X >= nx || Y < 0 || Y >= ny || Z < 0 || Z >= nz) continue;
                                const int64_t nb = X + (int64_t)nx * (Y + (int64_t)ny * Z);
                                for (int32_t e = 0; e < dof; ++e) {
                                    const int64_t c = nb * dof + e;
                                    ci.push_back((int32_t)c);
                                    if (c == i) {
                                        diag_slot = va.size();
                                        va.push_back(0.0);
                                    } else {  // symmetric: keyed on the unordered pair
                                        const int64_t a = std::min(i, c), b = std::max(i, c);
                                        const double v = -unit_double(seed ^ (uint64_t)b, a, 0);
                                        offsum += std::fabs(v);
                                        va.push_back(v);
                                    }
                                }
                            }
                    va[diag_slot] = 1.0 + offsum;
                }
            }
    rp[(size_t)n] = (int32_t)ci.size();
    return emit(out, (int32_t)n, (int32_t)n, rp, ci, va);
}

int mpg_gen_fem27(int32_t nx, int32_t ny, int32_t nz, int32_t dof, int32_t keep_pct, uint64_t seed,
                  mpg_host_csr* out) {
    if (!out || nx <= 0 || ny <= 0 || nz <= 0 || dof <= 0 || dof > 8 || keep_pct < 0 || keep_pct > 100) return -2;
    const int64_t nodes = (int64_t)nx * ny * nz, n = nodes * dof;
    if (n > INT32_MAX || n * 27 * dof > INT32_MAX) return -2;
    // an undirected node pair {a, b} is coupled when its hash falls under
    // keep_pct %: the same decision from both ends, so the pattern (and, with
    // the values keyed on the unordered unknown pair, A) is symmetric
    auto kept = [&](int64_t a, int64_t b) {
        if (a == b) return true;
        const int64_t lo = std::min(a, b), hi = std::max(a, b);
        return mix64(seed * 0x2545f4914f6cdd1dULL ^ mix64((uint64_t)lo * 0x9e3779b97f4a7c15ULL + (uint64_t)hi)) % 100 <
               (uint64_t)keep_pct;
    };
    std::vector<int32_t> rp((size_t)n + 1), ci;
    std::vector<double> va;
    ci.reserve((size_t)(n * 27 * dof * (keep_pct + 5) / 100));
    va.reserve(ci.capacity());
    for (int32_t z = 0; z < nz; ++z)
        for (int32_t y = 0; y < ny; ++y)
            for (int32_t x = 0; x < nx; ++x) {
                const int64_t node = x + (int64_t)nx * (y + (int64_t)ny * z);
                for (int32_t d = 0; d < dof; ++d) {
                    const int64_t i = node * dof + d;
                    rp[(size_t)i] = (int32_t)ci.size();
                    double offsum = 0.0;
                    size_t diag_slot = 0;
                    for (int dz = -1; dz <= 1; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                const int32_t X = x + dx, Y = y + dy, Z = z + dz;
                                if (X < 0 || X >= nx || Y < 0 || Y >= ny || Z < 0 || Z >= nz) continue;
                                const int64_t nb = X + (int64_t)nx * (Y + (int64_t)ny * Z);
                                if (!kept(node, nb)) continue;
                                for (int32_t e = 0; e < dof; ++e) {
                                    const int64_t c = nb * dof + e;
                                    ci.push_back((int32_t)c);
                                    if (c == i) {
                                        diag_slot = va.size();
                                        va.push_back(0.0);
                                    } else {
                                        const int64_t a = std::min(i, c), b = std::max(i, c);
                                        const double v = -unit_double(seed ^ (uint64_t)b, a, 0);
                                        offsum += std::fabs(v);
                                        va.push_back(v);
                                    }
                                }
                            }
                    va[diag_slot] = 1.0 + offsum;
                }
            }
    rp[(size_t)n] = (int32_t)ci.size();
    return emit(out, (int32_t)n, (int32_t)n, rp, ci, va);
}

int mpg_perm_node_blocks(int64_t nodes, int32_t dof, int32_t block, uint64_t seed, int32_t* perm) {
    if (nodes <= 0 || dof <= 0 || block <= 0 || !perm || nodes * dof > INT32_MAX) return -2;
    const int64_t nb = (nodes + block - 1) / block;
    std::mt19937_64 rng(seed);
    std::vector<int64_t> order((size_t)nb);
    std::iota(order.begin(), order.end(), 0);
    std::shuffle(order.begin(), order.end(), rng);  // block q goes to position pos[q]
    std::vector<int64_t> pos((size_t)nb);
    for (int64_t p = 0; p < nb; ++p) pos[(size_t)order[(size_t)p]] = p;
    // new node positions: the blocks in shuffled order, each block's nodes
    // shuffled inside it (the last, short block keeps its size wherever it lands)
    std::vector<int64_t> start((size_t)nb + 1, 0);
    for (int64_t p = 0; p < nb; ++p) {
        const int64_t q = order[(size_t)p];
        start[(size_t)p + 1] = start[(size_t)p] + std::min<int64_t>(block, nodes - q * block);
    }
    std::vector<int64_t> inner((size_t)block);
    for (int64_t q = 0; q < nb; ++q) {
        const int64_t len = std::min<int64_t>(block, nodes - q * block);
        std::iota(inner.begin(), inner.begin() + len, 0);
        std::shuffle(inner.begin(), inner.begin() + len, rng);
        for (int64_t t = 0; t < len; ++t) {
            const int64_t old_node = q * block + t, new_node = start[(size_t)pos[(size_t)q]] + inner[(size_t)t];
            for (int32_t d = 0; d < dof; ++d) perm[old_node * dof + d] = (int32_t)(new_node * dof + d);
        }
    }
    return 0;
}

int mpg_csr_permute_sym(const mpg_host_csr* a, const int32_t* perm, mpg_host_csr* out) {
    if (!a || !perm || !out || a->nrows != a->ncols || a->nrows < 0) return -2;
    const int64_t n = a->nrows;
    std::vector<int32_t> inv((size_t)n, -1);
    for (int64_t i = 0; i < n; ++i) {
        if (perm[i] < 0 || perm[i] >= n || inv[(size_t)perm[i]] >= 0) return -2;  // not a permutation
        inv[(size_t)perm[i]] = (int32_t)i;
    }
    std::vector<int32_t> rp((size_t)n + 1, 0), ci((size_t)a->nnz);
    std::vector<double> va((size_t)a->nnz);
    for (int64_t r = 0; r < n; ++r) {
        const int32_t i = inv[(size_t)r];
        rp[(size_t)r + 1] = rp[(size_t)r] + (a->rowptr[i + 1] - a->rowptr[i]);
    }
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t r = 0; r < n; ++r) {
        const int32_t i = inv[(size_t)r];
        row.clear();
        for (int32_t e = a->rowptr[i]; e < a->rowptr[i + 1]; ++e) row.emplace_back(perm[a->col[e]], a->val[e]);
        // each row sorted by column (LoadMatrix.hpp:128-145 semantics; stable for duplicates)
        std::stable_sort(row.begin(), row.end(), [](const auto& u, const auto& v) { return u.first < v.first; });
        for (size_t t = 0; t < row.size(); ++t) {
            ci[(size_t)rp[(size_t)r] + t] = row[t].first;
            va[(size_t)rp[(size_t)r] + t] = row[t].second;
        }
    }
    return emit(out, (int32_t)n, (int32_t)n, rp, ci, va);
}

int mpg_gen_spec(const char* spec, mpg_host_csr* out, char* err, int errlen) {
    auto fail = [&](const char* what) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", what);
        return -2;
    };
    if (!spec || !out) return fail("null argument");
    std::vector<std::string> f;
    std::string s(spec);
    for (size_t p = 0;;) {
        const size_t q = s.find(':', p);
        f.push_back(s.substr(p, q == std::string::npos ? std::string::npos : q - p));
        if (q == std::string::npos) break;
        p = q + 1;
    }
    auto num = [&](size_t i, long long def) { return f.size() > i ? std::atoll(f[i].c_str()) : def; };
    if (f[0] == "band" && f.size() >= 2) {
        const long long n = num(1, 0);
        if (mpg_gen_band(n, (int)num(2, 5), (int)num(3, 4), (uint64_t)num(4, 7), 0, n, out) != 0)
            return fail("bad band spec");
        return 0;
    }
    if (f[0] == "laplace" && f.size() >= 2) {
        const int nx = (int)num(1, 0);
        if (mpg_gen_laplace3d(nx, (int)num(2, nx), (int)num(3, nx), out) != 0) return fail("bad laplace spec");
        return 0;
    }
    if (f[0] == "stencil27" && f.size() >= 2) {
        const int nx = (int)num(1, 0);
        if (mpg_gen_stencil27(nx, nx, nx, (int)num(2, 3), (uint64_t)num(3, 11), out) != 0)
            return fail("bad stencil27 spec");
        return 0;
    }
    // stencil27p / fem27: the irregular stand-ins (a symmetric permutation of
    // node blocks; a randomly thinned 27-point coupling with variable rows)
    auto permute = [&](long long block, long long pseed, int dof) {
        if (block <= 0) return 0;
        const int64_t n = out->nrows;
        std::vector<int32_t> perm((size_t)n);
        if (mpg_perm_node_blocks(n / dof, dof, (int32_t)block, (uint64_t)pseed, perm.data()) != 0) return -2;
        mpg_host_csr b{};
        const int st = mpg_csr_permute_sym(out, perm.data(), &b);
        mpg_host_csr_free(out);
        *out = b;
        return st;
    };
    if (f[0] == "stencil27p" && f.size() >= 2) {
        const int nx = (int)num(1, 0), dof = (int)num(2, 3);
        if (mpg_gen_stencil27(nx, nx, nx, dof, (uint64_t)num(3, 11), out) != 0 ||
            permute(num(4, 64), num(5, 5), dof) != 0)
            return fail("bad stencil27p spec");
        return 0;
    }
    if (f[0] == "fem27" && f.size() >= 2) {
        const int nx = (int)num(1, 0), dof = (int)num(2, 3);
        if (mpg_gen_fem27(nx, nx, nx, dof, (int)num(3, 70), (uint64_t)num(4, 13), out) != 0 ||
            permute(num(5, 0), num(6, 5), dof) != 0)
            return fail("bad fem27 spec");
        return 0;
    }
    return fail("unknown --matrix spec (band:N[:LO:HI[:SEED]], laplace:NX[:NY:NZ], stencil27:NX[:DOF[:SEED]], "
                "stencil27p:NX[:DOF[:SEED[:BLOCK[:PSEED]]]] or fem27:NX[:DOF[:KEEP%[:SEED[:BLOCK[:PSEED]]]]])");
}

int mpg_load_mtx(const char* path, mpg_host_csr* out, char* err, int errlen) {
    if (!out || !path) return -2;
    FILE* f = std::fopen(path, "r");
    if (!f) { set_err(err, errlen, "Could not access file"); return -2; }
    MMHeader h;
    std::string why;
    if (!read_banner(f, h, why)) { std::fclose(f); set_err(err, errlen, why); return -2; }
    char line[1025];
    long M = 0, N = 0, L = 0;
    // mm_read_mtx_crd_size (mmio.c:189-217, which LoadMatrix.hpp:44 calls):
    // the first non-comment line, or, when it does not hold three integers,
    // whatever fscanf("%d %d %d") finds further on (an array file's "M N"
    // line then reads on into its values and fails the type check below,
    // as in the reference)
    bool size_ok = false;
    if (std::fgets(line, sizeof line, f)) {
        while (line[0] == '%' && std::fgets(line, sizeof line, f)) {
        }
        if (line[0] != '%') {
            if (std::sscanf(line, "%ld %ld %ld", &M, &N, &L) == 3) {
                size_ok = true;
            } else {
                // (a token that is not a number matches nothing and is never
                // consumed: mmio.c loops forever there, this stops)
                int got;
                do got = std::fscanf(f, "%ld %ld %ld", &M, &N, &L);
                while (got != EOF && got != 3 && got != 0);
                size_ok = got == 3;
            }
        }
    }
    if (!size_ok) {
        std::fclose(f);
        set_err(err, errlen, "Malformed matrix size information");
        return -2;
    }
    if (!(h.coordinate && (h.real || h.integer) && (h.general || h.symmetric))) {
        std::fclose(f);
        set_err(err, errlen, "Unsupported matrix type");
        return -2;
    }
    if (M != N || N <= 0 || N > INT32_MAX) {
        std::fclose(f);
        set_err(err, errlen, "Only square matrices are supported");
        return -2;
    }
    const bool symm = h.symmetric;
    std::vector<int32_t> I((size_t)L), J((size_t)L);
    std::vector<double> V((size_t)L);
    // counts per row: one diagonal slot each, plus every off-diagonal entry
    std::vector<int64_t> cnt((size_t)N, 1);
    for (long e = 0; e < L; ++e) {
        if (!next_data_line(f, line, sizeof line)) {
            std::fclose(f);
            set_err(err, errlen, "Premature end of file");
            return -2;
        }
        char* p = line;
        long r = std::strtol(p, &p, 10), c = std::strtol(p, &p, 10);
        double v = std::strtod(p, &p);
        if (r < 1 || r > N || c < 1 || c > N) {
            std::fclose(f);
            set_err(err, errlen, "Index out of range");
            return -2;
        }
        I[(size_t)e] = (int32_t)(r - 1);
        J[(size_t)e] = (int32_t)(c - 1);
        V[(size_t)e] = v;
        if (r != c) {
            cnt[(size_t)(r - 1)]++;
            if (symm) cnt[(size_t)(c - 1)]++;
        }
    }
    std::fclose(f);
    std::vector<int32_t> rp((size_t)N + 1, 0);
    int64_t total = 0;
    for (long i = 0; i < N; ++i) {
        rp[(size_t)i] = (int32_t)total;
        total += cnt[(size_t)i];
    }
    if (total > INT32_MAX) { set_err(err, errlen, "nnz exceeds int32"); return -2; }
    rp[(size_t)N] = (int32_t)total;
    std::vector<int32_t> ci((size_t)total, -1);
    std::vector<double> va((size_t)total, 0.0);
    std::vector<int32_t> fillp((size_t)N, 1);
    for (long i = 0; i < N; ++i) ci[(size_t)rp[(size_t)i]] = (int32_t)i;  // diagonal slot first, value 0
    for (long e = 0; e < L; ++e) {
        const int32_t r = I[(size_t)e], c = J[(size_t)e];
        const double v = V[(size_t)e];
        if (r == c) {
            va[(size_t)rp[(size_t)r]] = v;  // later diagonal duplicates overwrite
            continue;
        }
        size_t s = (size_t)rp[(size_t)r] + (size_t)fillp[(size_t)r]++;
        ci[s] = c;
        va[s] = v;
        if (symm) {
            size_t t = (size_t)rp[(size_t)c] + (size_t)fillp[(size_t)c]++;
            ci[t] = r;
            va[t] = v;
        }
    }
    // per-row stable sort by column (the reference's bubble sort is stable)
    std::vector<std::pair<int32_t, double>> tmp;
    for (long i = 0; i < N; ++i) {
        const size_t a = (size_t)rp[(size_t)i], b = (size_t)rp[(size_t)i + 1];
        bool sorted = true;
        for (size_t k = a + 1; k < b; ++k)
            if (ci[k - 1] > ci[k]) { sorted = false; break; }
        if (sorted) continue;
        tmp.clear();
        for (size_t k = a; k < b; ++k) tmp.emplace_back(ci[k], va[k]);
        std::stable_sort(tmp.begin(), tmp.end(),
                         [](const std::pair<int32_t, double>& x, const std::pair<int32_t, double>& y) {
                             return x.first < y.first;
                         });
        for (size_t k = a; k < b; ++k) {
            ci[k] = tmp[k - a].first;
            va[k] = tmp[k - a].second;
        }
    }
    return emit(out, (int32_t)N, (int32_t)N, rp, ci, va);
}

int mpg_load_mtx_vector(const char* path, int32_t col, double* out, int64_t n, char* err, int errlen) {
    if (!out || !path) return -2;
    FILE* f = std::fopen(path, "r");
    if (!f) { set_err(err, errlen, "Could not access file"); return -2; }
    MMHeader h;
    std::string why;
    if (!read_banner(f, h, why)) { std::fclose(f); set_err(err, errlen, why); return -2; }
    char line[1025];
    long M = 0, N = 0, L = 0;
    if (!next_data_line(f, line, sizeof line)) { std::fclose(f); set_err(err, errlen, "Malformed matrix size information"); return -2; }
    int got = h.array ? std::sscanf(line, "%ld %ld", &M, &N) : std::sscanf(line, "%ld %ld %ld", &M, &N, &L);
    if ((h.array && got != 2) || (!h.array && got != 3)) { std::fclose(f); set_err(err, errlen, "Malformed matrix size information"); return -2; }
    if (col >= N) { std::fclose(f); set_err(err, errlen, "Column " + std::to_string(col) + " is too large for the " + std::to_string(N) + " vectors"); return -2; }
    if (M != n) { std::fclose(f); set_err(err, errlen, "vector length does not match the matrix"); return -2; }
    if (h.array) {
        for (long k = 0; k < (long)col * M; ++k)
            if (!next_data_line(f, line, sizeof line)) { std::fclose(f); set_err(err, errlen, "Premature end of file"); return -2; }
        for (long j = 0; j < M; ++j) {
            if (!next_data_line(f, line, sizeof line)) { std::fclose(f); set_err(err, errlen, "Premature end of file"); return -2; }
            out[j] = std::strtod(line, nullptr);
        }
    } else {
        for (long j = 0; j < M; ++j) out[j] = 0.0;
        for (long e = 0; e < L; ++e) {
            if (!next_data_line(f, line, sizeof line)) { std::fclose(f); set_err(err, errlen, "Premature end of file"); return -2; }
            char* p = line;
            long r = std::strtol(p, &p, 10) - 1, c = std::strtol(p, &p, 10) - 1;
            double v = std::strtod(p, &p);
            if (c == col && r >= 0 && r < M) out[r] = v;
        }
    }
    std::fclose(f);
    return 0;
}

int mpg_rand_vect(int64_t n, uint32_t seed, double* out) {
    if (!out || n < 0) return -2;
    std::mt19937 engine(seed);
    std::uniform_real_distribution<float> dist;
    for (int64_t i = 0; i < n; ++i) out[i] = dist(engine);
    return 0;
}

int mpg_host_spmv(const mpg_host_csr* a, const double* x, double* y) {
    if (!a || !x || !y) return -2;
    for (int32_t i = 0; i < a->nrows; ++i) {
        double s = 0.0;
        for (int32_t k = a->rowptr[i]; k < a->rowptr[i + 1]; ++k) s += a->val[k] * x[a->col[k]];
        y[i] = s;
    }
    return 0;
}

}  // extern "C"
