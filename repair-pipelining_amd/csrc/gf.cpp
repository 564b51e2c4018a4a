// gf.cpp -- see gf.hpp.
#include "gf.hpp"

#include <algorithm>
#include <utility>

namespace ecx {

Field::Field() {
    // Successive powers of the generator 2 modulo 0x11D give the exp table;
    // log is its inverse (Galois.generateLogTable / generateExpTable,
    // Galois.java:259-289).  exp_ is doubled to 510 entries so that
    // log a + log b never needs a modulo.
    for (int i = 0; i < 256; ++i) log_[i] = -1;
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        exp_[i] = (uint8_t)v;
        exp_[i + 255] = (uint8_t)v;
        log_[v] = (int16_t)i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11D;
    }
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            prod_[a][b] = (a == 0 || b == 0) ? 0 : exp_[log_[a] + log_[b]];
}

const Field &Field::get() {
    static const Field f;
    return f;
}

uint8_t Field::div(uint8_t a, uint8_t b) const {
    if (b == 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "Argument 'divisor' is 0");
    if (a == 0) return 0;
    int d = log_[a] - log_[b];
    return exp_[d < 0 ? d + 255 : d];
}

uint8_t Field::pow(uint8_t a, int n) const {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return exp_[(int)(((long long)log_[a] * n) % 255)];
}

Matrix Matrix::identity(int n) {
    Matrix m(n, n);
    for (int i = 0; i < n; ++i) m.at(i, i) = 1;
    return m;
}

Matrix Matrix::operator*(const Matrix &rhs) const {
    if (c_ != rhs.r_)
        throw Error(ECX_E_ILLEGAL_ARGUMENT, "Columns on left (" + std::to_string(c_) +
                                                ") is different than rows on right (" + std::to_string(rhs.r_) + ")");
    const Field &f = Field::get();
    Matrix out(r_, rhs.c_);
    for (int r = 0; r < r_; ++r)
        for (int i = 0; i < c_; ++i) {
            const uint8_t a = at(r, i);
            if (!a) continue;
            const uint8_t *mrow = f.row(a);
            const uint8_t *b = rhs.row(i);
            uint8_t *o = out.row(r);
            for (int c = 0; c < rhs.c_; ++c) o[c] ^= mrow[b[c]];
        }
    return out;
}

// Gauss-Jordan on [A | I].  The inverse is unique, so the pivot rule only has
// to agree with Matrix.gaussianElimination (Matrix.java:296-346) on WHEN the
// matrix is singular: a zero column below and on the diagonal.
Matrix Matrix::inverse() const {
    if (r_ != c_) throw Error(ECX_E_ILLEGAL_ARGUMENT, "Only square matrices can be inverted");
    const Field &f = Field::get();
    const int n = r_;
    std::vector<std::vector<uint8_t>> w(n, std::vector<uint8_t>(2 * n, 0));
    for (int r = 0; r < n; ++r) {
        std::copy(row(r), row(r) + n, w[r].begin());
        w[r][n + r] = 1;
    }
    for (int col = 0; col < n; ++col) {
        int piv = col;
        while (piv < n && w[piv][col] == 0) ++piv;
        if (piv == n) throw Error(ECX_E_SINGULAR, "Matrix is singular");
        std::swap(w[col], w[piv]);
        const uint8_t inv = f.div(1, w[col][col]);
        if (inv != 1)
            for (auto &x : w[col]) x = f.mul(x, inv);
        for (int r = 0; r < n; ++r) {
            if (r == col || w[r][col] == 0) continue;
            const uint8_t *mrow = f.row(w[r][col]);
            for (int c = 0; c < 2 * n; ++c) w[r][c] ^= mrow[w[col][c]];
        }
    }
    Matrix out(n, n);
    for (int r = 0; r < n; ++r) std::copy(w[r].begin() + n, w[r].end(), out.row(r));
    return out;
}

}  // namespace ecx
