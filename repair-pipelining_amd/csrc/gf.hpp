// gf.hpp -- GF(2^8) field and dense GF matrices for the host-side planner.
//
// The field is the reference's: generating polynomial 29 (x^8+x^4+x^3+x^2+1,
// Galois.java:43), generator 2, log/exp tables as Galois.java:59-170.  The
// matrix algebra follows Matrix.java:193-346 (times, Gauss-Jordan inverse with
// the same "Matrix is singular" failure).  None of this runs per byte: it builds
// coefficient matrices that the HIP kernels apply.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ecx.h"

namespace ecx {

// Carries an ecx_status code across the C++ planner up to the C ABI.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &msg) : std::runtime_error(msg), code(c) {}
};

class Field {
public:
    static const Field &get();
    uint8_t mul(uint8_t a, uint8_t b) const { return prod_[a][b]; }
    const uint8_t *row(uint8_t c) const { return prod_[c]; }
    uint8_t div(uint8_t a, uint8_t b) const;
    uint8_t pow(uint8_t a, int n) const;
    int16_t log(uint8_t a) const { return log_[a]; }
    uint8_t exp(int i) const { return exp_[i]; }

private:
    Field();
    int16_t log_[256];
    uint8_t exp_[510];
    uint8_t prod_[256][256];
};

// Row-major byte matrix over GF(2^8).
class Matrix {
public:
    Matrix() = default;
    Matrix(int rows, int cols) : r_(rows), c_(cols), v_((size_t)rows * cols, 0) {}
    static Matrix identity(int n);
    int rows() const { return r_; }
    int cols() const { return c_; }
    uint8_t &at(int r, int c) { return v_[(size_t)r * c_ + c]; }
    uint8_t at(int r, int c) const { return v_[(size_t)r * c_ + c]; }
    const uint8_t *row(int r) const { return v_.data() + (size_t)r * c_; }
    uint8_t *row(int r) { return v_.data() + (size_t)r * c_; }
    const std::vector<uint8_t> &data() const { return v_; }
    Matrix operator*(const Matrix &rhs) const;
    Matrix inverse() const;  // throws Error(ECX_E_SINGULAR)

private:
    int r_ = 0, c_ = 0;
    std::vector<uint8_t> v_;
};

}  // namespace ecx
