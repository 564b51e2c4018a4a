// codes.hpp -- the planner: Reed-Solomon, Clay and LRC repair/encode composed
// into single GF(256) linear maps.
//
// Every reference stage (ReedSolomon.decodeMissing, the Clay pair transform,
// the per-plane RS decode, re-coupling, ...) is linear over GF(2^8) and acts on
// every byte position independently with the same coefficients.  The planner
// therefore runs the reference's stage SEQUENCE once on symbolic buffers --
// each buffer is its coefficient vector over the input slots -- and the result
// is the exact linear map the JVM path computes for ANY input bytes (valid
// codewords or not).  Aliasing and in-place writes follow the Java object
// semantics (SymBuf = shared pointer), so that corner cases such as
// non-null erased inputs in the multi-erasure path compose identically.
#pragma once

#include <memory>
#include <vector>

#include "gf.hpp"

namespace ecx {

// A dense composed map: out[o] = sum_j a[o][j] * in[j]; in_slot / out_slot are
// the slot indices of the caller's layout the rows / columns refer to.
struct LinearMap {
    int n_out = 0, n_in = 0;
    std::vector<uint8_t> a;  // n_out x n_in
    std::vector<int> in_slot, out_slot;
    uint8_t at(int o, int j) const { return a[(size_t)o * n_in + j]; }
    int nnz() const;
    // Drop all-zero columns (inputs the map never reads).
    LinearMap pruned() const;
};

using SymBuf = std::shared_ptr<std::vector<uint8_t>>;

// ReedSolomon.java: systematic code built from Vandermonde * inv(top k rows)
// (buildMatrix / vandermonde, ReedSolomon.java:373-404).
class RsCode {
public:
    RsCode(int data_shards, int parity_shards);
    int k() const { return k_; }
    int m() const { return m_; }
    int n() const { return k_ + m_; }
    const Matrix &matrix() const { return gen_; }
    const uint8_t *parity_row(int p) const { return gen_.row(k_ + p); }

    // decodeMissing's row selection (ReedSolomon.java:224-244): the first k
    // present rows in ascending order, and the inverse of their submatrix.
    Matrix data_decoder(const std::vector<bool> &present, std::vector<int> *rows_used) const;

    LinearMap encode_map() const;                                  // encodeParity :94-108
    LinearMap decode_map(const std::vector<bool> &present) const;  // decodeMissing :189-286

    // decodeMissing on symbolic shards, writing the non-present shard objects in place.
    void decode_missing(std::vector<SymBuf> &shards, const std::vector<bool> &present) const;

private:
    int k_, m_;
    Matrix gen_;
};

// LRC (LRCErasureCode.kt:5-9, LRCErasureUtil.kt:3-6): K = 12 data blocks in local
// groups of R = 3, each with one parity from RS(R, 1) (parity row [1,1,1]: XOR).
// Block order of LRCErasureCodeExample.kt:48: group g = blocks 4g..4g+3, parity 4g+3.
class LrcCode {
public:
    static constexpr int kK = 12, kR = 3, kGroups = kK / kR, kN = kK + kGroups;
    LrcCode() : group_(kR, 1) {}
    // encode / encodeUsingSingle (LRCErasureCodeExample.kt:30-98): every group parity.
    LinearMap encode_map() const;
    // decode (:100-131): per group, decodeMissing of the group's non-present blocks;
    // more than one missing block in a group -> ECX_E_NOT_ENOUGH_SHARDS.
    LinearMap decode_map(const std::vector<bool> &present) const;

private:
    RsCode group_;
};

// Single-node Clay repair (doDecodeSingle, ClayCodeErasureDecodingStep.java:118-221) as a
// program over its helper planes, the stage structure the per-plane kernel
// (clay_rtc.cpp) executes.  For helper plane p (plane z = helper_planes(e)[p]):
//   decouple (:435-492)   U_j = pair_a * C(z, j) + pair_b * C(z', j') for every node j
//                         outside e's column (a dot, j' = j and z' = z, gives U_j = C(z, j)
//                         because pair_a ^ pair_b == 1; virtual nodes read zeros)
//   plane decode (:542-597)  U(column row r) = sum_j dmat[r][j] * U_j
//   re-couple (:180-200)  out(z) = U(e's row); for each column mate x at row r,
//                         out(z'_x) = rc_c * C(z, x) + rc_u * U(r)
// `table` holds, per helper plane, kClayTab ints: own slot of each non-column node,
// its partner slot, the mates' slots (q - 1, column order without e) and the q output
// slots (e's plane, then the mates'), real slot numbers or -1 (= zeros).
struct ClayRepairProgram {
    int q = 0, n_planes = 0, n_noncol = 0, stride = 0;  // stride = ints per plane in `table`
    uint8_t pair_a = 0, pair_b = 0, rc_c = 0, rc_u = 0;
    int e_row = 0;
    std::vector<int> mate_row;     // q - 1 column rows
    std::vector<uint8_t> dmat;     // q x n_noncol
    std::vector<int32_t> table;    // n_planes x stride
    int max_in_slot = -1, max_out_slot = -1;
    // Grid geometry, for the plane-group kernel (clay_rtc.cpp), which derives slots from
    // the plane digits instead of `table`: node u = x + q*y of the q x t grid, plane
    // z = sum_y zvec[y] * q^(t-1-y), the erased node at (ex, ey), `real_of[u]` the real
    // slot index of underlying node u (-1 = virtual), `noncol[jj]` the node of column jj
    // of dmat, `column[r]` the node of dmat row r.
    int t = 0, ex = 0, ey = 0, n_real = 0;
    std::vector<int> real_of, noncol, column;
    // The program composed into a dense map over (out slot, in slot); tests compare it
    // with perform_coding_map (the reference's stage sequence).
    LinearMap compose(int n_in_slots, int n_out_slots) const;
};

// ClayCodeErasureDecodingStep.java + ClayCodeUtil (:676-944), symbolically.
//
// virtual_units > 0 builds a SHORTENED code: Clay(k + v, m) whose data nodes
// [k, k+v) are virtual, always-zero nodes (Clay(10,4) as
// Clay(12,4) with 2 zero data nodes).  All public slot numbering is over the
// k + m REAL nodes (real node r < k is underlying r, r >= k is r + v).
class ClayPlanner {
public:
    // is_test: the single-repair plane decode takes decodeDecoupledPlane's -DisTest=true branch
    // (ClayCodeErasureDecodingStep.java:571-581, decodeMissingSingle per helper, bug B2 included).
    ClayPlanner(int data_units, int parity_units, std::vector<int> erased, int virtual_units = 0,
                bool is_test = false);
    bool is_test() const { return is_test_; }
    int k() const { return k_; }
    int m() const { return m_; }
    int n() const { return k_ + m_; }           // underlying code
    int n_real() const { return k_ + m_ - v_; }  // nodes that exist (slot numbering)
    int virtual_units() const { return v_; }
    int q() const { return q_; }
    int t() const { return t_; }
    int alpha() const { return alpha_; }
    const std::vector<int> &erased() const { return erased_real_; }

    std::vector<int> helper_planes(int erased_index) const;  // getHelperPlanesIndexes :924-941

    // performCoding (:64-107) for a given null pattern of the n*alpha inputs:
    // returns the map (rows = |E|*alpha outputs, columns = n*alpha input slots).
    LinearMap perform_coding_map(const std::vector<bool> &input_present) const;
    // doDecodeSingle overload 2 (:225-282) for helper plane i: columns are the
    // nh*n helper_coupled slots, rows are the alpha output planes (only the q
    // planes this helper plane writes are non-empty; `written` marks them).
    LinearMap decode_single_helper_map(const std::vector<bool> &helper_present, int helper_i, int erased_index,
                                       std::vector<bool> *written) const;
    // Single-node repair of real node `erased_index` as a per-helper-plane program
    // (ClayRepairProgram).  Throws ECX_E_ILLEGAL_ARGUMENT when the code's pair
    // transform does not allow the dot trick (pair_a ^ pair_b != 1) or when the
    // program does not compose to perform_coding_map exactly.
    ClayRepairProgram repair_program(int erased_index) const;

private:
    int k_, m_, v_, q_, t_, alpha_;
    bool is_test_ = false;
    std::vector<int> erased_;       // underlying node indices
    std::vector<int> erased_real_;  // as given (real node indices)
    int under(int real_node) const { return real_node < k_ - v_ ? real_node : real_node + v_; }
    bool is_virtual(int u) const { return u >= k_ - v_ && u < k_; }
    RsCode pair_, rs_;

    std::vector<int> zvec(int z) const;
    int zindex(const std::vector<int> &v) const;
    int node(int x, int y) const { return x + q_ * y; }
    int nx(int i) const { return i % q_; }
    int ny(int i) const { return i / q_; }
    int couple_plane(int x, int y, int z) const;
    int erasure_type(int idx, int z) const;
    int intersection_score(int z) const;
    bool is_erased(int idx) const;

    SymBuf pair_couple(SymBuf a, SymBuf a2, SymBuf b, SymBuf b2, int width) const;
    void decode_plane(std::vector<SymBuf> &plane, const std::vector<int> &erased, int width,
                      bool single = false) const;
    void decode_plane_is_test(std::vector<SymBuf> &plane, const std::vector<int> &erased, int width) const;
    void single_plane(const std::vector<SymBuf> &helper, const std::vector<int> &hidx, int i, int e,
                      std::vector<SymBuf> &outputs, int width) const;
    void decode_multi(std::vector<SymBuf> in, std::vector<SymBuf> &outputs, int width) const;
};

}  // namespace ecx
