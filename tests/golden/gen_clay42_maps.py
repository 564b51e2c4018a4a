"""Closed-form Clay(4,2) maps, derived WITHOUT running the reference's stage sequence:
an independent pin for the planner (csrc/codes.cpp) and the oracle (oracle/ecx_oracle.c),
which both restate ClayCodeErasureDecodingStep.java stage by stage and so could share a
misreading of it.  Writes tests/golden/clay42_closed_form.json (data only); run by
gen_golden.py, or alone -- it needs only the Galois tables already in reference_kats.json.

What is used, and nothing else:
  * GF(2^8) from the reference's LOG_TABLE / EXP_TABLE literals (Galois.java:59-170);
  * ReedSolomon.buildMatrix (ReedSolomon.java:373-385): vandermonde(n, k) times the
    inverse of its top k x k square, for RS(2,2) (the pair transform) and RS(4,2) (the
    per-plane code);
  * the Clay geometry of ClayCodeUtil (:690-941): q = m = 2, t = (k+m)/m = 3,
    alpha = q^t = 8, node i = (x, y) = (i % q, i / q), plane z = sum zvec[i] q^(t-1-i),
    helper planes of node (x, y) = the planes with zvec[y] == x, couple plane of (x, y)
    in z = z with zvec[y] := x;
  * the pair transform as equations: for a vertex (node a, plane z) that is not a dot
    (zvec[y_a] != x_a) and its couple (node b = (zvec[y_a], y_a), plane z[y_a := x_a]),
    [U_a, U_b] = P [C_a, C_b] with P the RS(2,2) parity rows [[3, 2], [2, 3]]
    (getPairWiseCouple :630-666: shards (C_a, C_b, U_a, U_b)); a dot has U = C;
  * per plane, the uncoupled symbols form an RS(4,2) codeword, and exactly k = 4 of the 6
    are known in every plane used below, so the unknown ones are the unique solution
    (data = inverse of the known rows' submatrix times the known values; parity = the
    parity rows times the data) -- no first-k choice arises.

Single repair of node e = (ex, ey): in each helper plane z the four nodes outside column ey
are decoupled from helper sub-chunks, the column's two U follow from the RS(4,2) equations,
C(e, z) = U(e, z) (a dot), and for the column mate m = (x', ey) the couple of (e, z[ey := x'])
is (m, z), so C(e, z[ey := x']) solves [U_m, ...] from (C_m, U_m):
C_e = (3/2) C_m + (1/2) U_m.
Encode (erasing the parity column {4, 5}): U of the data nodes from the pair transform, U of
the parity nodes = RS(4,2) parity rows times them, C of the parity nodes = P^-1 (U_p, U_p').

Any m-node erasure (solve_map): the erased sub-chunks are the unique solution of every
plane's RS parity checks on the decoupled symbols -- the code's definition as a linear
system, solved by Gaussian elimination, with no decoding order at all.  The tests compare it
with the planner's multi-node maps (doDecodeMulti's composition) of Clay(4,2), (6,3), (8,4),
(12,4) and the shortened (10,4).

Slots are the reference's: input z*n + node (ClayCodeErasureDecodingStep.java:84-97),
output z*|E| + j.  Maps are stored as {"out": [...], "in": [...], "coef": [...]} triples.
"""
import json
from pathlib import Path

HERE = Path(__file__).resolve().parent

K, M = 4, 2  # the committed maps; the functions below take any Clay(k, m) with m | k + m


class Geo:
    """ClayCodeUtil's geometry (ClayCodeErasureDecodingStep.java:690-941)."""

    def __init__(self, k, m):
        self.k, self.m, self.n = k, m, k + m
        self.q, self.t = m, (k + m) // m
        self.alpha = self.q ** self.t


class GF:
    def __init__(self, log_table, exp_table):
        self.log, self.exp = log_table, exp_table

    def mul(self, a, b):
        return 0 if a == 0 or b == 0 else self.exp[self.log[a] + self.log[b]]

    def inv(self, a):
        assert a != 0
        return self.exp[255 - self.log[a]]

    def div(self, a, b):
        return self.mul(a, self.inv(b))

    def power(self, a, n):  # Galois.exp: a^0 = 1 for every a
        r = 1
        for _ in range(n):
            r = self.mul(r, a)
        return r

    def mat_mul(self, A, B):
        return [[self._dot(row, [B[r][c] for r in range(len(B))]) for c in range(len(B[0]))] for row in A]

    def _dot(self, u, v):
        s = 0
        for a, b in zip(u, v):
            s ^= self.mul(a, b)
        return s

    def mat_inv(self, A):
        n = len(A)
        W = [list(A[r]) + [1 if c == r else 0 for c in range(n)] for r in range(n)]
        for c in range(n):
            p = next(r for r in range(c, n) if W[r][c])
            W[c], W[p] = W[p], W[c]
            f = self.inv(W[c][c])
            W[c] = [self.mul(f, x) for x in W[c]]
            for r in range(n):
                if r != c and W[r][c]:
                    g = W[r][c]
                    W[r] = [x ^ self.mul(g, y) for x, y in zip(W[r], W[c])]
        return [row[n:] for row in W]

    def rs_matrix(self, k, m):
        """ReedSolomon.buildMatrix: vandermonde(k+m, k) x inverse(top k x k)."""
        V = [[self.power(r, c) for c in range(k)] for r in range(k + m)]
        return self.mat_mul(V, self.mat_inv(V[:k]))


# ---- symbolic values: {input slot: coefficient} (a linear form over the map's inputs)
def lin_add(*terms):
    out = {}
    for t in terms:
        for k, v in t.items():
            out[k] = out.get(k, 0) ^ v
    return {k: v for k, v in out.items() if v}


def lin_scale(gf, c, t):
    return {k: gf.mul(c, v) for k, v in t.items() if gf.mul(c, v)}


def zvec(g, z):
    v = [0] * g.t
    for i in range(g.t - 1, -1, -1):
        v[i] = z % g.q
        z //= g.q
    return v


def zidx(g, v):
    z = 0
    for d in v:
        z = z * g.q + d
    return z


def node(g, x, y):
    return x + g.q * y


def coords(g, i):
    return i % g.q, i // g.q


def C(g, z, j):
    """The coupled (stored) sub-chunk of node j in plane z: an input slot."""
    return {z * g.n + j: 1}


def decoupled(gf, g, z, j):
    """U(j, z) from stored sub-chunks: a dot, or the pair transform with its couple."""
    x, y = coords(g, j)
    v = zvec(g, z)
    if v[y] == x:
        return C(g, z, j)
    partner = node(g, v[y], y)
    v2 = list(v)
    v2[y] = x
    return lin_add(lin_scale(gf, 3, C(g, z, j)), lin_scale(gf, 2, C(g, zidx(g, v2), partner)))


def solve_plane(gf, g, rs, U, missing):
    """RS(k, m) per plane: fill U[j] for the `missing` nodes from the k known."""
    known = [j for j in range(g.n) if j not in missing]
    assert len(known) == g.k
    sub_inv = gf.mat_inv([rs[j] for j in known])
    data = [lin_add(*[lin_scale(gf, sub_inv[d][c], U[known[c]]) for c in range(g.k)]) for d in range(g.k)]
    for j in missing:
        U[j] = data[j] if j < g.k else lin_add(*[lin_scale(gf, rs[j][d], data[d]) for d in range(g.k)])
    return U


def repair_map(gf, g, rs, e):
    """Single repair of node e: output slot z (|E| = 1) -> linear form over input slots."""
    ex, ey = coords(g, e)
    helpers = [z for z in range(g.alpha) if zvec(g, z)[ey] == ex]
    column = [node(g, x, ey) for x in range(g.q)]
    out = {}
    for z in helpers:
        U = {j: decoupled(gf, g, z, j) for j in range(g.n) if j not in column}
        solve_plane(gf, g, rs, U, column)
        out[z] = U[e]  # a dot in its helper plane: C(e, z) = U(e, z)
        for mate in column:
            if mate == e:
                continue
            v = zvec(g, z)
            v[ey] = coords(g, mate)[0]
            # couple of (e, z[ey := x']) is (mate, z): shards (C_e, C_m, U_e, U_m), C_m and U_m known
            out[zidx(g, v)] = lin_add(lin_scale(gf, gf.div(3, 2), C(g, z, mate)),
                                      lin_scale(gf, gf.div(1, 2), U[mate]))
    return out


def encode_map(gf, g, rs):
    """The parity column (the last node row) from the data nodes, every plane."""
    parity = [node(g, x, g.t - 1) for x in range(g.q)]
    U = {}
    for z in range(g.alpha):
        Uz = {j: decoupled(gf, g, z, j) for j in range(g.k)}
        for p in parity:
            Uz[p] = lin_add(*[lin_scale(gf, rs[p][d], Uz[d]) for d in range(g.k)])
        U[z] = Uz
    pinv = gf.mat_inv([[3, 2], [2, 3]])
    out = {}
    for z in range(g.alpha):
        v = zvec(g, z)
        for jj, p in enumerate(parity):
            x, y = coords(g, p)
            if v[y] == x:
                out[z * len(parity) + jj] = U[z][p]
            else:
                partner = node(g, v[y], y)
                v2 = list(v)
                v2[y] = x
                # [C_p, C_p'] = P^-1 [U_p, U_p'] with P = [[3, 2], [2, 3]] (its own inverse)
                out[z * len(parity) + jj] = lin_add(lin_scale(gf, pinv[0][0], U[z][p]),
                                                    lin_scale(gf, pinv[0][1], U[zidx(g, v2)][partner]))
    return out


def solve_map(gf, g, rs, erased):
    """Any m-node erasure, from the code's definition alone: the unknowns are the erased
    nodes' stored sub-chunks C(e, z), every plane's decoupled symbols must satisfy the
    RS(k, m) parity checks U_p = sum_d G[p][d] U_d (m equations per plane, m * alpha in
    all -- as many as unknowns), and Gaussian elimination over GF(2^8) expresses each
    unknown in the known sub-chunks.  No decoding order, helper choice or stage sequence
    is involved, and with |E| = m the result is unique (k * alpha known symbols carry
    the whole codeword), so every correct decoder composes to exactly this map.
    Output slot z * |E| + j for the j-th erased node in ascending order; the result is
    {output slot: {input slot: coefficient}} like repair_map's."""
    import numpy as np
    erased = sorted(erased)
    assert len(erased) == g.m
    unk = {z * g.n + e: j * g.alpha + z for j, e in enumerate(erased) for z in range(g.alpha)}
    known = sorted(s for s in range(g.alpha * g.n) if s not in unk)
    col_of = dict(unk)
    col_of.update({s: len(unk) + i for i, s in enumerate(known)})
    mul = np.zeros((256, 256), np.uint8)
    for a in range(1, 256):
        for b in range(1, 256):
            mul[a, b] = gf.mul(a, b)
    inv = np.zeros(256, np.uint8)
    inv[1:] = [gf.inv(a) for a in range(1, 256)]
    W = np.zeros((g.m * g.alpha, len(col_of)), np.uint8)  # [A | B]: A x = B y over GF(2^8)
    r = 0
    for z in range(g.alpha):
        U = [decoupled(gf, g, z, j) for j in range(g.n)]
        for p in range(g.k, g.n):
            # U_p + sum_d G[p][d] U_d = 0; a known term moves across unchanged (characteristic 2)
            for slot, c in lin_add(U[p], *[lin_scale(gf, rs[p][d], U[d]) for d in range(g.k)]).items():
                W[r, col_of[slot]] ^= c
            r += 1
    n = len(unk)
    for col in range(n):
        piv = col + int(np.flatnonzero(W[col:, col])[0])
        W[[col, piv]] = W[[piv, col]]
        W[col] = mul[inv[W[col, col]], W[col]]
        h = W[:, col].copy()
        h[col] = 0
        rows = np.flatnonzero(h)
        cols = np.flatnonzero(W[col])
        W[np.ix_(rows, cols)] ^= mul[h[rows][:, None], W[col, cols][None, :]]
    assert (W[:, :n] == np.eye(n, dtype=np.uint8)).all()
    out = {}
    for j in range(len(erased)):
        for z in range(g.alpha):
            row = W[j * g.alpha + z, n:]
            out[z * len(erased) + j] = {known[i]: int(row[i]) for i in np.flatnonzero(row)}
    return out


def field_and_code(k, m):
    kats = json.loads((HERE / "reference_kats.json").read_text())
    gf = GF(kats["galois"]["log_table"], kats["galois"]["exp_table"])
    return gf, Geo(k, m), gf.rs_matrix(k, m)


def triples(m):
    o, i, c = [], [], []
    for out_slot in sorted(m):
        for in_slot in sorted(m[out_slot]):
            o.append(out_slot)
            i.append(in_slot)
            c.append(m[out_slot][in_slot])
    return {"out": o, "in": i, "coef": c, "nnz": len(c)}


def main():
    kats = json.loads((HERE / "reference_kats.json").read_text())
    gf, g, rs = field_and_code(K, M)
    assert rs[K:] == kats["rs_parity_rows"]["4,2"], rs[K:]
    assert gf.rs_matrix(2, 2)[2:] == [[3, 2], [2, 3]]
    doc = {
        "source": "closed-form Clay(4,2) maps (tests/golden/gen_clay42_maps.py); no reference stage sequence run",
        "repair_e1": triples(repair_map(gf, g, rs, 1)),
        "repair_e4": triples(repair_map(gf, g, rs, 4)),
        "encode_45": triples(encode_map(gf, g, rs)),
    }
    (HERE / "clay42_closed_form.json").write_text(json.dumps(doc) + "\n")
    print("wrote", HERE / "clay42_closed_form.json", {k: v["nnz"] for k, v in doc.items() if k != "source"})


if __name__ == "__main__":
    main()
