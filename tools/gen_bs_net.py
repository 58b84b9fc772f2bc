#!/usr/bin/env python3
"""Generate the bit-sliced XOR network of a fixed GF(2^8) parity matrix (dev tool, round 4).

A byte product c*x over GF(2^8)/0x11D is GF(2)-linear in the bits of x: bit i of c*x is the XOR of
the bits j of x where bit i of c*2^j is set.  With 32 bytes of a shard held as 8 bit planes (plane j
= bit j of every byte), a whole parity row is therefore a fixed XOR network over the 8 * k input
planes: no table lookups, no selectors.  This script writes that network for the EC16P20L2 parity
(the 20 KRS global rows over 16 data rows, then the two AZ-local rows expressed over the data) as
straight-line C++, one block per output row; common subexpressions are shared inside a row only
(Paar's greedy pairing), which bounds the live temporaries to what one row needs.

The matrix is built here with a plain restatement of KRS buildMatrix (vandermonde(k + m, k) times
the inverse of its top k rows, reedsolomon.go:220-244) and of the CubeFS local rows
(lrcencoder.go: the (18, 1) local code over an AZ's 8 data and 10 global parities); the library
checks its engine's coefficients against these constants before it takes the network
(gf_bs16.hip), and the probes tools/bs_probe.hip / bs_repair_probe.hip use it too.

  python3 tools/gen_bs_net.py ec16p20l2 > chubaofs_amd/csrc/bs_net_ec16p20l2.hpp
  python3 tools/gen_bs_net.py ec15p12 | ec12p9   (measured, not shipped: profiles/r04/bsk_ab.txt)
"""
import sys

import numpy as np

EXP = [0] * 512
LOG = [0] * 256
_v = 1
for _i in range(255):
    EXP[_i] = _v
    LOG[_v] = _i
    _v <<= 1
    if _v & 0x100:
        _v ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gmul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def gpow(a, n):
    if n == 0:
        return 1
    return 0 if a == 0 else EXP[(LOG[a] * n) % 255]


def inverse(M):
    n = len(M)
    A = [row[:] + [int(i == j) for j in range(n)] for i, row in enumerate(M)]
    for c in range(n):
        p = next(r for r in range(c, n) if A[r][c])
        A[c], A[p] = A[p], A[c]
        iv = EXP[255 - LOG[A[c][c]]]
        A[c] = [gmul(iv, x) for x in A[c]]
        for r in range(n):
            if r != c and A[r][c]:
                f = A[r][c]
                A[r] = [x ^ gmul(f, y) for x, y in zip(A[r], A[c])]
    return [row[n:] for row in A]


def parity_rows(k, m):
    V = [[gpow(r, c) for c in range(k)] for r in range(k + m)]
    T = inverse(V[:k])
    out = []
    for r in range(k, k + m):
        row = []
        for c in range(k):
            acc = 0
            for t in range(k):
                acc ^= gmul(V[r][t], T[t][c])
            row.append(acc)
        out.append(row)
    return out


def ec16p20l2_rows():
    g = parity_rows(16, 20)
    lc = parity_rows(18, 1)[0]
    rows = [r[:] for r in g]
    for a in range(2):  # AZ a: data 8a..8a+7, global parities 10a..10a+9, one local parity
        row = [0] * 16
        for t in range(8):
            row[8 * a + t] ^= lc[t]
        for t in range(10):
            for c in range(16):
                row[c] ^= gmul(lc[8 + t], g[10 * a + t][c])
        rows.append(row)
    return rows


def bitmat(c):
    """8x8 GF(2) matrix of x -> c*x: column j = bits of c * 2^j."""
    M = np.zeros((8, 8), np.int32)
    p = c
    for j in range(8):
        for i in range(8):
            M[i, j] = (p >> i) & 1
        p = gmul(p, 2)
    return M


def row_network(row):
    """Paar's greedy CSE over one output row: 8 planes x 8k input planes."""
    k = len(row)
    B = np.concatenate([bitmat(c) for c in row], axis=1)  # 8 x 8k
    n_in = B.shape[1]
    temps = []
    while True:
        C = B.T @ B
        np.fill_diagonal(C, 0)
        i, j = np.unravel_index(np.argmax(C), C.shape)
        if C[i, j] < 2:
            break
        col = B[:, i] & B[:, j]
        B[:, i] -= col
        B[:, j] -= col
        B = np.concatenate([B, col[:, None]], axis=1)
        temps.append((int(i), int(j)))
    outs = [[int(s) for s in np.nonzero(B[o])[0]] for o in range(8)]
    return n_in, temps, outs


def emit_row(name, r, row, lines):
    """Row r's network as a specialization bs_row_<name><r>(x, o)."""
    n_in, temps, outs = row_network(row)
    nx = n_in
    tname = lambda s_: f"x[{s_}]" if s_ < n_in else f"t{s_ - n_in}"
    done = set()
    body = []

    def need(s_):
        if s_ < n_in or s_ in done:
            return
        a_, b_ = temps[s_ - n_in]
        need(a_)
        need(b_)
        done.add(s_)
        body.append(f"  const uint32_t {tname(s_)} = {tname(a_)} ^ {tname(b_)};")

    ops = 0
    for o, sig in enumerate(outs):
        for s_ in sig:
            need(s_)
        terms = [tname(s_) for s_ in sig]
        if not terms:
            expr = "0u"
        else:
            # a balanced tree of 3-input XORs (depth log3 of the terms, not a serial chain)
            while len(terms) > 1:
                nxt = []
                for i in range(0, len(terms), 3):
                    g = terms[i:i + 3]
                    if len(g) == 3:
                        nxt.append(f"bs_x3({g[0]}, {g[1]}, {g[2]})")
                    elif len(g) == 2:
                        nxt.append(f"({g[0]} ^ {g[1]})")
                    else:
                        nxt.append(g[0])
                    ops += len(g) > 1
                terms = nxt
            expr = terms[0]
        body.append(f"  o[{o}] = {expr};")
    ops += len(temps)
    lines.append(f"// row {r}: {len(temps)} shared pairs, {ops} VALU ops per 32-byte column")
    lines.append("template <>")
    lines.append(f"__device__ __forceinline__ void bs_row_{name}<{r}>(const uint32_t (&x)[{nx}], uint32_t (&o)[8]) {{")
    lines += body
    lines.append("}")
    return ops


BARRIER = "--no-barrier" not in sys.argv

CODES = {
    # name: (title, rows, note on NR)
    "ec16p20l2": ("The EC16P20L2 parity (20 KRS global rows, then the 2 AZ-local rows over the data)",
                  ec16p20l2_rows, "NR = 20: EC16P20's global parity; 22: with the local rows"),
    "ec15p12": ("The EC15P12 parity (KRS buildMatrix(15, 27) rows 15..26)", lambda: parity_rows(15, 12), "NR = 12"),
    "ec12p9": ("The EC12P9 parity (KRS buildMatrix(12, 21) rows 12..20)", lambda: parity_rows(12, 9), "NR = 9"),
}


def main():
    code = next((a for a in sys.argv[1:] if not a.startswith("--")), "ec16p20l2")
    title, make_rows, nr_note = CODES[code]
    rows = make_rows()
    m, k = len(rows), len(rows[0])
    nx = 8 * k
    lines = []
    total = 0
    for r, row in enumerate(rows):
        total += emit_row(code, r, row, lines)
    Name = "Bs" + code[0].upper() + code[1:]
    out = sys.stdout
    out.write(f"// bs_net_{code}.hpp -- GENERATED by tools/gen_bs_net.py {code}; do not edit.\n")
    out.write(f"//\n// {title} as a\n")
    out.write(f"// bit-sliced XOR network: {total} VALU ops per 32-byte column for all {m} rows.\n")
    out.write("// x[8c + j]: bit plane j of data row c; o: the output row's 8 planes.\n")
    out.write("#pragma once\n#include <cstdint>\n\nnamespace cfsec {\nnamespace dev {\n\n")
    out.write(f"constexpr uint8_t k{Name}Rows[{m}][{k}] = {{\n")
    for row in rows:
        out.write("    {" + ", ".join(f"0x{v:02x}" for v in row) + "},\n")
    out.write("};\n\n")
    out.write("#ifndef CFSEC_BS_X3\n#define CFSEC_BS_X3\n")
    out.write("__device__ __forceinline__ uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) {\n"
              "  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);\n}\n#endif\n\n")
    out.write(f"template <int R>\n__device__ __forceinline__ void bs_row_{code}(const uint32_t (&x)[{nx}], uint32_t (&o)[8]);\n\n")
    out.write("\n".join(lines) + "\n\n")
    out.write(f"// rows 0 .. NR-1 in order ({nr_note}); emit(r, o) consumes row r's planes\n")
    out.write(f"template <int NR = {m}, class Emit>\n__device__ __forceinline__ void bs_net_{code}(const uint32_t (&x)[{nx}], Emit&& emit) {{\n")
    for r in range(m):
        out.write(f"  if constexpr ({r} < NR) {{\n    uint32_t o[8];\n    bs_row_{code}<{r}>(x, o);\n    emit({r}, o);\n")
        if BARRIER:
            out.write("    __builtin_amdgcn_sched_barrier(0);\n")
        out.write("  }\n")
    out.write("}\n\n")
    out.write("// row r chosen at run time (uniform)\n")
    out.write(f"__device__ __forceinline__ void bs_row_{code}_rt(int r, const uint32_t (&x)[{nx}], uint32_t (&o)[8]) {{\n  switch (r) {{\n")
    for r in range(m):
        out.write(f"    case {r}: bs_row_{code}<{r}>(x, o); break;\n")
    out.write("    default: for (int j = 0; j < 8; ++j) o[j] = 0u;\n  }\n}\n\n")
    out.write(f"// the network as a type for the K-input kernels (gf_bs16.hip)\n")
    out.write(f"struct {Name} {{\n  static constexpr int K = {k}, M = {m};\n")
    out.write(f"  static const uint8_t* rows() {{ return &k{Name}Rows[0][0]; }}\n")
    out.write(f"  template <int NR, class Emit>\n  __device__ static __forceinline__ void net(const uint32_t (&x)[{nx}], Emit&& emit) {{\n")
    out.write(f"    bs_net_{code}<NR>(x, static_cast<Emit&&>(emit));\n  }}\n}};\n\n")
    out.write("}  // namespace dev\n}  // namespace cfsec\n")


if __name__ == "__main__":
    main()
