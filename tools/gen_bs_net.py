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

  python3 tools/gen_bs_net.py ec16p20l2 --paired --joint > chubaofs_amd/csrc/bs_net_ec16p20l2.hpp
  python3 tools/gen_bs_net.py ec15p12 | ec12p9   (measured, not shipped: profiles/r04/bsk_ab.txt)
  python3 tools/gen_bs_net.py ec6p10l2 --paired --joint > chubaofs_amd/csrc/bs_net_ec6p10l2.hpp
  python3 tools/gen_bs_net.py ec12p4 --paired --joint > chubaofs_amd/csrc/bs_net_ec12p4.hpp
  python3 tools/gen_bs_net.py ec12p9 --paired --joint > chubaofs_amd/csrc/bs_net_ec12p9.hpp
  python3 tools/gen_bs_net.py ec15p12 > chubaofs_amd/csrc/bs_net_ec15p12.hpp   (k odd: no paired basis)
  python3 tools/gen_bs_net.py ec10p4 --paired --joint > chubaofs_amd/csrc/bs_net_ec10p4.hpp
  python3 tools/gen_bs_net.py ec4p4 --paired --joint > chubaofs_amd/csrc/bs_net_ec4p4.hpp
  python3 tools/gen_bs_net.py ec3p3 > chubaofs_amd/csrc/bs_net_ec3p3.hpp
  python3 tools/gen_bs_net.py ec6p3l3 --paired --joint > chubaofs_amd/csrc/bs_net_ec6p3l3.hpp
  python3 tools/gen_bs_net.py ec4p4l2 --paired --joint > chubaofs_amd/csrc/bs_net_ec4p4l2.hpp
  python3 tools/gen_bs_net.py ec6p6l9 --paired --joint > chubaofs_amd/csrc/bs_net_ec6p6l9.hpp
  python3 tools/gen_bs_net.py ec6p8l10 --paired --joint > chubaofs_amd/csrc/bs_net_ec6p8l10.hpp
    (round 6: the fused encode + checksum kernels, gf_bs_crc.hip; EC6P8 / EC6P10 use the first 8 / 10
    rows of the EC6P10L2 network -- a KRS parity row does not depend on m)
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


def lrc_rows(k, m, azs, ln, lm=1):
    """An LRC's fused encode rows (as the engine's ECEncoder::create builds them): the m KRS global
    rows, then each AZ's lm local parities over the data -- AZ a holds data k/azs * a .. and global
    parities m/azs * a .., its local rows are the KRS (ln, lm) parity rows over those ln members."""
    g = parity_rows(k, m)
    lc = parity_rows(ln, lm)
    rows = [r[:] for r in g]
    dk, dm = k // azs, m // azs
    for a in range(azs):
        for j in range(lm):
            row = [0] * k
            for t in range(dk):
                row[dk * a + t] ^= lc[j][t]
            for t in range(dm):
                for c in range(k):
                    row[c] ^= gmul(lc[j][dk + t], g[dm * a + t][c])
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


def _paar(B, allowed=None, limit=None):
    """Greedy Paar on B (outputs x columns, 0/1), appending one column per chosen pair; allowed(B,
    col) may veto a pair, limit caps the pairs taken.  Returns the new pairs."""
    temps = []
    while limit is None or len(temps) < limit:
        C = B.T @ B
        np.fill_diagonal(C, 0)
        picked = None
        while True:
            i, j = np.unravel_index(np.argmax(C), C.shape)
            if C[i, j] < 2:
                break
            col = B[:, i] & B[:, j]
            if allowed is None or allowed(col):
                picked = (int(i), int(j), col)
                break
            C[i, j] = C[j, i] = 0
        if picked is None:
            break
        i, j, col = picked
        B[:, i] -= col
        B[:, j] -= col
        B = np.concatenate([B, col[:, None]], axis=1)
        temps.append((i, j))
    return B, temps


def group_network(rows, shared=None):
    """Paar's greedy CSE over the 8 * len(rows) output planes of a group of rows, with pairs shared
    across the group's rows too (fewer XORs, more temporaries live across the group).  shared caps
    the pairs used by more than one row (registers live across a row boundary); past it each row
    continues with its own pairs, which may use the shared ones."""
    B = np.concatenate([np.concatenate([bitmat(c) for c in row], axis=1) for row in rows], axis=0)
    n_in = B.shape[1]
    nr = len(rows)
    if shared is None:
        B, temps = _paar(B)
    else:
        spans = lambda col: len({o // 8 for o in np.nonzero(col)[0]}) > 1
        count = [0]

        def allowed(col):
            if spans(col):
                if count[0] >= shared:
                    return False
                count[0] += 1
            return True
        B, temps = _paar(B, allowed)
        # the pairs a row found only among its own outputs after the cap are still row-private
    outs = [[int(s) for s in np.nonzero(B[o])[0]] for o in range(B.shape[0])]
    return n_in, temps, outs


def xor_tree(terms):
    """A balanced tree of 3-input XORs over the terms: (expression, VALU ops)."""
    if not terms:
        return "0u", 0
    ops = 0
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
    return terms[0], ops


def emit_group(name, gi, r0, rows, nx, lines):
    """Rows r0 .. r0 + len(rows) - 1 as one function with the pairs shared across them; a row
    whose index is >= NR is dropped at compile time (its private temporaries die as dead code)."""
    n_in, temps, outs = group_network(rows, SHARED)
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

    ops = len(temps)
    for q in range(len(rows)):
        r = r0 + q
        body.append(f"  uint32_t o{q}[8];")
        for o in range(8):
            sig = outs[8 * q + o]
            for s_ in sig:
                need(s_)
            expr, n = xor_tree([tname(s_) for s_ in sig])
            ops += n
            body.append(f"  o{q}[{o}] = {expr};")
        body.append(f"  if constexpr ({r} < NR) {{")
        body.append(f"    emit({r}, o{q});")
        if BARRIER:
            body.append("    __builtin_amdgcn_sched_barrier(0);")
        body.append("  }")
    lines.append(f"// rows {r0}..{r0 + len(rows) - 1}: {len(temps)} shared pairs, {ops} VALU ops per 32-byte column")
    lines.append("template <int NR, class Emit>")
    lines.append(f"__device__ __forceinline__ void bs_grp_{name}_{gi}(const uint32_t (&x)[{nx}], Emit&& emit) {{")
    lines += body
    lines.append("}")
    return ops


def paired_row(row):
    """A row's coefficients in the paired basis: inputs (u_p = x_2p ^ x_2p+1, x_2p+1), so
    c x_2p + d x_2p+1 = c u_p + (c ^ d) x_2p+1."""
    out = []
    for p in range(0, len(row), 2):
        out += [row[p], row[p] ^ row[p + 1]]
    return out


def half_network(coefs, parity, prefix, body, ops_out, extra=None):
    """sum_p coefs[p] * plane set p, the plane set p being x[8 (2p + parity) + j]; Paar per output
    block; extra[j] (an expression) joins output j's XOR tree.  Appends the code to body and returns
    the 8 output expressions.  coefs may also be a list of coefficient lists: one Paar over all
    their outputs (pairs shared between them), 8 expressions per list, concatenated."""
    if coefs and isinstance(coefs[0], (list, tuple)):
        B = np.concatenate([np.concatenate([bitmat(c) for c in cl], axis=1) for cl in coefs], axis=0)
        n_in = B.shape[1]
        B, temps = _paar(B)
        outs = [[int(s) for s in np.nonzero(B[o])[0]] for o in range(B.shape[0])]
        extra = (extra or []) * len(coefs) if extra else None
    else:
        n_in, temps, outs = row_network(list(coefs))
    xi = lambda s_: f"x[{8 * (2 * (s_ // 8) + parity) + s_ % 8}]"
    tname = lambda s_: xi(s_) if s_ < n_in else f"{prefix}{s_ - n_in}"
    done = set()

    def need(s_):
        if s_ < n_in or s_ in done:
            return
        a_, b_ = temps[s_ - n_in]
        need(a_)
        need(b_)
        done.add(s_)
        body.append(f"  const uint32_t {tname(s_)} = {tname(a_)} ^ {tname(b_)};")

    exprs = []
    ops = len(temps)
    for o, sig in enumerate(outs):
        for s_ in sig:
            need(s_)
        terms = [tname(s_) for s_ in sig] + ([extra[o]] if extra else [])
        e, n = xor_tree(terms)
        ops += n
        exprs.append(e)
    ops_out.append(ops)
    return exprs


def emit_pair(name, q, rows, nx, lines):
    """Rows 2q and 2q + 1 of a dyadic pair (row 2q+1 = row 2q with columns c and c^1 swapped) in
    the paired basis: out_2q = A(u) ^ B(x_odd), out_2q+1 = A'(u) ^ B(x_odd) with B shared."""
    r = 2 * q
    a, b = rows[r], rows[r + 1]
    assert all(b[c] == a[c ^ 1] for c in range(len(a))), "not a dyadic row pair"
    body = []
    ops = []
    bexp = half_network([a[2 * p] ^ a[2 * p + 1] for p in range(len(a) // 2)], 1, "tb", body, ops)
    body.append("  uint32_t b[8];")
    body += [f"  b[{j}] = {e};" for j, e in enumerate(bexp)]
    bref = [f"b[{j}]" for j in range(8)]
    if JOINT:  # A and A' from one Paar: their pairs shared too
        e01 = half_network([[a[2 * p] for p in range(len(a) // 2)], [a[2 * p + 1] for p in range(len(a) // 2)]],
                           0, "ta", body, ops, bref)
        body += [f"  o0[{j}] = {e};" for j, e in enumerate(e01[:8])]
        body += [f"  o1[{j}] = {e};" for j, e in enumerate(e01[8:])]
    else:
        e0 = half_network([a[2 * p] for p in range(len(a) // 2)], 0, "ta", body, ops, bref)
        body += [f"  o0[{j}] = {e};" for j, e in enumerate(e0)]
        e1 = half_network([a[2 * p + 1] for p in range(len(a) // 2)], 0, "tc", body, ops, bref)
        body += [f"  o1[{j}] = {e};" for j, e in enumerate(e1)]
    total = sum(ops)
    lines.append(f"// rows {r}, {r + 1} (a dyadic pair): {total} VALU ops per 32-byte column")
    lines.append("template <>")
    lines.append(f"__device__ __forceinline__ void bs_pair_{name}<{q}>(const uint32_t (&x)[{nx}], uint32_t (&o0)[8], uint32_t (&o1)[8]) {{")
    lines += body
    lines.append("}")
    return total


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
GROUP = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--group=")), 1)
PAIRED = "--paired" in sys.argv
JOINT = "--joint" in sys.argv
SHARED = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--shared=")), None)

CODES = {
    # name: (title, rows, note on NR)
    "ec16p20l2": ("The EC16P20L2 parity (20 KRS global rows, then the 2 AZ-local rows over the data)",
                  ec16p20l2_rows, "NR = 20: EC16P20's global parity; 22: with the local rows"),
    "ec6p10l2": ("The EC6P10L2 fused LRC encode rows (10 KRS global rows, then the 2 AZ-local rows over the data)",
                 lambda: lrc_rows(6, 10, 2, 8), "NR = 12"),
    "ec12p4": ("The EC12P4 parity (KRS buildMatrix(12, 16) rows 12..15)", lambda: parity_rows(12, 4), "NR = 4"),
    "ec6p3l3": ("The EC6P3L3 fused LRC encode rows (3 global, then 3 AZ-local rows over the data)",
                lambda: lrc_rows(6, 3, 3, 3), "NR = 6"),
    "ec4p4l2": ("The EC4P4L2 fused LRC encode rows (4 global, then 2 AZ-local rows over the data)",
                lambda: lrc_rows(4, 4, 2, 4), "NR = 6"),
    "ec6p6l9": ("The EC6P6L9 fused LRC encode rows (6 global, then 3 AZs x 3 local rows over the data)",
                lambda: lrc_rows(6, 6, 3, 4, 3), "NR = 15"),
    "ec6p8l10": ("The EC6P8L10 fused LRC encode rows (8 global, then 2 AZs x 5 local rows over the data)",
                 lambda: lrc_rows(6, 8, 2, 7, 5), "NR = 18"),
    "ec4p4": ("The EC4P4 parity (KRS buildMatrix(4, 8) rows 4..7)", lambda: parity_rows(4, 4), "NR = 4"),
    "ec3p3": ("The EC3P3 parity (KRS buildMatrix(3, 6) rows 3..5)", lambda: parity_rows(3, 3), "NR = 3"),
    "ec10p4": ("The EC10P4 parity (KRS buildMatrix(10, 14) rows 10..13)", lambda: parity_rows(10, 4), "NR = 4"),
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
    npairs = 0
    if PAIRED:
        # rows in the paired basis; the leading dyadic row pairs share their odd-column half
        prow = [paired_row(row) for row in rows]
        while 2 * npairs + 1 < m and all(rows[2 * npairs + 1][c] == rows[2 * npairs][c ^ 1] for c in range(k)):
            npairs += 1
        for r, row in enumerate(prow):
            emit_row(code, r, row, lines)
        plines = []
        for q in range(npairs):
            total += emit_pair(code, q, rows, nx, plines)
        rest = 0
        if JOINT and m - 2 * npairs > 1:  # the rows after the pairs as one group (pairs shared)
            rest = emit_group(code, 0, 2 * npairs, prow[2 * npairs:], nx, plines)
        else:
            for r in range(2 * npairs, m):
                n_in, temps, outs = row_network(prow[r])
                rest += len(temps) + sum(xor_tree(["a"] * len(sg))[1] for sg in outs)
        total += rest
    else:
        for r, row in enumerate(rows):
            total += emit_row(code, r, row, lines)
    Name = "Bs" + code[0].upper() + code[1:]
    out = sys.stdout
    out.write(f"// bs_net_{code}.hpp -- GENERATED by tools/gen_bs_net.py {code}; do not edit.\n")
    out.write(f"//\n// {title} as a\n")
    out.write(f"// bit-sliced XOR network: {total} VALU ops per 32-byte column for all {m} rows.\n")
    if PAIRED:
        out.write(f"// Paired basis (k{Name}Paired): x[8c + j] is bit plane j of data row c for odd c and of\n"
                  "// (row c ^ row c + 1) for even c -- the caller XORs each odd column's planes into the even\n"
                  f"// one's after the transposes.  Rows 0..{2 * npairs - 1} come as dyadic pairs sharing the odd-column half\n"
                  "// (bs_pair_*); every row also as a single network in that basis (bs_row_*).\n")
    else:
        out.write("// x[8c + j]: bit plane j of data row c; o: the output row's 8 planes.\n")
    out.write("#pragma once\n#include <cstdint>\n\nnamespace cfsec {\nnamespace dev {\n\n")
    out.write(f"constexpr uint8_t k{Name}Rows[{m}][{k}] = {{\n")
    for row in rows:
        out.write("    {" + ", ".join(f"0x{v:02x}" for v in row) + "},\n")
    out.write("};\n\n")
    out.write("#ifndef CFSEC_BS_X3\n#define CFSEC_BS_X3\n")
    out.write("__device__ __forceinline__ uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) {\n"
              "  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);\n}\n#endif\n\n")
    out.write(f"constexpr bool k{Name}Paired = {'true' if PAIRED else 'false'};\n\n")
    out.write(f"template <int R>\n__device__ __forceinline__ void bs_row_{code}(const uint32_t (&x)[{nx}], uint32_t (&o)[8]);\n\n")
    out.write("\n".join(lines) + "\n\n")
    if PAIRED:
        out.write(f"template <int Q>\n__device__ __forceinline__ void bs_pair_{code}(const uint32_t (&x)[{nx}], uint32_t (&o0)[8], uint32_t (&o1)[8]);\n\n")
        out.write("\n".join(plines) + "\n\n")
        out.write(f"// rows 0 .. NR-1 in order ({nr_note}); emit(r, o) consumes row r's planes\n")
        out.write(f"template <int NR = {m}, class Emit>\n__device__ __forceinline__ void bs_net_{code}(const uint32_t (&x)[{nx}], Emit&& emit) {{\n")
        bar = "    __builtin_amdgcn_sched_barrier(0);\n" if BARRIER else ""
        for q in range(npairs):
            out.write(f"  if constexpr ({2 * q} < NR) {{\n    uint32_t o0[8], o1[8];\n    bs_pair_{code}<{q}>(x, o0, o1);\n"
                      f"    emit({2 * q}, o0);\n{bar}    if constexpr ({2 * q + 1} < NR) emit({2 * q + 1}, o1);\n{bar}  }}\n")
        if JOINT and m - 2 * npairs > 1:
            out.write(f"  if constexpr ({2 * npairs} < NR) bs_grp_{code}_0<NR>(x, emit);\n")
        else:
            for r in range(2 * npairs, m):
                out.write(f"  if constexpr ({r} < NR) {{\n    uint32_t o[8];\n    bs_row_{code}<{r}>(x, o);\n    emit({r}, o);\n{bar}  }}\n")
        out.write("}\n\n")
    if PAIRED:
        pass
    elif GROUP > 1:
        glines = []
        gtotal = 0
        groups = [(r0, rows[r0:r0 + GROUP]) for r0 in range(0, m, GROUP)]
        for gi, (r0, grows) in enumerate(groups):
            gtotal += emit_group(code, gi, r0, grows, nx, glines)
        out.write(f"// the full network with pairs shared inside groups of {GROUP} rows: {gtotal} VALU ops per\n"
                  f"// 32-byte column (rows alone: {total})\n")
        out.write("\n".join(glines) + "\n\n")
        out.write(f"// rows 0 .. NR-1 in order ({nr_note}); emit(r, o) consumes row r's planes\n")
        out.write(f"template <int NR = {m}, class Emit>\n__device__ __forceinline__ void bs_net_{code}(const uint32_t (&x)[{nx}], Emit&& emit) {{\n")
        for gi, (r0, grows) in enumerate(groups):
            out.write(f"  if constexpr ({r0} < NR) bs_grp_{code}_{gi}<NR>(x, emit);\n")
        out.write("}\n\n")
    else:
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
    out.write(f"  static constexpr bool Paired = k{Name}Paired;  // inputs in the paired basis (see the top)\n")
    out.write(f"  static const uint8_t* rows() {{ return &k{Name}Rows[0][0]; }}\n")
    out.write(f"  template <int NR, class Emit>\n  __device__ static __forceinline__ void net(const uint32_t (&x)[{nx}], Emit&& emit) {{\n")
    out.write(f"    bs_net_{code}<NR>(x, static_cast<Emit&&>(emit));\n  }}\n}};\n\n")
    out.write("}  // namespace dev\n}  // namespace cfsec\n")


if __name__ == "__main__":
    main()
