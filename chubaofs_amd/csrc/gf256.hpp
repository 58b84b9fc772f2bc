// gf256.hpp -- host-side GF(2^8) arithmetic and matrix algebra for the engine.
//
// Field: polynomial 0x11D (KRS/galois.go:25, generatingPolynomial = 29).
// Matrix algebra follows KRS/matrix.go: vandermonde (:271-282), Multiply
// (:103-118), Invert via Gauss-Jordan with pivot swap (:193-266).  All of this
// is O(n^3) on <= 38x38 byte matrices and runs once per code mode / erasure
// pattern; the shard bytes never touch the host.
#pragma once
#include <array>
#include <cstdint>
#include <vector>

namespace cfsec {

class GF {
 public:
  static const GF& get() {
    static const GF g;
    return g;
  }
  uint8_t mul(uint8_t a, uint8_t b) const { return mul_[a][b]; }
  // galDivide (KRS/galois.go:873-887); b != 0.
  uint8_t div(uint8_t a, uint8_t b) const {
    if (a == 0) return 0;
    int r = int(log_[a]) - int(log_[b]);
    if (r < 0) r += 255;
    return exp_[r];
  }
  // galExp (KRS/galois.go:892-906): a^0 == 1 even for a == 0.
  uint8_t pow(uint8_t a, int n) const {
    if (n == 0) return 1;
    if (a == 0) return 0;
    int r = int(log_[a]) * n;
    r %= 255;
    return exp_[r];
  }

 private:
  GF() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp_[i] = exp_[i + 255] = uint8_t(x);
      log_[x] = uint8_t(i);
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    log_[0] = 0;
    for (int a = 0; a < 256; ++a)
      for (int b = 0; b < 256; ++b)
        mul_[a][b] = (a == 0 || b == 0) ? 0 : exp_[log_[a] + log_[b]];
  }
  std::array<uint8_t, 256> log_{};
  std::array<uint8_t, 510> exp_{};
  uint8_t mul_[256][256]{};
};

// Row-major byte matrix.
struct Matrix {
  int rows = 0, cols = 0;
  std::vector<uint8_t> v;
  Matrix() = default;
  Matrix(int r, int c) : rows(r), cols(c), v(size_t(r) * c, 0) {}
  uint8_t* row(int r) { return v.data() + size_t(r) * cols; }
  const uint8_t* row(int r) const { return v.data() + size_t(r) * cols; }
  uint8_t& at(int r, int c) { return v[size_t(r) * cols + c]; }
  uint8_t at(int r, int c) const { return v[size_t(r) * cols + c]; }
};

inline Matrix mat_mul(const Matrix& a, const Matrix& b) {
  const GF& gf = GF::get();
  Matrix out(a.rows, b.cols);
  for (int r = 0; r < a.rows; ++r)
    for (int c = 0; c < b.cols; ++c) {
      uint8_t v = 0;
      for (int i = 0; i < a.cols; ++i) v ^= gf.mul(a.at(r, i), b.at(i, c));
      out.at(r, c) = v;
    }
  return out;
}

// Returns false when singular (errSingular, KRS/matrix.go:185).
inline bool mat_invert(const Matrix& m, Matrix& inv) {
  const GF& gf = GF::get();
  const int n = m.rows;
  Matrix w(n, 2 * n);
  for (int r = 0; r < n; ++r) {
    for (int c = 0; c < n; ++c) w.at(r, c) = m.at(r, c);
    w.at(r, n + r) = 1;
  }
  const int cols = 2 * n;
  for (int r = 0; r < n; ++r) {
    if (w.at(r, r) == 0) {
      for (int below = r + 1; below < n; ++below)
        if (w.at(below, r) != 0) {
          for (int c = 0; c < cols; ++c) std::swap(w.at(r, c), w.at(below, c));
          break;
        }
    }
    if (w.at(r, r) == 0) return false;
    if (w.at(r, r) != 1) {
      const uint8_t s = gf.div(1, w.at(r, r));
      for (int c = 0; c < cols; ++c) w.at(r, c) = gf.mul(w.at(r, c), s);
    }
    for (int below = r + 1; below < n; ++below) {
      const uint8_t s = w.at(below, r);
      if (s)
        for (int c = 0; c < cols; ++c) w.at(below, c) ^= gf.mul(s, w.at(r, c));
    }
  }
  for (int d = 0; d < n; ++d)
    for (int above = 0; above < d; ++above) {
      const uint8_t s = w.at(above, d);
      if (s)
        for (int c = 0; c < cols; ++c) w.at(above, c) ^= gf.mul(s, w.at(d, c));
    }
  inv = Matrix(n, n);
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) inv.at(r, c) = w.at(r, n + c);
  return true;
}

// buildMatrix (KRS/reedsolomon.go:220-244): vandermonde(total, k) * inv(top k x k).
inline bool build_matrix(int k, int total, Matrix& out) {
  const GF& gf = GF::get();
  Matrix vm(total, k);
  for (int r = 0; r < total; ++r)
    for (int c = 0; c < k; ++c) vm.at(r, c) = gf.pow(uint8_t(r), c);
  Matrix top(k, k);
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) top.at(r, c) = vm.at(r, c);
  Matrix top_inv;
  if (!mat_invert(top, top_inv)) return false;
  out = mat_mul(vm, top_inv);
  return true;
}

}  // namespace cfsec
