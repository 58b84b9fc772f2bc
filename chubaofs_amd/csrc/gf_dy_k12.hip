// gf_dy_k12.hip -- 4x4-dyadic kernels for k = 12 (EC12P4 encode and coset-aligned repairs); see
// gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

namespace cfsec {
template <>
hipError_t launch_dy<12>(int m, int B, int E, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  return dy_dispatch<12, 4>(Ms<4, 8, 12>{}, Ms<>{}, m, B, E, mode, a, ns, st);
}
}  // namespace cfsec
