// gf_dy_k16.hip -- 4x4-dyadic kernels for k = 16: EC16P4 / EC16P20 encode, their coset-aligned
// repairs, and the EC16P20L2 fused encode (20 dyadic global rows + 2 local rows); see gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

namespace cfsec {
template <>
hipError_t launch_dy<16>(int m, int B, int E, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  return dy_dispatch<16, 4>(Ms<4, 8, 12, 16, 20>{}, Ms<22>{}, m, B, E, mode, a, ns, st);
}
}  // namespace cfsec
