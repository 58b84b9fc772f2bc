// gf_dy_k6.hip -- 2x2-dyadic kernels for k = 6: EC6P6 / EC6P10 encode, their coset-aligned
// repairs, and the EC6P10L2 fused encode (10 dyadic global rows + 2 local rows); see gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

namespace cfsec {
template <>
hipError_t launch_dy<6>(int m, int B, int E, MatVecMode mode, const dev::GfArgs& a, unsigned ns, hipStream_t st) {
  return dy_dispatch<6, 2>(Ms<6, 8, 10, 12>{}, Ms<12>{}, m, B, E, mode, a, ns, st);
}
}  // namespace cfsec
