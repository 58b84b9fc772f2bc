// gf_lut_k12.hip -- lookup-product kernels for k = 12 (m = 5..9); see gf_lut.hpp.
#include "gf_lut_inst.hpp"

namespace cfsec {
template <>
hipError_t launch_lut_k<12>(int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (m) {
    case 5: return lutinst::go<12, 5>(mode, a, grid, st);
    case 6: return lutinst::go<12, 6>(mode, a, grid, st);
    case 7: return lutinst::go<12, 7>(mode, a, grid, st);
    case 8: return lutinst::go<12, 8>(mode, a, grid, st);
    case 9: return lutinst::go<12, 9>(mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cfsec
