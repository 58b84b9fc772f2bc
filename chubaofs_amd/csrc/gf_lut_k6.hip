// gf_lut_k6.hip -- lookup-product kernels for k = 6 (m = 5..12); see gf_lut.hpp.
#include "gf_lut_inst.hpp"

namespace cfsec {
template <>
hipError_t launch_lut_k<6>(int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (m) {
    case 5: return lutinst::go<6, 5>(mode, a, grid, st);
    case 6: return lutinst::go<6, 6>(mode, a, grid, st);
    case 7: return lutinst::go<6, 7>(mode, a, grid, st);
    case 8: return lutinst::go<6, 8>(mode, a, grid, st);
    case 9: return lutinst::go<6, 9>(mode, a, grid, st);
    case 10: return lutinst::go<6, 10>(mode, a, grid, st);
    case 11: return lutinst::go<6, 11>(mode, a, grid, st);
    case 12: return lutinst::go<6, 12>(mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cfsec
