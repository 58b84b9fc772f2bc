// gf_lut_k15.hip -- lookup-product kernels for k = 15 (m = 5..12); see gf_lut.hpp.
#include "gf_lut_inst.hpp"

namespace cfsec {
template <>
hipError_t launch_lut_k<15>(int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (m) {
    case 5: return lutinst::go<15, 5>(mode, a, grid, st);
    case 6: return lutinst::go<15, 6>(mode, a, grid, st);
    case 7: return lutinst::go<15, 7>(mode, a, grid, st);
    case 8: return lutinst::go<15, 8>(mode, a, grid, st);
    case 9: return lutinst::go<15, 9>(mode, a, grid, st);
    case 10: return lutinst::go<15, 10>(mode, a, grid, st);
    case 11: return lutinst::go<15, 11>(mode, a, grid, st);
    case 12: return lutinst::go<15, 12>(mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cfsec
