// gf_lut_k16.hip -- lookup-product kernels for k = 16 (m = 5..16); see gf_lut.hpp.
#include "gf_lut_inst.hpp"

namespace cfsec {
template <>
hipError_t launch_lut_k<16>(int m, MatVecMode mode, const dev::GfArgs& a, dim3 grid, hipStream_t st) {
  switch (m) {
    case 5: return lutinst::go<16, 5>(mode, a, grid, st);
    case 6: return lutinst::go<16, 6>(mode, a, grid, st);
    case 7: return lutinst::go<16, 7>(mode, a, grid, st);
    case 8: return lutinst::go<16, 8>(mode, a, grid, st);
    case 9: return lutinst::go<16, 9>(mode, a, grid, st);
    case 10: return lutinst::go<16, 10>(mode, a, grid, st);
    case 11: return lutinst::go<16, 11>(mode, a, grid, st);
    case 12: return lutinst::go<16, 12>(mode, a, grid, st);
    case 13: return lutinst::go<16, 13>(mode, a, grid, st);
    case 14: return lutinst::go<16, 14>(mode, a, grid, st);
    case 15: return lutinst::go<16, 15>(mode, a, grid, st);
    case 16: return lutinst::go<16, 16>(mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace cfsec
