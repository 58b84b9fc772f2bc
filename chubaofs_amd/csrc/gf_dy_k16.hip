// gf_dy_k16.hip -- 4x4-dyadic kernels for k = 16 (EC16P4, EC16P20); see gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

CFSEC_DY_INSTANTIATE(16, 4, 4, 8, 12, 16, 20)
