// gf_dy_k6.hip -- 2x2-dyadic kernels for k = 6 (EC6P6, EC6P10, EC6P10L2 global parities and their
// coset-aligned repairs); see gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

CFSEC_DY_INSTANTIATE(6, 2, 6, 8, 10, 12)
