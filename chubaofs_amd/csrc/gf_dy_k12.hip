// gf_dy_k12.hip -- 4x4-dyadic kernels for k = 12 (EC12P4 encode and coset-aligned repairs); see
// gf_dyadic.hpp.
#include "gf_dy_fixed.hpp"

CFSEC_DY_INSTANTIATE(12, 4, 4, 8, 12)
