// gf_k10.hip -- fixed-K (k = 10) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(10)
