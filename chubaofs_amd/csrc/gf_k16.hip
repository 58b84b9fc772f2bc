// gf_k16.hip -- fixed-K (k = 16) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(16)
