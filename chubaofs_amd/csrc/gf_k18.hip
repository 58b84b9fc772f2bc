// gf_k18.hip -- fixed-K (k = 18) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(18)
