// gf_k15.hip -- fixed-K (k = 15) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(15)
