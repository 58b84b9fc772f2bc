// gf_k6.hip -- fixed-K (k = 6) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(6)
