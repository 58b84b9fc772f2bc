// gf_k7.hip -- fixed-K (k = 7) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(7)
