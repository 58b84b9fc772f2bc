// gf_k4.hip -- fixed-K (k = 4) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(4)
