// gf_k3.hip -- fixed-K (k = 3) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(3)
