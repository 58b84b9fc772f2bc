// gf_k8.hip -- fixed-K (k = 8) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(8)
