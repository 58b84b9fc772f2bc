// gf_k12.hip -- fixed-K (k = 12) GF matvec kernels; see gf_fixed.hpp.
#include "gf_fixed.hpp"

CFSEC_INSTANTIATE_K(12)
