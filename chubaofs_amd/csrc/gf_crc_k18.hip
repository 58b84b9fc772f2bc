// gf_crc_k18.hip -- fused matvec + CRC kernels for k = 18; see gf_crc.hpp.
#include "gf_crc.hpp"

CFSEC_CRC_INSTANTIATE(18)
