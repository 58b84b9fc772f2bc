// gf_crc_k6.hip -- fused matvec + CRC kernels for k = 6; see gf_crc.hpp.
#include "gf_crc.hpp"

CFSEC_CRC_INSTANTIATE(6)
