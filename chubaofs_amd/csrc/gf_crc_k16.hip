// gf_crc_k16.hip -- fused matvec + CRC kernels for k = 16; see gf_crc.hpp.
#include "gf_crc.hpp"

CFSEC_CRC_INSTANTIATE(16)
