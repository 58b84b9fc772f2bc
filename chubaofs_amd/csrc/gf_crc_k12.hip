// gf_crc_k12.hip -- fused matvec + CRC kernels for k = 12; see gf_crc.hpp.
#include "gf_crc.hpp"

CFSEC_CRC_INSTANTIATE(12)
