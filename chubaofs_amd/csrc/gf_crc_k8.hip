// gf_crc_k8.hip -- fused matvec + CRC kernels for k = 8; see gf_crc.hpp.
#include "gf_crc.hpp"

CFSEC_CRC_INSTANTIATE(8)
