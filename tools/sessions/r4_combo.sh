# Round 4 combined session (GPU pool congested): the sync-poll A/B with the GPU tests, then the C4
# checksum A/B.
set -e
bash tools/r4_sync_ab.sh
bash tools/r4_c4_crc_ab.sh
