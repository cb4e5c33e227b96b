# ring A/B of library variants, interleaved, 2 rounds: tools/ab_ring_libs.sh "<windows>" lib...
set -o pipefail
W=$1; shift
bash tools/ab_ring.sh "--batches 6000 --depths 8 --groups 4 --window-abs $W" "$@"
