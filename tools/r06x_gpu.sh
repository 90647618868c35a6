# round 6: the driver's multi-rank bench flow rehearsed with 4 ranks on the one GPU (final tree)
set -eo pipefail
bash tools/rehearse_multi.sh 4
