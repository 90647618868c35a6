#!/bin/bash
# Round-4 A/B session (one GPU box): the upload-stream layouts (tools/ab_queues.sh, one pass) and the NTT / evaluator
# kernel variants at 2^20 (tools/ab_variants.sh, alternating), each bench line with --ab.
set -o pipefail
O=gpurun_out
mkdir -p $O
AB_REPS=${AB_REPS:-3} bash tools/ab_queues.sh > $O/ab_queues.txt 2>&1; cat $O/ab_queues.txt
BENCH_ARGS="--ab" bash tools/ab_variants.sh base glast nostash grp2 base glast nostash grp2 base glast nostash grp2 > $O/ab_kernels.txt 2>&1
cat $O/ab_kernels.txt
