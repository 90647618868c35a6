# round 6: per-kernel time of one sharded 2^22 proof at G = 8 and G = 2 (loopback, measurement mode), and the
# single-GPU 2^22 proof's kernels for comparison
set -eo pipefail
R=$(pwd); O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for G in 8 2; do
  for np in 1 3; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shk_g${G}_$np -o k -- \
      python3 $R/tools/shard_kernels.py 22 $G device $np > $O/shk_g${G}_$np.log 2>&1
  done
  python3 $R/tools/shard_kernels.py --diff $O/shk_g${G}_1/k_kernel_stats.csv $O/shk_g${G}_3/k_kernel_stats.csv $G > $O/r06h_shard_kernels_g$G.txt
  head -30 $O/r06h_shard_kernels_g$G.txt
  find $O/shk_g${G}_1 $O/shk_g${G}_3 -name '*kernel_trace.csv' -delete
done
