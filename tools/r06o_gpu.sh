# round 6: the lead-only window of one sharded 2^22 proof at G = 8 (kernel trace)
set -eo pipefail
R=$(pwd); O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/lead_g8 -o k -- python3 $R/tools/shard_kernels.py 22 8 device 2 > $O/lead_g8.log 2>&1
python3 $R/tools/lead_window.py $(ls $O/lead_g8/*kernel_trace.csv | head -1) > $O/r06o_lead_window_g8.txt
cat $O/r06o_lead_window_g8.txt
find $O/lead_g8 -name '*kernel_trace.csv' -delete
