# round 6: addsub asm lab + full GPU suite + A/B of the interleaved add/sub against the compiler's chains
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 120 ./tools/ubench/addsub_lab > $O/r06a_addsub_lab.txt 2>&1 || { cat $O/r06a_addsub_lab.txt; exit 1; }
cat $O/r06a_addsub_lab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/r06a_gpu_tests.log 2>&1
rc=$?
tail -30 $O/r06a_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
AB_STEPS=30 bash tools/ab_variants.sh base noasm base noasm base noasm > $O/r06a_ab_addsub.txt 2>&1
cat $O/r06a_ab_addsub.txt
