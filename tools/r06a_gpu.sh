set -o pipefail
O=gpurun_out
timeout -k 10 120 ./tools/ubench/addsub_lab > $O/r06a_addsub_lab.txt 2>&1 && cat $O/r06a_addsub_lab.txt &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r06a_gpu_tests.log 2>&1 && tail -1 $O/r06a_gpu_tests.log &&
AB_STEPS=30 bash tools/ab_variants.sh base noasm base noasm base noasm > $O/r06a_ab_addsub.txt 2>&1; cat $O/r06a_ab_addsub.txt
