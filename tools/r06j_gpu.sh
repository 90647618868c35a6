# round 6: the coset pass 1's two-part inter-pass twiddle -- parity, then A/B against the fe_mul form
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r06j_parity.log 2>&1
rc=$?
tail -3 $O/r06j_parity.log
if [ $rc -ne 0 ]; then echo "parity rc=$rc: stopping"; exit $rc; fi
AB_STEPS=60 bash tools/ab_variants.sh base nopw2 base nopw2 base nopw2 > $O/r06j_ab_pass_w2.txt 2>&1
cat $O/r06j_ab_pass_w2.txt
