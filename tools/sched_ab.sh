# Same-box A/B of throughput-kernel variants (build_variants/*: tools/build_variant.sh) + the variant's
# bit-exactness (tests/test_pbs_gpu.py against its library); output gpurun_out/qpair_ab.txt
set -o pipefail
O=gpurun_out/qpair_ab.txt
FHE_ROCM_LIB=$PWD/build_variants/qpair/lib/libfhe_rocm.so timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || exit 3
for r in 1 2; do
for v in fhe-sign_amd build_variants/qpair; do timeout -k 10 150 python3 tools/variant_probe.py $v 32768 3 >> $O 2>&1 || exit 2; done
done
