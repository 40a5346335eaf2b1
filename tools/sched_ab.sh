# Same-box A/B of latency-kernel variants (build_variants/*: tools/build_variant.sh) + the variant's
# bit-exactness (tests/test_pbs_gpu.py against its library); output gpurun_out/wsplit2_ab.txt
set -o pipefail
O=gpurun_out/wsplit2_ab.txt
FHE_ROCM_LIB=$PWD/build_variants/wsplit2/lib/libfhe_rocm.so timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || exit 3
for r in 1 2; do
for mb in 1 0; do for B in 1 256; do for v in fhe-sign_amd build_variants/wsplit2; do FHE_PROBE_MB=$mb timeout -k 10 150 python3 tools/variant_probe.py $v $B 5 >> $O 2>&1 || exit 2; done; done; done
done
