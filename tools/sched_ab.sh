# Same-box A/B of throughput-kernel variants (build_variants/*: tools/build_variant.sh); output gpurun_out/qpst_ab.txt
set -o pipefail
O=gpurun_out/qpst_ab.txt
for r in 1 2; do
for mb in 0 1; do for v in fhe-sign_amd build_variants/qpst; do FHE_PROBE_MB=$mb timeout -k 10 150 python3 tools/variant_probe.py $v 32768 3 >> $O 2>&1 || exit 2; done; done
done
