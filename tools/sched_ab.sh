# Same-box A/B of latency-kernel variants (build_variants/*: tools/build_variant.sh); output gpurun_out/wpair_ab2.txt
set -o pipefail
O=gpurun_out/wpair_ab2.txt
for r in 1 2; do
for B in 1 128 256; do for v in fhe-sign_amd build_variants/wpair build_variants/wpair_def; do timeout -k 10 150 python3 tools/variant_probe.py $v $B 5 >> $O 2>&1 || exit 2; done; done
done
