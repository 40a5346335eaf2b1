# Same-box A/B of throughput-kernel variants (build_variants/*: tools/build_variant.sh); output gpurun_out/stag_ab.txt
set -o pipefail
O=gpurun_out/stag_ab.txt
for r in 1 2; do
for B in 768 1536 5200 32768; do for v in fhe-sign_amd build_variants/stag4 build_variants/stag8; do R=5; [ $B = 32768 ] && R=2; timeout -k 10 150 python3 tools/variant_probe.py $v $B $R >> $O 2>&1 || exit 2; done; done
done
