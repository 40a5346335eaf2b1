# Same-box A/B of latency-kernel variants (build_variants/*: tools/build_variant.sh with EXTRA_FLAGS);
# output gpurun_out/sched_ab4.txt
set -o pipefail
O=gpurun_out/sched_ab4.txt
for r in 1 2; do
for B in 1 256; do for v in fhe-sign_amd build_variants/w1_p1 build_variants/w1_p2 build_variants/w1_p3; do timeout -k 10 150 python3 tools/variant_probe.py $v $B 5 >> $O 2>&1 || exit 2; done; done
done
