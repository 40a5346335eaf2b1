# Same-box A/B of machine-scheduler strategy variants (build_variants/quad_mr, wide_*: tools/build_variant.sh with
# EXTRA_FLAGS="-mllvm -amdgpu-sched-strategy=..."); output gpurun_out/sched_ab2.txt
set -o pipefail
O=gpurun_out/sched_ab2.txt
for r in 1 2; do
for mb in 0 1; do for B in 1 256; do for v in fhe-sign_amd build_variants/wide_mi build_variants/wide_mi2; do FHE_PROBE_MB=$mb timeout -k 10 150 python3 tools/variant_probe.py $v $B 5 >> $O 2>&1 || exit 2; done; done; done
done
