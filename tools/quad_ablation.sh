# (Round-1 ablations of the textbook-CMUX kernel: its variant sources are not kept; the script records how
# profiles/r1/quad_ablation_r1o.txt was made.)
# Quad-kernel ablations (timing only: each variant removes one piece and so decrypts wrongly) plus
# the PBS tests and the latency sweep.  Variants: built with tools/build_variant.sh NAME SRC "" br_quad.
set -o pipefail
timeout -k 10 400 python -m pytest tests/test_pbs_gpu.py -x -q > gpurun_out/t_pbs.log 2>&1 || exit 1
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/latency_w3.txt 2>&1 || exit 2
timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 3 > gpurun_out/abl.txt 2>&1 || exit 3
for v in q_nobar7 q_norot q_nobsk q_nost9 q_notw; do
  timeout -k 10 120 python tools/variant_probe.py build_variants/$v 8192 3 >> gpurun_out/abl.txt 2>&1 || exit 4
done
