set -u
for r in 1 2; do
  for B in 512 1536 32768; do
    timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd 4 $B 3 || exit $?
    for v in qy_q1 qy_q2; do timeout -k 10 120 python -u tools/qy2_probe.py build_variants/$v 4 $B 3 || exit $?; done
  done
done
