set -u
for r in 1 2 3; do
  for B in 512 1536 32768; do
    timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd 4 $B 3 || exit $?
    timeout -k 10 120 python -u tools/qy2_probe.py build_variants/qy_p1 4 $B 3 || exit $?
  done
done
