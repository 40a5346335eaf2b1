set -u
for r in 1 2 3; do
  for K in 5 6; do timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd $K 32768 3 || exit $?; done
done
