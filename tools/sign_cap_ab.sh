# A/B of the signer with the first compression round capped (CAP0: an environment hook of the A/B build only,
# since removed -- the product always caps) and qy vs qy2 at 1012 bootstraps.
set -u
for r in 1 2 3; do
  for c in 0 4; do CAP0=$c timeout -k 10 100 python3 tools/sign_probe.py 2>&1 | grep "sign_fhe_with_k0" | sed "s/^/cap$c /" || exit $?; done
done
for r in 1 2; do for K in 4 5; do timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd $K 1012 3 || exit $?; done; done
