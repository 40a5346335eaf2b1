set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 600 python3 -u -m pytest tests/test_radix_gpu.py tests/test_sign_gpu.py tests/test_fanout_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5c/tests.txt 2>&1 || { tail -40 gpurun_out/r5c/tests.txt; exit 2; }
tail -3 gpurun_out/r5c/tests.txt
timeout -k 10 600 python3 -u tools/compat_ab.py 3 > gpurun_out/r5c/compat_ab.txt 2>&1 || { tail -30 gpurun_out/r5c/compat_ab.txt; exit 3; }
tail -8 gpurun_out/r5c/compat_ab.txt
