set -u
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_fanout_gpu.py -k world2 > gpurun_out/r6c_world2.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_pbs_gpu.py::test_noise_budget_lwe_bound tests/test_noise_gpu.py > gpurun_out/r6c_noise.txt 2>&1
rc2=$?; if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python -u tools/fanout_projection.py 1 2 4 8 > gpurun_out/r6c_fanout_projection.txt 2>&1
