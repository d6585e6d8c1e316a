# Round-4: in-workgroup k-groups for the glds GEMM (tiles 19-21) - tests, then the fc1 sweep.
set -o pipefail
O=gpurun_out/r4kg
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_glds_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python3 bench/gemm_sweep.py --iters 30 --tiles 8,12,14,19,20,21 > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
grep -v amdgpu.ids $O/sweep.txt
