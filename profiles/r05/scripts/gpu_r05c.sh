# the device-resident line searches: GPU tests, the A/B at n = 1e4 / 1e5, a
# seeded soak against the oracle; the vector-free layout probe with the product's 256-B offset
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r05c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_device_search.py tests/test_gpu_coop_safety.py tests/test_gpu_speculative.py tests/test_gpu_knobs.py > gpurun_out/r05c/pytest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05c/smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/search_ab.py 1e4 gpurun_out/r05c/search_ab_n1e4.json > gpurun_out/r05c/search_ab_n1e4.txt 2>&1 &&
timeout -k 10 300 python -u tools/search_ab.py 1e5 gpurun_out/r05c/search_ab_n1e5.json > gpurun_out/r05c/search_ab_n1e5.txt 2>&1 &&
timeout -k 10 600 python -u tools/search_soak.py 300 gpurun_out/r05c/search_soak_300.json > gpurun_out/r05c/search_soak.txt 2>&1 &&
timeout -k 10 120 tools/vfilprobe > gpurun_out/r05c/vfilprobe_n1e8.txt 2>&1
