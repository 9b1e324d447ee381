# the two fetch-soak mismatches (quad_sep, Wolfe) in detail (tools/fetch_case.py)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/soak
timeout -k 10 300 python -u tools/fetch_case.py 1829114 2 quad_sep wolfe 24 722348 > gpurun_out/soak/case21.txt 2>&1 &&
timeout -k 10 300 python -u tools/fetch_case.py 617189 20 quad_sep wolfe 13 398147 > gpurun_out/soak/case26.txt 2>&1
