# seeded soak of the slot fetches that poll a k_slot_publish word (tools/fetch_soak.py) against the
# oracle's canonical restatement, bit for bit
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/soak
timeout -k 10 800 python -u tools/fetch_soak.py 150 gpurun_out/soak/fetch_soak_150.json > gpurun_out/soak/fetch_soak.txt 2>&1
