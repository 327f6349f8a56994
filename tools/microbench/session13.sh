set -u
# C5 set tile test: PMC counter passes (pipeline issue / LDS / L2 picture of k_tile_probe_set)
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 tools/pmc_passes.sh gpurun_out/pmc_c5 --config c5 --no-host-c5 --no-compare || exit $?
python tools/pmc_summary.py gpurun_out/pmc_c5 > gpurun_out/pmc_c5_summary.txt 2>&1; head -60 gpurun_out/pmc_c5_summary.txt
