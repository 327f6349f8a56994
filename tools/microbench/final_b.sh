set -u
# final records B: PMC traffic of C3 / C4 / C5, C3 and C4 benches
cd /root/repo
bash tools/gpu_session.sh final_b bench_c3 bench_c4 || exit $?
