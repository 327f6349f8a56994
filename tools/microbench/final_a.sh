set -u
# final records A: smoke, GPU suite, C2 bench + profile + traffic, C1 bench, C2 PMC passes
cd /root/repo
bash tools/gpu_session.sh final_a bench_c1 pmcall || exit $?
