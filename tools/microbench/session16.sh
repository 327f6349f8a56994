set -u
# tile test words in flight per wave: 8 (default) vs 12 (build/variants/u12.so), C2 and C5
cd /root/repo
bash tools/gpu_session.sh ab ab_c5 || exit $?
