set -u
# tile test without fill masking, packed u16 table, DPP result words: GPU suite, then A/B
# against the previous sources (build/variants/base.so) on C2, C5 and C3
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/t14.log 2>&1
rc=$?; tail -5 gpurun_out/t14.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_session.sh ab1 ab_c5 ab_c3
