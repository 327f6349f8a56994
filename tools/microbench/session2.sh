set -u
cd /root/repo
tools/microbench/run_rb.sh rb_new rb_full rb_fullplain || exit 1
cd tools/microbench && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d ../../gpurun_out/fetch_cal -o run -- ./fetch_cal > ../../gpurun_out/fetch_cal.log 2>&1; echo "fetch_cal rc=$?"
cd /root/repo && bash tools/gpu_session.sh c5sim
tools/microbench/run_rb.sh rb_synth rb_synthnost
bash tools/microbench/session3.sh
