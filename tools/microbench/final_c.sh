set -u
# final records C: C5 / C5mixed / SSTable benches, C3 / C4 / C5 profiles, multi-rank rehearsal
cd /root/repo
bash tools/gpu_session.sh bench_c5 bench_c5mixed bench_sst final_d || exit $?
export PBF_BENCH_DEVICE=0 PBF_BENCH_BACKEND=gloo
cd /root/repo && mkdir -p gpurun_out && timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-host-c5 > gpurun_out/sl_c5_n2.log 2>&1; echo "sl_c5_n2 rc=$?"
