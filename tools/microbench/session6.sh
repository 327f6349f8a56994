set -u
# A/B: tile index by bit-field extract (rb_bfe vs rb_nobfe); gather with branch-free LDS ANDs
# (pb_gbf vs pb_gbr); then the per-key latency and headline benches on the library with both
cd /root/repo
rm -f gpurun_out/rb.txt gpurun_out/pb6.txt
tools/microbench/run_rb.sh rb_nobfe rb_bfe rb_nobfe rb_bfe || exit 1
cd tools/microbench
for b in pb_gbr pb_gbf pb_gbr pb_gbf; do
  echo "== $b" >> ../../gpurun_out/pb6.txt
  timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb6.txt 2>&1 || { echo "$b rc=$?"; cat ../../gpurun_out/pb6.txt; exit 1; }
done
cat ../../gpurun_out/pb6.txt
cd /root/repo
bash tools/gpu_session.sh bench_c1 bench
