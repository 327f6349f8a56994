set -u
# A/B: keys prefetched two batches ahead (rb_d2 / pb_d2) against one (rb_cur / pb_cur)
cd /root/repo
rm -f gpurun_out/rb.txt gpurun_out/pb8.txt
tools/microbench/run_rb.sh rb_cur rb_d2 rb_cur rb_d2 || exit 1
cd tools/microbench
for b in pb_cur pb_d2 pb_cur pb_d2; do
  echo "== $b" >> ../../gpurun_out/pb8.txt
  timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb8.txt 2>&1 || { echo "$b rc=$?"; cat ../../gpurun_out/pb8.txt; exit 1; }
done
cat ../../gpurun_out/pb8.txt
