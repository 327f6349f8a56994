set -u
# gather: quads per lane x regions in flight (pb_q1u4 = shipped, pb_q2u2, pb_q4u1), alternated;
# then the multi-rank launch rehearsal on the final library (all ranks on device 0 over gloo)
cd /root/repo/tools/microbench
rm -f ../../gpurun_out/pb10.txt
for b in pb_q1u4 pb_q2u2 pb_q4u1 pb_q1u4 pb_q2u2 pb_q4u1; do
  echo "== $b" >> ../../gpurun_out/pb10.txt
  timeout -k 5 120 ./$b 20 >> ../../gpurun_out/pb10.txt 2>&1 || { echo "$b rc=$?"; cat ../../gpurun_out/pb10.txt; exit 1; }
done
cat ../../gpurun_out/pb10.txt
cd /root/repo
bash tools/gpu_session.sh selflaunch
